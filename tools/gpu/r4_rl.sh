# A/B: the relabel's staged scatter (default) against the direct LDS-cursor scatter
# (SHEEP_RELABEL_DIRECT=1: 512 threads x 8, =2: 256 x 16).  gpurun_out/r4rl/.
set -o pipefail
mkdir -p gpurun_out/r4rl && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4rl
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
SHEEP_RELABEL_DIRECT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_d1.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/d0.json 2> $O/d0.err || exit 1
SHEEP_RELABEL_DIRECT=1 timeout -k 10 200 $B > $O/d1.json 2> $O/d1.err || exit 1
SHEEP_RELABEL_DIRECT=2 timeout -k 10 200 $B > $O/d2.json 2> $O/d2.err || exit 1
SHEEP_RELABEL_DIRECT=1 timeout -k 10 200 $B --shuffle > $O/d1_shuf.json 2> $O/d1_shuf.err || exit 1
timeout -k 10 200 $B --shuffle > $O/d0_shuf.json 2> $O/d0_shuf.err || exit 1
