# A/B: the early cut's LDS window (SHEEP_BIG_HOT_BITS 15 / 14 / 13: one or two workgroups
# per CU), 2^20 and 2^19 cuts.  gpurun_out/r4hot/.
set -o pipefail
mkdir -p gpurun_out/r4hot && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4hot
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
SHEEP_BIG_HOT_BITS=13 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/h15.json 2> $O/h15.err || exit 1
SHEEP_BIG_HOT_BITS=14 timeout -k 10 200 $B > $O/h14.json 2> $O/h14.err || exit 1
SHEEP_BIG_HOT_BITS=13 timeout -k 10 200 $B > $O/h13.json 2> $O/h13.err || exit 1
SHEEP_BIG_BITS=19 SHEEP_BIG_HOT_BITS=14 timeout -k 10 200 $B > $O/b19h14.json 2> $O/b19h14.err || exit 1
