# The early MSF cut of the top subproblem: parity with it, then 2^18 / 2^19 / 2^20 / off;
# one map's level debug line; 8 shards.  gpurun_out/r4big/.
set -o pipefail
mkdir -p gpurun_out/r4big && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4big
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --eval-reps 0 --no-cpu-baseline --no-verify > $O/dbg.json 2> $O/dbg.err || exit 1
timeout -k 10 200 $B > $O/b19.json 2> $O/b19.err || exit 1
SHEEP_BIG_BITS=0 timeout -k 10 200 $B > $O/off.json 2> $O/off.err || exit 1
SHEEP_BIG_BITS=18 timeout -k 10 200 $B > $O/b18.json 2> $O/b18.err || exit 1
SHEEP_BIG_BITS=20 timeout -k 10 200 $B > $O/b20.json 2> $O/b20.err || exit 1
timeout -k 10 200 $B --shards 8 > $O/s8_b19.json 2> $O/s8_b19.err || exit 1
