# A/B: the early cut's hot window as u16 distances over 2^16 positions (SHEEP_BIG_HOT16)
# against u32 picks over 2^15.  gpurun_out/r4h16/.
set -o pipefail
mkdir -p gpurun_out/r4h16 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4h16
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
SHEEP_BIG_HOT16=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rmat or C3 or C4 or tree" > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/h15a.json 2> $O/h15a.err || exit 1
SHEEP_BIG_HOT16=1 timeout -k 10 200 $B > $O/h16a.json 2> $O/h16a.err || exit 1
timeout -k 10 200 $B > $O/h15b.json 2> $O/h15b.err || exit 1
SHEEP_BIG_HOT16=1 timeout -k 10 200 $B > $O/h16b.json 2> $O/h16b.err || exit 1
