# The early MSF cut with LDS has-upper windows: parity, 2^20 (default) / 2^19 / off, 8 shards, a
# kernel trace of the default.  gpurun_out/r4big3/.
set -o pipefail
mkdir -p gpurun_out/r4big3 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4big3
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/b20.json 2> $O/b20.err || exit 1
SHEEP_BIG_BITS=19 timeout -k 10 200 $B > $O/b19.json 2> $O/b19.err || exit 1
SHEEP_BIG_BITS=0 timeout -k 10 200 $B > $O/off.json 2> $O/off.err || exit 1
timeout -k 10 200 $B --shards 8 > $O/s8_def.json 2> $O/s8_def.err || exit 1
timeout -k 10 400 python -u bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline --eval-reps 0 > $O/c4.json 2> $O/c4.err || exit 1
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify > t.log 2>&1 || exit 1
python ../../tools/trace_step.py $(find t -name '*kernel_trace.csv' | head -1) --levels > step.txt || exit 1
rm -rf t
