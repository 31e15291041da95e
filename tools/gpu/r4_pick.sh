# The early cut with any-lower-neighbour picks (plain stores): the GPU suite, a bench line,
# 8 shards, C4 and a kernel trace.  gpurun_out/r4pick/.
set -o pipefail
mkdir -p gpurun_out/r4pick && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4pick
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/b20.json 2> $O/b20.err || exit 1
SHEEP_BIG_BITS=21 timeout -k 10 200 $B > $O/b21.json 2> $O/b21.err || exit 1
timeout -k 10 400 python -u bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline --eval-reps 0 > $O/c4.json 2> $O/c4.err || exit 1
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify > t.log 2>&1 || exit 1
python ../../tools/trace_step.py $(find t -name '*kernel_trace.csv' | head -1) --levels > step.txt || exit 1
rm -rf t
