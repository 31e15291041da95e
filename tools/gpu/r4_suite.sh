# The GPU suite with the round-4 defaults, a default bench line and the top-block kernel trace.
set -o pipefail
mkdir -p gpurun_out/r4suite && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4suite
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b26.json 2> $O/b26.err || exit 1
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify > t.log 2>&1 || exit 1
python ../../tools/top_trace.py $(find t -name '*kernel_trace.csv' | head -1) > top_trace.txt || exit 1
python ../../tools/trace_step.py $(find t -name '*kernel_trace.csv' | head -1) --levels > step.txt || exit 1
rm -rf t
