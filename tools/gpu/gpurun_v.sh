# validate the current build: GPU tests, then RMAT-26 and RMAT-22 benches and a RMAT-22 kernel trace
set -o pipefail
mkdir -p gpurun_out/v && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v/tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/v/b26.json 2> gpurun_out/v/b26.err || exit 1
timeout -k 10 200 python bench.py --scale 22 --k 16 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/v/b22.json 2> gpurun_out/v/b22.err || exit 1
(cd gpurun_out/v && timeout -k 10 200 rocprofv3 --kernel-trace -d t22 -o run --output-format csv -- python ../../bench.py --scale 22 --k 16 --steps 2 --warmup 1 --eval-reps 1 --no-cpu-baseline > t22.log 2>&1) || exit 1
python tools/trace_step.py $(find gpurun_out/v/t22 -name '*kernel_trace.csv' | head -1) --levels > gpurun_out/v/step22.txt
