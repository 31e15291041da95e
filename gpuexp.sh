set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt9.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --scale 22 --k 16 --no-cpu-baseline > gpurun_out/b22t.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify > gpurun_out/b26t.log 2>&1 || exit 1
