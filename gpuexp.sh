# A/B: fused degree pass vs k_degree + separate head count; GPU tests first
set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify > gpurun_out/b26f.log 2>&1 || exit 1
SHEEP_SPLIT_DEGREE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b26sd.log 2>&1 || exit 1
