set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e1.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/x26.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline > gpurun_out/x4.log 2>&1 || exit 1
