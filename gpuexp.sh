set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gt2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --eval-reps 1 > gpurun_out/b26.log 2>&1 || exit 1
cd gpurun_out && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks26 -o run --output-format csv -- python ../bench.py --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 > ks26.log 2>&1 || exit 1
