set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py tests/test_cli.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gt_all.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --eval-reps 1 > gpurun_out/new26.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --scale 22 --k 16 --steps 5 --no-cpu-baseline --eval-reps 1 > gpurun_out/new22.log 2>&1 || exit 1
