set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e2.log 2>&1 || exit 1
$T 300 python -u bench.py --steps 3 --no-cpu-baseline --eval-reps 0 > gpurun_out/b1.log 2> gpurun_out/b1.err || exit 1
$T 300 python -u bench.py --graph powerlaw --k 128 --steps 2 --no-cpu-baseline --eval-reps 0 > gpurun_out/b4.log 2> gpurun_out/b4.err || exit 1
