set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e2.log 2>&1 || exit 1
$T 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 1 --warmup 1 --no-cpu-baseline --eval-reps 0 > gpurun_out/b5.log 2> gpurun_out/b5.err || exit 1
