set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt7.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify > gpurun_out/b26xa_$r.log 2>&1 || exit 1
done
