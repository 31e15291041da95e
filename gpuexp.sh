set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt8.log 2>&1 || exit 1
for r in 1 2; do for hb in 1 0; do
SHEEP_HOOK_BATCH=$hb timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify > gpurun_out/b26hb${hb}_$r.log 2>&1 || exit 1
done; done
