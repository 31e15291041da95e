# relabel sub-tile size sweep
set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
for p in 16 8 4; do
SHEEP_RL_PER=$p timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b26_per$p.log 2>&1 || exit 1
done
