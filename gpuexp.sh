# round-2 exploration: etree per-level stats at RMAT-26 and RMAT-22
set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
SHEEP_DEBUG_ETREE=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dbg26.log 2>&1 || exit 1
SHEEP_DEBUG_ETREE=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --scale 22 --k 16 --no-cpu-baseline > gpurun_out/dbg22.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b26.log 2>&1 || exit 1
