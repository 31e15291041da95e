# Block-size distribution of the late etree levels (SHEEP_DEBUG_ETREE) at RMAT-26, 8 shards + merge, and C4.
set -o pipefail
mkdir -p gpurun_out/r4blocks && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/r4blocks
SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python ../../bench.py --scale 26 --k 64 --steps 1 --warmup 0 --eval-reps 0 \
  --no-cpu-baseline --no-verify > dbg26.json 2> dbg26.err || exit 1
SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python ../../bench.py --scale 26 --k 64 --shards 8 --steps 1 --warmup 0 --eval-reps 0 \
  --no-cpu-baseline --no-verify > dbg26s8.json 2> dbg26s8.err || exit 1
