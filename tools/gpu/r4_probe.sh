# Round-4 probe: per-level etree stats (SHEEP_DEBUG_ETREE) of the RMAT-26 map, of one
# 1/8 shard's map and of the 8-tree K-way merge; plus plain bench lines.  Output under
# gpurun_out/r4probe/.
set -o pipefail
mkdir -p gpurun_out/r4probe && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/r4probe
SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python ../../bench.py --scale 26 --k 64 --steps 1 --warmup 0 --eval-reps 0 \
  --no-cpu-baseline --no-verify > dbg26.json 2> dbg26.err || exit 1
SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python ../../bench.py --scale 26 --k 64 --shards 8 --steps 1 --warmup 0 --eval-reps 0 \
  --no-cpu-baseline --no-verify > dbg26s8.json 2> dbg26s8.err || exit 1
timeout -k 10 300 python ../../bench.py --scale 26 --k 64 --steps 5 --warmup 1 --eval-reps 1 --no-cpu-baseline \
  > b26.json 2> b26.err || exit 1
timeout -k 10 300 python ../../bench.py --scale 26 --k 64 --shards 8 --steps 3 --warmup 1 --eval-reps 0 --no-cpu-baseline \
  > b26s8.json 2> b26s8.err || exit 1
