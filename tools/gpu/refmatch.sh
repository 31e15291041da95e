# The reference lib/ flow on the bench's own records (--cpu-same-graph): C4 (Chung-Lu,
# 1.47 G records) and C5 (RMAT-28, 4.24 G records, 2 shards), each line's
# cpu_baseline.matches_gpu comparing the reference's sequence, tree and parts with the GPU's.
# gpurun_out/$OUT/.
set -o pipefail
O=gpurun_out/${OUT:-refmatch}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
if [ -n "$C4" ]; then
  timeout -k 10 900 python -u bench.py --graph powerlaw --k 128 --steps 2 --warmup 1 --eval-reps 1 --cpu-same-graph \
    --cpu-configs 16x1 > $O/c4.json 2> $O/c4.err || exit 1
fi
timeout -k 10 1080 python -u bench.py --scale 28 --k 256 --shards 2 --steps 2 --warmup 1 --eval-reps 1 --cpu-same-graph \
  --cpu-configs 8x1 > $O/c5.json 2> $O/c5.err || exit 1
