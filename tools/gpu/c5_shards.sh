# C5 (RMAT-28 ef16, k = 256) on one GPU with fewer, larger edge shards: 4 shards (1.06 G
# records each, the size of the whole RMAT-26 graph) on 1 and 2 streams, and 2 shards.
# Every line checks its merged tree against the pairwise merges of the same shard trees.
# gpurun_out/$OUT/.
set -o pipefail
OUT=${OUT:-c5s}
O=gpurun_out/$OUT
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
for cfg in "4 1" "4 2" "2 1"; do
  set -- $cfg
  timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards $1 --streams $2 --steps 2 --warmup 1 \
    --no-cpu-baseline --eval-reps 1 > $O/c5_sh$1_st$2.json 2> $O/c5_sh$1_st$2.err || exit 1
done
