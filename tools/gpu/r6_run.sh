# Round-6 probe: the one-GPU shard forms with the shards' maps on 1 / 2 / 4 streams
# (bench.py --streams): the 8-shard RMAT-26 line and C5.
set -o pipefail
O=gpurun_out/r6/streams
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
for st in 1 2 4 2 1; do
  timeout -k 10 300 python -u bench.py --scale 26 --k 64 --shards 8 --streams $st --steps 3 --warmup 1 --no-cpu-baseline \
    --eval-reps 1 > $O/s8_st${st}_$RANDOM.json 2> $O/s8_st$st.err || exit 1
done
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --streams 2 --steps 2 --warmup 1 --no-cpu-baseline \
  --eval-reps 1 > $O/c5_st2.json 2> $O/c5_st2.err || exit 1
