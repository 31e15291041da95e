# Round-4 measurement set, part 2: C4, C5, shuffled C3, a 2-rank rehearsal on one GPU,
# SQ counters of the bucket passes and level kernels.
set -o pipefail
mkdir -p gpurun_out/r4res && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
O=gpurun_out/r4res
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 200 $B --shards 8 --tune fin_merge_bits=13 > $O/ab_s8_merge13.json 2> $O/ab_s8_merge13.err || exit 1
timeout -k 10 200 $B --scale 22 --k 16 --steps 20 --tune fin_map_bits=12 > $O/ab_b22_fin12.json 2> $O/ab_b22_fin12.err || exit 1
timeout -k 10 400 python -u bench.py --shuffle --steps 5 --no-cpu-baseline > $O/bench_rmat26_k64_shuffled.json 2> $O/shuf.err || exit 1
timeout -k 10 500 python -u bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline > $O/bench_c4_powerlaw_k128.json 2> $O/c4.err || exit 1
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/bench_c5_rmat28_k256_8shards.json 2> $O/c5.err || exit 1
timeout -k 10 300 python -u bench.py --scale 26 --k 64 --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 0 \
  > $O/bench_rmat26_k64_8shards.json 2> $O/s8.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/bench_rehearsal_2ranks_rmat24.json 2> $O/reh.err || exit 1
W=26 bash tools/gpu/gpupmc2.sh || exit 1
