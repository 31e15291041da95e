# Final measurement set, part 2 (see profiles/rN/README.md): the sparse-input etree
# phase by phase (one 1/8 shard map, the 8-tree merge, the binomial schedule's hops), the
# 8-shard RMAT-26 bench with one step's kernel trace (and with the maps on 2 streams), shuffled RMAT-26, C4, C5 and the
# 2-rank rehearsal.  gpurun_out/$FIN/.
set -o pipefail
R=$(pwd)
FIN=${FIN:-fin}
mkdir -p gpurun_out/$FIN/s8 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
O=gpurun_out/$FIN
OUT=$FIN/shard bash tools/gpu/shard_phases.sh || exit 1
cd $O/s8 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks -o run --output-format csv -- \
  python $R/bench.py --scale 26 --k 64 --shards 8 --steps 3 --warmup 1 --eval-reps 1 --no-cpu-baseline > ks.log 2>&1 || exit 1
python $R/tools/trace_step.py $(find ks -name '*kernel_trace.csv' | head -1) --levels > step_trace.txt || exit 1
cp $(find ks -name '*kernel_stats.csv' | head -1) kernel_stats.csv && rm -rf ks && cd $R || exit 1
timeout -k 10 300 python -u bench.py --scale 26 --k 64 --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/bench_rmat26_k64_8shards.json 2> $O/s8.err || exit 1
timeout -k 10 300 python -u bench.py --scale 26 --k 64 --shards 8 --streams 2 --steps 3 --warmup 1 --no-cpu-baseline \
  --eval-reps 1 > $O/bench_rmat26_k64_8shards_2streams.json 2> $O/s8s2.err || exit 1
timeout -k 10 400 python -u bench.py --shuffle --steps 5 --no-cpu-baseline > $O/bench_rmat26_k64_shuffled.json 2> $O/shuf.err || exit 1
timeout -k 10 500 python -u bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline > $O/bench_c4_powerlaw_k128.json 2> $O/c4.err || exit 1
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/bench_c5_rmat28_k256_8shards.json 2> $O/c5.err || exit 1
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --streams 2 --steps 2 --warmup 1 --no-cpu-baseline \
  --eval-reps 1 > $O/bench_c5_rmat28_k256_8shards_2streams.json 2> $O/c5s2.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/bench_rehearsal_2ranks_rmat24.json 2> $O/reh.err || exit 1
