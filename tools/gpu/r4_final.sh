# Round-4 final measurement set with the round's last code: the GPU suite, the RMAT-26 and
# RMAT-22 profiles (kernel stats + trace, PMC passes, bench lines), shuffled, C4, C5,
# 8 shards, the 2-rank rehearsal.  gpurun_out/r4fin/, gpurun_out/p26, gpurun_out/p22.
set -o pipefail
mkdir -p gpurun_out/r4fin && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
O=gpurun_out/r4fin
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
W=26 K=64 bash tools/gpu/gpuprof.sh || exit 1
W=22 K=16 bash tools/gpu/gpuprof.sh || exit 1
timeout -k 10 400 python -u bench.py --shuffle --steps 5 --no-cpu-baseline > $O/bench_rmat26_k64_shuffled.json 2> $O/shuf.err || exit 1
timeout -k 10 500 python -u bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline > $O/bench_c4_powerlaw_k128.json 2> $O/c4.err || exit 1
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/bench_c5_rmat28_k256_8shards.json 2> $O/c5.err || exit 1
timeout -k 10 300 python -u bench.py --scale 26 --k 64 --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 0 \
  > $O/bench_rmat26_k64_8shards.json 2> $O/s8.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/bench_rehearsal_2ranks_rmat24.json 2> $O/reh.err || exit 1
