# C4, C5 and shuffled C3 bench lines with the current build
set -o pipefail
mkdir -p gpurun_out/r3 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u bench.py --graph powerlaw --k 128 --steps 5 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/r3/bench_c4_powerlaw_k128.json 2> gpurun_out/r3/c4.err || exit 1
timeout -k 10 300 python -u bench.py --shuffle --steps 5 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/r3/bench_rmat26_k64_shuffled.json 2> gpurun_out/r3/shuf.err || exit 1
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/r3/bench_c5_rmat28_k256_8shards.json 2> gpurun_out/r3/c5.err || exit 1
timeout -k 10 300 python -u tools/merge_trace.py 26 3 8 > gpurun_out/r3/merge_kway_rmat26_k8.txt 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 || exit 1
