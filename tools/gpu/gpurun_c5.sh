# C5 with the corrected verification labels + the 2-rank rehearsal on one GPU
set -o pipefail
mkdir -p gpurun_out/c5 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/c5/bench_c5_rmat28_k256_8shards.json 2> gpurun_out/c5/c5.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/c5/bench_rehearsal_2ranks_rmat24.json 2> gpurun_out/c5/reh.err || exit 1
