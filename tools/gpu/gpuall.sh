# Round-2 measurement set: profiles (RMAT-26 k=64, RMAT-22 k=16), C4 / C5 / shuffled bench
# lines, the reduce step alone, a 2-rank rehearsal of the multi-GPU bench on one GPU.
# Everything lands under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
W=26 K=64 bash tools/gpu/gpuprof.sh || exit 1
W=22 K=16 bash tools/gpu/gpuprof.sh || exit 1
timeout -k 10 400 python -u bench.py --graph powerlaw --k 128 --steps 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 1
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit 1
timeout -k 10 400 python -u bench.py --shuffle --steps 5 --no-cpu-baseline > gpurun_out/bench_r26_shuffled.json 2> gpurun_out/bench_r26s.err || exit 1
timeout -k 10 300 python -u tools/merge_probe.py 26 3 8 > gpurun_out/merge_probe_rmat26_k8.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --dist-backend gloo --same-device --scale 24 --k 64 --steps 2 --verify --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/bench_rehearsal_2ranks.json 2> gpurun_out/bench_rehearsal.err || exit 1
