# Round 5: tight workspaces (list bound m + n, exact finish buffers, relabel scratch aliased
# with the etree lists, generator buffers trimmed): the GPU suite, then the RMAT-26 bench
# line with its HBM high-water mark, and C5 (RMAT-28, 8 shards).
set -o pipefail
O=gpurun_out/r5mem
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> $O/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > $O/b26.json 2> $O/b26.err || exit 1
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/c5.json 2> $O/c5.err || exit 1
