# Round-3 validation + profile set: full GPU suite, then (gpuprof.sh) kernel stats +
# generation-free PMC traffic + a 10-step bench line with the CPU baseline, RMAT-26 k=64
# and RMAT-22 k=16.
set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --durations 30 --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || exit 1
W=26 K=64 bash tools/gpu/gpuprof.sh || exit 1
W=22 K=16 bash tools/gpu/gpuprof.sh
