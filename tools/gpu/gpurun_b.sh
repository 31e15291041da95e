set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || exit 1
SCALES="22 26" bash tools/gpu/gpuprobe.sh
