# Round-4 measurement set, part 1: the GPU suite, the profiles of RMAT-26 k=64 and
# RMAT-22 k=16 (kernel stats + trace, PMC FETCH/WRITE passes, a bench line each).
set -o pipefail
mkdir -p gpurun_out/r4res && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4res/gpu_tests.log 2>&1 || exit 1
W=26 K=64 bash tools/gpu/gpuprof.sh || exit 1
W=22 K=16 bash tools/gpu/gpuprof.sh || exit 1
