# Final measurement set, part 1 (see profiles/rN/README.md): the GPU suite, the
# RMAT-26 and RMAT-22 profiles (kernel stats + trace, FETCH/WRITE PMC passes, bench lines with
# the CPU baseline), one RMAT-26 step's per-level kernel trace and the SQ stall counters of
# the step's top kernels.  gpurun_out/$FIN/, gpurun_out/p26, gpurun_out/p22.
set -o pipefail
R=$(pwd)
FIN=${FIN:-fin}
mkdir -p gpurun_out/$FIN && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
O=gpurun_out/$FIN
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
W=26 K=64 bash tools/gpu/gpuprof.sh || exit 1
W=22 K=16 bash tools/gpu/gpuprof.sh || exit 1
OUT=$FIN/prof bash tools/gpu/prof_step.sh || exit 1
