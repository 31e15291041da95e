# Round-6: the group tests after the parent-plane reduce, then final set part 2.
set -o pipefail
mkdir -p gpurun_out/r6 && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "group or rccl or concurrent" > gpurun_out/r6/group_tests.log 2>&1 || exit 1
FIN=r6fin bash tools/gpu/final_set2.sh
