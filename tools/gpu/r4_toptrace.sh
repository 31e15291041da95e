# Kernel trace of the dense-top-block kernels (RMAT-26, 4 blocks, 11-bit finish).  gpurun_out/toptrace/.
set -o pipefail
mkdir -p gpurun_out/toptrace && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/toptrace
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=11 timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify > t.log 2>&1 || exit 1
python ../../tools/top_trace.py $(find t -name '*kernel_trace.csv' | head -1) > top_trace.txt || exit 1
python ../../tools/trace_step.py $(find t -name '*kernel_trace.csv' | head -1) --levels > step.txt || exit 1
