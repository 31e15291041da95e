# Probe: per-level etree stats (SHEEP_DEBUG_ETREE) and a kernel trace of one bench step
# at RMAT-22 and RMAT-26; bench lines.  Output under gpurun_out/probe/.
set -o pipefail
mkdir -p gpurun_out/probe && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/probe
for W in ${SCALES:-22 26}; do
  K=16; [ "$W" = 26 ] && K=64
  SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python ../../bench.py --scale $W --k $K --steps 1 --warmup 1 --eval-reps 0 \
    --no-cpu-baseline --no-verify > dbg$W.json 2> dbg$W.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d t$W -o run --output-format csv -- \
    python ../../bench.py --scale $W --k $K --steps 2 --warmup 1 --eval-reps 1 --no-cpu-baseline > t$W.log 2>&1 || exit 1
  python ../../tools/trace_step.py $(find t$W -name '*kernel_trace.csv' | head -1) --levels > step$W.txt || exit 1
  timeout -k 10 300 python ../../bench.py --scale $W --k $K --steps 5 --no-cpu-baseline > b$W.json 2> b$W.err || exit 1
done
