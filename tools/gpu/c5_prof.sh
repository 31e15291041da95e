# C5 as 2 shards on one GPU: a kernel trace + stats of a 1-step run (tools/trace_step.py
# splits the step), and the etree's per-level debug lines.  gpurun_out/$OUT/.
set -o pipefail
R=$(pwd)
OUT=${OUT:-c5p}
O=gpurun_out/$OUT
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
cd $O && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d ks -o run --output-format csv -- \
  python $R/bench.py --scale 28 --k 256 --shards 2 --steps 1 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify \
  > ks.log 2>&1 || exit 1
python $R/tools/trace_step.py $(find ks -name '*kernel_trace.csv' | head -1) > step_trace.txt || exit 1
cp $(find ks -name '*kernel_stats.csv' | head -1) kernel_stats.csv && rm -rf ks && cd $R || exit 1
SHEEP_DEBUG=etree timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 2 --steps 1 --warmup 0 --eval-reps 0 \
  --no-cpu-baseline --no-verify > $O/dbg.json 2> $O/etree_debug.txt || exit 1
