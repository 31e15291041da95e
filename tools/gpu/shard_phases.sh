# The sparse-input etree, phase by phase.  A kernel trace of one 1/8 RMAT-26 shard
# map and the 8-tree K-way merge (tools/shard_trace.py -> tools/trace_phases.py), and the
# same run with SHEEP_DEBUG=etree for the per-level list sizes.  SHEEP_TUNE="field=v ..."
# (read by shard_trace.py) selects sheep_tuning variants.
set -o pipefail
R=$(pwd)
O=gpurun_out/${OUT:-shard}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python $R/tools/shard_trace.py ${SCALE:-26} 2 8 > shard.json 2> shard.err || exit 1
python $R/tools/trace_phases.py $(find t -name '*kernel_trace.csv' | head -1) --levels > phases.txt || exit 1
rm -rf t
SHEEP_DEBUG=etree timeout -k 10 300 python $R/tools/shard_trace.py ${SCALE:-26} 1 8 > dbg.json 2> dbg.err || exit 1
