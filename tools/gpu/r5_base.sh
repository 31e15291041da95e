# Round 5 baseline: the -t CLI tests, and a kernel trace of one 1/8 RMAT-26 shard map and
# the 8-tree K-way merge cut into phases (tools/shard_trace.py, tools/trace_phases.py).
set -o pipefail
O=gpurun_out/${OUT:-r5base}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_cli.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "print or world_ir" > $O/cli.log 2>&1 || exit 1
fi
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../tools/shard_trace.py ${SCALE:-26} 2 8 > shard.json 2> shard.err || exit 1
python ../../tools/trace_phases.py $(find t -name '*kernel_trace.csv' | head -1) --levels > phases.txt || exit 1
rm -rf t
