# The D&C finish with unrolled list loads and long lists first: 11 / 12 / 13 bits, 8 shards,
# and a kernel trace of the default.  gpurun_out/r4dc3/.
set -o pipefail
mkdir -p gpurun_out/r4dc3 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4dc3
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/dc12.json 2> $O/dc12.err || exit 1
SHEEP_FIN_MAP=13 timeout -k 10 200 $B > $O/dc13.json 2> $O/dc13.err || exit 1
SHEEP_FIN_MAP=11 timeout -k 10 200 $B > $O/dc11.json 2> $O/dc11.err || exit 1
timeout -k 10 200 $B --shards 8 > $O/s8_dc12.json 2> $O/s8_dc12.err || exit 1
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify > t.log 2>&1 || exit 1
python ../../tools/trace_step.py $(find t -name '*kernel_trace.csv' | head -1) --levels > step.txt || exit 1
rm -rf t
