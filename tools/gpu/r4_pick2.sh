# The early cut with a picked bitmap for the read checks: the GPU parity tests, 2^20 / 2^21
# / 2^22 cuts, a kernel trace at 2^21.  gpurun_out/r4pick2/.
set -o pipefail
mkdir -p gpurun_out/r4pick2 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4pick2
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/b20.json 2> $O/b20.err || exit 1
SHEEP_BIG_BITS=21 timeout -k 10 200 $B > $O/b21.json 2> $O/b21.err || exit 1
SHEEP_BIG_BITS=22 timeout -k 10 200 $B > $O/b22.json 2> $O/b22.err || exit 1
cd $O && SHEEP_BIG_BITS=21 timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify > t.log 2>&1 || exit 1
python ../../tools/trace_step.py $(find t -name '*kernel_trace.csv' | head -1) --levels > step.txt || exit 1
rm -rf t
