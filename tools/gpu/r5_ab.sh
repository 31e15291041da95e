# Round 5 A/B driver: the GPU parity tests that do not need C4/C5, two RMAT-26 bench lines
# and the kernel stats of a 3-step RMAT-26 run (compare per-kernel averages against
# profiles/r5/rmat26_k64_kernel_stats.csv).
set -o pipefail
O=gpurun_out/${OUT:-r5ab}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py -x -q --timeout 300 \
  --timeout-method thread -k "not C4 and not C5" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --eval-reps 1 > $O/b26_$i.json 2> $O/b26_$i.err || exit 1
done
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks -o run --output-format csv -- python ../../bench.py --steps 3 --warmup 1 --eval-reps 1 --no-cpu-baseline > ks.log 2>&1 || exit 1
if [ -n "$KS2" ]; then   # a second profiled run: the box's run-to-run spread per kernel
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks2 -o run --output-format csv -- python ../../bench.py --steps 3 --warmup 1 --eval-reps 1 --no-cpu-baseline > ks2.log 2>&1
fi
