# Round 5: quick check of the packing-event kernels — partition parity tests, one RMAT-26
# run with SHEEP_DEBUG=part (per-event phases), one C4 bench line.
set -o pipefail
O=gpurun_out/${OUT:-r5evq}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "partition or rmat_vs_oracle" > $O/tests.log 2>&1 || exit 1
SHEEP_DEBUG=part timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 0 \
  > $O/dbg.json 2> $O/dbg.err || exit 1
timeout -k 10 300 python -u bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline --eval-reps 0 \
  > $O/c4.json 2> $O/c4.err || exit 1
