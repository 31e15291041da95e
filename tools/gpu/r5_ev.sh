# Round 5: the persistent packing-event kernel (sheep_tuning event_loop) — partition parity
# tests, then RMAT-26 and C4 bench lines with the default and with one launch per event.
set -o pipefail
O=gpurun_out/${OUT:-r5ev}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "partition or rmat_vs_oracle" > $O/tests.log 2>&1 || exit 1
for v in 4096 0; do
  timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --eval-reps 0 --tune "event_loop=$v" \
    > $O/b26_ev$v.json 2> $O/b26_ev$v.err || exit 1
done
for v in 4096 0; do
  timeout -k 10 300 python -u bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline --eval-reps 0 \
    --tune "event_loop=$v" > $O/c4_ev$v.json 2> $O/c4_ev$v.err || exit 1
done
for v in 4096 0; do
  SHEEP_DEBUG=part timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 0 \
    --tune "event_loop=$v" > $O/dbg_ev$v.json 2> $O/dbg_ev$v.err || exit 1
done
