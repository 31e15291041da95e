# Round 5: the evaluator from the step's position-space edges (sheep_evaluate_step) —
# parity tests, then RMAT-26 / C4 bench lines timing it beside the record evaluator.
set -o pipefail
O=gpurun_out/${OUT:-r5evs}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "evaluate" > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline --eval-records > $O/b26.json 2> $O/b26.err || exit 1
timeout -k 10 400 python -u bench.py --graph powerlaw --k 128 --steps 2 --no-cpu-baseline --eval-records \
  > $O/c4.json 2> $O/c4.err || exit 1
