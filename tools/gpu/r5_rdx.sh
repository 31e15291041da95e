# Round 5: the radix sort's ranking per wave chunk — the tests that sort (RMAT generation's
# dedup, sequences, kid tables, the etree finish, C2), then RMAT-26 / C4 bench lines.
set -o pipefail
O=gpurun_out/${OUT:-r5rdx}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py -x -q --timeout 300 \
  --timeout-method thread -k "not C3 and not C4 and not C5" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --eval-reps 1 > $O/b26_$i.json 2> $O/b26_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --graph powerlaw --k 128 --steps 3 --no-cpu-baseline --eval-reps 1 > $O/c4.json 2> $O/c4.err || exit 1
