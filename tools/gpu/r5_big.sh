# Round 5: the early cut's k_big_min0 software-pipelined — parity (tuning tests, C3 / C4
# digests) and two RMAT-26 bench lines plus C4.
set -o pipefail
O=gpurun_out/r5big
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> $O/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests/test_tuning.py tests/test_scale_parity.py -m gpu -x -v --timeout 500 \
  --timeout-method thread -k "tuning or TestC3 or TestC4" > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 5 --eval-reps 0 --no-cpu-baseline > $O/b26_$i.json 2> $O/b26_$i.err || exit 1
done
timeout -k 10 400 python -u bench.py --graph powerlaw --k 128 --steps 3 --eval-reps 0 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 1
