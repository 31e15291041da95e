# Round 5, A/B set 4: the early cut's LDS window (big_hot_bits 15 default, 14 and 13 with
# two workgroups per CU) on the RMAT-26 line and C4; parity through the tuning tests.
set -o pipefail
O=gpurun_out/r5ab4
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tuning.py -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python -u bench.py --steps 5 --eval-reps 0 --no-cpu-baseline"
for v in 15 14 13; do
  timeout -k 10 300 $B --tune big_hot_bits=$v > $O/b26_hot$v.json 2> $O/b26_hot$v.err || exit 1
done
timeout -k 10 400 $B --graph powerlaw --k 128 --steps 3 --tune big_hot_bits=14 > $O/c4_hot14.json 2> $O/c4_hot14.err || exit 1
