# Round 5, first A/B set: the tuning tests, default bench, relabel_per 12 / 15, and the
# shard/merge phase trace with the default and with cross_win_levels=4.
set -o pipefail
R=$(pwd)
O=gpurun_out/r5ab1
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> $O/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests/test_tuning.py -m gpu -v --timeout 500 --timeout-method thread > $O/tuning_tests.log 2>&1
for v in 8 12 15; do
  timeout -k 10 300 python -u bench.py --steps 5 --eval-reps 0 --no-cpu-baseline --no-verify --tune relabel_per=$v \
    > $O/b26_per$v.json 2> $O/b26_per$v.err || exit 1
done
OUT=r5ab1/shard bash tools/gpu/r5_shard.sh || exit 1
SHEEP_TUNE="cross_win_levels=4 fin_merge_bits=13" OUT=r5ab1/shard_xw4 bash tools/gpu/r5_shard.sh || exit 1
