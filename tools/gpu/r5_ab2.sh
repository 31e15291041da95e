# Round 5, A/B set 2: batched hook rounds (hook_batch 1: merges, 2: maps too) on the
# shard/merge phase trace and the 8-shard bench line; relabel_per=4 on the RMAT-26 line.
set -o pipefail
O=gpurun_out/r5ab2
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> $O/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests/test_tuning.py -m gpu -v --timeout 500 --timeout-method thread > $O/tuning_tests.log 2>&1 || exit 1
SHEEP_TUNE="hook_batch=2" OUT=r5ab2/shard_hb2 bash tools/gpu/r5_shard.sh || exit 1
B="python -u bench.py --steps 3 --warmup 1 --eval-reps 0 --no-cpu-baseline"
timeout -k 10 300 $B --shards 8 > $O/s8.json 2> $O/s8.err || exit 1
timeout -k 10 300 $B --shards 8 --tune hook_batch=1 > $O/s8_hb1.json 2> $O/s8_hb1.err || exit 1
timeout -k 10 300 $B --steps 5 --tune relabel_per=4 > $O/b26_per4.json 2> $O/b26_per4.err || exit 1
