# A/B and config lines after the round-4 changes: RMAT-26 with / without the dense top block,
# the 8-shard form (per-shard trees + K-way merge), shuffled records, C2 and C4.
# Output under gpurun_out/r4ab/.
set -o pipefail
mkdir -p gpurun_out/r4ab && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4ab
B="python -u bench.py --no-cpu-baseline"
timeout -k 10 300 $B --steps 10 --warmup 2 > $O/b26_top.json 2> $O/b26_top.err || exit 1
SHEEP_NO_TOP=1 timeout -k 10 300 $B --steps 10 --warmup 2 > $O/b26_notop.json 2> $O/b26_notop.err || exit 1
timeout -k 10 300 $B --steps 10 --warmup 2 > $O/b26_top2.json 2> $O/b26_top2.err || exit 1
timeout -k 10 300 $B --shards 8 --steps 5 --warmup 1 --eval-reps 0 > $O/b26_s8.json 2> $O/b26_s8.err || exit 1
timeout -k 10 300 $B --shuffle --steps 5 --warmup 1 --eval-reps 1 > $O/b26_shuf.json 2> $O/b26_shuf.err || exit 1
timeout -k 10 300 $B --scale 22 --k 16 --steps 20 --warmup 3 > $O/b22.json 2> $O/b22.err || exit 1
timeout -k 10 400 $B --graph powerlaw --k 128 --steps 5 --warmup 1 --eval-reps 1 > $O/c4.json 2> $O/c4.err || exit 1
