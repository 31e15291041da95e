# Round-4 check in one call: the etree debug run at RMAT-26 (top-block and block stats), the
# GPU suite, bench lines (RMAT-26 with / without the dense top block, 8 shards, shuffled,
# C2, C4), a 2-rank rehearsal on one GPU and the partition event split.  gpurun_out/r4all/.
set -o pipefail
mkdir -p gpurun_out/r4all && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4all
B="python -u bench.py --no-cpu-baseline"
SHEEP_DEBUG_ETREE=1 timeout -k 10 300 $B --steps 1 --warmup 0 --eval-reps 0 --no-verify > $O/dbg26.json 2> $O/dbg26.err || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 $B --steps 10 --warmup 2 > $O/b26_top.json 2> $O/b26_top.err || exit 1
SHEEP_NO_TOP=1 timeout -k 10 300 $B --steps 10 --warmup 2 > $O/b26_notop.json 2> $O/b26_notop.err || exit 1
SHEEP_TOP_BITS=16 timeout -k 10 300 $B --steps 10 --warmup 2 > $O/b26_top16.json 2> $O/b26_top16.err || exit 1
SHEEP_TOP_BLOCKS=4 timeout -k 10 300 $B --steps 10 --warmup 2 > $O/b26_top4blk.json 2> $O/b26_top4blk.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_DEBUG_ETREE=1 timeout -k 10 300 $B --steps 1 --warmup 0 --eval-reps 0 --no-verify \
  > $O/dbg26_4blk.json 2> $O/dbg26_4blk.err || exit 1
timeout -k 10 300 $B --shards 8 --steps 5 --warmup 1 --eval-reps 0 > $O/b26_s8.json 2> $O/b26_s8.err || exit 1
timeout -k 10 300 $B --shuffle --steps 5 --warmup 1 --eval-reps 1 > $O/b26_shuf.json 2> $O/b26_shuf.err || exit 1
timeout -k 10 300 $B --scale 22 --k 16 --steps 20 --warmup 3 > $O/b22.json 2> $O/b22.err || exit 1
timeout -k 10 400 $B --graph powerlaw --k 128 --steps 5 --warmup 1 --eval-reps 1 > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 300 $B --gpus 2 --same-device --scale 24 --steps 3 --warmup 1 --eval-reps 1 > $O/reh2_rmat24.json 2> $O/reh2.err || exit 1
SHEEP_DEBUG_PART=1 timeout -k 10 300 $B --steps 2 --warmup 1 --eval-reps 0 > $O/part_dbg.json 2> $O/part_dbg.err || exit 1
