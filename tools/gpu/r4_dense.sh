# A/B: the early cut's density rule (SHEEP_BIG_DENSE 256 default / 48) on edge shards:
# RMAT-26 as 8 shards (2^19 / 2^21 cuts) and C5.  gpurun_out/r4dense/.
set -o pipefail
mkdir -p gpurun_out/r4dense && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4dense
B="python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --eval-reps 0"
SHEEP_BIG_DENSE=48 SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python -u bench.py --shards 8 --steps 1 --warmup 0 --eval-reps 0 --no-cpu-baseline > $O/dbg_s8.json 2> $O/dbg_s8.err || exit 1
SHEEP_BIG_DENSE=48 timeout -k 10 300 $B --shards 8 > $O/s8_d48.json 2> $O/s8_d48.err || exit 1
SHEEP_BIG_DENSE=48 SHEEP_BIG_BITS=19 timeout -k 10 300 $B --shards 8 > $O/s8_d48_b19.json 2> $O/s8_d48_b19.err || exit 1
timeout -k 10 300 $B --shards 8 > $O/s8_def.json 2> $O/s8_def.err || exit 1
SHEEP_BIG_DENSE=48 timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 0 --no-verify > $O/c5_d48.json 2> $O/c5_d48.err || exit 1
