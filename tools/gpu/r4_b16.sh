# A/B: the map's top-block cut at 2^15 (default) against 2^16 positions; parity with the
# 2^16 cut; one map and 8 shard maps.  gpurun_out/r4b16/.
set -o pipefail
mkdir -p gpurun_out/r4b16 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4b16
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
SHEEP_TOP_BITS=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_b16.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/b15.json 2> $O/b15.err || exit 1
SHEEP_TOP_BITS=16 timeout -k 10 200 $B > $O/b16.json 2> $O/b16.err || exit 1
SHEEP_TOP_BITS=16 SHEEP_TOP_BLOCKS=2 timeout -k 10 200 $B > $O/b16_nb2.json 2> $O/b16_nb2.err || exit 1
timeout -k 10 200 $B --shards 8 > $O/s8_b15.json 2> $O/s8_b15.err || exit 1
SHEEP_TOP_BITS=16 timeout -k 10 200 $B --shards 8 > $O/s8_b16.json 2> $O/s8_b16.err || exit 1
