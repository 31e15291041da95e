# A/B: priority-hashed hooks x top blocks x finishing bits; 8 shards.  gpurun_out/r4ab4/.
set -o pipefail
mkdir -p gpurun_out/r4ab4 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4ab4
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "rmat or tree or merge or shards" > $O/quick_tests.log 2>&1 || exit 1
SHEEP_HOOK_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "rmat or tree or merge or shards" > $O/quick_tests_prio.log 2>&1 || exit 1
SHEEP_NO_TOP=1 timeout -k 10 200 $B > $O/notop.json 2> $O/notop.err || exit 1
SHEEP_NO_TOP=1 SHEEP_HOOK_PRIO=1 timeout -k 10 200 $B > $O/notop_prio.json 2> $O/notop_prio.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=10 timeout -k 10 200 $B > $O/top4_fin10.json 2> $O/top4_fin10.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=10 SHEEP_HOOK_PRIO=1 timeout -k 10 200 $B > $O/top4_fin10_prio.json 2> $O/top4_fin10_prio.err || exit 1
SHEEP_TOP_BLOCKS=8 SHEEP_FIN_MAP=10 timeout -k 10 200 $B > $O/top8_fin10.json 2> $O/top8_fin10.err || exit 1
SHEEP_TOP_BLOCKS=8 SHEEP_FIN_MAP=11 timeout -k 10 200 $B > $O/top8_fin11.json 2> $O/top8_fin11.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=10 SHEEP_TOP_BITS=16 timeout -k 10 200 $B > $O/top4_b16_fin10.json 2> $O/top4_b16_fin10.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=10 timeout -k 10 200 $B --shards 8 > $O/s8_top4_fin10.json 2> $O/s8_top4_fin10.err || exit 1
SHEEP_NO_TOP=1 timeout -k 10 200 $B --shards 8 > $O/s8_notop.json 2> $O/s8_notop.err || exit 1
SHEEP_NO_TOP=1 SHEEP_HOOK_PRIO=1 timeout -k 10 200 $B --shards 8 > $O/s8_notop_prio.json 2> $O/s8_notop_prio.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=10 timeout -k 10 200 $B --scale 22 --k 16 --steps 20 > $O/b22_top4.json 2> $O/b22_top4.err || exit 1
SHEEP_NO_TOP=1 timeout -k 10 200 $B --scale 22 --k 16 --steps 20 > $O/b22_notop.json 2> $O/b22_notop.err || exit 1
