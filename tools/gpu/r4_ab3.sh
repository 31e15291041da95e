# A/B of the cheaper top-block cut (one extraction pass, LDS round 0, one sync): off / 1 / 4 /
# 8 blocks x finishing bits, the 8-shard form, plus a kernel trace.  gpurun_out/r4ab3/.
set -o pipefail
mkdir -p gpurun_out/r4ab3 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4ab3
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "rmat or tree or merge or shards" > $O/quick_tests.log 2>&1 || exit 1
SHEEP_NO_TOP=1 timeout -k 10 200 $B > $O/notop.json 2> $O/notop.err || exit 1
timeout -k 10 200 $B > $O/top1.json 2> $O/top1.err || exit 1
SHEEP_TOP_BLOCKS=4 timeout -k 10 200 $B > $O/top4.json 2> $O/top4.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=10 timeout -k 10 200 $B > $O/top4_fin10.json 2> $O/top4_fin10.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=11 timeout -k 10 200 $B > $O/top4_fin11.json 2> $O/top4_fin11.err || exit 1
SHEEP_TOP_BLOCKS=8 SHEEP_FIN_MAP=11 timeout -k 10 200 $B > $O/top8_fin11.json 2> $O/top8_fin11.err || exit 1
SHEEP_TOP_BLOCKS=8 SHEEP_FIN_MAP=10 timeout -k 10 200 $B > $O/top8_fin10.json 2> $O/top8_fin10.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=11 timeout -k 10 200 $B --shards 8 > $O/s8_top4_fin11.json 2> $O/s8_top4_fin11.err || exit 1
SHEEP_NO_TOP=1 timeout -k 10 200 $B --shards 8 > $O/s8_notop.json 2> $O/s8_notop.err || exit 1
SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=11 SHEEP_DEBUG_ETREE=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 1 \
  --warmup 0 --eval-reps 0 --no-verify > $O/dbg.json 2> $O/dbg.err || exit 1
cd $O && SHEEP_TOP_BLOCKS=4 SHEEP_FIN_MAP=11 timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify > t.log 2>&1 || exit 1
python ../../tools/top_trace.py $(find t -name '*kernel_trace.csv' | head -1) > top_trace.txt || exit 1
python ../../tools/trace_step.py $(find t -name '*kernel_trace.csv' | head -1) --levels > step.txt || exit 1
rm -rf t
