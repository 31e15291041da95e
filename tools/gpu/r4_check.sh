# The etree debug run at RMAT-26 (top-block stats), GPU suite, a default bench line, a
# 2-rank rehearsal on one GPU (per-rank split, clean JSON) and the partition event timing
# split (SHEEP_DEBUG_PART).  Output under gpurun_out/r4check/.
set -o pipefail
mkdir -p gpurun_out/r4check && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4check
SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --eval-reps 0 --no-cpu-baseline --no-verify \
  > $O/dbg26.json 2> $O/dbg26.err || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/b26.json 2> $O/b26.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > $O/reh2_rmat24.json 2> $O/reh2.err || exit 1
SHEEP_DEBUG_PART=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 0 \
  > $O/part_dbg.json 2> $O/part_dbg.err || exit 1
