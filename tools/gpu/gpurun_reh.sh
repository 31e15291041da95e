# 2-rank rehearsal on one GPU (world > 1 verification path)
set -o pipefail
mkdir -p gpurun_out/reh && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/reh/bench_rehearsal_2ranks_rmat24.json 2> gpurun_out/reh/reh.err || exit 1
