set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --graph powerlaw --k 128 --steps 2 --no-cpu-baseline --eval-reps 1 > gpurun_out/b_c4.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 1 > gpurun_out/b_c5.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > gpurun_out/b_26.log 2>&1 || exit 1
