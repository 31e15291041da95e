# round-2: bench smoke (evaluator leg, MPI cpu baseline) + shuffled + rocprof stats
set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --scale 22 --k 16 --steps 5 > gpurun_out/b22.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/b26.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --shuffle > gpurun_out/b26s.log 2>&1 || exit 1
cd gpurun_out && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks26 -o run --output-format csv -- python ../bench.py --steps 3 --warmup 1 --no-cpu-baseline > ks26.log 2>&1 || exit 1
