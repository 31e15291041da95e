set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "relabel or c2 or tree or wide" > gpurun_out/e2.log 2>&1 || exit 1
cd gpurun_out
SHEEP_RL_PER=16 $T 300 rocprofv3 --kernel-trace --stats -d k16 -o run --output-format csv -- python ../bench.py --steps 3 --warmup 1 --eval-reps 0 --no-cpu-baseline > k16.log 2>&1 || exit 1
$T 300 rocprofv3 --kernel-trace --stats -d k8 -o run --output-format csv -- python ../bench.py --steps 3 --warmup 1 --eval-reps 0 --no-cpu-baseline > k8.log 2>&1 || exit 1
SHEEP_RL_PER=16 $T 300 rocprofv3 --kernel-trace --stats -d k16b -o run --output-format csv -- python ../bench.py --steps 3 --warmup 1 --eval-reps 0 --no-cpu-baseline > k16b.log 2>&1 || exit 1
