set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T 500 $P tests/test_gpu_parity.py tests/test_scale_parity.py -m gpu -k "partition or oracle or c2 or c3_rmat26_k64" > gpurun_out/e2.log 2>&1 || exit 1
$T 300 python -u bench.py --steps 3 --no-cpu-baseline --eval-reps 0 > gpurun_out/b1.log 2> gpurun_out/b1.err || exit 1
cd gpurun_out && $T 300 rocprofv3 --kernel-trace --stats -d ks2 -o run --output-format csv -- python ../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline > ks2.log 2>&1 || exit 1
