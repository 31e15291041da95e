# GPU suite + shuffled RMAT-26 bench (tail-bucket pre-pass) + sorted RMAT-26 bench
set -o pipefail
mkdir -p gpurun_out/t && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --shuffle --steps 5 --warmup 1 --no-cpu-baseline --eval-reps 1 > gpurun_out/t/shuf.json 2> gpurun_out/t/shuf.err || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/t/b26.json 2> gpurun_out/t/b26.err || exit 1
