# GPU parity suite (with per-test durations) + smoke + bench checks; round 3
set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations 30 --timeout 900 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gt.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
# --gpus 2 on a one-GPU box must fail loudly (exit 2), not run one GPU
timeout -k 10 120 python bench.py --gpus 2 --scale 20 --steps 1 > gpurun_out/b_gpus2.log 2>&1; echo "rc=$?" >> gpurun_out/b_gpus2.log
# two ranks rehearsed on one GPU over the world's host link (sheep_group_join), verified
timeout -k 10 300 python bench.py --gpus 2 --same-device --scale 24 --k 64 --steps 2 --eval-reps 1 > gpurun_out/b_rehearsal2.json 2> gpurun_out/b_rehearsal2.err || exit 1
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/b26.json 2> gpurun_out/b26.err || exit 1
