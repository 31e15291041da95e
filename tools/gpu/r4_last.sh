# The GPU suite and smoke() with the round's last code.  gpurun_out/r4last/.
set -o pipefail
mkdir -p gpurun_out/r4last && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4last
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --eval-reps 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
