# Round 5: the GPU parity suite, smoke, a default bench line (no CPU baseline), then the
# sparse-etree phase trace (r5_shard.sh).
set -o pipefail
O=gpurun_out/${OUT:-r5suite}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > $O/b26.json 2> $O/b26.err || exit 1
[ -n "$NO_SHARD" ] || OUT=${OUT:-r5suite}/shard bash tools/gpu/r5_shard.sh
