# A/B: the relabel scatter's stage as two u32 planes (SHEEP_RELABEL_PLANES) against one
# u64 array.  gpurun_out/r4planes/.
set -o pipefail
mkdir -p gpurun_out/r4planes && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4planes
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
SHEEP_RELABEL_PLANES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "relabel or rmat or tree" > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/u64.json 2> $O/u64.err || exit 1
SHEEP_RELABEL_PLANES=1 timeout -k 10 200 $B > $O/planes.json 2> $O/planes.err || exit 1
timeout -k 10 200 $B > $O/u64b.json 2> $O/u64b.err || exit 1
SHEEP_RELABEL_PLANES=1 timeout -k 10 200 $B > $O/planesb.json 2> $O/planesb.err || exit 1
