# A/B: the finishing levels per block as a workgroup-wide D&C (SHEEP_FIN_DC=1) at 10-13
# bits against Liu's sweep per block (default); parity first.  gpurun_out/r4dc/.
set -o pipefail
mkdir -p gpurun_out/r4dc && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4dc
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
SHEEP_FIN_DC=1 SHEEP_FIN_MAP=13 SHEEP_FIN_MERGE=13 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_dc13.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/base.json 2> $O/base.err || exit 1
SHEEP_FIN_DC=1 SHEEP_FIN_MAP=13 timeout -k 10 200 $B > $O/dc13.json 2> $O/dc13.err || exit 1
SHEEP_FIN_DC=1 SHEEP_FIN_MAP=12 timeout -k 10 200 $B > $O/dc12.json 2> $O/dc12.err || exit 1
SHEEP_FIN_DC=1 SHEEP_FIN_MAP=11 timeout -k 10 200 $B > $O/dc11.json 2> $O/dc11.err || exit 1
SHEEP_FIN_DC=1 SHEEP_FIN_MAP=10 timeout -k 10 200 $B > $O/dc10.json 2> $O/dc10.err || exit 1
timeout -k 10 200 $B --shards 8 > $O/s8_base.json 2> $O/s8_base.err || exit 1
SHEEP_FIN_DC=1 SHEEP_FIN_MAP=13 SHEEP_FIN_MERGE=13 timeout -k 10 200 $B --shards 8 > $O/s8_dc13.json 2> $O/s8_dc13.err || exit 1
SHEEP_FIN_DC=1 SHEEP_FIN_MAP=12 SHEEP_FIN_MERGE=12 timeout -k 10 200 $B --shards 8 > $O/s8_dc12.json 2> $O/s8_dc12.err || exit 1
