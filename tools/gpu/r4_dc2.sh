# The D&C finish with its list in LDS for short blocks: default (12 bits) against 11 / 13
# bits and Liu's sweep; the GPU suite with the defaults.  gpurun_out/r4dc2/.
set -o pipefail
mkdir -p gpurun_out/r4dc2 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4dc2
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 $B > $O/dc12.json 2> $O/dc12.err || exit 1
SHEEP_FIN_MAP=13 timeout -k 10 200 $B > $O/dc13.json 2> $O/dc13.err || exit 1
SHEEP_FIN_MAP=11 timeout -k 10 200 $B > $O/dc11.json 2> $O/dc11.err || exit 1
SHEEP_FIN_DC=0 SHEEP_FIN_MAP=10 timeout -k 10 200 $B > $O/liu10.json 2> $O/liu10.err || exit 1
timeout -k 10 200 $B --shards 8 > $O/s8_dc12.json 2> $O/s8_dc12.err || exit 1
SHEEP_FIN_MAP=13 SHEEP_FIN_MERGE=13 timeout -k 10 200 $B --shards 8 > $O/s8_dc13.json 2> $O/s8_dc13.err || exit 1
timeout -k 10 200 $B --scale 22 --k 16 --steps 20 > $O/b22_dc12.json 2> $O/b22_dc12.err || exit 1
SHEEP_FIN_DC=0 SHEEP_FIN_MAP=10 SHEEP_FIN_MERGE=11 timeout -k 10 200 $B --scale 22 --k 16 --steps 20 > $O/b22_liu.json 2> $O/b22_liu.err || exit 1
