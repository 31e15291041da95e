# A/B: the early cut at 2^22 positions with a density rule of 150 (the default rule, 256,
# keeps 2^22 out) against the 2^21 default.  gpurun_out/r4b22/.
set -o pipefail
mkdir -p gpurun_out/r4b22 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4b22
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --eval-reps 0"
SHEEP_BIG_BITS=22 SHEEP_BIG_DENSE=150 SHEEP_DEBUG_ETREE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --eval-reps 0 --no-cpu-baseline > $O/dbg.json 2> $O/dbg.err || exit 1
timeout -k 10 200 $B > $O/b21a.json 2> $O/b21a.err || exit 1
SHEEP_BIG_BITS=22 SHEEP_BIG_DENSE=150 timeout -k 10 200 $B > $O/b22a.json 2> $O/b22a.err || exit 1
timeout -k 10 200 $B > $O/b21b.json 2> $O/b21b.err || exit 1
SHEEP_BIG_BITS=22 SHEEP_BIG_DENSE=150 timeout -k 10 200 $B > $O/b22b.json 2> $O/b22b.err || exit 1
