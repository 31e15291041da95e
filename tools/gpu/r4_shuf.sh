# Records in any order: the three-pass relabel (default) against the two-pass form, and a
# kernel trace of one shuffled step.  gpurun_out/r4shuf/.
set -o pipefail
mkdir -p gpurun_out/r4shuf && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4shuf
B="python -u bench.py --no-cpu-baseline --steps 5 --warmup 1 --eval-reps 0 --shuffle"
timeout -k 10 300 $B > $O/three.json 2> $O/three.err || exit 1
SHEEP_RELABEL_2PASS=1 timeout -k 10 300 $B > $O/two.json 2> $O/two.err || exit 1
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace -d t -o run --output-format csv -- \
  python ../../bench.py --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify --shuffle > t.log 2>&1 || exit 1
python ../../tools/trace_step.py $(find t -name '*kernel_trace.csv' | head -1) > step.txt || exit 1
rm -rf t
