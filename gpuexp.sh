set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
T="timeout -k 10"
for G in 16 32 64 128 256; do SHEEP_EV_WG=$G SHEEP_DEBUG_PART=1 $T 200 python -u bench.py --steps 2 --no-cpu-baseline --eval-reps 0 > gpurun_out/bg$G.log 2> gpurun_out/bg$G.err || exit 1; done
