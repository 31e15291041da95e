set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "partition or facts or oracle or c2" > gpurun_out/e2.log 2>&1 || exit 1
for cfg in "2 63" "1 63" "3 63" "2 31" "2 127"; do set -- $cfg
SHEEP_RAKE=$1 SHEEP_RULER=$2 $T 300 python -u bench.py --steps 3 --no-cpu-baseline --eval-reps 0 > gpurun_out/bp_$1_$2.log 2> gpurun_out/bp_$1_$2.err || exit 1
done
SHEEP_RAKE=1 $T 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "partition or facts or c2" > gpurun_out/e3.log 2>&1 || exit 1
SHEEP_RULER=127 $T 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "partition or facts or c2" > gpurun_out/e4.log 2>&1 || exit 1
