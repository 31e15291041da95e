# kernel trace of the shuffled RMAT-26 step
set -o pipefail
mkdir -p gpurun_out/t2 && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
(cd gpurun_out/t2 && timeout -k 10 300 rocprofv3 --kernel-trace -d ts -o run --output-format csv -- python ../../bench.py --shuffle --steps 2 --warmup 1 --eval-reps 1 --no-cpu-baseline > ts.log 2>&1) || exit 1
python tools/trace_step.py $(find gpurun_out/t2/ts -name '*kernel_trace.csv' | head -1) > gpurun_out/t2/step.txt
