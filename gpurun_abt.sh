# A/B of kernel variants with a kernel trace each (per-level etree breakdown), RMAT-26 k=64
set -o pipefail
mkdir -p gpurun_out/abt && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/abt
for V in base ${VARIANTS}; do
  L=""; [ $V != base ] && L=$GRAFT_REPO_ROOT/sheep_amd/lib/variants/libsheep_hip_$V.so
  SHEEP_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d t_$V -o run --output-format csv -- \
    python ../../bench.py --scale ${W:-26} --k 64 --steps 2 --warmup 1 --eval-reps 1 --no-cpu-baseline > t_$V.log 2>&1 || exit 1
  python ../../tools/trace_step.py $(find t_$V -name '*kernel_trace.csv' | head -1) --levels > step_$V.txt || exit 1
done
