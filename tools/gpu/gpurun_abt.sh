# A/B of kernel variants with a kernel trace each (per-level etree breakdown), RMAT-26 k=64.
# Each variant first passes C3's tree digest test (parity against the recorded oracle run).
set -o pipefail
mkdir -p gpurun_out/abt && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
for V in base ${VARIANTS}; do
  L=""; [ $V != base ] && L=$GRAFT_REPO_ROOT/sheep_amd/lib/variants/libsheep_hip_$V.so
  if [ $V != base ]; then
    SHEEP_HIP_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
      tests/test_scale_parity.py -m gpu -k "TestC3 and sequence_and_tree" > gpurun_out/abt/p_$V.log 2>&1 || exit 1
  fi
  (cd gpurun_out/abt && SHEEP_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d t_$V -o run --output-format csv -- \
    python ../../bench.py --scale ${W:-26} --k 64 --steps 2 --warmup 1 --eval-reps 1 --no-cpu-baseline > t_$V.log 2>&1) || exit 1
  python tools/trace_step.py $(find gpurun_out/abt/t_$V -name '*kernel_trace.csv' | head -1) --levels > gpurun_out/abt/step_$V.txt || exit 1
done
