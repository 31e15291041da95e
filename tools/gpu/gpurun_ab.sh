# A/B of kernel variants (sheep_amd/lib/variants) on the RMAT-26 / RMAT-22 bench
set -o pipefail
mkdir -p gpurun_out/ab && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
ls gpurun_marker* > gpurun_out/ab/marker.txt 2>&1
for W in 26 22; do
  K=64; [ $W = 22 ] && K=16
  for V in base ${VARIANTS}; do
    L=""; [ $V != base ] && L=sheep_amd/lib/variants/libsheep_hip_$V.so
    SHEEP_HIP_LIB=$L timeout -k 10 300 python bench.py --scale $W --k $K --steps 5 --no-cpu-baseline --eval-reps 1 \
      > gpurun_out/ab/b${W}_$V.json 2> gpurun_out/ab/b${W}_$V.err || exit 1
  done
done
