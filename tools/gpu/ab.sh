# A/B bench lines on one box: the in-tree library ("base") against
# sheep_amd/lib/variants/libsheep_hip_$V.so (make variant V=... DEFS=...) for every V in
# $VARIANTS, alternating, $REPS rounds, for each bench argument set in $CONFIGS
# (';'-separated).  Output: gpurun_out/$OUT/c<config>_<variant>_<rep>.json and summary.txt
# (tools/ab_summary.py: median ms per step and the regions that moved).
set -o pipefail
O=gpurun_out/${OUT:-ab}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
IFS=';' read -ra CF <<< "${CONFIGS:---steps 5}"
printf '%s\n' "${CF[@]}" > $O/configs.txt
i=0
for c in "${CF[@]}"; do
  for r in $(seq 1 ${REPS:-2}); do
    for v in base $VARIANTS; do
      lib=""
      [ "$v" != base ] && lib=sheep_amd/lib/variants/libsheep_hip_$v.so
      SHEEP_HIP_LIB=$lib timeout -k 10 ${LIMIT:-400} python -u bench.py $c --no-cpu-baseline ${EVAL:---eval-reps 1} \
        > $O/c${i}_${v}_$r.json 2> $O/c${i}_${v}_$r.err || exit 1
    done
  done
  i=$((i+1))
done
python tools/ab_summary.py $O > $O/summary.txt
