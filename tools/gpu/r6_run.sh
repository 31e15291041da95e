# Round-6 probe: the direct relabel (random pos[head] gathers, k_relabel) against the
# head-bucketed one, C3 and C2 (no evaluator leg: the direct form leaves no step edges).
set -o pipefail
mkdir -p gpurun_out/r6 && export HSA_ENABLE_IPC_MODE_LEGACY=0
EVAL="--eval-reps 0" OUT=r6/ab_direct VARIANTS="direct" REPS=2 CONFIGS="--steps 5;--scale 22 --k 16 --steps 10" bash tools/gpu/ab.sh
