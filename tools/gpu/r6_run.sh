# Round-6 probe: record (tail, head) in one 8-byte load (variant "pre": two dword loads)
set -o pipefail
mkdir -p gpurun_out/r6 && export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=r6/ab_thload VARIANTS="pre" REPS=3 CONFIGS="--steps 5;--scale 22 --k 16 --steps 10;--shuffle --steps 3" bash tools/gpu/ab.sh
