# Stall breakdown (SQ counters) of the bucket passes and the etree's level kernels on one
# RMAT-26 step: where do the waves wait.  Output under gpurun_out/sq/.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/${SQOUT:-sq} && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/${SQOUT:-sq}
RX=${RX:-'k_relabel|k_hist_scatter|k_lo_scatter|k_degree_fused|k_hist_final|k_cross|k_hook_round|k_split|k_light_top|k_big_min0'}
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex "$RX" -d s1 -o run --output-format csv -- \
  python $R/bench.py --scale ${W:-26} --k 64 --steps 1 --warmup 0 --eval-reps 0 --no-cpu-baseline --no-verify > s1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU \
  --kernel-include-regex "$RX" -d s2 -o run --output-format csv -- \
  python $R/bench.py --scale ${W:-26} --k 64 --steps 1 --warmup 0 --eval-reps 0 --no-cpu-baseline --no-verify > s2.log 2>&1 || exit 1
