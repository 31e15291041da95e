# Profile probe: kernel stats + one step's kernel trace of the RMAT-26 bench
# (tools/trace_step.py --levels), and the SQ stall counters of the step's top kernels.
set -o pipefail
R=$(pwd)
O=gpurun_out/${OUT:-prof}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks -o run --output-format csv -- \
  python $R/bench.py --scale ${W:-26} --k ${K:-64} --steps 3 --warmup 1 --eval-reps 1 --no-cpu-baseline > ks.log 2>&1 || exit 1
python $R/tools/trace_step.py $(find ks -name '*kernel_trace.csv' | head -1) --levels > step_trace.txt || exit 1
cp $(find ks -name '*kernel_stats.csv' | head -1) kernel_stats.csv
rm -rf ks/*/*kernel_trace.csv
cd $R
RX=${RX:-'k_big_min0|k_relabel_scatter|k_relabel_gather|k_cross_find|k_cross_apply|k_hook_round|k_lo_scatter_staged|k_hist_scatter|k_degree_fused|k_split'} \
  SQOUT=${OUT:-prof}/sq bash tools/gpu/sq_counters.sh || exit 1
