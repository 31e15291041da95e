# 512-thread staged scatters for degree_heads / pst_group against the current build
set -o pipefail
W=22 VARIANTS="h512" bash gpurun_abt.sh && mkdir -p gpurun_out/ab22 && mv gpurun_out/abt/* gpurun_out/ab22/ && \
W=26 VARIANTS="h512" bash gpurun_abt.sh
