# degree pass records per thread against the current build
set -o pipefail
W=22 VARIANTS="dpt16 dpt4" bash tools/gpu/gpurun_abt.sh && mkdir -p gpurun_out/ab22 && mv gpurun_out/abt/* gpurun_out/ab22/ && \
W=26 VARIANTS="dpt16 dpt4" bash tools/gpu/gpurun_abt.sh
