# current build (fused clean, hook finish from shards, adaptive window chunks) against the previous commit, then the GPU suite
set -o pipefail
W=22 VARIANTS="old" bash gpurun_abt.sh && mkdir -p gpurun_out/ab22 && mv gpurun_out/abt/* gpurun_out/ab22/ && \
W=26 VARIANTS="old" bash gpurun_abt.sh && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abt/tests.log 2>&1
