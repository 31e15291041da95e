# plain-store hooks A/B at RMAT-22 and RMAT-26 (parity first, then traced bench per variant)
set -o pipefail
W=22 VARIANTS="plainhook" bash gpurun_abt.sh && mkdir -p gpurun_out/ab22 && mv gpurun_out/abt/* gpurun_out/ab22/ && \
W=26 VARIANTS="plainhook" bash gpurun_abt.sh
