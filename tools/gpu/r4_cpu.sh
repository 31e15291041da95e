# Reference CPU baselines on the box's host cores (oracle/_ref, test infrastructure):
# the literal -ir sequence (mpiSequence, sequence.h:85) at C1 and RMAT-20, and a ranks x
# OpenMP-threads sweep of the -r -p flow at RMAT-26 k=64.  Output under gpurun_out/r4cpu/.
set -o pipefail
mkdir -p gpurun_out/r4cpu && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
O=gpurun_out/r4cpu
nproc > $O/nproc.txt; lscpu > $O/lscpu.txt 2>&1; (cat /sys/fs/cgroup/cpu.max; python -c "import os; print(len(os.sched_getaffinity(0)))") > $O/cpu_quota.txt 2>&1
timeout -k 10 600 python -u tools/cpu_ir.py $O/cpu_ir_literal.json --rmat-ranks 1 2 --hep-ranks 1 2 4 8 --timeout 240 \
  > $O/cpu_ir.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/cpu_sweep.py $O/cpu_sweep_rmat26_k64.json --scale 26 --k 64 \
  --configs 8x1 16x1 16x4 16x16 32x1 32x8 > $O/cpu_sweep.log 2>&1 || exit 1
