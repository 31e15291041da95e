set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u tools/merge_probe.py 26 3 8 2 > gpurun_out/mp8.log 2>&1 || exit 1
$T 300 python -u tools/merge_probe.py 26 3 4 2 > gpurun_out/mp4.log 2>&1 || exit 1
$T 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 3 --dist-backend gloo --same-device --scale 22 --k 16 --steps 2 --verify --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/reh3.json 2> gpurun_out/reh3.err || exit 1
$T 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 4 --dist-backend gloo --same-device --scale 22 --k 16 --steps 2 --verify --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/reh4.json 2> gpurun_out/reh4.err || exit 1
