set -o pipefail
mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
T="timeout -k 10"
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T 400 $P tests/test_gpu_parity.py -m gpu -k "merge" > gpurun_out/e2.log 2>&1 || exit 1
$T 300 python -u tools/merge_probe.py 26 3 8 > gpurun_out/mp8.log 2>&1 || exit 1
$T 300 python -u tools/merge_probe.py 26 3 4 > gpurun_out/mp4.log 2>&1 || exit 1
$T 300 python -u tools/merge_probe.py 26 3 2 > gpurun_out/mp2.log 2>&1 || exit 1
$T 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --dist-backend gloo --same-device --scale 22 --k 16 --steps 2 --verify --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/reh2.json 2> gpurun_out/reh2.err || exit 1
$T 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 4 --dist-backend gloo --same-device --scale 22 --k 16 --steps 2 --verify --no-cpu-baseline --eval-reps 1 \
  > gpurun_out/reh4.json 2> gpurun_out/reh4.err || exit 1
