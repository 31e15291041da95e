mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || exit 1
SHEEP_DEBUG_ETREE=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --scale 22 --k 16 --no-cpu-baseline > gpurun_out/dbg22.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --scale 22 --k 16 --no-cpu-baseline > gpurun_out/b22.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify > gpurun_out/b26.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 --scale 22 --k 16 --dist-backend gloo --same-device --verify > gpurun_out/dist2.log 2>&1
