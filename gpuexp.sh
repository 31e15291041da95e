mkdir -p gpurun_out && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt.log 2>&1 || exit 1
SHEEP_DEBUG_ETREE=1 timeout -k 10 200 python tools/merge_probe.py 26 1 2 > gpurun_out/mpdbg.log 2>&1 || exit 1
for k in 2 8; do
  timeout -k 10 200 python tools/merge_probe.py 26 3 $k > gpurun_out/mp26_k$k.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b26.log 2>&1 || exit 1
