# GPU checks of the current build + a kernel trace of the K-way merge alone (RMAT-26, 8 trees)
set -o pipefail
mkdir -p gpurun_out/m && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_scale_parity.py tests/test_gpu_parity.py -m gpu > gpurun_out/m/tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/m/bench.json 2> gpurun_out/m/bench.err || exit 1
(cd gpurun_out/m && timeout -k 10 300 rocprofv3 --kernel-trace -d tm -o run --output-format csv -- python ../../tools/merge_trace.py 26 3 8 > merge.log 2>&1) || exit 1
python tools/trace_step.py $(find gpurun_out/m/tm -name '*kernel_trace.csv' | head -1) --levels --from k_tree_count > gpurun_out/m/merge_step.txt
