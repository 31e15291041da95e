mkdir -p gpurun_out/q && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/q
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d pf -o run --output-format csv -- python ../../bench.py --steps 1 --warmup 0 --no-cpu-baseline > pf.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d pw -o run --output-format csv -- python ../../bench.py --steps 1 --warmup 0 --no-cpu-baseline > pw.log 2>&1 || exit 1
cd ../..
python tools/pmc_traffic.py gpurun_out/q/pf/run_counter_collection.csv gpurun_out/q/pw/run_counter_collection.csv gpurun_out/q/pmc.json --workload "RMAT-26 ef16, k=64" --steps 1
