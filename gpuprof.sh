# Round-1 profile set for RMAT-26 ef16 k=64 (see profiles/r1/README.md)
set -o pipefail
mkdir -p gpurun_out/p && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/p
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks -o run --output-format csv -- python ../../bench.py --steps 3 --warmup 1 --no-cpu-baseline > ks.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d pf -o run --output-format csv -- python ../../bench.py --steps 1 --warmup 0 --no-cpu-baseline > pf.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d pw -o run --output-format csv -- python ../../bench.py --steps 1 --warmup 0 --no-cpu-baseline > pw.log 2>&1 || exit 1
cd ../..
python tools/pmc_traffic.py gpurun_out/p/pf/run_counter_collection.csv gpurun_out/p/pw/run_counter_collection.csv gpurun_out/p/pmc_traffic_rmat26.json --workload "RMAT-26 ef16, k=64" --steps 1 || exit 1
mkdir -p profiles/r1 && cp gpurun_out/p/pmc_traffic_rmat26.json profiles/r1/
timeout -k 10 400 python bench.py > gpurun_out/p/bench_rmat26.json 2> gpurun_out/p/bench_rmat26.err || exit 1
