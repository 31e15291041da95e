# Round-2 profile set (see profiles/r4/README.md): kernel stats + trace of a bench run,
# generation-free PMC traffic per path step (2-step minus 1-step runs), bench lines
set -o pipefail
W=${W:-26}; K=${K:-64}
mkdir -p gpurun_out/p$W && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
cd gpurun_out/p$W
B="../../bench.py --scale $W --k $K --no-cpu-baseline --warmup 0 --eval-reps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks -o run --output-format csv -- python ../../bench.py --scale $W --k $K --steps 3 --warmup 1 --eval-reps 1 --no-cpu-baseline > ks.log 2>&1 || exit 1
for S in 1 2; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d pf$S -o run --output-format csv -- python $B --steps $S > pf$S.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d pw$S -o run --output-format csv -- python $B --steps $S > pw$S.log 2>&1 || exit 1
done
cd ../..
python tools/pmc_traffic.py gpurun_out/p$W/pmc_traffic_rmat${W}_k${K}.json --workload "RMAT-$W ef16, k=$K" --eval-reps 1 \
  --fetch gpurun_out/p$W/pf1/run_counter_collection.csv gpurun_out/p$W/pf2/run_counter_collection.csv \
  --write gpurun_out/p$W/pw1/run_counter_collection.csv gpurun_out/p$W/pw2/run_counter_collection.csv || exit 1
timeout -k 10 900 python bench.py --scale $W --k $K --steps 10 > gpurun_out/p$W/bench.json 2> gpurun_out/p$W/bench.err || exit 1
