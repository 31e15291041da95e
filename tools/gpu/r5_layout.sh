# Round 5: the relabel reusing the degree pass's head layout when the layout's key range
# sits below the sequence's (shards): parity tests, the 8-shard line with its kernel stats.
set -o pipefail
R=$(pwd)
O=gpurun_out/${OUT:-r5layout}; mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py tests/test_dist.py -x -q --timeout 300 --timeout-method thread -k "not C4" > $O/t.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 0 > $O/s8.json 2> $O/s8.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 0 > $O/reh.json 2> $O/reh.err || exit 1
cd $O && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ks -o run --output-format csv -- python $R/bench.py --shards 8 --steps 2 --warmup 1 --eval-reps 0 --no-cpu-baseline --no-verify > ks.log 2>&1
