# Round 5: one more cross-window level for sparse maps — the parity and tuning tests, the 8-shard line twice and C3.
set -o pipefail
O=gpurun_out/cw; mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_parity.py tests/test_tuning.py -x -q --timeout 300 --timeout-method thread -k "not C4 and not C5" > $O/t.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 0 --no-verify > $O/s8a.json 2> $O/s8a.err || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --eval-reps 0 > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 300 python -u bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 0 --no-verify > $O/s8b.json 2> $O/s8b.err || exit 1
