set -o pipefail
O=gpurun_out/pipe
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-reps 1 > $O/seq_$r.json 2> $O/seq_$r.err || exit 1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --eval-reps 1 --pipeline > $O/pipe_$r.json 2> $O/pipe_$r.err || exit 1
done
timeout -k 10 300 python -u bench.py --scale 22 --k 16 --steps 20 --warmup 2 --no-cpu-baseline --eval-reps 1 > $O/c2seq.json 2> $O/c2seq.err || exit 1
timeout -k 10 300 python -u bench.py --scale 22 --k 16 --steps 20 --warmup 2 --no-cpu-baseline --eval-reps 1 --pipeline > $O/c2pipe.json 2> $O/c2pipe.err || exit 1
