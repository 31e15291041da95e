# Sequential steps against whole steps on N concurrent contexts (--concurrent N, a stream of
# graphs), interleaved, at C3 and C2.  gpurun_out/$OUT/.
set -o pipefail
O=gpurun_out/${OUT:-conc}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --eval-reps 1 > $O/seq_$r.json 2> $O/seq_$r.err || exit 1
  for n in 2 3; do
    timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --eval-reps 1 --concurrent $n > $O/conc${n}_$r.json 2> $O/conc${n}_$r.err || exit 1
  done
done
timeout -k 10 300 python -u bench.py --scale 22 --k 16 --steps 24 --warmup 3 --no-cpu-baseline --eval-reps 1 > $O/c2seq.json 2> $O/c2seq.err || exit 1
for n in 2 3 4; do
  timeout -k 10 300 python -u bench.py --scale 22 --k 16 --steps 24 --warmup 4 --no-cpu-baseline --eval-reps 1 --concurrent $n > $O/c2conc$n.json 2> $O/c2conc$n.err || exit 1
done
