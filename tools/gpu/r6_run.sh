# Round-6 probe: sheep_tuning sweep on C4 (Chung-Lu, twitter-2010 scale): the defaults were
# measured on RMAT-26.  One bench line per variant, base twice.
set -o pipefail
O=gpurun_out/r6/c4sweep
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
run() {
  timeout -k 10 300 python -u bench.py --graph powerlaw --k 128 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 0 \
    $2 > $O/$1.json 2> $O/$1.err || exit 1
}
run base ""
run big22 "--tune big_bits=22"
run big23 "--tune big_bits=23"
run big20 "--tune big_bits=20"
run win3 "--tune cross_win_levels=3"
run fin12 "--tune fin_map_bits=12"
run base2 ""
