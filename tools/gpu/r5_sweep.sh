# Round 5: a sweep of sheep_tuning knobs on the round's final code (RMAT-26 k=64, 5 steps
# each, alternating with the defaults so box drift shows), results in gpurun_out/r5sweep/.
set -o pipefail
O=gpurun_out/${OUT:-r5sweep}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> $O/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
run() {   # name, tune args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --eval-reps 0 "$@" > $O/$n.json 2> $O/$n.err || exit 1
}
run def1
run cw3 --tune cross_win_levels=3
run cw1 --tune cross_win_levels=1
run def2
run bb20 --tune big_bits=20
run bb22 --tune big_bits=22
run def3
run fin12 --tune fin_map_bits=12
run tb15 --tune top_bits=15
run def4
