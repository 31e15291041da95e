# Round 5: sheep_tuning knobs on sparse maps — RMAT-26 as 8 shards on one GPU (the 8-GPU
# per-rank work, serialised) and C5, alternating with the defaults; gpurun_out/r5sweep8/.
set -o pipefail
O=gpurun_out/${OUT:-r5sweep8}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date >> $O/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
run() {   # name, tune args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --eval-reps 0 --no-verify "$@" > $O/$n.json 2> $O/$n.err || exit 1
}
run5() {
  local n=$1; shift
  timeout -k 10 600 python -u bench.py --scale 28 --k 256 --shards 8 --steps 2 --warmup 1 --no-cpu-baseline --eval-reps 0 --no-verify "$@" > $O/$n.json 2> $O/$n.err || exit 1
}
run a_def1
run a_cw3 --tune cross_win_levels=3
run b_def2
run b_cw3 --tune cross_win_levels=3
run c_def3
run c_cw3 --tune cross_win_levels=3
run5 c5_def
run5 c5_cw3 --tune cross_win_levels=3
