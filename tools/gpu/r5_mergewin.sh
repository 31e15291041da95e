# Round 5: the 8-tree K-way merge (tools/shard_trace.py) with 0 / 1 / 2 cross-window levels.
set -o pipefail
O=gpurun_out/${OUT:-r5mw}
mkdir -p $O && export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 2 1 0 2 1 0; do
  SHEEP_TUNE="cross_win_levels=$v" timeout -k 10 300 python tools/shard_trace.py 26 2 8 > $O/w${v}_$RANDOM.json 2>> $O/err.log || exit 1
done
