# Round 5, A/B set 3: the early MSF cut forced on the K-way merge (merge_cut_bits 21 / 19 /
# 17) — the shard/merge phase trace with per-level stats and the cut's outcome.
set -o pipefail
for b in 21 19 17; do
  SHEEP_TUNE="merge_cut_bits=$b" OUT=r5ab3/mc$b bash tools/gpu/r5_shard.sh || exit 1
done
