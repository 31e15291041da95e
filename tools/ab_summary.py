"""Summary of a tools/gpu/ab.sh run: per config and variant, the median step time over the
repetitions and every region whose median moved by more than 2 % against base."""
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab")
configs = (d / "configs.txt").read_text().splitlines() if (d / "configs.txt").exists() else []
runs = defaultdict(list)   # (config, variant) -> bench lines
for f in sorted(d.glob("c*_*_*.json")):
    ci, rest = f.stem[1:].split("_", 1)
    v, _ = rest.rsplit("_", 1)
    lines = [ln for ln in f.read_text().splitlines() if ln.startswith("{")]
    if lines:
        runs[(int(ci), v)].append(json.loads(lines[-1]))
for ci in sorted({k[0] for k in runs}):
    print(f"config {ci}: {configs[ci] if ci < len(configs) else ''}")
    base = runs.get((ci, "base"), [])
    med = lambda js, key: statistics.median(j["phases"][key]["ms_per_step"] for j in js if key in j["phases"])
    for v in ["base"] + sorted({k[1] for k in runs if k[0] == ci and k[1] != "base"}):
        js = runs[(ci, v)]
        if not js:
            continue
        ms = statistics.median(j["ms_per_step"] for j in js)
        moved = {}
        if v != "base" and base:
            for key in js[0]["phases"]:
                try:
                    a, b = med(base, key), med(js, key)
                except statistics.StatisticsError:
                    continue
                if a > 0.05 and abs(b - a) > 0.02 * a:
                    moved[key] = f"{a:.3f} -> {b:.3f}"
        print(f"  {v:>12}: {ms:.3f} ms/step (runs {[j['ms_per_step'] for j in js]}) {moved}")
