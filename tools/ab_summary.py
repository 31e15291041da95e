"""Summary of a gpurun_abt.sh run: per variant, its parity line, step time and the phases asked for."""
import json
import sys
from pathlib import Path

d = Path(sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/abt")
variants, phases = sys.argv[1].split(), sys.argv[2].split() if len(sys.argv) > 2 else []
for v in ["base"] + variants:
    p = d / f"p_{v}.log"
    par = p.read_text().strip().splitlines()[-1] if p.exists() else ""
    t = d / f"t_{v}.log"
    line = [l for l in t.read_text().splitlines() if l.startswith("{")] if t.exists() else []
    if not line:
        print(f"{v}: no bench line {par}")
        continue
    j = json.loads(line[-1])
    ph = {k: j["phases"][k]["ms_per_step"] for k in phases if k in j["phases"]}
    print(f"{v}: {j['ms_per_step']} ms {ph} {par}")
