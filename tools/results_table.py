#!/usr/bin/env python3
"""BASELINE.md §4 rows from bench.py JSON lines (one file per config).

    python tools/results_table.py profiles/r2/bench_rmat22_k16.json profiles/r2/bench_rmat26_k64.json ...

Columns: t_seq = degree + degree_heads + sequence, t_tree = relabel + pst_group + etree
(+ merge), t_part = kids + partition (ms per step, HIP events on the context stream);
edges/s = the line's value; B_alg and the path roofline fraction from `path_roofline`;
the dominant leaf region and its fraction from `roofline`; the evaluator's wall time."""
import json
import sys


def row(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    ph = {k: v["ms_per_step"] for k, v in d["phases"].items()}
    g = lambda *ks: sum(ph.get(k, 0.0) for k in ks)
    t_seq = g("degree", "degree_heads", "sequence")
    t_tree = g("relabel", "pst_group", "etree", "merge")
    t_part = g("kids", "partition")
    roof, path_r, ev = d["roofline"] or {}, d["path_roofline"], d.get("evaluator") or {}
    cpu = d.get("cpu_baseline") or {}
    return (f"| {d['config']['workload']} | {d['n_gpus']} | {t_seq:.1f} / {t_tree:.1f} / {t_part:.1f} | "
            f"**{d['value'] / 1e9:.2f} G** | {d['ms_per_step']:.1f} | {path_r['alg_bytes'] / 1e9:.2f} | "
            f"{100 * path_r['frac']:.1f}% | {roof.get('kernel')} ({roof.get('frac')}) | "
            f"{ev.get('ms', '—')} ms | "
            + (f"{cpu['value'] / 1e6:.1f} M ({cpu['cores']} ranks)" if cpu.get("value") else "—") + " |")


if __name__ == "__main__":
    print("| Config | GPUs | t_seq / t_tree / t_part (ms) | edges/s | ms/step | B_alg (GB) | path roofline | "
          "dominant region (frac) | evaluator | CPU baseline |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for p in sys.argv[1:]:
        print(row(p))
