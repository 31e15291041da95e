#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter CSVs (one or more passes): the counters
summed over a kernel's dispatches, and for the SQ stall counters the share of the waves'
cycles (SQ_WAIT_ANY = parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stalls,
SQ_ACTIVE_INST_ANY = issuing; MI355X_MICROARCH.md counter notes).

    python tools/sq_summary.py s1/run_counter_collection.csv [s2/...csv]
"""
import csv
import re
import sys
from collections import defaultdict


def base(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    tot = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = base(r["Kernel_Name"])
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0)
        line = f"{k:24s} n={len(calls[k]):4d}"
        if wc:
            for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if name in c:
                    line += f" {name[3:]}={c[name] / wc:5.2f}"
            if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
                line += f" LDSconf/active={c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:5.2f}"
            line += f" wave_cycles={wc:.3g}"
        for name in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_WAVES"):
            if name in c:
                line += f" {name[3:]}={c[name]:.3g}"
        print(line)


if __name__ == "__main__":
    main()
