#!/usr/bin/env python3
"""Per-op PMC counters of one forward (the model's own launches, split layout
included), from rocprofv3 passes over tools/trace_forward.py.

usage: tools/pmc_ops.sh OUTDIR [trace_forward args]    (collect: one pass per counter group)
       python tools/pmc_ops.py OUTDIR [--op NAME]      (print per-op medians + derived ratios)
"""
import argparse
import csv
import glob
import json
import os
import statistics


def load(outdir):
    ops = json.load(open(os.path.join(outdir, "ops.json")))
    n = len(ops)
    vals = {}  # counter -> position -> [values]
    for d in sorted(glob.glob(os.path.join(outdir, "p*"))):
        if not os.path.isdir(d):
            continue
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                rows += [r for r in csv.DictReader(fh) if "spi" in r["Kernel_Name"]]
        by_counter = {}
        for r in rows:
            by_counter.setdefault(r["Counter_Name"], []).append(r)
        for cname, rs in by_counter.items():
            rs.sort(key=lambda r: int(r["Dispatch_Id"]))
            fwds = [rs[i:i + n] for i in range(0, len(rs) - n + 1, n)][3:]
            for pos in range(n):
                vals.setdefault(cname, {}).setdefault(pos, []).extend(float(f[pos]["Counter_Value"]) for f in fwds)
    return ops, {c: {p: statistics.median(v) for p, v in pv.items()} for c, pv in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--op", default="")
    a = ap.parse_args()
    ops, med = load(a.outdir)
    for pos, name in enumerate(ops):
        if a.op and a.op not in name:
            continue
        c = {k: v[pos] for k, v in med.items() if pos in v}
        line = [f"{k}={c[k]:.0f}" for k in sorted(c)]
        der = []
        if c.get("SQ_WAVE_CYCLES"):
            wc = c["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
                if k in c:
                    der.append(f"{k[3:]}/wave={c[k] / wc:.2f}")
        if c.get("SQ_INSTS_MFMA"):
            der.append(f"valu/mfma={c.get('SQ_INSTS_VALU', 0) / c['SQ_INSTS_MFMA']:.1f}")
        if c.get("SQ_LDS_IDX_ACTIVE"):
            der.append(f"lds_conflict={c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.2f}")
        print(f"[{pos:2d}] {name}\n     " + " ".join(line) + ("\n     " + " ".join(der) if der else ""))


if __name__ == "__main__":
    main()
