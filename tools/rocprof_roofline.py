#!/usr/bin/env python3
"""Record the rocprofv3 average duration of the roofline op's kernel next to the bench line.

tools/roofline_profile.sh runs `bench.py --roofline-only --roofline-op OP` under
`rocprofv3 --kernel-trace --stats`; that process launches only the op's kernel back to
back (after one warm-up task), so the kernel with the most calls in its
*_kernel_stats.csv is the op's.  Writes profiles/<round>/roofline_rocprof.json, which
bench.py reads to print `rocprof_avg_launch_ms` / `frac_rocprof` beside the hipEvents
figure (the profiler serialises dispatches and adds per-kernel cache maintenance, so its
per-kernel time reads higher than back-to-back events on short kernels).

usage: tools/rocprof_roofline.py KERNEL_STATS.csv OP_NAME OUT.json [KERNEL_TRACE.csv]
"""
import csv
import json
import os
import sys


def longest_run(trace):
    """The longest run of consecutive dispatches of one kernel and grid in a kernel trace: the
    op's back-to-back launches (kernel-stats averages also count the warm-up forward's launches
    of the same template instance by other ops -- ViT-L's out-proj beside FFN2)."""
    with open(trace) as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    best, cur = [], []
    for r in rows:
        key = (r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"])
        if cur and key != (cur[-1]["Kernel_Name"], cur[-1]["Grid_Size_X"], cur[-1]["Grid_Size_Y"]):
            cur = []
        cur.append(r)
        if len(cur) > len(best):
            best = list(cur)
    return best


def main():
    stats, op, out = sys.argv[1:4]
    trace = sys.argv[4] if len(sys.argv) > 4 else ""
    rec = {}
    if os.path.exists(out):
        with open(out) as f:
            rec = json.load(f)
    if trace:
        run = longest_run(trace)
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in run]
        rec[op] = {"kernel": run[0]["Kernel_Name"][:160], "calls": len(run),
                   "avg_ms": round(sum(durs) / len(durs), 5), "min_ms": round(min(durs), 5),
                   "selection": "longest run of back-to-back dispatches in the kernel trace",
                   "source": os.path.relpath(trace)}
    else:
        with open(stats) as f:
            rows = list(csv.DictReader(f))
        top = max(rows, key=lambda r: int(r["Calls"]))
        rec[op] = {"kernel": top["Name"][:160], "calls": int(top["Calls"]),
                   "avg_ms": round(float(top["AverageNs"]) / 1e6, 5),
                   "min_ms": round(float(top["MinNs"]) / 1e6, 5),
                   "source": os.path.relpath(stats)}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec[op]))


if __name__ == "__main__":
    main()
