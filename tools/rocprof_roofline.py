#!/usr/bin/env python3
"""Record the rocprofv3 average duration of the roofline op's kernel next to the bench line.

tools/roofline_profile.sh runs `bench.py --roofline-only --roofline-op OP` under
`rocprofv3 --kernel-trace --stats`; that process launches only the op's kernel back to
back (after one warm-up task), so the kernel with the most calls in its
*_kernel_stats.csv is the op's.  Writes profiles/<round>/roofline_rocprof.json, which
bench.py reads to print `rocprof_avg_launch_ms` / `frac_rocprof` beside the hipEvents
figure (the profiler serialises dispatches and adds per-kernel cache maintenance, so its
per-kernel time reads higher than back-to-back events on short kernels).

usage: tools/rocprof_roofline.py KERNEL_STATS.csv OP_NAME OUT.json
"""
import csv
import json
import os
import sys


def main():
    stats, op, out = sys.argv[1:4]
    with open(stats) as f:
        rows = list(csv.DictReader(f))
    top = max(rows, key=lambda r: int(r["Calls"]))
    rec = {}
    if os.path.exists(out):
        with open(out) as f:
            rec = json.load(f)
    rec[op] = {"kernel": top["Name"][:160], "calls": int(top["Calls"]),
               "avg_ms": round(float(top["AverageNs"]) / 1e6, 5),
               "min_ms": round(float(top["MinNs"]) / 1e6, 5),
               "source": os.path.relpath(stats)}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec[op]))


if __name__ == "__main__":
    main()
