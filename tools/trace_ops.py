#!/usr/bin/env python3
"""Per-op durations from a rocprofv3 kernel trace (--kernel-trace --output-format csv).

One kernel instance (e.g. gemm_kernel<3, 64, 64, 3, 1>) serves several ops of a
forward; the grid shape tells them apart (tiles x split-K slices).  Groups every
dispatch by (kernel name, grid X, grid Y) and prints count / mean / median / p10
/ p90 in microseconds, largest total first.  With --ops OPS_JSON and --plan
(grid X, grid Y) pairs a caller can name a group.

usage: python tools/trace_ops.py TRACE_CSV [--top 20] [--csv OUT]
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--csv", default="", help="write the table here as CSV")
    a = ap.parse_args()
    groups = collections.defaultdict(list)
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            name = (r["Kernel_Name"].replace("(spi::(anonymous namespace)::KArgs)", "")
                    .replace("void spi::(anonymous namespace)::", "").replace("_ZN3spi12_GLOBAL__N_1", ""))
            wg = int(r["Workgroup_Size_X"])
            key = (name, int(r["Grid_Size_X"]) // max(wg, 1), int(r["Grid_Size_Y"]))
            groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for (name, gx, gy), d in groups.items():
        d.sort()
        q = lambda p: d[min(len(d) - 1, int(p * (len(d) - 1)))]
        rows.append((name, gx, gy, len(d), sum(d), statistics.mean(d), statistics.median(d), q(0.1), q(0.9)))
    rows.sort(key=lambda x: -x[4])
    hdr = ("kernel", "workgroups_x", "grid_y", "calls", "total_us", "mean_us", "median_us", "p10_us", "p90_us")
    print(f"{'kernel':58s} {'wg_x':>5s} {'y':>2s} {'calls':>6s} {'total_us':>10s} {'mean':>7s} {'median':>7s} "
          f"{'p10':>7s} {'p90':>7s}")
    for r in rows[: a.top]:
        print(f"{r[0][:58]:58s} {r[1]:5d} {r[2]:2d} {r[3]:6d} {r[4]:10.1f} {r[5]:7.2f} {r[6]:7.2f} {r[7]:7.2f} {r[8]:7.2f}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(hdr)
            for r in rows:
                w.writerow([r[0], r[1], r[2], r[3]] + [round(x, 3) for x in r[4:]])


if __name__ == "__main__":
    main()
