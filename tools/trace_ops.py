#!/usr/bin/env python3
"""Per-op durations from a rocprofv3 kernel trace (--kernel-trace --output-format csv).

One kernel instance (e.g. gemm_kernel<1, 64, 64, 3, 1, 4>) serves several ops of a
forward; the grid shape tells them apart (tiles x split-K slices).  Groups every
dispatch by (kernel, grid X in workgroups, grid Y) and prints count / total / mean /
median / p10 / p90 in microseconds, largest total first.

--launches TABLE.tsv names the groups: the table is one profiled eager forward's launch
list (bench.py --loop-only --launch-table, from spi_model_launch_table: op index, op
name, kernel, grid), so every (kernel, grid) group gets the op(s) that launch it and
their launches per forward.  The first row of the written CSV is then the op that
bounds the timed loop (bench.py's roofline picks it from the committed CSV).

usage: python tools/trace_ops.py TRACE_CSV [--launches TABLE.tsv] [--top 20] [--csv OUT]
"""
import argparse
import collections
import csv
import re
import statistics


def base_key(kernel: str) -> str:
    """A kernel's name without namespaces, return type and parameter list, keeping its
    template arguments: 'gemm_kernel<1, 64, 64, 3, 1, 4>'.  rocprofv3 leaves some names
    mangled ('..16stem_pool_kernelILi2ELi8ELb1ELi0EEEvPKf..'): those keep the mangled
    template part, which is unique per instance too."""
    k = kernel.strip()
    m = re.search(r"_GLOBAL__N_1(\d+)", k)
    if "(" not in k and m:  # mangled: <len><name>I<literal args>E
        n, pos = int(m.group(1)), m.end()
        name, rest = k[pos:pos + n], k[pos + n:]
        end = rest.find("EE")
        return name + (rest[:end + 2] if rest.startswith("I") and end >= 0 else "")
    k = re.sub(r"^void\s+", "", k).replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(k):  # drop the parameter list (the first '(' outside <...>)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            k = k[:i]
            break
    k = k.replace("spi::", "")
    return k.replace("_ZN3spi12_GLOBAL__N_1", "")


def mangled_key(kernel: str):
    """The same key for a demangled table name, in the mangled spelling (for the names
    rocprofv3 did not demangle): name + ILi..E template args."""
    m = re.match(r"([A-Za-z_][A-Za-z0-9_]*)<(.*)>$", kernel)
    if not m:
        return None
    args = []
    for a in m.group(2).split(","):
        a = a.strip()
        if a in ("true", "false"):
            args.append(f"Lb{1 if a == 'true' else 0}E")
        elif re.fullmatch(r"-?\d+", a):
            args.append(f"Li{a.replace('-', 'n')}E")
        else:
            return None
    return m.group(1) + "I" + "".join(args) + "E"


def read_launches(path):
    """op index -> name, and (kernel key, gx, gy) -> {op name: launches per forward}."""
    by_key = collections.defaultdict(collections.Counter)
    with open(path) as f:
        for line in f:
            if not line.strip() or line.startswith("#"):
                continue
            idx, name, kernel, gx, gy, gz, block = line.rstrip("\n").split("\t")
            k = base_key(kernel)
            by_key[(k, int(gx), int(gy))][name] += 1
            mk = mangled_key(k)
            if mk:
                by_key[(mk, int(gx), int(gy))][name] += 1
    return by_key


def strip_args(k: str) -> str:
    """A kernel key without its template arguments (demangled '<...>' or mangled 'I...E')."""
    k = k.split("<", 1)[0]
    m = re.match(r"([A-Za-z_][A-Za-z0-9_]*?)I(L[ib].*)?$", k)
    return m.group(1) if m else k


def read_table(path):
    """The launch table as a list of (op, kernel name without template args, gx, gy)."""
    rows = []
    with open(path) as f:
        for line in f:
            if not line.strip() or line.startswith("#"):
                continue
            idx, name, kernel, gx, gy, gz, block = line.rstrip("\n").split("\t")
            rows.append((name, strip_args(base_key(kernel)), int(gx), int(gy)))
    return rows


def attribute_by_sequence(dispatches, table):
    """Op of every dispatch by walking each hardware queue's dispatches (start-time order) along
    the launch table: one forward's launch sequence, replayed back to back by every worker
    stream.  Kernel names alone cannot tell two launches of one template instance and grid apart
    (ViT-L's out-proj and FFN2: the same gemm256 instance on 52 workgroups), their position in
    the forward can.  A dispatch that does not fit the next table entry resynchronises on the
    nearest entry it fits (warm-up copies and fills fit none: left unattributed)."""
    n = len(table)
    by_q = collections.defaultdict(list)
    for i, d in enumerate(dispatches):
        by_q[d["queue"]].append(i)
    ops = [""] * len(dispatches)
    for q, idx in by_q.items():
        idx.sort(key=lambda i: dispatches[i]["start"])
        p = 0
        for i in idx:
            d = dispatches[i]
            key = (d["name"], d["gx"], d["gy"])
            for step in range(n):
                j = (p + step) % n
                if table[j][1:] == key:
                    ops[i] = table[j][0]
                    p = (j + 1) % n
                    break
    return ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--launches", default="", help="launch table TSV of one eager forward (op attribution)")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--csv", default="", help="write the table here as CSV")
    a = ap.parse_args()
    dispatches = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            wg = int(r["Workgroup_Size_X"])
            k = base_key(r["Kernel_Name"])
            dispatches.append(dict(key=k, name=strip_args(k), gx=int(r["Grid_Size_X"]) // max(wg, 1),
                                   gy=int(r["Grid_Size_Y"]), start=int(r["Start_Timestamp"]),
                                   queue=r.get("Queue_Id") or r.get("Stream_Id") or "0",
                                   us=(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    launches = read_launches(a.launches) if a.launches else {}
    table = read_table(a.launches) if a.launches else []
    # the table's kernel ids carry no template arguments (clang's __PRETTY_FUNCTION__ prints the
    # specialisation's name only): attribute by position in the forward instead
    seq_ops = attribute_by_sequence(dispatches, table) if table else [""] * len(dispatches)
    per_fwd_of = collections.Counter(t[0] for t in table)
    groups = collections.defaultdict(list)
    for d, op in zip(dispatches, seq_ops):
        groups[(op, d["key"], d["gx"], d["gy"])].append(d["us"])
    rows = []
    total_all = sum(sum(d) for d in groups.values())
    for (op, kname, gx, gy), d in groups.items():
        d.sort()
        q = lambda p: d[min(len(d) - 1, int(p * (len(d) - 1)))]
        if not op:  # fall back to the (kernel, grid) match of a table with template arguments
            ops = launches.get((kname, gx, gy), {})
            op = "|".join(sorted(ops)) if ops else ""
            per_fwd = sum(ops.values()) if ops else 0
        else:
            per_fwd = per_fwd_of[op]
        rows.append((op, kname, gx, gy, per_fwd, len(d), sum(d), sum(d) / total_all, statistics.mean(d),
                     statistics.median(d), q(0.1), q(0.9)))
    rows.sort(key=lambda x: -x[6])
    hdr = ("op", "kernel", "workgroups_x", "grid_y", "launches_per_forward", "calls", "total_us", "share", "mean_us",
           "median_us", "p10_us", "p90_us")
    print(f"{'op':44s} {'kernel':40s} {'wg_x':>5s} {'y':>2s} {'n/fw':>4s} {'calls':>6s} {'total_us':>10s} "
          f"{'share':>6s} {'mean':>7s} {'median':>7s} {'p10':>7s} {'p90':>7s}")
    for r in rows[: a.top]:
        print(f"{r[0][:44]:44s} {r[1][:40]:40s} {r[2]:5d} {r[3]:2d} {r[4]:4d} {r[5]:6d} {r[6]:10.1f} {r[7]:6.3f} "
              f"{r[8]:7.2f} {r[9]:7.2f} {r[10]:7.2f} {r[11]:7.2f}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(hdr)
            for r in rows:
                w.writerow(list(r[:6]) + [round(x, 4) for x in r[6:]])


if __name__ == "__main__":
    main()
