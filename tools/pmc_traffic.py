#!/usr/bin/env python3
"""HBM traffic per op of one forward, from rocprofv3 PMC passes.

Collection (tools/pmc_traffic.sh): two separate passes over isolated forwards
(tools/trace_forward.py), one with --pmc FETCH_SIZE and one with --pmc
WRITE_SIZE (they do not fit one pass: 3 + 2 of the 4 TCC slots,
MI355X_MICROARCH.md "rocprofv3 PMC slots").  Corrections from the guide's HBM
section: both counters are KB; on gfx950 FETCH_SIZE reports half the bytes of a
wide (16 B/lane) streaming read, so it is doubled; WRITE_SIZE is exact for
16 B/lane stores.  Infinity-Cache hits are counted too (the counters sit on the
L2's fabric side), so these are L2-miss bytes, an upper bound on HBM bytes.

MFMA pass (--mfma DIR): SQ_VALU_MFMA_BUSY_CYCLES is the MFMA-busy SIMD-cycles summed over the
chip (= 16 x N for v_mfma_f32_16x16x32_f16, MI355X_MICROARCH.md cycle table); GRBM_GUI_ACTIVE is
summed over the 8 XCDs, so wall cycles = GRBM_GUI_ACTIVE / 8 and
MFMA-busy % = 100 x SQ_VALU_MFMA_BUSY_CYCLES / (wall cycles x 256 CUs x 4 SIMDs).

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OPS_JSON [-o OUT_JSON] [--mfma DIR --mfma-out JSON]
Dispatches are grouped into forwards of len(OPS_JSON) kernels (the model's
launch order); the first forwards (the eager profiled one, warm-up) are skipped.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_dispatch(path, counter):
    """(kernel, grid, value) per model dispatch, in dispatch order."""
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if r["Counter_Name"] == counter]
    # torch's own fills / copies run outside the model: keep the model's kernels only
    rows = [r for r in rows if "spi::" in r["Kernel_Name"] or "_ZN3spi" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"])) for r in rows]


def by_op(disp, ops, skip):
    n = len(ops)
    fwds = [disp[i:i + n] for i in range(0, len(disp) - n + 1, n)][skip:]
    out = {}
    for pos, name in enumerate(ops):
        vals = [f[pos][2] for f in fwds]
        out.setdefault(name, []).append(statistics.median(vals))
    kern = {name: fwds[0][pos][0] for pos, name in enumerate(ops)} if fwds else {}
    return {k: (statistics.mean(v), len(v), kern.get(k, "")) for k, v in out.items()}, len(fwds)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("ops_json")
    ap.add_argument("-o", "--out", default="")
    ap.add_argument("--mfma", default="", help="directory of the MFMA-busy pass")
    ap.add_argument("--mfma-out", default="mfma.json")
    ap.add_argument("--skip", type=int, default=3, help="forwards to skip (profiled eager forward + warm-up)")
    a = ap.parse_args()
    ops = json.load(open(a.ops_json))
    fetch, nf = by_op(per_dispatch(a.fetch_dir, "FETCH_SIZE"), ops, a.skip)
    write, nw = by_op(per_dispatch(a.write_dir, "WRITE_SIZE"), ops, a.skip)
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), isolated forwards",
           "correction": "bytes = FETCH_SIZE KB * 1024 * 2 (gfx950 half-count) + WRITE_SIZE KB * 1024",
           "forwards": min(nf, nw), "ops": {}}
    for name in dict.fromkeys(ops):
        fb = fetch[name][0] * 1024 * 2
        wb = write[name][0] * 1024
        res["ops"][name] = {"kernel": fetch[name][2][:120], "launches_per_forward": fetch[name][1],
                            "fetch_bytes": round(fb), "write_bytes": round(wb), "hbm_bytes_per_launch": round(fb + wb)}
        print(f"{name:36s} x{fetch[name][1]:2d}  fetch {fb / 1e6:8.2f} MB  write {wb / 1e6:8.2f} MB")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    if a.mfma:
        busy, _ = by_op(per_dispatch(a.mfma, "SQ_VALU_MFMA_BUSY_CYCLES"), ops, a.skip)
        gui, _ = by_op(per_dispatch(a.mfma, "GRBM_GUI_ACTIVE"), ops, a.skip)
        cu, _ = by_op(per_dispatch(a.mfma, "SQ_BUSY_CU_CYCLES"), ops, a.skip)
        m = {"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE, isolated forwards",
             "formula": "mfma_busy_pct = 100 * SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 * 4)",
             "ops": {}}
        for name in dict.fromkeys(ops):
            wall = gui[name][0] / 8.0
            pct = 100.0 * busy[name][0] / max(wall * 1024.0, 1.0)
            m["ops"][name] = {"mfma_busy_cycles": round(busy[name][0]), "grbm_gui_active": round(gui[name][0]),
                              "sq_busy_cu_cycles": round(cu[name][0]), "wall_cycles": round(wall),
                              "mfma_busy_pct": round(pct, 3)}
            print(f"{name:36s} mfma busy {pct:6.2f} %  ({busy[name][0]:.0f} cyc over {wall:.0f} wall)")
        with open(a.mfma_out, "w") as f:
            json.dump(m, f, indent=1)


if __name__ == "__main__":
    main()
