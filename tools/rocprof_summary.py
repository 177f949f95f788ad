#!/usr/bin/env python3
"""Summarise a rocprofv3 output dir (kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE
PMC passes) into the markdown table committed under profiles/.

usage: rocprof_summary.py <dir> <title> [--fetch-x2] [--json out.json]
HBM bytes per launch = FETCH_SIZE*1024 (*2 with --fetch-x2: gfx950 reports half of the bytes
read, MI355X_MICROARCH.md 'HBM'; tools/fetch_calib.hip measures the factor for the 16-, 4- and
1-byte-per-lane reads the VO kernels issue, profiles/r2_fetch_calibration.md) + WRITE_SIZE*1024
(exact for 16-, 4- and 1-byte stores).
VALU (a third pass, "valu*": SQ_INSTS_VALU, SQ_WAVES, GRBM_GUI_ACTIVE): issue fraction =
SQ_INSTS_VALU x 4 cycles (a wave64 instruction per SIMD, profiles/r2_valu_calibration.md) / (1024 SIMDs x GRBM_GUI_ACTIVE / 8
XCDs), i.e. the share of the dispatch's SIMD cycles spent issuing VALU at the f32/integer rate
(f64 FMAs and transcendentals take longer, so f64 kernels read low).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void\s+)?(?:vo::)?(\w+(?:<[^>]*>)?)", name)
    return m.group(1).replace(" ", "") if m else name[:40]


def pmc(d, prefix, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, f"{prefix}*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d, title = sys.argv[1], sys.argv[2]
    x2 = "--fetch-x2" in sys.argv
    stats = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_stats.csv"))[0])))
    fetch = pmc(d, "fetch", "FETCH_SIZE")
    write = pmc(d, "write", "WRITE_SIZE")
    vinst = pmc(d, "valu", "SQ_INSTS_VALU")
    waves = pmc(d, "valu", "SQ_WAVES")
    grbm = pmc(d, "valu", "GRBM_GUI_ACTIVE")
    table = {}
    print(f"# {title}\n")
    print("rocprofv3 --kernel-trace --stats (durations) and separate --pmc passes: FETCH_SIZE, WRITE_SIZE, and "
          "SQ_INSTS_VALU + SQ_WAVES + GRBM_GUI_ACTIVE.  VALU issue = SQ_INSTS_VALU x 4 / (1024 x "
          "GRBM_GUI_ACTIVE / 8).\n")
    print("| kernel | calls | avg us | share % | FETCH_SIZE KB/launch | WRITE_SIZE KB/launch | HBM bytes/launch | "
          "VALU insts/launch | waves/launch | VALU issue |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for r in stats:
        k = short(r["Name"])
        f, w = fetch.get(k), write.get(k)
        vi, wv, gc = vinst.get(k), waves.get(k), grbm.get(k)
        issue = vi * 4 / (1024 * gc / 8) if vi is not None and gc else None
        hb = "" if f is None or w is None else f"{(f * (2 if x2 else 1) + w) * 1024:,.0f}"
        table[k] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                    "fetch_kb": f, "write_kb": w,
                    "hbm_bytes_per_launch": None if f is None or w is None else (f * (2 if x2 else 1) + w) * 1024,
                    "valu_insts": vi, "waves": wv, "grbm_cycles": gc, "valu_issue_frac": issue}
        print(f"| {k} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} | "
              f"{'' if f is None else f'{f:.1f}'} | {'' if w is None else f'{w:.1f}'} | {hb} | "
              f"{'' if vi is None else f'{vi:,.0f}'} | {'' if wv is None else f'{wv:,.0f}'} | "
              f"{'' if issue is None else f'{issue:.3f}'} |")

    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        json.dump({"title": title, "fetch_x2": x2, "kernels": table}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
