#!/usr/bin/env python3
"""Per-frame timeline of a rocprofv3 --kernel-trace CSV of bench.py (two-stream pipeline).

usage: timeline.py <trace_kernel_trace.csv> [frames_per_step]
Prints, over the last timed step: the frame period (successive k_triangulate ends), each
kernel's median duration and VGPR/SGPR/scratch, and the median gap in front of each pose-chain
kernel (the dependent-launch boundary plus any wait for the extract stream)."""
import csv
import re
import sys
from collections import defaultdict

import numpy as np


def short(n):
    m = re.match(r"(?:void\s+)?(?:vo::)?(\w+)", n)
    return m.group(1) if m else n


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ks = [dict(name=short(r["Kernel_Name"]), q=r["Queue_Id"], s=int(r["Start_Timestamp"]),
               e=int(r["End_Timestamp"]), vgpr=r["VGPR_Count"], sgpr=r["SGPR_Count"], scratch=r["Scratch_Size"],
               lds=r["LDS_Block_Size"]) for r in rows]
    ks.sort(key=lambda k: k["s"])
    tri = [k for k in ks if k["name"] == "k_triangulate"]
    last = tri[-F:]
    t0, t1 = last[0]["s"], last[-1]["e"]
    sel = [k for k in ks if t0 - 1 <= k["s"] and k["e"] <= t1 + 1]
    ends = np.array([k["e"] for k in last], dtype=np.float64)
    per = np.diff(ends) / 1e3
    print(f"frames {len(last)}: period median {np.median(per):.1f} us, mean {per.mean():.1f} us "
          f"-> {1e6 / per.mean():.0f} frames/s (span {(t1 - t0) / 1e3:.0f} us)")
    dur = defaultdict(list)
    meta = {}
    for k in sel:
        dur[k["name"]].append((k["e"] - k["s"]) / 1e3)
        meta[k["name"]] = (k["q"], k["vgpr"], k["sgpr"], k["scratch"], k["lds"])
    print(f"{'kernel':16s} {'n':>5s} {'med us':>8s} {'mean us':>8s}  queue vgpr sgpr scratch lds")
    for n, v in sorted(dur.items(), key=lambda x: -np.sum(x[1])):
        q, vg, sg, sc, l = meta[n]
        print(f"{n:16s} {len(v):5d} {np.median(v):8.2f} {np.mean(v):8.2f}  {q:>5s} {vg:>4s} {sg:>4s} {sc:>7s} {l:>5s}")
    byq = defaultdict(list)
    for k in sel:
        byq[k["q"]].append(k)
    print("gap in front of each kernel on its queue (median us):")
    for q, lst in byq.items():
        gaps = defaultdict(list)
        for a, b in zip(lst, lst[1:]):
            gaps[b["name"]].append((b["s"] - a["e"]) / 1e3)
        busy = sum(k["e"] - k["s"] for k in lst) / (t1 - t0)
        print(f"  queue {q}: busy {busy * 100:.0f}%  " +
              "  ".join(f"{n}:{np.median(g):.1f}" for n, g in gaps.items()))


if __name__ == "__main__":
    main()
