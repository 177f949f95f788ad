#!/usr/bin/env python3
"""Queue-level anatomy of a rocprofv3 --kernel-trace CSV of bench.py (two-queue pipeline).

usage: pass_timeline.py <trace_kernel_trace.csv> [n_last_launches]
Over the last n launches (default: all of the last 40 % of the trace): per queue, the busy
fraction, the time per kernel (sum, count, mean), the gaps in front of each kernel, and one
pose pass (k_match .. k_finalize) launch by launch with start offsets and durations."""
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
    ks = [dict(name=short(r["Kernel_Name"]), q=r["Queue_Id"], s=int(r["Start_Timestamp"]), e=int(r["End_Timestamp"]))
          for r in rows]
    ks.sort(key=lambda k: k["s"])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else int(len(ks) * 0.4)
    sel = ks[-n:]
    t0, t1 = sel[0]["s"], max(k["e"] for k in sel)
    span = (t1 - t0) / 1e3
    print(f"{len(sel)} launches over {span:.0f} us")
    byq = defaultdict(list)
    for k in sel:
        byq[k["q"]].append(k)
    for q, lst in byq.items():
        busy = sum(k["e"] - k["s"] for k in lst) / 1e3
        print(f"queue {q}: busy {busy:.0f} us ({100 * busy / span:.0f} %)")
        per = defaultdict(list)
        gaps = defaultdict(list)
        for a, b in zip(lst, lst[1:]):
            gaps[b["name"]].append((b["s"] - a["e"]) / 1e3)
        for k in lst:
            per[k["name"]].append((k["e"] - k["s"]) / 1e3)
        for name, v in sorted(per.items(), key=lambda x: -sum(x[1])):
            g = gaps.get(name, [0.0])
            print(f"   {name:28s} n {len(v):4d}  sum {sum(v):8.1f}  mean {np.mean(v):7.1f}  gap-before mean "
                  f"{np.mean(g):6.1f}")
    # one pose pass in the middle of the selection
    m = [i for i, k in enumerate(sel) if k["name"].startswith("k_match")]
    if len(m) >= 3:
        i0 = m[len(m) // 2]
        q = sel[i0]["q"]
        lst = [k for k in sel[i0:] if k["q"] == q]
        base = lst[0]["s"]
        print("one pose pass (us from k_match start: start / duration):")
        for k in lst:
            print(f"   {k['name']:28s} {(k['s'] - base) / 1e3:8.1f} {(k['e'] - k['s']) / 1e3:8.1f}")
            if k["name"] == "k_finalize":
                break


if __name__ == "__main__":
    main()
