#!/usr/bin/env python3
"""Per-call timeline of the single-frame path (tools/pf_loop.py under rocprofv3 --kernel-trace
[--memory-copy-trace]): for the calls after the first few, the median duration of each kernel and
copy, the median gap in front of it, and the device span of a call (first op start -> last op end).

usage: pf_timeline.py <dir with *kernel_trace.csv [+ *memory_copy_trace.csv]>"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

import numpy as np


def short(n):
    m = re.match(r"(?:void\s+)?(?:vo::)?(\w+)", n)
    return m.group(1) if m else n


def main():
    d = sys.argv[1]
    ops = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy_" + r.get("Direction", "?"), "copy"))
    ops.sort()
    starts = [i for i, o in enumerate(ops) if o[2].startswith("k_stencil")]
    calls = [ops[a:b] for a, b in zip(starts, starts[1:])][5:]
    dur, gap, span = defaultdict(list), defaultdict(list), []
    for c in calls:
        # ops of the call: up to the last k_traj (later ops belong to the next call's upload)
        last = max(i for i, o in enumerate(c) if o[2] == "k_traj") if any(o[2] == "k_traj" for o in c) else len(c) - 1
        c = c[:last + 1]
        span.append((c[-1][1] - c[0][0]) / 1e3)
        prev_end = None
        for s, e, n, q in c:
            dur[n].append((e - s) / 1e3)
            if prev_end is not None:
                gap[n].append((s - prev_end) / 1e3)
            prev_end = max(prev_end or 0, e)
    print(f"calls {len(calls)}: device span per call median {np.median(span):.1f} us (stencil start -> k_traj end)")
    print(f"{'op':22s} {'n/call':>6s} {'med us':>8s} {'gap before':>10s}")
    for n in dur:
        print(f"{n:22s} {len(dur[n]) / max(len(calls), 1):6.1f} {np.median(dur[n]):8.2f} "
              f"{np.median(gap[n]) if gap[n] else 0:10.2f}")
    print(f"sum of op medians x count: {sum(np.median(v) * len(v) for v in dur.values()) / max(len(calls), 1):.1f} us")


if __name__ == "__main__":
    main()
