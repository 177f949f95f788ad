#!/usr/bin/env python3
"""Pose-pass anatomy of one bench step from a rocprofv3 --kernel-trace CSV (tools/gpu_trace.sh).

usage: step_timeline.py <tr_kernel_trace.csv> [step index (default: the 4th k_reset interval)]
Steps are the intervals between k_reset launches (bench.py resets before every run); prints the
interval's span, per-queue busy time, and every pose pass (k_match .. k_finalize) with its start,
span and per-kernel durations, plus the extract batches' stencil start times."""
import csv
import re
import sys
from collections import Counter, defaultdict


def short(n):
    m = re.match(r"(?:void\s+)?(?:vo::)?(\w+)", n)
    return m.group(1) if m else n


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted([dict(n=short(r["Kernel_Name"]), q=r["Queue_Id"], s=int(r["Start_Timestamp"]),
                      e=int(r["End_Timestamp"])) for r in rows], key=lambda k: k["s"])
    resets = [i for i, k in enumerate(ks) if k["n"] == "k_reset"] + [len(ks)]
    spans = list(zip(resets, resets[1:]))
    for a, b in spans:
        seg = ks[a:b]
        c = Counter(k["n"] for k in seg)
        busy = defaultdict(float)
        for k in seg:
            busy[k["q"]] += (k["e"] - k["s"]) / 1e3
        print(f"interval: span {(max(k['e'] for k in seg) - seg[0]['s']) / 1e3:8.0f} us  batches {c['k_stencil']:3d}"
              f"  passes {c['k_match']:3d}  busy " + " ".join(f"q{q}:{v:.0f}" for q, v in busy.items()))
    idx = int(sys.argv[2]) if len(sys.argv) > 2 else min(4, len(spans) - 1)
    a, b = spans[idx]
    seg = ks[a:b]
    t0 = seg[0]["s"]
    pq = Counter(k["q"] for k in seg if k["n"].startswith("k_match")).most_common(1)[0][0]
    print("interval", idx, "stencil starts (us):", [round((k["s"] - t0) / 1e3) for k in seg if k["n"] == "k_stencil"])
    passes, cur = [], None
    for k in seg:
        if k["q"] != pq or not k["n"].startswith("k_"):
            continue
        if k["n"].startswith("k_match"):
            cur = [k]
            passes.append(cur)
        elif cur is not None:
            cur.append(k)
    for i, p in enumerate(passes):
        print(f"pass {i:2d} start {(p[0]['s'] - t0) / 1e3:8.0f} span {(p[-1]['e'] - p[0]['s']) / 1e3:6.1f} "
              + " ".join(f"{k['n'][2:6]}:{(k['e'] - k['s']) / 1e3:.0f}" for k in p))


if __name__ == "__main__":
    main()
