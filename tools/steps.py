#!/usr/bin/env python3
"""Per-step phases of a bench kernel trace: from each k_reset (step start) to the first
extract, the first pose pass, the last extract and the last finalize of that step."""
import csv
import re
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("vo::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2] == "k_reset"]
starts.append(len(rows))
t_prev_end = None
for a, b in zip(starts[:-1], starts[1:]):
    seg = rows[a:b]
    t0 = seg[0][0]
    first = lambda name: next((s for s, e, k in seg if k.startswith(name)), None)
    last_end = lambda name: max((e for s, e, k in seg if k.startswith(name)), default=None)
    us = lambda t: None if t is None else round((t - t0) / 1e3, 1)
    nfin = sum(1 for r in seg if r[2] == "k_finalize")
    print(f"step: first stencil {us(first('k_stencil'))}  first match {us(first('k_match'))}  "
          f"last describe end {us(last_end('k_describe'))}  last finalize end {us(last_end('k_finalize'))}  "
          f"next step in {us(rows[b][0]) if b < len(rows) else None}  passes {nfin}")
