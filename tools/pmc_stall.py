#!/usr/bin/env python3
"""Per-kernel stall anatomy from tools/gpu_pmc_stall.sh: per wave, the cycles it existed
(SQ_WAVE_CYCLES / SQ_WAVES), the share spent waiting on anything / on an instruction dependency
(SQ_WAIT_ANY, SQ_WAIT_INST_ANY), and the VALU / LDS issue shares (SQ_ACTIVE_INST_*).
usage: pmc_stall.py <stall_counter_collection.csv>"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.match(r"(?:void\s+)?(?:vo::)?(\w+)", n)
    return m.group(1) if m else n[:40]


acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = short(r["Kernel_Name"])
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
print(f"{'kernel':28s} {'disp':>5s} {'waves':>9s} {'cyc/wave':>9s} {'wait%':>6s} {'dep%':>6s} {'valu%':>6s} {'lds%':>6s} {'lds/wave':>8s}")
for k, c in sorted(acc.items(), key=lambda x: -x[1].get("SQ_WAVE_CYCLES", 0)):
    w = c.get("SQ_WAVES", 0) or 1
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k:28s} {len(disp[k]):5d} {w:9.0f} {wc / w:9.0f} {100 * c.get('SQ_WAIT_ANY', 0) / wc:6.1f} "
          f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} {100 * c.get('SQ_ACTIVE_INST_VALU', 0) / wc:6.1f} "
          f"{100 * c.get('SQ_ACTIVE_INST_LDS', 0) / wc:6.1f} {c.get('SQ_INSTS_LDS', 0) / w:8.0f}")
