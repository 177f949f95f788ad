#!/usr/bin/env python3
"""Mean of one PMC counter per launch, per kernel, from a rocprofv3 --pmc CSV directory
(tools/gpu_pmc_ab.sh).  usage: pmc_mean.py <dir> <counter>"""
import csv
import glob
import re
import sys
from collections import defaultdict

d, c = sys.argv[1], sys.argv[2]
f = sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True))
if not f:
    sys.exit(f"no counter_collection.csv under {d}")
per = defaultdict(lambda: defaultdict(float))          # kernel -> dispatch -> value
for r in csv.DictReader(open(f[0])):
    if r.get("Counter_Name") != c:
        continue
    n = re.match(r"(?:void\s+)?(?:vo::)?([\w<>, ]+?)(?:\(|$)", r["Kernel_Name"])
    per[n.group(1) if n else r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1].values()) / len(kv[1])):
    vals = list(v.values())
    print(f"  {k:40s} launches {len(vals):4d}  mean {sum(vals) / len(vals):14.1f}")
