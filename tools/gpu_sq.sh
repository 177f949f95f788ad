# one SQ PMC pass over the default bench (serial queue), summarised per kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sq}; mkdir -p $O
shift
export VO_SERIAL=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O -o sq -- python3 bench.py --steps 1 --warmup 1 --no-cpu "$@" > $O/bench.json 2> $O/bench.err || { echo PMC_FAIL; tail -5 $O/bench.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, re
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(lambda: defaultdict(int))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("vo::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[k][r["Counter_Name"]] += 1
for k, d in acc.items():
    n = cnt[k]["SQ_WAVES"] or 1
    print(k, "launches", n, " ".join(f"{c}={v / n:.4g}" for c, v in sorted(d.items())))
PY
