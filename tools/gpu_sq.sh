# one SQ PMC pass over the default bench (serial queue), summarised per kernel and per frame
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
frames = 3 * 200          # warmup + timing pass + 1 step
tot = 0.0
for k, d in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0)):
    if not k.startswith("k_"): continue
    v = d["SQ_INSTS_VALU"] / frames; tot += v
    print(f"{k:22s} VALU/frame {v/1e3:8.1f}k  LDS/frame {d['SQ_INSTS_LDS']/frames/1e3:7.1f}k  waves/frame {d['SQ_WAVES']/frames:7.1f}  "
          f"wave-cycles/frame {d['SQ_WAVE_CYCLES']/frames/1e6:6.2f}M  wait {d['SQ_WAIT_ANY']/max(d['SQ_WAVE_CYCLES'],1):.2f} issue-stall {d['SQ_WAIT_INST_ANY']/max(d['SQ_WAVE_CYCLES'],1):.2f}")
print(f"total VALU wave-instr per frame {tot/1e3:.1f}k -> {tot*4/1024/2.4e3:.2f} us/frame at 4 cycles each over 1024 SIMDs at 2.4 GHz")
PY
