# A/B of queue priorities (VO_PRIO 0 / 1 / -1), alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-prio}; mkdir -p $O
for i in 1 2 3; do for P in 0 1 -1; do
VO_PRIO=$P timeout -k 10 300 python -u bench.py --no-cpu --no-variants --no-check > $O/b_${P}_$i.json 2> $O/b_${P}_$i.err || { echo BENCH_FAIL; tail -20 $O/b_${P}_$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_${P}_$i.json'));print('PRIO=$P', round(d['value']))"
done; done
