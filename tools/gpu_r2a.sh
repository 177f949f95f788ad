set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2a; mkdir -p $O
for m in 1.0 0.12 0.05; do
timeout -k 10 300 python -u bench.py --no-cpu --breakdown --motion $m > $O/bench_$m.json 2> $O/bench_$m.err || { echo BENCH_FAIL; tail -20 $O/bench_$m.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$m.json'));c=d['config'];print('$m VALUE',round(d['value'],1),'hyp',c['mean_hypotheses'],'inl',c['mean_inliers'],'M',c['mean_matches'])"
cat $O/bench_$m.err
done
