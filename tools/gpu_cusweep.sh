# bench.py under different CU splits of the two frame-pipeline queues (VO_CU_POSE)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cusweep; mkdir -p $O
for cu in 0 64 96 128 160; do
  VO_CU_POSE=$cu timeout -k 10 120 python -u bench.py --no-cpu --breakdown > $O/b$cu.json 2> $O/b$cu.err || { echo BENCH_FAIL $cu; tail -5 $O/b$cu.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$cu.json'));print('CU_POSE $cu VALUE',round(d['value'],1),{k:round(v*1e3,1) for k,v in d['kernels_ms_per_frame'].items()})"
done
