# bench sweep over frame_batch / sequence length (no CPU leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-sweep}; mkdir -p $O
for cfg in "--batch 8" "--batch 16" "--batch 32" "--batch 64" "--batch 16 --frames 1000" "--batch 32 --frames 1000"; do
  timeout -k 10 200 python -u bench.py --no-cpu $cfg > $O/b.json 2> $O/b.err || { echo FAIL $cfg; tail -5 $O/b.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/b.json'));print('$cfg', round(d['value'],1), d['roofline']['kernel'])"
done
