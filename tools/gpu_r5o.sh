# drain: the chunk's last B frames in smaller batches (VO_LAST), KITTI and 0.12 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5o}; mkdir -p $O
for rep in 1 2; do for e in "VO_LAST=0" "VO_LAST=16" "VO_LAST=32"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo "KITTI BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('KITTI $e', round(d['value']))"
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('0.12 $e', round(d['value']))"
done; done
echo DONE
