# KITTI: extract batch size A/B (64 default vs 72 / 80 / 96)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5t}; mkdir -p $O
for rep in 1 2 3; do for b in 64 72 80 96; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-variants --batch $b > $O/b.json 2> $O/b.err || { echo "KITTI BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('KITTI batch $b', round(d['value']))"
done; done
echo DONE
