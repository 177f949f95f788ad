# frames/s over frame_batch and first-batch sizes (no CPU leg): gpu_sweep_batch.sh [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sweep_batch; mkdir -p $O
for cfg in "64 0" "64 16" "64 32" "64 8"; do
  set -- $cfg
  VO_FIRST=$2 timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --batch $1 "${@:3}" > $O/b.json 2> $O/b.err || { echo FAIL $cfg; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('batch $1 first $2', round(d['value'],1))"
done
