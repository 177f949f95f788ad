# A/B of an environment knob over the bench (no CPU leg): gpu_ab_env.sh <tag> "<env A>" "<env B>" [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O; A="$2"; Bv="$3"; shift 3
for rep in 1 2; do
for e in "$A" "$Bv"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu "$@" > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$e', round(d['value'],1))"
done
done
