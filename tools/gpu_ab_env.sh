# A/B of environment knobs over the bench (no CPU leg, no variants), two alternating rounds:
#   gpu_ab_env.sh <tag> "<env A>" "<env B>" [...] -- [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O; shift
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ "$1" == "--" ] && shift
for rep in 1 2; do
for e in "${ENVS[@]}"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants "$@" > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
