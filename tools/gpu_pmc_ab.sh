# One PMC counter over several bench argument sets (VO_SERIAL=1 as in profile.sh), per-kernel mean
# per launch printed for each:  gpu_pmc_ab.sh <tag> <counter> "<bench args A>" "<bench args B>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp VO_SERIAL=1
O=gpurun_out/$1; C=$2; shift 2; mkdir -p $O
n=0
for a in "$@"; do
  n=$((n + 1))
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/p$n -o pmc -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu --no-variants --no-check $a > $O/p$n.json 2> $O/p$n.err || { echo "PMC_FAIL $a"; tail -5 $O/p$n.err; exit 1; }
  echo "== $a"
  python3 tools/pmc_mean.py $O/p$n $C
done
