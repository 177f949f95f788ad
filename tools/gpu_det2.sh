# determinism stress of the headline stream under execution knobs (args: out-tag repeats knob...)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det2}; mkdir -p $O
R=$2
shift 2
for e in "$@"; do
  echo "== $e"
  env $e timeout -k 10 240 python -u tools/det_stress.py $R 0 > $O/det.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det.txt; exit 1; }
  grep -E "DIFFERS|seq|frame|full path" $O/det.txt | head -24
done
echo DONE
