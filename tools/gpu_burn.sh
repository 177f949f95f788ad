# extract-only determinism next to unrelated MFMA / VALU load on a torch stream
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-burn}; mkdir -p $O
for m in mfma valu none mfma; do
  timeout -k 10 240 python -u tools/det_burn.py 12 $m > $O/burn_$m.txt 2>&1 || { echo BURN_FAIL $m; tail -20 $O/burn_$m.txt; exit 1; }
  grep -E "frames differ \[[0-9]|repeats differ" $O/burn_$m.txt | head -8
done
echo DONE
