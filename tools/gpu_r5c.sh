set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 60 ./tools/valu_rate > $O/valu_rate.txt 2>&1 || { echo VALU_FAIL; cat $O/valu_rate.txt; exit 1; }
cat $O/valu_rate.txt
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_nopk.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/nopk_tests.log 2>&1 || { echo NOPK_TESTS_FAIL; tail -30 $O/nopk_tests.log; exit 1; }
tail -1 $O/nopk_tests.log
bash tools/gpu_ab_reps.sh r5c_ab 4 "libvo_mi355x.so libvo_mi355x_nopk.so" || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('VALUE',round(d['value']));print(d['determinism']);print(json.dumps(d['cpu_baseline'])[:1500])"
