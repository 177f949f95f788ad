# per-frame call after describe_pf's term restructure and relaxed polls; RANSAC forms by kernel;
# stall anatomy of the 0.12 m/frame bench (one PMC pass, serial queues)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5i}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_regimes.py tests/test_gpu_reference_sampler.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so PF=1 timeout -k 10 200 python3 tools/stamps_describe.py > $O/stamps_describe_pf.txt 2>&1 || { echo STAMPS_DS_FAIL; tail $O/stamps_describe_pf.txt; exit 1; }
cat $O/stamps_describe_pf.txt
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 MOTION=0.12 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_stage.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_stage.txt; exit 1; }
cat $O/stamps_stage.txt
for e in "VO_X=0" "VO_RANSAC_FUSED=0" "VO_SEL_FUSED=1" "VO_X=0" "VO_RANSAC_FUSED=0" "VO_SEL_FUSED=1"; do
  env $e PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$e $(tail -1 $O/pf.txt)"
done
PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
for rep in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json')); print('0.12', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
VO_SERIAL=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d $O/stall -o stall -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-variants --sequences 1 --motion 0.12 > $O/stall.json 2> $O/stall.err || { echo PMC_FAIL; tail -5 $O/stall.err; exit 1; }
python3 tools/pmc_stall.py $(ls $O/stall/*counter_collection.csv | head -1)

timeout -k 10 60 ./tools/f64_lat > $O/f64_lat.txt 2>&1 && cat $O/f64_lat.txt
echo DONE
