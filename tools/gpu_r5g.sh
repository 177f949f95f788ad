# RANSAC anatomy at 0.12 m/frame: s_memtime phase stamps (batched and stage) and a kernel trace
# of the low-inlier bench variant for the queue timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5g}; mkdir -p $O
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so MOTION=0.12 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_batched.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_batched.txt; exit 1; }
cat $O/stamps_batched.txt
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 MOTION=0.12 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_stage.txt 2>&1 || { echo STAMPS2_FAIL; tail $O/stamps_stage.txt; exit 1; }
cat $O/stamps_stage.txt
timeout -k 10 300 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/bench012.json 2> $O/bench012.err || { echo BENCH_FAIL; tail $O/bench012.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench012.json'));print('VALUE012',round(d['value']))"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/trace.json 2>&1 || { echo TRACE_FAIL; exit 1; }
python3 tools/pass_timeline.py $(ls $O/trace/*kernel_trace.csv | head -1) > $O/pass_timeline.txt 2>&1; cat $O/pass_timeline.txt
echo DONE
