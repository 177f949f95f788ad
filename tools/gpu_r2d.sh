set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread -k "extract or config2 or windowed or host" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_env.sh r2d_xcd "VO_XCD=1" "VO_XCD=0" || exit 1
bash tools/gpu_ab_env.sh r2d_xcd1080 "VO_XCD=1" "VO_XCD=0" -- --width 1920 --height 1080 --max-kpts 4096 --frames 64 --sequences 2 || exit 1
for f in 0 8 16 32; do VO_FIRST=$f timeout -k 10 200 python -u tools/host_stream_diag.py > $O/hs_$f.json 2>$O/hs_$f.err || { echo HS_FAIL; tail $O/hs_$f.err; exit 1; }; cat $O/hs_$f.json; done
