# Round evidence, profiles first and the bench second from one build: rocprofv3 duration + PMC
# passes of the given workloads (tools/profile.sh), summarised into profiles/<round>_<w>_kernels.{md,json}
# on the box (bench.py reads them: PROFILES) and copied to gpurun_out; then the default bench line.
# Usage: gpu_evidence.sh <round: r4> <out-tag> <workloads: kitti kitti_012 1080 1080_512 ...> [bench]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r4}; shift
O=gpurun_out/${1:-${R}prof}; shift; mkdir -p $O
BUILD=$(tr "\n" " " < BUILD_ID 2>/dev/null || echo unknown)
for w in "$@"; do
  case $w in
    kitti) A="" ; T="kitti: bench.py --no-variants --no-check (8 sequences at 1.0 m/frame, the headline workload)";;
    kitti_012) A="--motion 0.12 --sequences 1" ; T="kitti 0.12 m/frame: bench.py --motion 0.12 --sequences 1 (the low-inlier variant's workload)";;
    1080) A="--width 1920 --height 1080 --max-kpts 4096 --frames 64 --sequences 1" ; T="1920x1080 N=4096 32-test: the config-4 variant's workload";;
    1080_512) A="--width 1920 --height 1080 --max-kpts 4096 --frames 64 --sequences 1 --match-bits 512" ; T="1920x1080 N=4096 512-test: the config-4 variant's workload";;
    bench) continue;;
    *) echo "unknown workload $w"; exit 1;;
  esac
  bash tools/profile.sh $O/prof_$w $A > $O/prof_$w.log 2>&1 || { echo PROF_FAIL $w; tail -20 $O/prof_$w.log; exit 1; }
  python3 tools/rocprof_summary.py $O/prof_$w "$R (build $BUILD) $T" --fetch-x2 --json profiles/${R}_${w}_kernels.json > profiles/${R}_${w}_kernels.md || { echo SUM_FAIL $w; exit 1; }
  cp $O/prof_$w/stats_kernel_stats.csv profiles/${R}_${w}_kernel_stats.csv
  cp profiles/${R}_${w}_kernels.* profiles/${R}_${w}_kernel_stats.csv $O/
  head -16 profiles/${R}_${w}_kernels.md | tail -12
done
case " $* " in *" bench "*)
  timeout -k 10 600 python -u bench.py --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('VALUE',round(d['value']),'dominant',r['kernel'],'live',r['avg_launch_ms'],'rocprof',r['rocprof_avg_launch_us'],r['traffic_source']);print(d['determinism']);print(json.dumps(d['variants'],indent=0)[:2500]);print(json.dumps(d['cpu_baseline'])[:500])"
  cat $O/bench.err;;
esac
echo DONE
