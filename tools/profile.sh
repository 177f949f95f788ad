#!/bin/bash
# Kernel-duration profile plus separate PMC passes of bench.py (MI355X_MICROARCH.md "rocprofv3
# PMC slots": FETCH_SIZE and WRITE_SIZE cannot share a pass; no trace domain is combined with
# --pmc).  Run on the GPU box:
#   tools/profile.sh gpurun_out/prof_<tag> [extra bench.py args]
# then summarise with tools/rocprof_summary.py <dir> "<title>" --fetch-x2 --json <file>.
set -eo pipefail
OUT=$(realpath -m "$1"); shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
# the headline workload (8 sequences as one stream), without the after-timing check runs, so the
# average launch of every kernel is the bench's own launch
B="--steps 3 --warmup 1 --no-cpu --no-variants --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o stats -- \
    python3 bench.py $B "$@" > "$OUT/bench_stats.json"
# PMC collection serializes dispatches, so the frame pipeline's cross-queue waits would spin
# into their timeouts: the counter passes run every kernel on one queue (same kernels, same
# bytes; VO_SERIAL=1)
export VO_SERIAL=1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o fetch -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu --no-variants --no-check "$@" > "$OUT/bench_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o write -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu --no-variants --no-check "$@" > "$OUT/bench_write.json"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$OUT" -o valu -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu --no-variants --no-check "$@" > "$OUT/bench_valu.json"
echo "profile written to $OUT"
