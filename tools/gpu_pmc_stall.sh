# stall anatomy per kernel: one rocprofv3 PMC pass (8 SQ counters) over the bench on one queue
#   gpu_pmc_stall.sh <tag>   then tools/pmc_stall.py gpurun_out/<tag>/stall_counter_collection.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp VO_SERIAL=1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d $O -o stall -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-variants --sequences 1 > $O/stall.json 2> $O/stall.err || { echo PMC_FAIL; tail -5 $O/stall.err; exit 1; }
echo PMC_OK
