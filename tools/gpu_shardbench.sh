# within-sequence sharding: GPU parity, bench at 1 rank, and 2 ranks sharing the box's GPU over gloo (rehearsal)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-shb}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -k "shard" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_shard.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest_shard.log; exit 1; }
tail -2 $O/pytest_shard.log
timeout -k 10 300 python -u bench.py --shard-sequence --steps 5 --warmup 1 > $O/shard1.json 2> $O/shard1.err || { echo SH1_FAIL; tail -20 $O/shard1.err; exit 1; }
cat $O/shard1.json
for M in 1.0 0.12; do
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --shard-sequence --gpus 2 --backend gloo --device 0 --steps 5 --warmup 1 --motion $M > $O/shard2_$M.json 2> $O/shard2_$M.err || { echo SH2_FAIL; tail -30 $O/shard2_$M.err; exit 1; }
cat $O/shard2_$M.json
done
