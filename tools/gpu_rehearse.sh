# the N > 1 bench line rehearsed on the one-GPU box: two ranks under torch.distributed.run sharing
# GPU 0 over gloo (the RCCL path differs in the backend and one device per rank).
# Usage: gpu_rehearse.sh <tag> [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-rehearse}; shift; mkdir -p $O
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --backend gloo --device 0 --steps 5 --warmup 2 "$@" > $O/bench2.json 2> $O/bench2.err || { echo REH_FAIL; tail -30 $O/bench2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench2.json').read().strip().splitlines()[-1]);print('VALUE',round(d['value']),d['n_gpus'],d['scaling']);print(d['determinism']);print(json.dumps(d['cpu_baseline'])[:900]);print(json.dumps(d.get('config5_strong'))[:900])"
