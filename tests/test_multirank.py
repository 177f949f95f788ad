"""bench.py's N>1 harness (replicas: barrier + max-over-ranks time, whole-job frames/s) on
world_size 2 over gloo (CPU).  On the GPU node the same functions run over RCCL."""
import os
import socket

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, ROOT)
    import bench
    dist = bench.dist_init(world, rank, backend="gloo")
    dist.barrier()
    dt = 1.0 + rank                       # rank 1 is the slow one
    dt_max, value = bench.aggregate(dist, dt, frames_per_rank=100, world=world, backend="gloo")
    q.put((rank, dt_max, value))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_bench_aggregate_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, dt_max, value in res:
        assert dt_max == float(world)               # max over ranks
        assert value == pytest.approx(100 * world / world)   # all ranks' frames / slowest time


def test_single_rank_has_no_collective():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    assert bench.dist_init(1, 0) is None
    assert bench.aggregate(None, 2.0, 50, 1) == (2.0, 25.0)
