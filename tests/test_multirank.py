"""bench.py's N>1 harness on world_size 2 over gloo (CPU): the config-5 partition (sequence s
on rank s mod G), the barrier + max-over-ranks time with the summed frames, and the all-reduce
that assembles every sequence's pose rows on every rank, checked against the rows one rank
computes alone.  On the GPU node the same functions run over RCCL."""
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


def _rows(s, nframes):
    """Stand-in for sequence s's pose rows: any deterministic function of (s, frame)."""
    import numpy as np
    rng = np.random.default_rng(1000 + s)
    r = rng.standard_normal((nframes, 13))
    r[:, 12] = rng.integers(0, 5, nframes)
    return r


def _rank(rank, world, port, q, n_seq=8, nframes=7):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, ROOT)
    import bench
    dist = bench.dist_init(world, rank, backend="gloo")
    dist.barrier()
    dt = 1.0 + rank                       # rank 1 is the slow one
    mine = bench.rank_sequences(n_seq, rank, world)
    dt_max, value = bench.aggregate(dist, dt, frames_per_rank=100 * len(mine), world=world, backend="gloo")
    gathered = bench.gather_poses(dist, {s: _rows(s, nframes) for s in mine}, n_seq, nframes, backend="gloo")
    q.put((rank, dt_max, value, mine, gathered))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_bench_aggregate_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    owned = sorted(s for r in res for s in r[3])
    assert owned == list(range(8))                  # every sequence on exactly one rank
    assert res[0][3] == [0, 2, 4, 6] and res[1][3] == [1, 3, 5, 7]
    single = np.stack([_rows(s, 7) for s in range(8)])
    for rank, dt_max, value, mine, gathered in res:
        assert dt_max == float(world)               # max over ranks
        assert value == pytest.approx(100 * 8 / world)   # all ranks' frames / slowest time
        assert np.array_equal(gathered, single)     # the gather equals one rank computing all


def test_single_rank_has_no_collective():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    assert bench.dist_init(1, 0) is None
    assert bench.aggregate(None, 2.0, 50, 1) == (2.0, 25.0)
    assert bench.rank_sequences(8, 0, 1) == list(range(8))
    assert [bench.rank_sequences(8, r, 4) for r in range(4)] == [[0, 4], [1, 5], [2, 6], [3, 7]]
