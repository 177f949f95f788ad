"""bench.py's N>1 harness on world_size 2 over gloo (CPU): the partitions (strong, config 5:
sequence s on rank s mod G; weak: every rank its own block of sequences), the barrier +
max-over-ranks time with the summed frames, and the all_gather of raw row bits that assembles
every sequence's pose rows on every rank -- checked against the rows one rank computes alone, -0.0
and NaN payloads included.  On the GPU node the same functions run over RCCL."""
import os
import socket

import numpy as np
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
    r[0, 0] = -0.0                        # a SUM all-reduce would return +0.0 here
    r[1, 1] = np.array([0x7FF8DEADBEEF0001], np.int64).view(np.float64)[0]   # NaN with a payload
    return r


def _rank(rank, world, port, q, n_seq=8, nframes=7, scaling="strong"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, ROOT)
    import bench
    dist = bench.dist_init(world, rank, backend="gloo")
    dist.barrier()
    dt = 1.0 + rank                       # rank 1 is the slow one
    mine = bench.rank_sequences(n_seq, rank, world, scaling)
    owners = [bench.rank_sequences(n_seq, r, world, scaling) for r in range(world)]
    dt_max, value = bench.aggregate(dist, dt, frames_per_rank=100 * len(mine), world=world, backend="gloo")
    gathered = bench.gather_poses(dist, {s: _rows(s, nframes) for s in mine}, owners, nframes, backend="gloo")
    q.put((rank, dt_max, value, mine, gathered))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,scaling", [(2, "strong"), (2, "weak")])
def test_bench_aggregate_gloo(world, scaling):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, 8, 7, scaling)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_all = 8 if scaling == "strong" else 8 * world
    owned = sorted(s for r in res for s in r[3])
    assert owned == list(range(n_all))              # every sequence on exactly one rank
    if scaling == "strong":
        assert res[0][3] == [0, 2, 4, 6] and res[1][3] == [1, 3, 5, 7]
    else:
        assert res[0][3] == list(range(8)) and res[1][3] == list(range(8, 16))
    single = np.stack([_rows(s, 7) for s in range(n_all)])
    for rank, dt_max, value, mine, gathered in res:
        assert dt_max == float(world)               # max over ranks
        assert value == pytest.approx(100 * n_all / world)   # all ranks' frames / slowest time
        # the gather equals one rank computing all, bit for bit (-0.0 and NaN payloads kept)
        assert np.array_equal(gathered.view(np.int64), single.view(np.int64))


def test_single_rank_has_no_collective():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    assert bench.dist_init(1, 0) is None
    assert bench.aggregate(None, 2.0, 50, 1) == (2.0, 25.0)
    assert bench.rank_sequences(8, 0, 1) == list(range(8))
    assert [bench.rank_sequences(8, r, 4) for r in range(4)] == [[0, 4], [1, 5], [2, 6], [3, 7]]
    assert [bench.rank_sequences(2, r, 3, "weak") for r in range(3)] == [[0, 1], [2, 3], [4, 5]]
    rows = {s: _rows(s, 5) for s in range(8)}
    out = bench.gather_poses(None, rows, [list(range(8))], 5)
    assert np.array_equal(out.view(np.int64), np.stack([rows[s] for s in range(8)]).view(np.int64))
