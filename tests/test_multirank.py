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


class _StandInContext:
    """The engine interface bench.main() drives (acs_visual_odometry_amd.Context), restated over the
    CPU oracle so the N > 1 harness runs end to end on a machine without a GPU.  Test infrastructure
    only: bench.context_class() returns the HIP library's Context everywhere else."""

    def __init__(self, W, H, K=None, max_kpts=2000, match_bits=32, **_):
        import types
        self.W, self.H, self.K, self.N, self.bits = W, H, K, max_kpts, match_bits
        self.cfg = types.SimpleNamespace(frame_batch=0)
        self.gt, self.starts = None, []

    class _Frames:
        def __init__(self, frames):
            self.frames, self.n = frames, frames.shape[0]

        def free(self):
            pass

    def device_frames(self, frames):
        return self._Frames(np.ascontiguousarray(frames))

    def reset(self):
        pass

    def set_ground_truth(self, gt):
        self.gt = gt

    def set_sequence_starts(self, starts):
        self.starts = list(starts)

    def process_frames_device(self, df, timing=0):
        import oracle as O
        cfg = O.config(self.W, self.H, K=np.asarray(self.K).reshape(9), max_kpts=self.N, match_bits=self.bits)
        bounds = [0] + self.starts + [df.n]
        poses, st, info = np.zeros((df.n, 3, 4)), np.zeros(df.n, np.int32), np.zeros((df.n, 8), np.int32)
        for a, b in zip(bounds[:-1], bounds[1:]):
            vo = O.VO(cfg, gt=self.gt[a:b])
            for f in range(a, b):
                p, s, i = vo.process(df.frames[f])
                poses[f], st[f], info[f, :len(i)] = p, s, i[:8]
            vo.close()
        return poses, st, info

    def kernel_stats(self):
        return {k: (0.01 * (i + 1), 4.0) for i, k in enumerate(["stencil", "select", "describe", "match", "ransac"])}

    def kernel_forms(self):
        import bench
        return {k: [v] for k, v in bench.ROCPROF_NAME.items()}

    def device_errors(self):
        return 0

    def close(self):
        pass


def _bench_rank(rank, world, port, q, argv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), VO_CPU_SHARE="2")
    import contextlib
    import io
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import bench
    from test_multirank import _StandInContext
    bench.context_class = lambda: _StandInContext
    sys.argv = ["bench.py"] + argv
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        bench.main()
    q.put((rank, out.getvalue()))


def test_bench_line_world2_gloo_is_complete():
    """bench.main() itself on two gloo ranks: the N > 1 line carries the CPU
    baseline (timed by rank 0 before dist_init, with its core counts), the oracle-row check of rank 0's
    first sequence, the headline roofline and config 5's own roofline -- the engine is the oracle-backed
    stand-in above, so this checks the harness, not the kernels (the one-GPU gloo rehearsal does that)."""
    import json
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    argv = ["--gpus", "2", "--backend", "gloo", "--device", "0", "--frames", "3", "--sequences", "1",
            "--steps", "1", "--warmup", "1", "--cpu-seconds", "0.2", "--no-variants"]
    procs = [ctx.Process(target=_bench_rank, args=(r, 2, port, q, argv)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] == ""                                   # rank 0 alone prints
    line = json.loads(res[0].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["sequences"] == 2
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["value"] > 0 and cpu["cores"] == 2
    assert cpu["host"]["share"] == 2 and cpu["host"]["affinity_logical_cpus"] >= 1
    assert "logical CPUs" in cpu["cores_note"]
    assert line["determinism"]["oracle_rows_equal"] is True
    assert line["determinism"]["gathered_rows_equal_separate_runs"] is True
    for roof in (line["roofline"], line["config5_strong"]["roofline"]):
        assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["achieved"] > 0
        assert roof["frac"] == pytest.approx(roof["achieved"] / roof["peak"])
    assert line["config5_strong"]["sequences_per_gpu"] == [4, 4]
