"""Within-sequence sharding (acs_visual_odometry_amd/shard.py) on the CPU.

The protocol is checked against a toy engine that restates the trajectory loop's rules
(VisualOdometry.cpp:68-189): missing images, < 8 matches, < 8 inliers with the model leak
(quirk 9), desc1 / last_valid advance (:164-166), a GT-like scale that depends on the last
valid frame (:161-162) and the T_curr chain (:184).  A frame's matches and its own fit are
deterministic functions of (partner, frame), as the device's are of (desc1, frame, sampler
index).  Sharded runs -- in-process (run_local) and over gloo with 2 and 3 ranks (run_shard) --
must return the unsplit run's rows and statuses bit for bit, including worlds whose shard
boundaries fall into runs of skipped frames (second runs) and worlds with no fit at all.
The GPU form of the same checks is tests/test_gpu_paths.py::test_sequence_shards_*."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from acs_visual_odometry_amd import shard  # noqa: E402

FLIPZ = np.diag([1.0, 1.0, -1.0, 1.0])


def _h(*xs):
    z = 0x9E3779B97F4A7C15
    for x in xs:
        z = (z ^ (x + 0x632BE59BD9B4E019)) * 0xBF58476D1CE4E5B9 & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
    return z


class ToyWorld:
    """p_skip: chance a (partner, frame) pair has < 8 matches; p_fit: chance of an own fit."""

    def __init__(self, nframes, seed, p_skip=0.15, p_fit=0.6, p_missing=0.03):
        self.F, self.seed = nframes, seed
        self.p_skip, self.p_fit, self.p_missing = p_skip, p_fit, p_missing

    def u(self, *xs):
        return (_h(self.seed, *xs) >> 11) / float(1 << 53)

    def missing(self, f):
        return f > 0 and self.u(1, f) < self.p_missing

    def matches(self, p, f):
        return 3 if self.u(2, p, f) < self.p_skip else 100

    def own_fit(self, p, f):
        return self.u(3, p, f) < self.p_fit

    def motion(self, p, f):
        a = self.u(4, p, f) * 0.2
        c, s = np.cos(a), np.sin(a)
        T = np.eye(4)
        T[0, 0], T[0, 2], T[2, 0], T[2, 2] = c, s, -s, c
        T[:3, 3] = [self.u(5, p, f) - 0.5, 0.1 * self.u(6, p, f), 1.0]
        return T


class ToyEngine:
    """The loop over frames [s, b) of a ToyWorld as a fresh sequence started at s."""

    def __init__(self, world):
        self.w = world
        self.rec = []
        self.T = np.eye(4)

    def run(self, s, b):
        self.rec, self.T, self.L, self.model, self.s, self.end = [], np.eye(4), s, None, s, s
        return self.extend(s, b)

    def extend(self, a, b):
        assert a == self.end
        w, s = self.w, self.s
        n = b - a
        poses = np.zeros((n, 3, 4))
        status = np.zeros(n, np.int32)
        info = np.zeros((n, 8), np.int32)
        T, L, model = self.T, self.L, self.model
        for k in range(n):
            i = a + k
            kind, Trel = 0, None
            if i == s:
                status[k], row = shard.ST_FIRST, T.copy()
            elif w.missing(i):
                status[k], row = shard.ST_MISSING, T.copy()
            elif w.matches(L, i) < 8:
                status[k], row = shard.ST_FEW_MATCHES, FLIPZ @ T
            else:
                if w.own_fit(L, i):
                    model = (L, i)
                    info[k, 5] = 1
                if model is None:
                    status[k], row = shard.ST_FEW_INLIERS, FLIPZ @ T
                else:
                    scale = 1.0 + 0.01 * (i - L)          # depends on the last valid frame
                    Trel = w.motion(*model).copy()
                    Trel[:3, 3] *= scale
                    L = i
                    T = T @ Trel
                    kind = 1
                    status[k], row = shard.ST_OK, FLIPZ @ T
            self.rec.append((kind, Trel, status[k] in (shard.ST_FIRST, shard.ST_MISSING)))
            poses[k] = row[:3]
        self.T, self.L, self.model, self.end = T, L, model, b
        return poses, status, info

    def rechain(self, T_in, f0, n):
        T = np.array(T_in, dtype=np.float64).reshape(4, 4)
        out = np.zeros((n, 3, 4))
        for k in range(n):
            kind, Trel, noflip = self.rec[f0 + k]
            if kind == 1:
                T = T @ Trel
            out[k] = (T if noflip else FLIPZ @ T)[:3]
        self.T = T
        return out

    def trajectory_state(self):
        return self.T.copy()


def _check(results, full):
    poses = np.concatenate([r.poses for r in results])
    status = np.concatenate([r.status for r in results])
    assert np.array_equal(status, full[1])
    assert np.array_equal(poses, full[0])


WORLDS = [(60, s, ps, pf) for s, (ps, pf) in enumerate([(0.15, 0.6), (0.4, 0.3), (0.0, 1.0), (0.6, 0.2),
                                                          (0.3, 0.05), (0.2, 0.0), (0.9, 0.5)])]


@pytest.mark.parametrize("F,seed,p_skip,p_fit", WORLDS)
@pytest.mark.parametrize("G", [1, 2, 3, 5, 8])
def test_run_local_equals_unsplit(F, seed, p_skip, p_fit, G):
    w = ToyWorld(F, seed, p_skip, p_fit)
    full = ToyEngine(w).run(0, F)
    res = shard.run_local([ToyEngine(w) for _ in range(G)], F)
    _check(res, full)


def test_second_runs_happen_and_stay_exact():
    """Worlds with long skip runs force shards to start again further back."""
    reruns = 0
    for seed in range(40):
        w = ToyWorld(48, 100 + seed, p_skip=0.5, p_fit=0.3)
        full = ToyEngine(w).run(0, 48)
        res = shard.run_local([ToyEngine(w) for _ in range(4)], 48)
        _check(res, full)
        reruns += sum(r.runs == 2 for r in res)
    assert reruns > 0


def test_more_shards_than_frames():
    w = ToyWorld(5, 7)
    full = ToyEngine(w).run(0, 5)
    _check(shard.run_local([ToyEngine(w) for _ in range(8)], 5), full)


def test_partition_and_restart_point():
    assert shard.partition(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert shard.partition(2, 3) == [(0, 1), (1, 2), (2, 2)]
    adv = np.array([1, 0, 1, 1, 0], bool)
    fit = np.array([0, 0, 0, 1, 0], np.int32)
    assert shard.restart_point(adv, fit, 5) == 2           # x' = 3: frame 2 advanced, 3 fitted
    assert shard.restart_point(adv, np.zeros(5, np.int32), 5) == 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q, worlds):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from acs_visual_odometry_amd import shard as S
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = S.TorchComm(dist)
    out = []
    for (F, seed, ps, pf) in worlds:
        r = S.run_shard(ToyEngine(ToyWorld(F, seed, ps, pf)), comm, F)
        out.append((r.a, r.b, r.poses, r.status, r.runs))
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_run_shard_gloo(world):
    worlds = WORLDS + [(40, 200 + i, 0.5, 0.3) for i in range(6)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, worlds)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i, (F, seed, ps, pf) in enumerate(worlds):
        full = ToyEngine(ToyWorld(F, seed, ps, pf)).run(0, F)
        parts = [res[r][1][i] for r in range(world)]
        assert [(p[0], p[1]) for p in parts] == shard.partition(F, world)
        assert np.array_equal(np.concatenate([p[3] for p in parts]), full[1])
        assert np.array_equal(np.concatenate([p[2] for p in parts]), full[0])


# -- failures: every rank raises ShardError, none is left blocked ---------------------------------
class FailingEngine(ToyEngine):
    """mode: 'halo' raises in the halo run, 'rerun' in the second run, 'rechain' in the hand-over;
    'capacity' reports a record ring shorter than the shard."""

    def __init__(self, world, mode):
        super().__init__(world)
        self.mode, self.halo_done = mode, False

    def run(self, s, b):
        if self.mode == "halo" or (self.mode == "rerun" and self.halo_done):
            raise ValueError(f"frames before {s + 1} are not resident on this shard")
        return super().run(s, b)

    def extend(self, a, b):
        out = super().extend(a, b)
        self.halo_done = True
        return out

    def rechain(self, T_in, f0, n):
        if self.mode == "rechain":
            raise RuntimeError("vo_rechain: invalid state (-5)")
        return super().rechain(T_in, f0, n)

    def capacity(self):
        return 3 if self.mode == "capacity" else None


def _rerun_world(world):
    """A ToyWorld in which shard 1 of `world` needs its second run."""
    for seed in range(300, 400):
        w = ToyWorld(48, seed, p_skip=0.5, p_fit=0.3)
        if shard.run_local([ToyEngine(w) for _ in range(world)], 48)[1].runs == 2:
            return (48, seed, 0.5, 0.3)
    raise AssertionError("no world with a second run on shard 1")


def _fail_rank(rank, world, port, q, wspec, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from acs_visual_odometry_amd import shard as S
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F, seed, ps, pf = wspec
    w = ToyWorld(F, seed, ps, pf)
    eng = FailingEngine(w, mode) if rank == 1 else ToyEngine(w)
    try:
        S.run_shard(eng, S.TorchComm(dist), F)
        q.put((rank, "ok"))
    except S.ShardError as e:
        q.put((rank, "raised: " + str(e)))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["halo", "rerun", "rechain", "capacity"])
def test_run_shard_failure_reaches_every_rank(mode):
    world = 3
    wspec = _rerun_world(world) if mode == "rerun" else (60, 1, 0.15, 0.6)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_rank, args=(r, world, port, q, wspec, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if mode == "rechain":
        # rank 0 chains before rank 1 and finishes; every rank after the failing one raises
        assert res[0] == "ok" and all(res[r].startswith("raised") for r in (1, 2)), res
    else:
        assert all(v.startswith("raised") for v in res.values()), res
    assert "rank 1" in res[1] or mode == "capacity"


def test_run_local_capacity_check():
    w = ToyWorld(60, 1)
    with pytest.raises(shard.ShardError):
        shard.run_local([FailingEngine(w, "capacity") for _ in range(2)], 60)
