"""One sequence split over GPUs (within-sequence sharding).

The reference runs a sequence as one loop (VisualOdometry::run, VisualOdometry.cpp:38-193)
whose state -- desc1 / last_valid_frame (:164-166), the FundamentalMatrix model that leaks
into frames without a fit of their own (:130,146, quirk 9) and T_curr (:184) -- makes every
frame depend on all earlier ones.  Rank r of G owns the contiguous frames [a_r, b_r) and
runs them as a stream that starts `halo` frames earlier (s_r = a_r - halo) as if a new
sequence started there (vo_set_frame_origin: identity pose, no model, desc1 = frame s_r; the
RANSAC sampler counts frames from the sequence start, so every frame draws the hypotheses of
the unsplit run).  No descriptor crosses GPUs: the halo frames are extracted again on the
shard, which costs a few microseconds per frame where shipping a predecessor's keypoints and
descriptors would serialise the shards.

Why the halo run gives the unsplit run's results.  A frame's match, RANSAC and refit depend
only on its partner (desc1 at that frame) and its sampler index.  If a frame x in (s_r, a_r]
has its predecessor x - 1 advancing desc1 in BOTH runs and fits a model of its own (>= 8
RANSAC inliers; `fitted`), both runs leave x with the same state (last_valid = desc1 = x,
model = x's fit), and every later frame is computed identically -- except T_curr, which the
halo run started from the identity.  So:
  1. every shard runs its halo stream in parallel (one all_gather of per-frame status and
     fitted flags afterwards); the halo grows (2, 4, 8, ... frames) until the halo run itself
     holds such an x, so step 2 rarely fails;
  2. shards are checked in rank order against the (final) flags of the frames before them;
     a shard whose halo shows no such x runs again from the latest frame x' < a_r of the
     unsplit run that advanced after an advancing predecessor (x' - 1 becomes the stream's
     first frame) -- or from frame 0 if there is none -- and broadcasts its new flags;
  3. T_curr crosses the shards in rank order (16 doubles, send/recv): shard r chains its
     frames' relative motions again from its predecessor's T_curr on the device
     (vo_rechain, the same f64 operations in the same order), so its rows equal the unsplit
     run's bit for bit.
Step 3 is the only sequential part: a 4x4 f64 product per frame on one wave.

The protocol is written once over two small interfaces -- an engine (a shard's VO context) and
a comm (torch.distributed, or the in-process driver run_local) -- so the CPU tests exercise the
same code with gloo and a toy engine (tests/test_shard.py).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

# statuses after the loop's rules (include/vo_mi355x.h)
ST_OK, ST_FIRST, ST_MISSING, ST_FEW_MATCHES, ST_FEW_INLIERS, ST_DEGENERATE = 0, 1, 2, 3, 4, 5
_ADVANCES = (ST_OK, ST_FIRST, ST_DEGENERATE)    # desc1 / last_valid moved to the frame (:164-166)

DEFAULT_HALO = 2


def partition(nframes: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous, balanced frame ranges [a_r, b_r) of the G shards (ranges may be empty)."""
    q, rem = divmod(nframes, world)
    out, a = [], 0
    for r in range(world):
        b = a + q + (1 if r < rem else 0)
        out.append((a, b))
        a = b
    return out


def advanced(status: np.ndarray) -> np.ndarray:
    return np.isin(status, _ADVANCES)


def entry_holds(true_adv: np.ndarray, s: int, a: int, halo_status: np.ndarray, halo_fit: np.ndarray) -> bool:
    """True when the halo run that started at frame s reaches frame a in the unsplit run's state
    (up to T_curr): some x in (s, a] has x - 1 advancing in both runs and a fit of its own.
    true_adv covers frames < a (final), halo_* the halo run's frames s.. (index f - s)."""
    if s == 0:
        return True                  # the stream starts where the sequence starts: the unsplit run
    hadv = advanced(halo_status)
    for x in range(s + 1, a + 1):
        if true_adv[x - 1] and hadv[x - 1 - s] and halo_fit[x - s]:
            return True
    return False


def halo_reaches(s: int, a: int, status: np.ndarray, fit: np.ndarray) -> bool:
    """The halo side of entry_holds over the halo frames alone (x < a): some x in (s, a) follows
    an advancing frame of the halo run and fits its own model."""
    hadv = advanced(status)
    return any(hadv[x - 1 - s] and fit[x - s] for x in range(s + 1, a))


def halo_run(engine, a: int, b: int, halo: int):
    """Phase 1 of a shard: the halo frames [a - h, a) first, h doubling until the halo run holds a
    frame that makes it reach the unsplit state (or h reaches the sequence start) -- at the survey's
    1.0 m/frame only a quarter of the frames fit a model of their own, so two halo frames would
    often fail the check -- then the shard's own frames continue the same stream."""
    if a == 0:
        return 0, engine.run(0, b)
    h = max(1, halo)
    while True:
        s = max(0, a - h)
        o1 = engine.run(s, a)
        if s == 0 or halo_reaches(s, a, o1[1], o1[2][:, 5]):
            break
        h *= 2
    o2 = engine.extend(a, b)
    return s, tuple(np.concatenate([x, y]) for x, y in zip(o1, o2))


def restart_point(true_adv: np.ndarray, true_fit: np.ndarray, a: int) -> int:
    """First frame of a shard's second run: x' - 1 for the latest x' < a that fitted its own model
    after an advancing predecessor in the unsplit run, else 0 (the sequence start)."""
    for x in range(a - 1, 0, -1):
        if true_adv[x - 1] and true_fit[x]:
            return x - 1
    return 0


class ShardResult:
    """A shard's rows and per-frame outputs for its own frames [a, b) of the sequence."""

    def __init__(self, a, b, poses, status, info, start, runs):
        self.a, self.b = a, b
        self.poses, self.status, self.info = poses, status, info
        self.start = start           # first frame of the stream the rows came from
        self.runs = runs             # 1, or 2 when the halo did not reach the unsplit state


def _resolve(parts, flags, nframes, rerun):
    """Steps 2 of the protocol over every shard in rank order.  flags[q] = (s, status, fitted) of
    shard q's stream; rerun(q, s2) runs shard q again from frame s2 and returns its new flags
    (every caller gets them).  Returns the final stream start of every shard."""
    true_st = np.full(nframes, -1, np.int32)
    true_fit = np.zeros(nframes, np.int32)
    starts = []
    for q, (a, b) in enumerate(parts):
        s, st, fit = flags[q]
        if b > a and not entry_holds(advanced(true_st[:a]), s, a, st, fit):
            s2 = restart_point(advanced(true_st[:a]), true_fit[:a], a)
            s, st, fit = rerun(q, s2)
        starts.append(s)
        if b > a:
            true_st[a:b] = st[a - s:]
            true_fit[a:b] = fit[a - s:]
    return starts


class ShardError(RuntimeError):
    """Raised on every rank when one rank's engine failed (or a shard cannot be chained), so no
    rank is left blocked in a collective or a recv."""


def _capacity(engine) -> Optional[int]:
    cap = getattr(engine, "capacity", None)
    return cap() if cap is not None else None


def check_capacity(parts, caps) -> None:
    """vo_rechain chains a shard's frames from trajectory records that must still be resident:
    a shard longer than its engine's record ring cannot be handed its T_curr."""
    for q, ((a, b), cap) in enumerate(zip(parts, caps)):
        if cap is not None and b - a > cap:
            raise ShardError(f"shard {q} holds {b - a} frames, more than its engine keeps for vo_rechain ({cap}); "
                             f"use more shards or a larger ring (VO_RING_SLOTS)")


def _poison_T():
    T = np.full((4, 4), np.nan)
    return T


def run_shard(engine, comm, nframes: int, halo: int = DEFAULT_HALO) -> ShardResult:
    """This rank's shard of one sequence (comm: rank, world, allgather, broadcast, send, recv).
    A failure on any rank -- a capacity check, an engine error in the halo run, the second run or
    the re-chain -- raises ShardError on every rank: the failing rank's error travels in the flag
    exchange, the second-run broadcast or (as a NaN T_curr) the hand-over."""
    r, G = comm.rank, comm.world
    parts = partition(nframes, G)
    a, b = parts[r]
    check_capacity(parts, comm.allgather(_capacity(engine)))      # every rank raises together
    err = None
    try:
        s, out = halo_run(engine, a, b, halo) if b > a else (max(0, a - halo), None)
    except Exception as e:                                        # noqa: BLE001 -- re-raised on every rank
        s, out, err = max(0, a - halo), None, f"rank {r}: halo run failed: {e!r}"
    mine = (s, out[1], out[2][:, 5]) if out is not None else (s, np.zeros(0, np.int32), np.zeros(0, np.int32))
    flags = comm.allgather(mine + (err,))
    errs = [f[3] for f in flags if f[3]]
    if errs:
        raise ShardError("; ".join(errs))
    flags = [f[:3] for f in flags]
    runs = [1]

    def rerun(q, s2):
        nonlocal out
        payload = None
        if q == r:
            try:
                out = engine.run(s2, b)
                runs[0] = 2
                payload = (s2, out[1], out[2][:, 5], None)
            except Exception as e:                                # noqa: BLE001
                payload = (s2, None, None, f"rank {r}: second run from frame {s2} failed: {e!r}")
        got = comm.broadcast(payload, q)
        if got[3]:
            raise ShardError(got[3])
        return got[:3]

    starts = _resolve(parts, flags, nframes, rerun)
    s = starts[r]
    # step 3: T_curr in rank order; a rank that cannot chain passes a NaN T_curr on, so every later
    # rank raises instead of waiting
    T = None
    failed = None
    if r > 0:
        T = comm.recv(r - 1)
        if not np.isfinite(np.asarray(T, np.float64)).all():
            failed = "an earlier rank failed to chain its shard"
    if b > a and failed is None:
        poses = out[0][a - s:]
        try:
            if r > 0:
                poses = engine.rechain(T, a - s, b - a)
            T = engine.trajectory_state()
        except Exception as e:                                    # noqa: BLE001
            failed = f"rank {r}: re-chain failed: {e!r}"
    if r < G - 1:
        comm.send(_poison_T() if failed else T, r + 1)
    if failed:
        raise ShardError(failed)
    if b <= a:
        return ShardResult(a, b, np.zeros((0, 3, 4)), np.zeros(0, np.int32), np.zeros((0, 8), np.int32), s, runs[0])
    return ShardResult(a, b, poses, out[1][a - s:], out[2][a - s:], s, runs[0])


def run_local(engines: Sequence, nframes: int, halo: int = DEFAULT_HALO) -> List[ShardResult]:
    """The protocol with every shard in this process (engines[r] = shard r's engine, e.g. several
    contexts on one GPU): the same steps in the order the ranks would reach them."""
    G = len(engines)
    parts = partition(nframes, G)
    check_capacity(parts, [_capacity(e) for e in engines])
    outs, flags = [], []
    for r, (a, b) in enumerate(parts):
        s, o = halo_run(engines[r], a, b, halo) if b > a else (max(0, a - halo), None)
        outs.append(o)
        flags.append((s, o[1], o[2][:, 5]) if o is not None else (s, np.zeros(0, np.int32), np.zeros(0, np.int32)))
    runs = [1] * G

    def rerun(q, s2):
        outs[q] = engines[q].run(s2, parts[q][1])
        runs[q] = 2
        return s2, outs[q][1], outs[q][2][:, 5]

    starts = _resolve(parts, flags, nframes, rerun)
    res, T = [], None
    for r, (a, b) in enumerate(parts):
        s = starts[r]
        if b <= a:
            res.append(ShardResult(a, b, np.zeros((0, 3, 4)), np.zeros(0, np.int32), np.zeros((0, 8), np.int32), s, 1))
            continue
        o = outs[r]
        poses = o[0][a - s:] if r == 0 or T is None else engines[r].rechain(T, a - s, b - a)
        T = engines[r].trajectory_state()
        res.append(ShardResult(a, b, poses, o[1][a - s:], o[2][a - s:], s, runs[r]))
    return res


class ContextEngine:
    """A shard's engine over a Context: the sequence's frames and GT rows.  frames: host
    (F x H x W u8, uploaded per run) or a DeviceFrames batch of the whole sequence, or of the
    frames from `base` on (resident in HBM; a run uses a view of it)."""

    def __init__(self, ctx, frames, gt: Optional[np.ndarray] = None, base: int = 0):
        self.ctx, self.frames, self.gt, self.base = ctx, frames, gt, base

    def run(self, s: int, b: int):
        ctx = self.ctx
        if not isinstance(self.frames, np.ndarray):
            if s < self.base:
                raise ValueError(f"frames before {self.base} are not resident on this shard (run from {s})")
            df = self.frames.view(s - self.base, b - self.base)
        else:
            df = ctx.device_frames(np.ascontiguousarray(self.frames[s:b]))
        try:
            ctx.reset()
            ctx.set_sequence_starts([])
            ctx.set_frame_origin(s)
            ctx.set_ground_truth(None if self.gt is None else self.gt[s:])
            return ctx.process_frames_device(df)
        finally:
            df.free()

    def extend(self, a: int, b: int):
        """Frames [a, b) continuing the stream of the last run (which ended at frame a)."""
        ctx = self.ctx
        if not isinstance(self.frames, np.ndarray):
            return ctx.process_frames_device(self.frames.view(a - self.base, b - self.base))
        df = ctx.device_frames(np.ascontiguousarray(self.frames[a:b]))
        try:
            return ctx.process_frames_device(df)
        finally:
            df.free()

    def rechain(self, T_in, f0: int, n: int):
        return self.ctx.rechain(T_in, f0, n)

    def capacity(self) -> int:
        """Frames whose trajectory records stay resident for rechain (the context's ring)."""
        return self.ctx.ring_slots()

    def trajectory_state(self):
        return self.ctx.trajectory_state()


class TorchComm:
    """comm over torch.distributed: object collectives for the flags; T_curr as a 16-double tensor
    (on the rank's GPU under "nccl" = RCCL over xGMI, on the CPU under gloo)."""

    def __init__(self, dist, device=None):
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.device = device

    def allgather(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def broadcast(self, obj, src: int):
        box = [obj]
        self.dist.broadcast_object_list(box, src=src)
        return box[0]

    def send(self, T, dst: int):
        import torch
        self.dist.send(torch.as_tensor(np.asarray(T, np.float64).reshape(16), device=self.device), dst)

    def recv(self, src: int):
        import torch
        t = torch.zeros(16, dtype=torch.float64, device=self.device)
        self.dist.recv(t, src)
        return t.cpu().numpy().reshape(4, 4)
