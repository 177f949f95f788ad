"""Seeded synthetic KITTI-shape sequences.

The KITTI images the reference runs on (README.md:52) are not available offline, so
tests and benchmarks use:

* ``scene``: a forward-moving camera (+1 m/frame along z, 0.1 deg/frame yaw) over a
  random 3-D point field; each point is drawn as a square of intensity U[30,225]
  (half-size 40/z px, 2..12) over a far background of 8x8 blocks U[40,215] that
  shifts with the yaw, plus U[-3,3] pixel noise.  Ground truth is returned in the
  KITTI pose-file layout (3x4 camera-to-world rows), so the trajectory loop's
  GT-derived scale (VisualOdometry.cpp:161-162) is 1.0 per frame.
* ``noise``: iid U[0,255] frames (throughput stress).

Seeds follow splitmix64(0xACE0 ^ (seq << 32) ^ frame).
"""
from __future__ import annotations

import math

import numpy as np

KITTI_K = np.array([[718.856, 0.0, 607.1928], [0.0, 718.856, 185.2157], [0.0, 0.0, 1.0]])
KITTI_W, KITTI_H = 1241, 376


def splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def frame_seed(seq: int, frame: int) -> int:
    return splitmix64(0xACE0 ^ (seq << 32) ^ frame)


def intrinsics(width: int, height: int) -> np.ndarray:
    """KITTI K, principal point / focal length scaled for other frame sizes."""
    if (width, height) == (KITTI_W, KITTI_H):
        return KITTI_K.copy()
    sx = width / KITTI_W
    return np.array([[718.856 * sx, 0.0, 607.1928 * sx], [0.0, 718.856 * sx, height * 185.2157 / KITTI_H],
                     [0.0, 0.0, 1.0]])


def _yaw(psi: float) -> np.ndarray:
    c, s = math.cos(psi), math.sin(psi)
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


class SceneSequence:
    """Deterministic scene sequence; frame(f) renders frame f, gt() gives KITTI rows."""

    def __init__(self, width=KITTI_W, height=KITTI_H, nframes=64, seq=0, density=None,
                 step=1.0, yaw_deg=0.1, size_k=40.0):
        self.W, self.H, self.n, self.seq = width, height, nframes, seq
        self.K = intrinsics(width, height)
        self.step, self.yaw = step, math.radians(yaw_deg)
        self.size_k = size_k
        rng = np.random.default_rng(splitmix64(0xACE0 ^ (seq << 32) ^ 0xFFFFFFFF))
        zmax = 60.0 + step * nframes + 5.0
        if density is None:
            density = 200.0 * (width * height) / (KITTI_W * KITTI_H)  # points per metre of depth
        npts = int(density * (zmax - 4.0))
        self.P = np.stack([rng.uniform(-30, 30, npts), rng.uniform(-3, 3, npts),
                           rng.uniform(4.0, zmax, npts)], axis=1)
        self.I = rng.integers(30, 226, npts).astype(np.uint8)
        # far background (at infinity: moves with the yaw only), 8x8-pixel blocks
        bw = width + 2 * int(self.K[0, 0] * self.yaw * nframes) + 64
        blocks = rng.integers(40, 216, size=((height + 7) // 8, (bw + 7) // 8)).astype(np.uint8)
        self.bg = np.kron(blocks, np.ones((8, 8), np.uint8))[:height, :bw]
        self.bg_x0 = int(self.K[0, 0] * self.yaw * nframes) + 32

    def pose(self, f: int):
        R = _yaw(self.yaw * f)
        C = np.array([0.0, 0.0, self.step * f])
        return R, C

    def gt(self) -> np.ndarray:
        rows = []
        for f in range(self.n):
            R, C = self.pose(f)
            rows.append(np.concatenate([R, C[:, None]], axis=1).reshape(12))
        return np.array(rows)

    def frame(self, f: int) -> np.ndarray:
        rng = np.random.default_rng(frame_seed(self.seq, f))
        R, C = self.pose(f)
        x0 = self.bg_x0 + int(round(self.K[0, 0] * self.yaw * f))
        img = np.clip(self.bg[:, x0:x0 + self.W].astype(np.int16)
                      + rng.integers(-3, 4, size=(self.H, self.W)), 0, 255).astype(np.uint8)
        Xc = (self.P - C) @ R          # world -> camera: R^T (X - C), row-vector form
        z = Xc[:, 2]
        vis = (z > 4.0) & (z < 60.0)
        Xc, I, z = Xc[vis], self.I[vis], z[vis]
        u = self.K[0, 0] * Xc[:, 0] / z + self.K[0, 2]
        v = self.K[1, 1] * Xc[:, 1] / z + self.K[1, 2]
        ui = np.rint(u).astype(np.int64)
        vi = np.rint(v).astype(np.int64)
        ok = (ui >= 2) & (ui < self.W - 2) & (vi >= 2) & (vi < self.H - 2)
        ui, vi, I, z = ui[ok], vi[ok], I[ok], z[ok]
        order = np.argsort(-z, kind="stable")       # painter's order: far to near
        half = np.clip(np.rint(self.size_k / z), 2, 12).astype(np.int64)
        for k in order:
            h = half[k]
            img[max(vi[k] - h, 0):vi[k] + h + 1, max(ui[k] - h, 0):ui[k] + h + 1] = I[k]
        return img

    def frames(self) -> np.ndarray:
        return np.stack([self.frame(f) for f in range(self.n)])


def noise_frames(width=KITTI_W, height=KITTI_H, nframes=8, seq=0) -> np.ndarray:
    out = np.empty((nframes, height, width), np.uint8)
    for f in range(nframes):
        rng = np.random.default_rng(frame_seed(seq, f))
        out[f] = rng.integers(0, 256, size=(height, width), dtype=np.uint8)
    return out


# -- parallel rendering (bench: several sequences of 200+ frames) ------------------------
_SEQ_CACHE: dict = {}


def _render(args):
    W, H, n, seq, step, f = args
    key = (W, H, n, seq, step)
    s = _SEQ_CACHE.get(key)
    if s is None:
        s = _SEQ_CACHE[key] = SceneSequence(W, H, nframes=n, seq=seq, step=step)
    return s.frame(f)


def render_sequences(specs, workers: int = 1):
    """Frames of several scene sequences, specs = [(W, H, nframes, seq, step), ...], rendered by
    `workers` forked processes (call before the process touches the GPU).  Identical to
    SceneSequence(W, H, nframes=n, seq=seq, step=step).frames() for each spec."""
    tasks = [(W, H, n, s, st, f) for (W, H, n, s, st) in specs for f in range(n)]
    if workers <= 1:
        flat = [_render(t) for t in tasks]
    else:
        import multiprocessing as mp
        # close + join (not the context manager's terminate): workers exit normally, no SIGTERM
        # (a profiler preloaded into the forked workers handles SIGTERM badly)
        pool = mp.get_context("fork").Pool(workers)
        try:
            flat = pool.map(_render, tasks, chunksize=max(1, len(tasks) // (4 * workers)))
        finally:
            pool.close()
            pool.join()
    out, k = [], 0
    for (W, H, n, s, st) in specs:
        out.append(np.stack(flat[k:k + n]))
        k += n
    return out
