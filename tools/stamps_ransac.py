#!/usr/bin/env python3
"""k_ransac_hyp anatomy from s_memtime stamps (diagnostic VO_STAMPS build): median cycles per
phase of a first-chunk hypothesis wave (eight hypotheses; slot = its first hypothesis, written by
the last frame), over a 64-frame batched run.
usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so python tools/stamps_ransac.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context, load  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence  # noqa: E402

# STAGE=1: one frame pair's matches through the stage call (vo_ransac_F: one writer per stamp slot,
# so the phases are one wave's); MOTION sets the camera step (0.12: hundreds of hypotheses)
STAGE = os.environ.get("STAGE", "0") == "1"
MOTION = float(os.environ.get("MOTION", "1.0"))
seq = SceneSequence(nframes=64 if not STAGE else 2, step=MOTION)
fr = seq.frames()
ctx = Context(seq.W, seq.H, K=seq.K)
ctx.set_ground_truth(seq.gt())
L = load()
L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
names = ["sample8", "point loads + normalisation", "Gauss-Jordan (8 steps)", "back substitution + denormalize", "rank 2 (3x3 min eigenvector)", "hypF store + Sampson count"]
idx = [0, 1, 3, 4, 2, 5, 6]
rows = []
if STAGE:
    import oracle as O
    cfg = O.config(seq.W, seq.H, K=seq.K.reshape(9))
    k0, d0, _ = O.extract(fr[0], cfg)
    k1, d1, _ = O.extract(fr[1], cfg)
    m = O.match(d0, d1)
    pts = np.concatenate([k0[m[:, 0]], k1[m[:, 1]]], axis=1).astype(np.float64)
    print(f"stage call: {len(pts)} matches")
for rep in range(10):
    if STAGE:
        g = ctx.ransac(pts, 7 + rep)
        if rep == 0:
            print(f"hypotheses evaluated {g['n_evaluated']}")
    else:
        df = ctx.device_frames(fr)
        ctx.reset()
        ctx.process_frames_device(df)
        df.free()
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    nk = 2000 if STAGE else 100
    t = buf[:nk * 16].reshape(nk, 16)[:, idx].astype(np.int64)
    t = t[(t > 0).all(axis=1)]
    # order: 0 entry, 1 after sample8, 3 after the normalisation, 4 after Gauss-Jordan, 2 after the fit,
    # 5 after rank 2, 6 after the count (a wave = 8 hypotheses)
    d = np.diff(t, axis=1)
    rows.append(d)
R = np.concatenate(rows)
print(f"hypothesis waves sampled: {len(R)}")
for i, n in enumerate(names):
    print(f"  {n:28s} median {int(np.median(R[:, i])):7d}  p90 {int(np.percentile(R[:, i], 90)):7d}")
print(f"  total median {int(np.median(R.sum(axis=1)))} cycles")
