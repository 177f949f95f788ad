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

seq = SceneSequence(nframes=64, step=1.0)
fr = seq.frames()
ctx = Context(seq.W, seq.H, K=seq.K)
ctx.set_ground_truth(seq.gt())
L = load()
L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
names = ["sample8", "fit (normalize, Gauss-Jordan, rank 2)", "hypF store + Sampson count"]
idx = [0, 1, 5, 6]
rows = []
for rep in range(10):
    df = ctx.device_frames(fr)
    ctx.reset()
    ctx.process_frames_device(df)
    df.free()
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    t = buf[:100 * 16].reshape(100, 16)[:, idx].astype(np.int64)
    t = t[(t > 0).all(axis=1)]
    # order: 0 entry, 1 after sample8, 5 after the fit, 6 after the count (a wave = 8 hypotheses)
    d = np.stack([t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]], 1)
    rows.append(d)
R = np.concatenate(rows)
print(f"hypothesis waves sampled: {len(R)}")
for i, n in enumerate(names):
    print(f"  {n:28s} median {int(np.median(R[:, i])):7d}  p90 {int(np.percentile(R[:, i], 90)):7d}")
print(f"  total median {int(np.median(R.sum(axis=1)))} cycles")
