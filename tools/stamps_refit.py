#!/usr/bin/env python3
"""k_refit anatomy from s_memtime stamps (diagnostic VO_STAMPS build): cycles per phase of one
frame's refit (slot 1995, the last frame to write it) over repeated 64-frame batched runs.
usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so python tools/stamps_refit.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context, load  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence  # noqa: E402

seq = SceneSequence(nframes=64, step=float(sys.argv[1]) if len(sys.argv) > 1 else 0.05)
fr = seq.frames()
ctx = Context(seq.W, seq.H, K=seq.K)
ctx.set_ground_truth(seq.gt())
L = load()
L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
names = ["inlier compaction", "means", "scales", "45 moments", "hypF load", "null vector (inverse iteration)",
         "denormalize + rank 2 (thread 0)", "getPose prologue: E, SVD, 4 candidates (thread 0)"]
rows = []
for rep in range(10):
    df = ctx.device_frames(fr)
    ctx.reset()
    ctx.process_frames_device(df)
    df.free()
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data, buf.size)
    st = buf[1995 * 16: 1995 * 16 + 16].astype(np.int64)
    if st[0] and st[8]:
        rows.append(np.diff(st[:9]))
rows = np.array(rows)
print(f"frames sampled: {len(rows)}; inliers of the last: {int(buf[1995 * 16 + 15])}")
for i, nm in enumerate(names):
    print(f"  {nm:52s} median {int(np.median(rows[:, i])):8d}")
print(f"  total median {int(np.median(rows.sum(1)))} cycles")
