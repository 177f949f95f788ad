#!/usr/bin/env python3
"""Per-phase cycles of k_refit / k_triangulate over a synthetic sequence (diagnostic VO_STAMPS
build).  usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so python tools/stamps_frame.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context, load  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence  # noqa: E402

seq = SceneSequence(nframes=24, step=0.05)
fr = seq.frames()
ctx = Context(seq.W, seq.H, K=seq.K)
ctx.set_ground_truth(seq.gt())
L = load()
L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
rows_r, rows_t, rows_n, rows_m = [], [], [], []
for f in range(seq.n):
    _, st, info = ctx.process_frame(fr[f])
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    if st == 0:
        r = buf[1995 * 16:1995 * 16 + 16].astype(np.int64)
        t = buf[1996 * 16:1996 * 16 + 16].astype(np.int64)
        rows_r.append(np.concatenate([np.diff(r[:9]), r[14:16]]))
        rows_t.append(np.diff(t[:4]))
        nv = buf[1994 * 16:1994 * 16 + 16].astype(np.int64)
        rows_n.append(np.diff(nv[:5]))
        mt = buf[1993 * 16:1993 * 16 + 16].astype(np.int64)
        rows_m.append(np.diff(mt[:4]))
R = np.array(rows_r)
T = np.array(rows_t)
names = ["compaction", "means", "spread", "moments", "modelp+sync", "nullvec9", "denorm+rank2", "pose_prep"]
print(f"k_refit cycles per phase (median over {len(R)} frames); nullvec iterations {np.median(R[:, 8])} "
      f"(max {R[:, 8].max()}), inliers {np.median(R[:, 9])}")
for i, nm in enumerate(names):
    print(f"  {nm:14s} {int(np.median(R[:, i])):8d}")
print(f"  {'total':14s} {int(np.median(R[:, :8].sum(1))):8d}")
print("k_triangulate (block 0): cheirality", int(np.median(T[:, 0])), " arrive", int(np.median(T[:, 1])),
      " finalize", int(np.median(T[:, 2])))
NV = np.median(np.array(rows_n), axis=0)
print("nullvec9 phases: cholesky", int(NV[0]), " inverse+W", int(NV[1]), " squarings", int(NV[2]), " power", int(NV[3]))
MT = np.median(np.array(rows_m), axis=0)
print("k_match (block 0 / last block): scoring", int(MT[0]), " arrive", int(MT[1]), " compaction", int(MT[2]))
