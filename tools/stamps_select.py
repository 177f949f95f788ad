#!/usr/bin/env python3
"""k_select anatomy from s_memtime stamps (diagnostic VO_STAMPS build): cycles per phase of one
frame's select (the stage API: one workgroup writes slot 1990), median over frames.
usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so python tools/stamps_select.py"""
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
names = ["A+B tile counts, scan, key staging", "C histogram boundary bin", "C boundary keys gathered",
         "C rank (threshold key) + clear", "D bitmap + segment counts, E scan", "F keypoint emission"]
rows = []
for rep in range(20):
    ctx.extract(fr[rep % len(fr)])
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    t = buf[1990 * 16:1990 * 16 + 7].astype(np.int64)
    rows.append(np.diff(t))
    nb = int(buf[1990 * 16 + 10])
R = np.median(np.array(rows), axis=0)
print(f"boundary-bin keys (last run): {nb}")
for n, v in zip(names, R):
    print(f"  {n:40s} {int(v):8d}")
print(f"  total {int(R.sum())} cycles = {R.sum() / 2.4e3:.1f} us at 2.4 GHz")
