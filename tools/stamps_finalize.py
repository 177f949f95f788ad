#!/usr/bin/env python3
"""k_finalize anatomy from s_memtime stamps (diagnostic VO_STAMPS build): cycles per step of the
window commit, over the pose passes of a batched run (the stamp slot holds the last pass).
usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so python tools/stamps_finalize.py"""
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
names = ["entry->0", "0 (work loads, choose_pose)", "1 (rules)", "2 (GT scale, T_rel)", "3 (T chain)",
         "4 (rows, state)"]
rows = []
for rep in range(20):
    df = ctx.device_frames(fr)
    ctx.reset()
    ctx.process_frames_device(df)
    df.free()
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    t = buf[1996 * 16:1996 * 16 + 8].astype(np.int64)
    seqv = [t[7], t[0], t[1], t[2], t[3], t[4], t[5]]
    rows.append(np.diff(seqv))
R = np.median(np.array(rows), axis=0)
print("median cycles per k_finalize step (last pass of a 64-frame run):")
for n, v in zip(names, R):
    print(f"  {n:32s} {int(v):8d}")
print(f"  total {int(R.sum())} cycles = {R.sum() / 2.4e3:.1f} us at 2.4 GHz")
