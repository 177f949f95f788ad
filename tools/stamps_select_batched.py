#!/usr/bin/env python3
"""k_select anatomy in the batched path (diagnostic VO_STAMPS build): cycles per phase of each
frame's select workgroup (slot 1900 + frame of the batch), median over the frames of a 64-frame
batched run, KITTI motion.  usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so
python tools/stamps_select_batched.py   (VO_SERIAL=1: every kernel on one queue, the select alone)"""
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
rows, spans = [], []
for rep in range(6):
    df = ctx.device_frames(fr)
    ctx.reset()
    ctx.process_frames_device(df)
    df.free()
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    t = buf[1900 * 16:1964 * 16].reshape(64, 16)[:, :7].astype(np.int64)
    t = t[(t > 0).all(axis=1)]
    if rep:
        rows.append(np.diff(t, axis=1))
        spans.append((t[:, 6].max() - t[:, 0].min()))
R = np.concatenate(rows)
print(f"select workgroups sampled: {len(R)}; launch span (first stamp .. last) median {np.median(spans):.0f} cycles")
for i, n in enumerate(names):
    print(f"  {n:40s} median {int(np.median(R[:, i])):7d}  p90 {int(np.percentile(R[:, i], 90)):7d}")
print(f"  workgroup total median {int(np.median(R.sum(axis=1)))} cycles")
