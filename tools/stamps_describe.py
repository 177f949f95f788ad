#!/usr/bin/env python3
"""k_describe anatomy from s_memtime stamps (diagnostic VO_STAMPS build): median cycles per
phase of a describe wave (32 keypoints), over the waves of a 64-frame batched run.
usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so [PF=1] python tools/stamps_describe.py
PF=1: one vo_process_frame call per sample (the per-frame path's k_describe_pf launch, wave 0 of
each 8-wave workgroup: its phase 2 is the in-order sum of the terms the other waves computed)."""
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
names = ["1 pattern gathers -> LDS", "2 orientation sums (903 terms)", "3 atan2 / sincos",
         "4 rotated gathers -> LDS", "5 512 tests (ballots)"]
rows, spans = [], []
PF = int(os.environ.get("PF", "0"))        # PF=1: the per-frame call (vo_process_frame), stamps of each call's describe
for rep in range(10):
    if PF:
        if rep == 0:
            ctx.reset()
        ctx.process_frame(fr[rep + 1])
    else:
        df = ctx.device_frames(fr)
        ctx.reset()
        ctx.process_frames_device(df)
        df.free()
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    t = buf[1000 * 16:1900 * 16].reshape(900, 16)[:, :6].astype(np.int64)
    if PF:
        t = t[:256:8]         # k_describe_pf: wave 0 of each workgroup (slot 1000 + 8 b + wave)
    t = t[(t > 0).all(axis=1)]
    rows.append(np.diff(t, axis=1))
    spans.append(t[:, 5].max() - t[:, 0].min())
R = np.concatenate(rows)
print(f"describe waves sampled: {len(R)}; launch span (first stamp .. last): median {np.median(spans):.0f} cycles")
for i, n in enumerate(names):
    print(f"  {n:34s} median {int(np.median(R[:, i])):7d}  p90 {int(np.percentile(R[:, i], 90)):7d}")
print(f"  wave total median {int(np.median(R.sum(axis=1)))} cycles")
