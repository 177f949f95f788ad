#!/usr/bin/env python3
"""Per-phase cycle breakdown of one RANSAC hypothesis wave (diagnostic VO_STAMPS build).
usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so python tools/stamps.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context, load  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence  # noqa: E402

seq = SceneSequence(nframes=2, step=0.05)
fr = seq.frames()
ctx = Context(seq.W, seq.H, K=seq.K)
k0, d0 = ctx.extract(fr[0])
k1, d1 = ctx.extract(fr[1])
m = ctx.match(d0, d1)
pts = np.concatenate([k0[m[:, 0]], k1[m[:, 1]]], 1).astype(np.float64)
L = load()
L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
for rep in range(3):
    r = ctx.ransac(pts, 7 + rep)
buf = np.zeros(2000 * 16, np.uint64)
n = L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
st = buf[:256 * 16].reshape(256, 16).astype(np.int64)
names = ["sample8", "load+normalize", "gauss-jordan", "denorm+rank2", "(ret)", "sampson"]
d = np.diff(st[:, :7], axis=1)
print(f"M={len(pts)} n_eval={r['n_evaluated']}; cycles per phase (median over 256 hypotheses)")
for i, nm in enumerate(names):
    print(f"  {nm:16s} {int(np.median(d[:, i])):8d}")
print(f"  {'total':16s} {int(np.median(st[:, 6] - st[:, 0])):8d}")
print("spread of start stamps (cycles):", int(st[:, 0].max() - st[:, 0].min()))
