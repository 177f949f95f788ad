#!/usr/bin/env python3
"""Phase breakdown of k_select (VO_STAMPS build)."""
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
L = load()
L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
names = ["tilerows+scan+stage", "hist scan", "boundary collect", "boundary rank", "count pass", "scan+write pass"]
rows = []
for rep in range(5):
    ctx.extract(fr[rep % 2])
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    st = buf[1990 * 16:1990 * 16 + 16].astype(np.int64)
    rows.append(np.diff(st[:7]))
    nb = st[10]
med = np.median(np.array(rows), axis=0)
for n, v in zip(names, med):
    print(f"  {n:18s} {int(v):8d} cycles")
print("  boundary keys", nb)
