#!/usr/bin/env python3
"""Per-frame RANSAC first-launch anatomy in the frame pipeline (diagnostic VO_STAMPS build):
hypothesis-wave phases, the spread of wave start times and the replay by the last wave.
usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so python tools/stamps_ransac.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context, load  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence  # noqa: E402

seq = SceneSequence(nframes=40, step=0.05)
fr = seq.frames()
ctx = Context(seq.W, seq.H, K=seq.K)
ctx.set_ground_truth(seq.gt())
L = load()
L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
names = ["sample8", "load+normalize", "gauss-jordan", "denorm+rank2", "(ret)", "sampson"]
rows = []
print("frame  M  n_eval | wave start spread | wave total p50/max | replay | launch span (kcycles)")
for f in range(seq.n):
    _, st, info = ctx.process_frame(fr[f])
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    if st != 0:
        continue
    s = buf[:256 * 16].reshape(256, 16).astype(np.int64)
    rp = buf[1997 * 16:1997 * 16 + 2].astype(np.int64)
    tot = s[:, 6] - s[:, 0]
    rows.append(np.median(np.diff(s[:, :7], axis=1), axis=0))
    print(f"{f:5d} {info[1]:4d} {info[4]:5d} | {(s[:, 0].max() - s[:, 0].min()) / 1e3:8.1f} | "
          f"{np.median(tot) / 1e3:6.1f} / {tot.max() / 1e3:6.1f} | {(rp[1] - rp[0]) / 1e3:6.1f} | "
          f"{(rp[1] - s[:, 0].min()) / 1e3:7.1f}")
    w = int(np.argmax(tot))
    if tot[w] > 2 * np.median(tot):
        print(f"      slowest wave: hypothesis {w}, phases (kcycles)",
              {n: round(v / 1e3, 1) for n, v in zip(names, np.diff(s[w, :7]))})
R = np.median(np.array(rows), axis=0)
print("median cycles per phase:", {n: int(v) for n, v in zip(names, R)})
