#!/usr/bin/env python3
"""The per-frame call's fused select (k_select_fused, VO_SEL_BANDS workgroups) from s_memtime
stamps (diagnostic VO_STAMPS build): cycles per phase of each band, median over calls, and the
wait for the last band's ranking.
usage: VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so python tools/stamps_select_pf.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context, load  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence  # noqa: E402

seq = SceneSequence(nframes=32, step=1.0)
fr = seq.frames()
ctx = Context(seq.W, seq.H, K=seq.K)
ctx.set_ground_truth(seq.gt())
L = load()
L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
names = ["count: band table (+ histogram loads)", "count: boundary bin", "count: band keys scanned",
         "wait: last band's rank + publish", "emit: band table", "emit: bitmap + segment counts",
         "emit: segment scan", "emit: keypoints written"]
rows, spans, rank = [], [], []
for rep in range(30):
    ctx.process_frame(fr[rep + 1])
    buf = np.zeros(2000 * 16, np.uint64)
    L.vo_debug_stamps(ctx.h, buf.ctypes.data_as(C.c_void_p), buf.size)
    t = buf[1960 * 16:1968 * 16].reshape(8, 16)[:, :10].astype(np.int64)
    t = t[(t[:, [0, 1, 2, 3, 5, 6, 7, 8, 9]] > 0).all(axis=1)]
    if rep < 2 or len(t) == 0:
        continue
    ph = np.stack([t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 5] - t[:, 3],
                   t[:, 6] - t[:, 5], t[:, 7] - t[:, 6], t[:, 8] - t[:, 7], t[:, 9] - t[:, 8]], axis=1)
    rows.append(ph)
    spans.append(t[:, 9].max() - t[:, 0].min())
    r = int(buf[1968 * 16])
    rank.append(r - t[:, 3].max())
R = np.concatenate(rows)
# (s_memtime counters are per XCD, so stamps of different bands are not compared: phases only)
print(f"select bands sampled: {len(R)}")
for i, n in enumerate(names):
    print(f"  {n:40s} median {int(np.median(R[:, i])):7d}  p90 {int(np.percentile(R[:, i], 90)):7d}")
ctx.close()
