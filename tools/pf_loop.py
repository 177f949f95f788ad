#!/usr/bin/env python3
"""vo_process_frame called once per frame (the reference loop's per-frame call): prints the
per-call latency (median over calls) for a kernel-trace profile of the single-frame path."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from acs_visual_odometry_amd import Context  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
seq = SceneSequence(nframes=n, step=1.0)
frames = seq.frames()
ctx = Context(seq.W, seq.H, K=seq.K)
ctx.set_ground_truth(seq.gt())
hf = ctx.host_frames(frames) if os.environ.get("PF_PINNED") == "1" else None   # frames in pinned memory
src = hf.array if hf is not None else frames
for rep in range(2):
    ctx.reset()
    ts = []
    for f in range(n):
        t0 = time.perf_counter()
        ctx.process_frame(src[f])
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts[5:]) * 1e6
    print(f"{'pinned' if hf is not None else 'pageable'} rep {rep}: per call median {np.median(ts):.1f} us, mean {ts.mean():.1f} us, min {ts.min():.1f} us")
if hf is not None:
    hf.free()
ctx.close()
