#!/usr/bin/env python3
"""Host-side anatomy of one bench step (S x 200 KITTI frames as one stream): wall time of
ctx.reset, set_ground_truth, set_sequence_starts, of the process_frames_device call, and of the
whole step, median over steps.  usage: python tools/step_host.py [steps] [sequences] [motion]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence, render_sequences  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
S = int(sys.argv[2]) if len(sys.argv) > 2 else 8
MOT = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
W, H, F = 1241, 376, 200
fr = render_sequences([(W, H, F, s, MOT) for s in range(S)], 8)
seqs = [SceneSequence(W, H, nframes=F, seq=s, step=MOT) for s in range(S)]
ctx = Context(W, H, K=seqs[0].K)
dall = ctx.device_frames(np.concatenate(fr))
gt = np.concatenate([s.gt() for s in seqs])
starts = [F * i for i in range(1, S)]
rs, gs, ss, call, tot = [], [], [], [], []
for i in range(steps + 3):
    t0 = time.perf_counter()
    ctx.reset()
    ta = time.perf_counter()
    ctx.set_ground_truth(gt)
    tb = time.perf_counter()
    ctx.set_sequence_starts(starts)
    t1 = time.perf_counter()
    ctx.process_frames_device(dall)
    t2 = time.perf_counter()
    if i >= 3:
        rs.append(ta - t0); gs.append(tb - ta); ss.append(t1 - tb); call.append(t2 - t1); tot.append(t2 - t0)
m = lambda v: np.median(v) * 1e6
print(f"per step (us, median of {steps}): reset {m(rs):.1f}  gt {m(gs):.1f}  starts {m(ss):.1f}  "
      f"process_frames_device {m(call):.1f}  step {m(tot):.1f}  -> {S * F / np.median(tot):.0f} frames/s")
