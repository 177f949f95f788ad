#!/usr/bin/env python3
"""Two pipelines on one GPU: the bench's 8 x 200-frame workload as S streams (contexts) of 8/S
sequences each, driven from S host threads at once (ctypes releases the GIL in the library
call), against one context running all 8.  usage: python tools/two_ctx.py [steps] [streams]"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence, render_sequences  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
S = int(sys.argv[2]) if len(sys.argv) > 2 else 2
W, H, F, NS = 1241, 376, 200, 8
fr = render_sequences([(W, H, F, s, 1.0) for s in range(NS)], 8)
seqs = [SceneSequence(W, H, nframes=F, seq=s, step=1.0) for s in range(NS)]


def make(group):
    ctx = Context(W, H, K=seqs[0].K)
    df = ctx.device_frames(np.concatenate([fr[s] for s in group]))
    gt = np.concatenate([seqs[s].gt() for s in group])
    starts = [F * i for i in range(1, len(group))]
    return ctx, df, gt, starts


def step(c):
    ctx, df, gt, starts = c
    ctx.reset()
    ctx.set_ground_truth(gt)
    ctx.set_sequence_starts(starts)
    return ctx.process_frames_device(df)


def run(cs, n):
    if len(cs) == 1:
        t0 = time.perf_counter()
        for _ in range(n):
            step(cs[0])
        return time.perf_counter() - t0
    bar = threading.Barrier(len(cs) + 1)
    out = [None] * len(cs)

    def worker(i):
        bar.wait()
        for _ in range(n):
            out[i] = step(cs[i])
        bar.wait()
    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(cs))]
    for t in th:
        t.start()
    bar.wait()
    t0 = time.perf_counter()
    bar.wait()
    dt = time.perf_counter() - t0
    for t in th:
        t.join()
    return dt


one = [make(list(range(NS)))]
many = [make(list(range(i * NS // S, (i + 1) * NS // S))) for i in range(S)]
ref = step(one[0])
for c in many:
    step(c)
for rep in range(2):
    d1 = run(one, steps)
    dS = run(many, steps)
    print(f"rep {rep}: one context {NS * F * steps / d1:.0f} frames/s, {S} contexts x {NS // S} sequences "
          f"{NS * F * steps / dS:.0f} frames/s")
# the S streams' rows equal the single stream's
rows = [step(c) for c in many]
p = np.concatenate([r[0] for r in rows])
st = np.concatenate([r[1] for r in rows])
print("rows equal:", bool(np.array_equal(p, ref[0]) and np.array_equal(st, ref[1])))
