"""Determinism amplifier: the batched extract of the bench's 1600 KITTI frames, repeated on one
context and compared frame by frame with its first run, while a second context runs the full path
(matcher included) on the same frames in a host thread, back to back -- so every extract repeat
co-runs with pose passes.  The matcher form is the process's (VO_MATCH_MFMA).

  python tools/det_amp.py [extract_repeats] [background: full|none]
"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence, render_sequences  # noqa: E402

W, H, F, S = 1241, 376, 200, 8
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
bg = sys.argv[2] if len(sys.argv) > 2 else "full"
rendered = render_sequences([(W, H, F, s, 1.0) for s in range(S)], 16)
seqs = [SceneSequence(W, H, nframes=F, seq=s, step=1.0) for s in range(S)]
frames = np.concatenate(rendered)
ctx1 = Context(W, H, K=seqs[0].K, max_kpts=2000)
d1 = ctx1.device_frames(frames)
stop = threading.Event()
bg_steps = [0]


def background():
    ctx2 = Context(W, H, K=seqs[0].K, max_kpts=2000)
    d2 = ctx2.device_frames(frames)
    gt = np.concatenate([s.gt() for s in seqs])
    while not stop.is_set():
        ctx2.reset()
        ctx2.set_ground_truth(gt)
        ctx2.set_sequence_starts([F * i for i in range(1, S)])
        ctx2.process_frames_device(d2)
        bg_steps[0] += 1
    d2.free()
    ctx2.close()


th = threading.Thread(target=background) if bg == "full" else None
nk0, k0, ds0 = ctx1.extract_frames_device(d1, outputs=True)
if th:
    th.start()
t0 = time.time()
bad_reps = bad_frames = 0
for r in range(reps):
    nk, k, ds = ctx1.extract_frames_device(d1, outputs=True)
    diff = [f for f in range(len(nk)) if nk[f] != nk0[f] or not np.array_equal(k[f], k0[f])
            or not np.array_equal(ds[f], ds0[f])]
    if diff:
        bad_reps += 1
        bad_frames += len(diff)
        f = diff[0]
        kd = np.nonzero((k[f] != k0[f]).any(1))[0]
        print(f"rep {r}: {len(diff)} frames differ {diff[:6]}; frame {f}: n {nk0[f]} -> {nk[f]}, "
              f"{kd.size} keypoints differ from {kd[:1].tolist()} (ref {k0[f][kd[:2]].tolist()} now {k[f][kd[:2]].tolist()})",
              flush=True)
    if r % 25 == 0:
        print(f"rep {r}: {time.time() - t0:.1f} s, background steps {bg_steps[0]}", flush=True)
stop.set()
if th:
    th.join()
print(f"extract under background '{bg}': {bad_reps} of {reps} repeats differ ({bad_frames} frames of "
      f"{reps * len(nk0)}), background steps {bg_steps[0]}")
d1.free()
ctx1.close()
