"""Extract-only determinism next to an unrelated load on another stream: the batched extract of the
headline stream (8 x 200 KITTI frames) is repeated while torch runs large bf16 matrix products
(hipBLASLt, MFMA) or elementwise work on its own stream, and every repeat's keypoints and 32-test
prefixes are compared with a run without load.  Unrelated memory, no shared buffers: any difference
is interference, not a data race of the path.

  python tools/det_burn.py [repeats] [mode: mfma | valu | none]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence, render_sequences  # noqa: E402

W, H, F, S = 1241, 376, 200, 8
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
mode = sys.argv[2] if len(sys.argv) > 2 else "mfma"
rendered = render_sequences([(W, H, F, s, 1.0) for s in range(S)], 16)
seq0 = SceneSequence(W, H, nframes=F, seq=0, step=1.0)
ctx = Context(W, H, K=seq0.K, max_kpts=2000)
dall = ctx.device_frames(np.concatenate(rendered))


def extract():
    nk, kp, ds = ctx.extract_frames_device(dall, outputs=True)
    pre = [d[:, 0] & 0xFFFFFFFF for d in ds]
    return nk, kp, pre


ref = extract()
dev = torch.device("cuda:0")
side = torch.cuda.Stream(device=dev)
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
x = torch.randn(64 << 20, device=dev)
bad = 0
t0 = time.time()
for r in range(reps):
    if mode != "none":
        with torch.cuda.stream(side):
            for _ in range(40):                       # ~1 s of load queued ahead of the extract
                if mode == "mfma":
                    c = a @ b
                else:
                    x = torch.sin(x) * 1.0001 + 0.5
    nk, kp, pre = extract()
    diff = [f for f in range(len(nk)) if nk[f] != ref[0][f] or not np.array_equal(kp[f], ref[1][f])
            or not np.array_equal(pre[f], ref[2][f])]
    torch.cuda.synchronize()
    bad += bool(diff)
    print(f"rep {r} load {mode}: {len(diff)} frames differ {diff[:6]} ({time.time() - t0:.1f} s)", flush=True)
print(f"extract under {mode} load: {bad} of {reps} repeats differ")
dall.free()
ctx.close()
