"""WRITE_SIZE attribution of k_stencil: the batched extract of 64 synthetic KITTI
frames, repeated, through whichever library VO_LIB_PATH names -- the probe builds
(make variant NAME=wp<k> DEFS=-DST_PROBE_NOSTORE=<k>) drop the blurred-plane stores (1), the key and
tile-row stores (2) or the histogram atomics (4), so their selects see inconsistent frames: the
return code is ignored (the stencil's launches are what the PMC pass counts).
Usage (GPU box): rocprofv3 --pmc WRITE_SIZE -- python3 tools/stencil_write_probe.py [reps]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from acs_visual_odometry_amd import Context  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence, render_sequences  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
frames = render_sequences([(1241, 376, 64, 0, 1.0)], 8)[0]
ctx = Context(1241, 376, K=SceneSequence(1241, 376, nframes=1).K)
df = ctx.device_frames(frames)
nk = np.zeros(64, np.int32)
for _ in range(reps):
    rc = ctx.lib.vo_extract_frames_device(ctx.h, df.ptr, df.frame_bytes, 64, None, None, nk.ctypes.data_as(C.c_void_p))
    print("rc", rc, "mean kpts", float(nk.mean()))
df.free()
ctx.close()
