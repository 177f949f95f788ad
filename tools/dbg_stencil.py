"""Debug aid: compare the device blurred image and response map with the oracle on one frame
and print where they differ (GPU box)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import oracle as O
from acs_visual_odometry_amd import Context
from acs_visual_odometry_amd.synth import SceneSequence

seq = SceneSequence(nframes=1, step=0.05)
img = seq.frames()[0]
ctx = Context(seq.W, seq.H, K=seq.K)
k, dsc, bl = ctx.extract(img, want_blurred=True)
blr = O.blur7(img)
print("kps", len(k))
bd = np.argwhere(bl != blr)
print("blur mismatches", len(bd), bd[:10], bl.shape)
if len(bd):
    y, x = bd[0]
    print("gpu", bl[y, x - 3:x + 4], "ref", blr[y, x - 3:x + 4])
R = ctx.response(img)
Rr = O.response(blr)
rd = np.argwhere(R.view(np.uint32) != Rr.view(np.uint32))
print("resp mismatches", len(rd), rd[:4], "nonzero gpu", np.count_nonzero(R), "ref", np.count_nonzero(Rr))
if len(rd):
    y, x = rd[0]
    print("gpu", R[y, x - 2:x + 3], "ref", Rr[y, x - 2:x + 3])
# debug planes (VO_DBG=2..6 builds of vo_response): window sums / vertical sums / squares
b = blr.astype(np.int64)
H, W = b.shape
jx = np.zeros_like(b); jy = np.zeros_like(b); jxy = np.zeros_like(b)
a, m, e = b[:-2], b[1:-1], b[2:]
d = a - e; s = a + 2 * m + e
jx[1:-1, 1:-1] = d[:, :-2] + 2 * d[:, 1:-1] + d[:, 2:]
jy[1:-1, 1:-1] = s[:, :-2] - s[:, 2:]
jxy[1:-1, 1:-1] = d[:, :-2] - d[:, 2:]
planes = {2: jx * jx, 3: jy * jy, 4: jxy}
for dbg in (2, 3, 4, 5, 6):
    os.environ["VO_DBG"] = str(dbg)
    G = ctx.response(img).astype(np.int64)
    q = planes.get(dbg, jx * jx)
    if dbg in (2, 3, 4):
        ref = np.zeros_like(q)
        for yy in range(2, H - 2):
            ref[yy, 2:W - 2] = sum(q[yy + i, 2 + j:W - 2 + j] for i in range(-2, 3) for j in range(-2, 3))
        ref = ref  # window sum centred at yy
    elif dbg == 5:   # vertical 5-sum of jx^2 rows yr-2..yr+2
        ref = np.zeros_like(q)
        for yy in range(2, H - 2):
            ref[yy] = q[yy - 2:yy + 3].sum(0)
    else:            # qx4 = jx^2 of row yr + 2
        ref = np.zeros_like(q); ref[:-2] = q[2:]
    dd = np.argwhere(G[2:-2, 2:-2] != ref[2:-2, 2:-2])
    print("dbg", dbg, "mismatch", len(dd), dd[:6] + [2, 2] if len(dd) else "")
    if len(dd):
        y, x = dd[0] + [2, 2]
        print("   gpu", G[y, x - 2:x + 3], "ref", ref[y, x - 2:x + 3])
print("all resp mismatch rows", np.unique(rd[:, 0])[:20], "cols", np.unique(rd[:, 1])[:40])
