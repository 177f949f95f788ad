"""Repeat the bench's headline stream (8 x 200 KITTI frames, 1.0 m/frame) under changing timing
modes and report where a repeat first differs from the first run: per sequence the first frame
whose status / info / pose differs, with both rows, so the stage that diverged can be read off
(keypoint count: extract; matches: match; inliers: RANSAC; pose only: refit / pose).  Then the
batched extract alone, repeated, keypoints and descriptors compared frame by frame.

  python tools/det_stress.py [repeats] [extract_repeats]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acs_visual_odometry_amd import Context  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence, render_sequences  # noqa: E402

W, H, F, S = 1241, 376, 200, 8
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
xreps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rendered = render_sequences([(W, H, F, s, 1.0) for s in range(S)], 16)
seqs = [SceneSequence(W, H, nframes=F, seq=s, step=1.0) for s in range(S)]
# (after the forked renderers; torch initialises the GPU before the library does)
# DET_LOAD=gemm[:n]: n bf16 8192^3 GEMMs (torch / hipBLASLt, matrix cores) queued on a torch stream of
# their own before every step, so unrelated MFMA work co-runs with the path (whatever matcher runs)
load = os.environ.get("DET_LOAD", "")
if load.startswith("gemm"):
    import torch
    n_gemm = int(load.split(":")[1]) if ":" in load else 16
    ga = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    gb = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    gc = torch.empty(8192, 8192, device="cuda", dtype=torch.bfloat16)
    gstream = torch.cuda.Stream()


ctx = Context(W, H, K=seqs[0].K, max_kpts=2000)
dall = ctx.device_frames(np.concatenate(rendered))
gt_all = np.concatenate([s.gt() for s in seqs])
starts = [F * i for i in range(1, S)]


def layout():
    """The context's device buffers and the frames, and which of them the range
    [blurred + 1 GiB, + blurred bytes) overlaps: where round 3's soffset-dropped blurred-row
    stores land if the range check ignores soffset (tests/hip/buffer_range_probe.hip)."""
    import ctypes as C
    L = ctx.lib
    L.vo_debug_layout.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_uint64)]
    bufs = []
    for i in range(L.vo_debug_layout(ctx.h, -1, None, None, None)):
        nm, pt, nb = C.c_char_p(), C.c_uint64(), C.c_uint64()
        L.vo_debug_layout(ctx.h, i, C.byref(nm), C.byref(pt), C.byref(nb))
        bufs.append((nm.value.decode(), pt.value, nb.value))
    bufs.append(("frames", int(dall.ptr.value), int(dall.frame_bytes) * int(dall.n)))
    bl = [b for b in bufs if b[0] == "blurred"][0]
    lo, hi = bl[1] + (1 << 30), bl[1] + (1 << 30) + bl[2]
    for nm, pt, nb in sorted(bufs, key=lambda b: b[1]):
        hit = " <-- blurred + 1 GiB overlaps" if pt < hi and pt + nb > lo else ""
        print(f"  {nm:12s} {pt:#014x} {nb:12d}{hit}")
    print(f"  blurred + 1 GiB = [{lo:#014x}, {hi:#014x})", flush=True)


layout()


def background():
    if load.startswith("gemm"):
        with torch.cuda.stream(gstream):
            for _ in range(n_gemm):
                torch.matmul(ga, gb, out=gc)


def step(timing):
    background()
    ctx.reset()
    ctx.set_ground_truth(gt_all)
    ctx.set_sequence_starts(starts)
    return ctx.process_frames_device(dall, timing=timing)


modes = [0, 100, 1, 0, 104, 103, 0, 1, 105, 0, 100, 1]
if os.environ.get("DET_MODES"):
    modes = [int(m) for m in os.environ["DET_MODES"].split(",")]
dbg = os.environ.get("DET_DBG") == "1"       # MM_VERIFY builds: MFMA key / hand-off counters in d.dbg
if dbg:
    import ctypes as C
    L = ctx.lib
    L.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    dbuf = np.zeros(22000, np.uint64)

    def counters():
        L.vo_debug_stamps(ctx.h, dbuf.ctypes.data_as(C.c_void_p), dbuf.size)
        return dbuf[6000:6008].astype(np.int64).copy()
    c_prev = counters()
diag = os.environ.get("DET_DIAG") == "1"     # ST_DIAG builds: stencil -> select per-tile key checksums
if diag:
    import ctypes as C
    ctx.lib.vo_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    dgbuf = np.zeros(24040, np.uint64)

    def diag_read():
        ctx.lib.vo_debug_stamps(ctx.h, dgbuf.ctypes.data_as(C.c_void_p), dgbuf.size)
        return dgbuf[24000:24040].copy()
    dg_prev = None
    diag_frames, diag_tiles = 0, []
    ctx.lib.vo_debug_diag.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
    NFd = S * F

    def diag_arr(what, f0=0, n=NFd):
        per = ctx.lib.vo_debug_diag(ctx.h, what, 0, 0, None)
        out = np.zeros((n, per), np.uint64)
        assert ctx.lib.vo_debug_diag(ctx.h, what, f0, n, out.ctypes.data_as(C.c_void_p)) == per
        return out
    NTX = (W + 56) // 57

    def key_str(k):
        k = int(k)
        r = np.array([k >> 32], np.uint32).view(np.float32)[0]
        return f"(x {k & 0xFFFF}, y {(k >> 16) & 0xFFFF}, R {r:.7g})"
ring = os.environ.get("DET_RING") == "1"     # compare the extracted ring slots too (vo_debug_ring)
if ring:
    import ctypes as C
    ctx.lib.vo_debug_ring.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    NF = S * F

    def ring_read():
        nk = np.zeros(NF, np.int32)
        kp = np.zeros((NF, 2000, 2), np.int32)
        pr = np.zeros((NF, 2000), np.uint32)
        rc = ctx.lib.vo_debug_ring(ctx.h, 0, NF, nk.ctypes.data_as(C.c_void_p), kp.ctypes.data_as(C.c_void_p),
                                   pr.ctypes.data_as(C.c_void_p))
        assert rc == 0, rc
        return nk, kp, pr
ref = step(0)
if diag:
    dref = [diag_arr(w) for w in (0, 1, 2)]
    kref = diag_arr(3)
ring_ref = ring_read() if ring else None
if dbg:
    counters()
    sel_ref = dbuf[8000:21600].copy()
bad = 0
t0 = time.time()
for r in range(reps):
    m = modes[r % len(modes)]
    p, st, info = step(m)
    same = np.array_equal(p, ref[0]) and np.array_equal(st, ref[1]) and np.array_equal(info, ref[2])
    msg = ""
    if dbg:
        c_now = counters()
        dc = c_now - c_prev
        c_prev = c_now
        msg = (f" mfma keys wrong {dc[0]} of {dc[1]}, stale match_j {dc[2]} of {dc[3]},"
               f" select: hist total != keys {dc[4]}, need > boundary keys {dc[5]} of {dc[6]} frames")
    if diag:
        dg = diag_read()
        if dg_prev is None or not np.array_equal(dg[1:], dg_prev[1:]):
            msg += (f" diag: tiles {int(dg[0])} checksum mismatches {int(dg[1])} invalid keys {int(dg[2])}"
                    + (f"; first: frame {int(dg[3]) - 1} tile {int(dg[4])} stencil ck {int(dg[5]):#x} select ck"
                       f" {int(dg[6]):#x} n {int(dg[7])} bad index {int(dg[8]) - 1} keys"
                       f" {[hex(int(k)) for k in dg[10:10 + min(int(dg[7]), 24)]]}" if dg[3] else ""))
        dg_prev = dg
        dnow = [diag_arr(w) for w in (0, 1, 2)]
        names = ("select key ck", "stencil source ck", "stencil response ck")
        fr_d = sorted(set(int(f) for w in range(3) for f in np.nonzero((dnow[w] != dref[w]).any(1))[0]))
        diag_frames += len(fr_d)
        diag_tiles.extend(int(t) for f in fr_d for t in np.nonzero(dnow[0][f] != dref[0][f])[0])
        for f in fr_d[:3]:
            msg += f"\n    diag frame {f}:"
            for w in range(3):
                t = np.nonzero(dnow[w][f] != dref[w][f])[0]
                msg += f" {names[w]} tiles {[(int(x), divmod(int(x), NTX)) for x in t[:4]]}"
            kn = diag_arr(3, f, 1)[0]
            a, b = set(kref[f][kref[f] != 0].tolist()), set(kn[kn != 0].tolist())
            ts = np.nonzero(dnow[1][f] != dref[1][f])[0]
            for t in ts[:4]:
                msg += f"\n      source ck tile {int(t)}: ref {int(dref[1][f][t]):#018x} now {int(dnow[1][f][t]):#018x}"
            msg += (f"\n      keys only in ref: {[key_str(k) for k in sorted(a - b)[:6]]}"
                    f"\n      keys only now:   {[key_str(k) for k in sorted(b - a)[:6]]}")
    if ring:
        nk, kp, pr = ring_read()
        fd = [f for f in range(NF) if nk[f] != ring_ref[0][f] or not np.array_equal(kp[f, :nk[f]], ring_ref[1][f, :nk[f]])
              or not np.array_equal(pr[f, :nk[f]], ring_ref[2][f, :nk[f]])]
        msg += f" ring frames differing: {len(fd)}" + (f" {fd[:6]}" if fd else "")
        for f in fd[:2]:
            if dbg:
                sel = dbuf[8000:21600]
                msg += (f"\n    select frame {f}: key-list checksum {'same' if sel[f] == sel_ref[f] else 'DIFFERS'},"
                        f" C {sel_ref[4000 + f]} -> {sel[4000 + f]}, Tb {hex(int(sel_ref[8000 + f]))} -> {hex(int(sel[8000 + f]))},"
                        f" b {sel_ref[12000 + f]} -> {sel[12000 + f]}")
            n0 = ring_ref[0][f]
            kd = np.nonzero((kp[f, :n0] != ring_ref[1][f, :n0]).any(1))[0]
            pd = np.nonzero(pr[f, :n0] != ring_ref[2][f, :n0])[0]
            msg += (f"\n    ring frame {f}: n {n0} -> {nk[f]}; {kd.size} keypoints differ {kd[:6].tolist()}"
                    f" (ref {ring_ref[1][f, kd[:3]].tolist()} now {kp[f, kd[:3]].tolist()});"
                    f" {pd.size} prefixes differ {pd[:6].tolist()}"
                    f" (ref {[hex(v) for v in ring_ref[2][f, pd[:3]]]} now {[hex(v) for v in pr[f, pd[:3]]]})")
    print(f"rep {r} timing {m}: {'same' if same else 'DIFFERS'} ({time.time() - t0:.1f} s){msg}", flush=True)
    if same:
        continue
    bad += 1
    for s in range(S):
        sl = slice(s * F, (s + 1) * F)
        d = np.nonzero((st[sl] != ref[1][sl]) | (info[sl] != ref[2][sl]).any(1) |
                       (p[sl] != ref[0][sl]).reshape(F, -1).any(1))[0]
        if d.size == 0:
            continue
        f = int(d[0])
        print(f"  seq {s}: {d.size} frames differ, first {f}")
        for g in range(max(0, f - 1), min(F, f + 2)):
            print(f"    frame {g}: ref st {ref[1][s * F + g]} info {ref[2][s * F + g].tolist()}"
                  f" | now st {st[s * F + g]} info {info[s * F + g].tolist()}"
                  f" | pose diff {np.abs(p[s * F + g] - ref[0][s * F + g]).max():.3g}")
print(f"full path: {bad} of {reps} repeats differ", flush=True)
if diag:
    odd = sum(1 for t in diag_tiles if (t % NTX) % 2 == 1)
    print(f"diag: {diag_frames} frame computations differ over the repeats; tiles {len(diag_tiles)}, "
          f"of them in odd tile columns (lanes 32-63) {odd}", flush=True)

nk0, k0, d0 = ctx.extract_frames_device(dall, outputs=True)
xbad = 0
for r in range(xreps):
    background()
    nk, k, d = ctx.extract_frames_device(dall, timing=(0, 1, 100)[r % 3], outputs=True)
    diff = [f for f in range(len(nk)) if nk[f] != nk0[f] or not np.array_equal(k[f], k0[f])
            or not np.array_equal(d[f], d0[f])]
    print(f"extract rep {r}: {len(diff)} frames differ" + (f", first {diff[:5]}" if diff else ""), flush=True)
    for f in diff[:2]:
        kd = np.nonzero((k[f] != k0[f]).any(1))[0] if nk[f] == nk0[f] else None
        dd = np.nonzero((d[f] != d0[f]).any(1))[0] if nk[f] == nk0[f] else None
        print(f"    frame {f}: n {nk0[f]} -> {nk[f]}; kps differ at {None if kd is None else kd[:8].tolist()}"
              f"; desc differ at {None if dd is None else dd[:8].tolist()}")
    xbad += bool(diff)
print(f"extract: {xbad} of {xreps} repeats differ")
dall.free()
ctx.close()
