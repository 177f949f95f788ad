"""The round-4 r4j failure, reproduced on the CPU ("Select consistency").

Mid-round 4, the first FLAT stencil (branch-free rows: every lane stores its key and its histogram
count through a buffer offset that is out of range when the lane holds no maximum) took "is this
lane a maximum" from the 3x3 compare alone: ``mx0 = nb0 < rm0``.  The general form reaches its
stores only through the row's ballots, which the NMS row test ``rok`` (rows [35, H-35],
corner_detection_parallel_GPU.cpp:157) masks; the FLAT form stored on ``mx0`` directly, so every
strict maximum in the margin rows 2..34 and H-34..H-3 added a histogram count with no key behind it
(its key store landed on the tile's next free slot, overwritten or past the row counts).  The select
takes the top-N boundary bin and the count above it from the histogram and the keys from the tiles
(k_select phases C/D), so it emitted fewer than N keypoints while the slot count said N: the slot's
tail kept stale keypoints -- the "keypoints differ" of ``test_extract_bit_exact[scene0]``
(gpurun_out/r4j/tests.txt) -- and on a fresh context uninitialised ones, whose coordinates sent
k_describe's gathers out of the blurred plane: the HIP error 700 of gpurun_out/det_r4j/det_1.txt
(the first step of a fresh context).  The fix (commit 595354e) is ``mx0 = rok && nb0 < rm0``.

This test restates the stencil's key / histogram bookkeeping and the single-workgroup select
(vo_kernels.hip k_select) in numpy on the same frame, and shows (a) with the fixed rule the histogram
total equals the key count and the select equals the oracle's top-N, (b) with the r4j rule the
histogram holds the margin maxima, the select emits fewer than N keys, and the consistency check the
library now performs (histogram total == key count, emitted == min(C, N); a failure is
VO_STATUS_INCONSISTENT and VO_ERR_INTERNAL, never a silent OVERFLOW) fires.
"""
import numpy as np
import pytest

import oracle as O
from acs_visual_odometry_amd.synth import SceneSequence

HIST_BINS = 4096
N = 2000


def f32_bits(x):
    return np.asarray(x, np.float32).view(np.uint32).astype(np.int64)


def strict_maxima(R, rows, cols):
    """Strict 3x3 maxima (any neighbour >= the centre rejects, corner_detection_parallel_GPU.cpp:
    160-176) with R > 0 at the given row and column ranges (inclusive)."""
    H, W = R.shape
    P = np.full((H + 2, W + 2), -1.0, np.float32)
    P[1:-1, 1:-1] = R
    c = P[1:-1, 1:-1]
    ok = c > 0
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy or dx:
                ok &= c > P[1 + dy:H + 1 + dy, 1 + dx:W + 1 + dx]
    m = np.zeros_like(ok)
    r0, r1 = rows
    c0, c1 = cols
    m[r0:r1 + 1, c0:c1 + 1] = ok[r0:r1 + 1, c0:c1 + 1]
    return m


def keys_of(R, mask):
    ys, xs = np.nonzero(mask)
    bits = f32_bits(R[ys, xs])
    return (bits << 32) | (ys.astype(np.int64) << 16) | xs.astype(np.int64)


def hist_of(keys, thr_bits):
    b = np.minimum(((keys >> 32) - thr_bits) >> 15, HIST_BINS - 1)
    return np.bincount(b, minlength=HIST_BINS).astype(np.int64)


def select(keys, hist, thr_bits, n=N):
    """k_select (vo_kernels.hip, phases C-D): boundary bin and count above it from the histogram,
    the boundary keys from the key list, the need-th largest of them as the threshold key.
    Returns the selected keys (none of the boundary bin when no boundary key has that rank)."""
    C = len(keys)
    if C <= n:
        return keys.copy()
    suf = np.cumsum(hist[::-1])[::-1]                 # count at or above each bin
    above = np.concatenate([suf[1:], [0]])
    b = int(np.nonzero((above < n) & (above + hist >= n))[0][0])
    kb = np.minimum(((keys >> 32) - thr_bits) >> 15, HIST_BINS - 1)
    bnd = np.sort(keys[kb == b])[::-1]
    need = n - int(above[b])
    sel = keys[kb > b]
    if 0 < need <= len(bnd):
        sel = np.concatenate([sel, bnd[:need]])
    return sel


def raster(keys):
    rc = np.stack([(keys >> 16) & 0xFFFF, keys & 0xFFFF], 1)
    o = np.lexsort((rc[:, 1], rc[:, 0]))
    return np.stack([rc[o, 1], rc[o, 0]], 1).astype(np.int32)   # (x = col, y = row)


@pytest.mark.parametrize("frame", [0, 3])
def test_r4j_margin_maxima_break_the_select(frame):
    seq = SceneSequence(nframes=6, step=0.05)           # test_gpu_parity.py's ``scene``
    img = seq.frames()[frame]
    H, W = img.shape
    R = O.response(O.blur7(img))
    thr_bits = int(f32_bits(20000.0))
    cols = (37, W - 37)
    band = strict_maxima(R, (35, H - 35), cols)          # rok: the NMS rows
    every = strict_maxima(R, (0, H - 1), cols)           # r4j: every row the stencil visits
    keys = keys_of(R, band)
    assert len(keys) == O.nms_candidates(R)
    assert len(keys) > N                                 # the select ranks (C > N)

    # fixed rule: histogram == keys, select == oracle
    h_fix = hist_of(keys, thr_bits)
    assert h_fix.sum() == len(keys)
    sel = select(keys, h_fix, thr_bits)
    assert len(sel) == N
    assert np.array_equal(raster(sel), O.nms_topn(R))

    # r4j rule: the margin rows' maxima in the histogram, not in the keys
    spurious = keys_of(R, every & ~band)
    assert len(spurious) > 0
    h_r4j = h_fix + hist_of(spurious, thr_bits)
    assert h_r4j.sum() > len(keys)                       # the check that now fires
    sel_r4j = select(keys, h_r4j, thr_bits)
    assert len(sel_r4j) < N                              # fewer keypoints than the slot count claims
    print(f"frame {frame}: C={len(keys)} margin maxima={len(spurious)} emitted={len(sel_r4j)} of {N}")


def test_r4j_failure_output_reproduced():
    """The failing GPU output itself (gpurun_out/r4j/tests.txt:36): the r4j select's 1689 keypoints
    of scene frame 0, then the slot's stale tail -- the keypoints the previous extract on the same
    context wrote there (test_response_map_strong_edges_bit_exact's 0/255 block image, run just
    before).  pytest printed the head and the tail of both lists; the model gives exactly those."""
    H, W = 376, 1241
    yy, xx = np.mgrid[0:H, 0:W]
    prev = np.where(((yy // 9) + (xx // 11)) % 2 == 0, 0, 255).astype(np.uint8)
    prev[100:140, 300:700] = 255
    prev[200:260, 500:540] = 0
    stale, _, _ = O.extract(prev, O.config(W, H))
    img = SceneSequence(nframes=6, step=0.05).frames()[0]
    R = O.response(O.blur7(img))
    thr_bits = int(f32_bits(20000.0))
    band = strict_maxima(R, (35, H - 35), (37, W - 37))
    every = strict_maxima(R, (0, H - 1), (37, W - 37))
    keys = keys_of(R, band)
    sel = raster(select(keys, hist_of(keys, thr_bits) + hist_of(keys_of(R, every & ~band), thr_bits), thr_bits))
    out = stale.copy()
    out[:len(sel)] = sel
    assert len(sel) == 1689
    assert out[:3].tolist() == [[62, 35], [367, 35], [503, 35]]           # GPU head, as printed
    assert out[-3:].tolist() == [[1189, 340], [1197, 340], [1200, 340]]   # GPU tail, as printed
    assert O.nms_topn(R)[-3:].tolist() == [[759, 341], [776, 341], [913, 341]]   # oracle tail, as printed
