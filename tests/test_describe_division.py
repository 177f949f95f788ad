"""The orientation term (ic*d)/|d| (kernels/feature_extraction_kernel_functions.c:159-160, f32
with a correctly rounded division).  The oracle evaluates it as (float)((double)(ic*d) * (1/|d|));
the describe kernel as fmaf(ic, A, ic * B) with the unit direction d/|d| split into two f32
(A = f32(d/|d|), B = f32(d/|d| - A), the quotient in f64; round 2's kernel used fmaf(x, rh, x * rl)
with x = ic*d and the reciprocal 1/|d| split the same way).  This checks, for every pair of the FREAK
pattern, both components and every intensity difference ic in [-255, 255], that all four give
the same f32 value (the hi/lo form may return +0 where the division returns -0; the orientation
sums start at +0 and an f32 sum is -0 only if both addends are, so the sums are identical)."""
import os
import re

import numpy as np

HDR = os.path.join(os.path.dirname(__file__), "..", "include", "vo_freak_tables.h")


def freak_points():
    src = open(HDR).read()
    body = src.split("#define VO_FREAK_POINTS_LIST")[1].split("#define")[0]
    return [tuple(map(int, p)) for p in re.findall(r"\{(-?\d+), (-?\d+)\}", body)]


def fma32(a, b, c):
    """Exact IEEE fmaf (round to nearest even) on float32 arrays: the f64 sum rounded to odd
    (TwoSum error term), then to f32 -- round-to-odd at 53 >= 24 + 2 bits rounds correctly."""
    p = a.astype(np.float64) * b.astype(np.float64)       # exact: 24 + 24 bits
    cc = c.astype(np.float64)
    s = p + cc
    bb = s - p
    t = (p - (s - bb)) + (cc - bb)
    even = (s.view(np.uint64) & 1) == 0
    s = np.where((t != 0) & even, np.nextafter(s, np.where(t > 0, np.inf, -np.inf)), s)
    return s.astype(np.float32)


def test_fma32_emulation_is_exact():
    from fractions import Fraction as Fr
    rng = np.random.default_rng(7)
    a, b, c = (rng.normal(size=4000).astype(np.float32) * np.float32(s) for s in (1.0, 300.0, 0.01))
    got = fma32(a, b, c)
    for i in range(0, 4000, 7):
        v = Fr(float(a[i])) * Fr(float(b[i])) + Fr(float(c[i]))
        g = np.float32(float(v))
        cands = [np.nextafter(g, np.float32(-np.inf)), g, np.nextafter(g, np.float32(np.inf))]
        best = min(cands, key=lambda z: (abs(Fr(float(z)) - v), int(np.array(z).view(np.uint32)) & 1))
        assert got[i] == best


def test_orientation_term_forms_agree_exhaustively():
    pts = freak_points()
    assert len(pts) == 43
    ic = np.arange(-255, 256, dtype=np.float32)
    checked = 0
    for p in range(43):
        for q in range(p + 1, 43):
            dx = np.float32(pts[p][0] - pts[q][0])
            dy = np.float32(pts[p][1] - pts[q][1])
            nrm = np.sqrt(dx * dx + dy * dy, dtype=np.float32)
            assert nrm > 0
            rn = 1.0 / np.float64(nrm)
            rh = np.float32(rn)
            rl = np.float32(rn - np.float64(rh))
            for dd in (dx, dy):
                num = ic * dd                                   # exact: |ic*d| < 2^24
                ref = num / nrm
                alt = (num.astype(np.float64) * rn).astype(np.float32)
                assert np.array_equal(ref.view(np.uint32), alt.view(np.uint32))
                hl = fma32(num, np.full_like(num, rh), num * rl)
                assert np.array_equal(hl, ref)                  # value equality: +0 == -0
                assert np.array_equal(hl.view(np.uint32) & 0x7FFFFFFF, ref.view(np.uint32) & 0x7FFFFFFF)
                # the kernel's form (vo_kernels.hip ensure_tables / orient_term)
                u = np.float64(dd) / np.float64(nrm)
                A = np.float32(u)
                B = np.float32(u - np.float64(A))
                ab = fma32(ic, np.full_like(ic, A), ic * B)
                assert np.array_equal(ab, ref)
                assert np.array_equal(ab.view(np.uint32) & 0x7FFFFFFF, ref.view(np.uint32) & 0x7FFFFFFF)
                checked += num.size
    assert checked == 903 * 2 * 511
