"""The describe kernel evaluates the orientation term (ic*d)/|d| (kernels/
feature_extraction_kernel_functions.c:159-160, f32 with a correctly rounded division) as
(float)((double)(ic*d) * (1/|d|)).  This checks, for every pair of the FREAK pattern and
every intensity difference ic in [-255, 255], that both give the same f32 bits."""
import re
import os

import numpy as np

HDR = os.path.join(os.path.dirname(__file__), "..", "include", "vo_freak_tables.h")


def test_reciprocal_multiply_equals_f32_division_exhaustively():
    src = open(HDR).read()
    body = src.split("vo_freak_points[VO_FREAK_NPOINTS][2] = {")[1].split("};")[0]
    pts = [tuple(map(int, p)) for p in re.findall(r"\{(-?\d+), (-?\d+)\}", body)]
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
            for dd in (dx, dy):
                num = ic * dd                                   # exact: |ic*d| < 2^24
                ref = num / nrm
                alt = (num.astype(np.float64) * rn).astype(np.float32)
                assert np.array_equal(ref.view(np.uint32), alt.view(np.uint32))
                checked += num.size
    assert checked == 903 * 2 * 511
