"""Stencil strip / tile geometry (vo_internal.h VO_TILE_W, VO_STRIP_XL, VO_BLUR_X0, vo_blur_stride;
vo_kernels.hip k_stencil): every image column is an output column of exactly one strip, the lanes of
tile A / B are lanes 0..31 / 32..63, a tile's strict 3x3 maxima fit VO_TILE_CAP, and every blurred
store of a column pair lands inside the row stride.  CPU only; the constants are read from the header."""
import re
from pathlib import Path

import numpy as np
import pytest

HDR = Path(__file__).resolve().parents[1] / "acs_visual_odometry_amd" / "csrc" / "vo_internal.h"


def _define(name):
    m = re.search(rf"#define {name} (\d+)", HDR.read_text())
    assert m, name
    return int(m.group(1))


TW = _define("VO_TILE_W")
TH = _define("VO_TILE_H")
SW = 2 * TW
XL = 128 - SW - 7 - (128 - SW - 14) // 2          # VO_STRIP_XL
X0 = XL & 1                                        # VO_BLUR_X0
CAP = ((TW + 1) // 2) * ((TH + 1) // 2)            # VO_TILE_CAP


def blur_stride(W):
    return (((W + SW - 1) // SW) * SW + X0 + 1 + 3) & ~3


def test_layout_constants():
    assert SW + 14 <= 128                          # strip + 7 halo columns each side in 64 column pairs
    assert XL + TW - 1 == 63                       # tile A ends in lane 31 (its second column)
    assert XL >= 7 and 128 - XL - SW >= 7          # the halo both sides


@pytest.mark.parametrize("W", [64, 113, 114, 115, 913, 1000, 1025, 1241, 1280, 1920])
def test_columns_covered_once_and_stores_in_stride(W):
    nsx = ((W + TW - 1) // TW + 1) // 2
    owner = np.zeros(W, np.int32)
    Wb = blur_stride(W)
    for sxi in range(nsx):
        xs = sxi * SW
        for lane in range(64):
            c0 = xs - XL + 2 * lane
            for c in (c0, c0 + 1):
                if xs <= c < xs + SW and 0 <= c < W:
                    owner[c] += 1
                    # tile A: lanes 0..31, tile B: 32..63 (k_stencil isB)
                    assert (c - xs >= TW) == (lane >= 32)
            # blurred store of the pair: issued when either column is the strip's and c0 < W
            if (xs <= c0 < xs + SW or xs <= c0 + 1 < xs + SW) and c0 < W:
                off = c0 + X0
                assert 0 <= off and off + 1 < Wb, (W, sxi, lane, off, Wb)
    assert (owner == 1).all()


def test_tile_capacity_bounds_strict_maxima():
    # the densest strict 3x3 maxima pattern: every other column of every other row
    assert CAP == len(range(0, TW, 2)) * len(range(0, TH, 2))
