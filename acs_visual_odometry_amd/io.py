"""Trajectory-loop I/O: gray images, KITTI ground-truth rows, pose CSV.

readGTLine (PoseUpdate.cpp:43-50), writePoseCSV (PoseUpdate.cpp:52-69) and
cv::imread(..., IMREAD_GRAYSCALE) (VisualOdometry.cpp:76).
"""
from __future__ import annotations

import os
import math
import re
import sys
from typing import Optional, Sequence

import numpy as np


def read_gray(path: str) -> Optional[np.ndarray]:
    """cv::imread(path, cv::IMREAD_GRAYSCALE) (VisualOdometry.cpp:65,76) through the library's
    PNG / PGM decoder (vo_imread_gray, csrc/vo_io.cpp); None where imread returns an empty Mat."""
    import ctypes as C
    from ._lib import load
    L = load()
    w, h = C.c_int(), C.c_int()
    bp = os.fsencode(path)
    if L.vo_imread_gray(bp, None, 0, C.byref(w), C.byref(h)) != 0:
        return None
    img = np.empty((h.value, w.value), np.uint8)
    if L.vo_imread_gray(bp, img.ctypes.data_as(C.c_void_p), img.nbytes, C.byref(w), C.byref(h)) != 0:
        return None
    return img


def write_pgm(path: str, img: np.ndarray) -> None:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]))
        f.write(img.tobytes())


# the characters libstdc++'s num_get accumulates for a double (istream >> double): a sign, the
# mantissa, and -- once the mantissa has a digit -- 'e' / 'E' with an optional sign and digits.  The
# accumulated token is then converted whole: one that is not a complete number ("1e", "1e+", ".")
# stores 0 and fails the stream.
_MANT = re.compile(r"[+-]?(?:\d+\.?\d*|\.\d+)")
_EXP = re.compile(r"[eE][+-]?(\d*)")
_EYE34 = (1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0)


def read_gt_line(line: str) -> np.ndarray:
    """readGTLine (PoseUpdate.cpp:43-50): T starts as eye(4) and `ss >> T(i/4, i%4)` fills the
    12 entries in order.  As with std::istream: at end of line the extraction leaves the entry
    (and every later one) untouched; a token that is not a number writes 0 there and stops."""
    T = list(_EYE34)
    pos, n = 0, len(line)
    for i in range(12):
        while pos < n and line[pos] in " \t\n\r\v\f":
            pos += 1
        if pos >= n:
            break
        m = _MANT.match(line, pos)
        if not m:
            T[i] = 0.0
            break
        end = m.end()
        e = _EXP.match(line, end)
        if e:
            if not e.group(1):                # "1e", "1e+": the whole token is not a number
                T[i] = 0.0
                break
            end = e.end()
        v = float(line[pos:end])
        if math.isinf(v):
            # libstdc++ __convert_to_v (LWG 23): an out-of-range value stores +-DBL_MAX and fails the
            # stream, so every later entry keeps its identity value
            T[i] = math.copysign(sys.float_info.max, v)
            break
        T[i] = v
        pos = end
    return np.array(T, dtype=np.float64)


def read_kitti_poses(path: str) -> np.ndarray:
    """One 3x4 row-major pose per getline, blank or short lines included, exactly as
    VisualOdometry.cpp:50-52 pushes readGTLine(line) for every line (so the GT index of frame i
    stays line i)."""
    # std::getline splits on '\n' only (a lone '\r' stays in the line, where >> skips it as space);
    # text after the last '\n' is one more line, an empty remainder is none
    with open(path, "r", newline="") as f:
        text = f.read()
    lines = text.split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    rows = [read_gt_line(line) for line in lines]
    return np.array(rows, dtype=np.float64).reshape(-1, 12)


def _fmt9(v: float) -> str:
    # std::setprecision(9) on a default-formatted ostream == printf("%.9g")
    return "%.9g" % v


def write_pose_csv(path: str, poses: Sequence[np.ndarray]) -> None:
    with open(path, "w") as f:
        for T in poses:
            T = np.asarray(T, dtype=np.float64).reshape(3, 4)
            f.write(",".join(_fmt9(T[r, c]) for r in range(3) for c in range(4)) + "\n")
