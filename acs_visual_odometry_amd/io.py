"""Trajectory-loop I/O: gray images, KITTI ground-truth rows, pose CSV.

readGTLine (PoseUpdate.cpp:43-50), writePoseCSV (PoseUpdate.cpp:52-69) and
cv::imread(..., IMREAD_GRAYSCALE) (VisualOdometry.cpp:76).
"""
from __future__ import annotations

import os
import re
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


# what libstdc++'s num_get accepts for a double (istream >> double)
_NUM = re.compile(r"[+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?")
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
        m = _NUM.match(line, pos)
        if not m:
            T[i] = 0.0
            break
        T[i] = float(m.group(0))
        pos = m.end()
    return np.array(T, dtype=np.float64)


def read_kitti_poses(path: str) -> np.ndarray:
    """One 3x4 row-major pose per getline, blank or short lines included, exactly as
    VisualOdometry.cpp:50-52 pushes readGTLine(line) for every line (so the GT index of frame i
    stays line i)."""
    with open(path, newline=None) as f:
        rows = [read_gt_line(line.rstrip("\n")) for line in f]
    return np.array(rows, dtype=np.float64).reshape(-1, 12)


def _fmt9(v: float) -> str:
    # std::setprecision(9) on a default-formatted ostream == printf("%.9g")
    return "%.9g" % v


def write_pose_csv(path: str, poses: Sequence[np.ndarray]) -> None:
    with open(path, "w") as f:
        for T in poses:
            T = np.asarray(T, dtype=np.float64).reshape(3, 4)
            f.write(",".join(_fmt9(T[r, c]) for r in range(3) for c in range(4)) + "\n")
