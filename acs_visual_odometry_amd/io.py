"""Trajectory-loop I/O: gray images, KITTI ground-truth rows, pose CSV.

readGTLine (PoseUpdate.cpp:43-50), writePoseCSV (PoseUpdate.cpp:52-69) and
cv::imread(..., IMREAD_GRAYSCALE) (VisualOdometry.cpp:76).
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np


def read_gray(path: str) -> Optional[np.ndarray]:
    """8-bit gray image (PNG via PIL, binary PGM natively); None if it cannot be read."""
    if not os.path.exists(path):
        return None
    try:
        if path.endswith(".pgm"):
            with open(path, "rb") as f:
                data = f.read()
            parts = data.split(maxsplit=4)
            if parts[0] != b"P5":
                return None
            w, h, mx = int(parts[1]), int(parts[2]), int(parts[3])
            if mx > 255:
                return None
            return np.frombuffer(parts[4][:w * h], np.uint8).reshape(h, w).copy()
        from PIL import Image
        with Image.open(path) as im:
            if im.mode not in ("L", "I;16", "I"):
                # cv::IMREAD_GRAYSCALE uses ITU-R 601 luma like PIL's "L" conversion
                im = im.convert("L")
            a = np.asarray(im)
            if a.dtype != np.uint8:
                a = (a >> 8).astype(np.uint8) if a.max() > 255 else a.astype(np.uint8)
            return np.ascontiguousarray(a)
    except Exception:
        return None


def write_pgm(path: str, img: np.ndarray) -> None:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (img.shape[1], img.shape[0]))
        f.write(img.tobytes())


def read_kitti_poses(path: str) -> np.ndarray:
    """One 3x4 row-major pose per line (readGTLine reads 12 doubles)."""
    rows = []
    with open(path) as f:
        for line in f:
            vals = line.split()
            if not vals:
                continue
            r = [float(v) for v in vals[:12]]
            r += [0.0] * (12 - len(r))
            rows.append(r)
    return np.array(rows, dtype=np.float64).reshape(-1, 12)


def _fmt9(v: float) -> str:
    # std::setprecision(9) on a default-formatted ostream == printf("%.9g")
    return "%.9g" % v


def write_pose_csv(path: str, poses: Sequence[np.ndarray]) -> None:
    with open(path, "w") as f:
        for T in poses:
            T = np.asarray(T, dtype=np.float64).reshape(3, 4)
            f.write(",".join(_fmt9(T[r, c]) for r in range(3) for c in range(4)) + "\n")
