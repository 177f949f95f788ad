#!/usr/bin/env python3
"""Regenerates tests/golden/*.npz from the CPU oracle (oracle/), whose extract stages are
pinned against the reference's own OpenCL kernels (tests/test_ref_kernels.py) and whose
other stages are restated from the reference sources (DESIGN.md "Oracle").

Fixtures (inputs are the reference's own images/factory{1,2}.png, copied to tests/golden/,
and the seeded synthetic sequence acs_visual_odometry_amd/synth.py; its frames' sha256 is
stored so a generator change is caught rather than silently re-baselined):
  factory_pair.npz  extract(factory1), extract(factory2), match, RANSAC (T=8, seed=1), getPose
  scene_traj.npz    8-frame KITTI-shape trajectory: poses, statuses, per-frame info
usage: python tools/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle as O  # noqa: E402
from acs_visual_odometry_amd.io import read_gray  # noqa: E402
from acs_visual_odometry_amd.synth import SceneSequence  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def factory_pair():
    imgs = [read_gray(os.path.join(GOLD, f"factory{i}.png")) for i in (1, 2)]
    H, W = imgs[0].shape
    cfg = O.config(W, H)
    k1, d1, _ = O.extract(imgs[0], cfg)
    k2, d2, _ = O.extract(imgs[1], cfg)
    m = O.match(d1, d2)
    pts = np.concatenate([k1[m[:, 0]], k2[m[:, 1]]], axis=1).astype(np.float64)
    r = O.ransac(pts, 0.99, 1.0, T=8, seed=1)
    inl = pts[r["inliers"]]
    rc, R, t, cnt = O.pose(r["F"], np.array(cfg.K[:]), inl[:, :2], inl[:, 2:], 1.0)
    return dict(k1=k1, d1=d1, k2=k2, d2=d2, matches=m, ransac_counts=r["counts"], ransac_best_k=r["best_k"],
                ransac_n_eval=r["n_evaluated"], ransac_inliers=r["inliers"], F=r["F"], fitted=r["fitted"],
                pose_rc=rc, R=R, t=t, pose_counts=cnt)


def scene_traj(nframes=8):
    seq = SceneSequence(nframes=nframes, step=0.05)
    frames = seq.frames()
    cfg = O.config(seq.W, seq.H, K=seq.K.reshape(9))
    vo = O.VO(cfg, gt=seq.gt())
    poses, st, info = [], [], []
    for f in range(nframes):
        p, s, i = vo.process(frames[f])
        poses.append(p)
        st.append(s)
        info.append(i)
    vo.close()
    return dict(frames_sha256=np.frombuffer(hashlib.sha256(frames.tobytes()).digest(), np.uint8),
                poses=np.array(poses), status=np.array(st, np.int32), info=np.array(info))


def main():
    np.savez_compressed(os.path.join(GOLD, "factory_pair.npz"), **factory_pair())
    np.savez_compressed(os.path.join(GOLD, "scene_traj.npz"), **scene_traj())
    for f in ("factory_pair.npz", "scene_traj.npz"):
        print(f, os.path.getsize(os.path.join(GOLD, f)), "bytes")


if __name__ == "__main__":
    main()
