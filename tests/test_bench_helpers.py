"""bench.py's roofline bookkeeping on the committed profiles (CPU): every kernel of the three bench
configs has a profile row with a duration, PMC HBM bytes and a VALU issue fraction in (0, 1], the
512-test matcher is found under k_match512, and the algorithmic bytes follow SURVEY 8(d)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("W,H,bits", [(1241, 376, 32), (1920, 1080, 32), (1920, 1080, 512)])
def test_committed_profiles_have_every_kernel(W, H, bits):
    prof, src = bench.load_profile(W, H, bits)
    assert prof is not None and os.path.exists(os.path.join(ROOT, src))
    for k in ["stencil", "select", "describe", "match", "ransac", "refit", "triangulate", "finalize"]:
        row = bench.profile_row(prof, k)
        assert row is not None, k
        assert row["avg_us"] > 0 and row["hbm_bytes"] > 0, k
        if k in ("stencil", "describe", "match"):
            assert 0.0 < row["valu_issue_frac"] <= 1.0, (k, row)


def test_algorithmic_bytes_follow_the_survey():
    info = np.zeros((4, 8))
    info[:, 0], info[:, 1], info[:, 2] = 2000, 300, 10
    W, H = 1241, 376
    parts = sum(bench.algorithmic_bytes(k, W, H, info) for k in
                ("stencil", "select", "describe", "match", "ransac", "trajectory"))
    assert bench.algorithmic_bytes("path", W, H, info) == W * H + 80 * 2000 + 24 * 300 + 96 == parts
