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


def forms_of(prof, bits):
    """The stage -> kernel symbols map of the run a profile was taken from (its kernel list)."""
    base = {k.split("<")[0] for k in prof}
    match = [m for m in (["k_match_mfma", "k_match"] if bits == 32 else ["k_match512_mfma", "k_match512"])
             if m in base][:1]          # (round-3 profiles may hold the matrix-core matchers)
    sel = ["k_select"] if "k_select" in base else ["k_select_count", "k_select_emit"]
    return {"stencil": ["k_stencil"], "select": sel, "describe": ["k_describe"], "match": match,
            "ransac": ["k_ransac_hyp"], "refit": ["k_refit"], "triangulate": ["k_triangulate"],
            "finalize": ["k_finalize"], "trajectory": ["k_traj"]}


@pytest.mark.parametrize("W,H,bits", [(1241, 376, 32), (1920, 1080, 32), (1920, 1080, 512)])
def test_committed_profiles_have_every_kernel(W, H, bits):
    prof, src = bench.load_profile(W, H, bits)
    assert prof is not None and os.path.exists(os.path.join(ROOT, src))
    forms = forms_of(prof, bits)
    for k in ["stencil", "select", "describe", "match", "ransac", "refit", "triangulate", "finalize"]:
        row = bench.profile_row(prof, k, forms)
        assert row is not None, k
        assert row["avg_us"] > 0 and row["hbm_bytes"] > 0, k
        assert {s.split("<")[0] for s in row["symbols"]} == set(forms[k]), (k, row["symbols"])
        if k in ("stencil", "describe", "match"):
            assert 0.0 < row["valu_issue_frac"] <= 1.0, (k, row)


def test_profile_row_refuses_another_form():
    """A profile of the MFMA matcher is not read as the VALU matcher's (round 3 unioned them)."""
    prof = {"k_stencil<8,false>": {"calls": 10, "avg_us": 100.0, "hbm_bytes_per_launch": 1.0},
            "k_match_mfma": {"calls": 12, "avg_us": 80.0, "hbm_bytes_per_launch": 2.0}}
    forms = {"match": ["k_match"], "stencil": ["k_stencil"]}
    assert bench.profile_row(prof, "match", forms) is None
    forms["match"] = ["k_match_mfma"]
    row = bench.profile_row(prof, "match", forms)
    assert row["avg_us"] == 80.0 and row["symbols"] == ["k_match_mfma"]


def test_algorithmic_bytes_follow_the_survey():
    info = np.zeros((4, 8))
    info[:, 0], info[:, 1], info[:, 2] = 2000, 300, 10
    W, H = 1241, 376
    parts = sum(bench.algorithmic_bytes(k, W, H, info) for k in
                ("stencil", "select", "describe", "match", "ransac", "trajectory"))
    assert bench.algorithmic_bytes("path", W, H, info) == W * H + 80 * 2000 + 24 * 300 + 96 == parts


def test_dominant_kernel_is_on_the_critical_queue():
    """The roofline kernel is the largest kernel of the busier queue, not the largest of any queue:
    KITTI at round 4 has the matcher above the stencil but the extract queue ahead of the pose queue."""
    kitti = {"stencil": 1.49, "select": 0.61, "describe": 0.95, "match": 1.63, "ransac": 1.0, "refit": 0.6,
             "triangulate": 0.55, "finalize": 0.38, "trajectory": 0.5}
    assert bench.dominant_kernel(kitti) == "stencil"
    low_inlier = dict(kitti, ransac=4.2)
    assert bench.dominant_kernel(low_inlier) == "ransac"
    # "ransac" also times a pass's later chunks on the trajectory queue: the pose queue counts only
    # its first chunk ("ransac_pose") when the breakdown has it (round 6's evidence breakdown)
    r6 = {"stencil": 1.478, "select": 0.498, "describe": 0.937, "match": 1.593, "ransac": 1.370,
          "refit": 0.588, "triangulate": 0.524, "finalize": 0.349, "trajectory": 0.457}
    assert bench.dominant_kernel(r6) == "match"
    assert bench.dominant_kernel(dict(r6, ransac_pose=0.35)) == "stencil"
