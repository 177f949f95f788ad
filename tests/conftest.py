import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.lib()
    return oracle


def _have_gpu():
    try:
        return os.path.exists("/dev/kfd")
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _have_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def _oracle_rows(seq, frames, max_kpts=2000, match_bits=32, T=8):
    """The oracle's (pose, status, info) rows of a frame sequence (None = a missing image)."""
    import oracle as O
    cfg = O.config(seq.W, seq.H, K=seq.K.reshape(9), max_kpts=max_kpts, match_bits=match_bits,
                   ransac_chunk_threads=T)
    vo = O.VO(cfg, gt=seq.gt())
    ref = [vo.process(None if frames[f] is None else frames[f]) for f in range(len(frames))]
    vo.close()
    return ref


def _leak_sequence():
    """80 scene frames (0.05 m/frame) with frames of a far-moving sequence spliced in:
    frames 1-3 give < 8 inliers before any fit (FEW_INLIERS, VisualOdometry.cpp:147-153: the
    model has no inliers yet), the later splices give >= 8 matches but < 8 inliers after a fit,
    so the previous model leaks (quirk 9) -- at window starts, middles and ends for windows of
    8, 16 and 64 frames."""
    from acs_visual_odometry_amd.synth import SceneSequence
    seq = SceneSequence(nframes=80, step=0.05)
    frames = seq.frames()
    far = SceneSequence(nframes=80, step=1.0, seq=3)
    for j in (1, 2, 3, 8, 9, 16, 23, 24, 25, 40, 47, 63, 64):
        frames[j] = far.frame(j)
    return seq, frames


@pytest.fixture(scope="session")
def leak_case():
    seq, frames = _leak_sequence()
    ref = _oracle_rows(seq, frames)
    import numpy as np
    st = np.array([r[1] for r in ref])
    fitted = np.array([r[2][5] for r in ref])
    # the case exercises what it claims
    assert list(st[1:4]) == [4, 4, 4]
    leaks = [f for f in range(4, 80) if st[f] == 0 and fitted[f] == 0]
    assert {8, 9, 16, 23, 25, 40, 48, 64} <= set(leaks), leaks
    return seq, frames, ref


