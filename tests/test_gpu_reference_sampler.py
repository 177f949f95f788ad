"""VO_RNG_MT19937 on the GPU: with the reference's own sampler (std::mt19937 + std::sample drawn on the
host, tests/test_reference_sampler.py), every path matches the oracle in the same mode bit for bit --
per-hypothesis counts, best hypothesis, inliers and F of the stage call (Ransac::run, ransac.cpp:120-194),
and every trajectory row of the batched, host-streamed and per-frame paths (VisualOdometry.cpp:67-190).
The sample tables are drawn per pose pass once k_match has written each frame's match count."""
import numpy as np
import pytest

import oracle as O
from acs_visual_odometry_amd import Context
from acs_visual_odometry_amd.synth import SceneSequence

pytestmark = pytest.mark.gpu
MT = 1


def _two_view(outlier_frac=0.45, seed=4):
    """Two-view matches of a synthetic scene with a known fraction of outliers: the image-pair
    matches at 0.12 m/frame stay under 10 % inliers for this scorer, so maxIt falls to the 100
    floor (ransac.cpp:179-190) and the stage call never leaves the first chunk."""
    rng = np.random.default_rng(seed)
    X = np.column_stack([rng.uniform(-20, 20, 400), rng.uniform(-3, 3, 400), rng.uniform(8, 60, 400)])
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1.0]])
    R = np.array([[0.9998, 0, 0.0175], [0, 1, 0], [-0.0175, 0, 0.9998]])
    t = np.array([0.1, 0.0, -1.0])
    x1 = (K @ X.T).T
    x2 = (K @ (R @ X.T + t[:, None])).T
    pts = np.column_stack([x1[:, :2] / x1[:, 2:], x2[:, :2] / x2[:, 2:]])
    out = rng.random(400) < outlier_frac
    pts[out, 2:] += rng.uniform(-40, 40, (int(out.sum()), 2))
    return pts


@pytest.mark.parametrize("T,seed", [(8, 0x1234ABCD), (3, 7), (1, 0xFEDCBA9876543210)])
def test_stage_ransac_reference_sampler(T, seed):
    pts = _two_view()
    ctx = Context(1241, 376, ransac_chunk_threads=T, rng_mode=MT)
    g = ctx.ransac(pts, seed)
    r = O.ransac(pts, T=T, seed=seed, rng_mode=MT)
    assert r["n_evaluated"] > 100                       # past the first chunk (611 / 739 / 859)
    assert (g["n_evaluated"], g["best_k"], g["n_inl"], g["fitted"]) == \
           (r["n_evaluated"], r["best_k"], r["n_inl"], r["fitted"])
    assert np.array_equal(g["counts"], r["counts"])
    assert np.array_equal(g["inliers"], r["inliers"])
    assert np.array_equal(g["F"], r["F"])
    r0 = O.ransac(pts, T=T, seed=seed, rng_mode=0)
    assert not np.array_equal(r0["counts"][:100], r["counts"][:100])   # the modes draw differently
    ctx.close()


def _oracle_rows(seq, frames):
    cfg = O.config(seq.W, seq.H, K=seq.K.reshape(9), rng_mode=MT)
    vo = O.VO(cfg, gt=seq.gt())
    rows = [vo.process(f) for f in frames]
    vo.close()
    return rows


def _check(rows, poses, st, info):
    for f, (pr, sr, ir) in enumerate(rows):
        assert st[f] == sr, (f, st[f], sr)
        assert np.array_equal(info[f][:6], ir[:6]), (f, info[f], ir)
        assert np.array_equal(poses[f], pr), f


@pytest.mark.parametrize("motion,batch", [(0.12, 8), (1.0, 16)])
def test_trajectory_reference_sampler(motion, batch):
    seq = SceneSequence(nframes=24, step=motion)
    frames = seq.frames()
    rows = _oracle_rows(seq, frames)
    ctx = Context(seq.W, seq.H, K=seq.K, rng_mode=MT, frame_batch=batch)
    ctx.set_ground_truth(seq.gt())
    df = ctx.device_frames(frames)
    _check(rows, *ctx.process_frames_device(df))
    df.free()
    ctx.reset()
    _check(rows, *ctx.process_frames_host(frames))
    ctx.reset()
    out = [ctx.process_frame(f) for f in frames]
    _check(rows, np.stack([o[0] for o in out]), [o[1] for o in out], [o[2] for o in out])
    assert ctx.device_errors() == 0
    ctx.close()


def test_leak_sequence_reference_sampler(leak_case):
    """The leak sequence (skips, FEW_INLIERS before the first fit, the model leaking from earlier
    frames, repair windows with two records per frame) in the reference-sampler mode."""
    seq, frames, _ = leak_case
    rows = _oracle_rows(seq, frames)
    ctx = Context(seq.W, seq.H, K=seq.K, rng_mode=MT, frame_batch=16)
    ctx.set_ground_truth(seq.gt())
    df = ctx.device_frames(frames)
    _check(rows, *ctx.process_frames_device(df))
    df.free()
    ctx.close()
