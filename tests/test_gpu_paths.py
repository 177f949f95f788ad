"""GPU parity of the trajectory paths beyond the default device-resident run: the model-leak
and skip rules of k_finalize at every window position, the event-wait fallback of the frame
pipeline, host-frame streaming (vo_process_frames_host), the reference CLI / run() on a PNG
sequence, and the survey's full-path configs 1 (640x480) and 4 (1920x1080, N=4096, 32- and
512-test matching).  Every result is compared with the CPU oracle row for row, bit for bit."""
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

import oracle as O
from acs_visual_odometry_amd import Context, VisualOdometry, shard
from acs_visual_odometry_amd.synth import SceneSequence
from conftest import _leak_sequence  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "acs_visual_odometry_amd", "bin", "vo_cli")


def _oracle_rows(seq, frames, max_kpts=2000, match_bits=32, T=8):
    cfg = O.config(seq.W, seq.H, K=seq.K.reshape(9), max_kpts=max_kpts, match_bits=match_bits,
                   ransac_chunk_threads=T)
    vo = O.VO(cfg, gt=seq.gt())
    ref = [vo.process(None if frames[f] is None else frames[f]) for f in range(len(frames))]
    vo.close()
    return ref


def _check(ref, poses, st, info):
    for f, (pr, sr, ir) in enumerate(ref):
        assert st[f] == sr, (f, st[f], sr)
        assert np.array_equal(info[f, :6], ir[:6]), (f, info[f], ir)
        assert np.array_equal(poses[f], pr), f


def _device_run(seq, frames, ref=None, host=None, **ctx_kw):
    ref = ref or _oracle_rows(seq, frames, ctx_kw.get("max_kpts", 2000), ctx_kw.get("match_bits", 32))
    ctx = Context(seq.W, seq.H, K=seq.K, **ctx_kw)
    ctx.set_ground_truth(seq.gt())
    if host is None:
        df = ctx.device_frames(frames)
        out = ctx.process_frames_device(df)
        df.free()
    elif host == "pinned":
        hf = ctx.host_frames(frames)
        out = ctx.process_frames_host(hf)
        hf.free()
    else:
        out = ctx.process_frames_host(frames)
    ctx.close()
    _check(ref, *out)
    return ref


@pytest.mark.parametrize("batch", [8, 16, 64, 112, 128])
def test_finalize_leak_and_few_inliers_paths(leak_case, batch):
    """k_finalize's fallback model (fitted == 0, >= 8 matches): the leaked (R, t) comes from an
    earlier frame of the same window, from the previous pass (window start), or is absent
    (FEW_INLIERS before the first fit, which also holds desc1 back and forces re-passes)."""
    seq, frames, ref = leak_case
    _device_run(seq, frames, ref=ref, frame_batch=batch)


@pytest.mark.parametrize("mode", ["0", "1"])
def test_cross_queue_wait_modes(leak_case, monkeypatch, mode):
    """The pose queue waits for extract batches on events (VO_EVENT_WAIT=1, the default) or in a
    one-wave kernel polling the counter describe publishes (VO_EVENT_WAIT=0, no event on the extract
    queue); results are the same."""
    seq, frames, ref = leak_case
    monkeypatch.setenv("VO_EVENT_WAIT", mode)
    _device_run(seq, frames, ref=ref, frame_batch=16)


@pytest.mark.parametrize("host,batch", [("pinned", 64), ("pinned", 128), ("pinned", 8), ("pageable", 16), ("staged", 16)])
def test_host_streaming_matches_oracle(leak_case, host, batch, monkeypatch):
    """vo_process_frames_host: frames from host memory, H2D of batch k+1 on the copy queue
    while batch k is extracted (ring of 3 device batch slots).  pageable: registered for the
    call; staged (VO_HOST_STAGING=1): copied through the pinned staging ring."""
    seq, frames, ref = leak_case
    if host == "staged":
        monkeypatch.setenv("VO_HOST_STAGING", "1")
    _device_run(seq, frames, ref=ref, host="pinned" if host == "pinned" else "pageable", frame_batch=batch)


def test_host_streaming_across_chunks(monkeypatch):
    """1100 host frames on a 256-slot ring: five host chunks, ring wraps, and the device batch
    ring reused across them, with a skip run over a chunk boundary."""
    monkeypatch.setenv("VO_RING_SLOTS", "256")
    seq = SceneSequence(320, 192, nframes=1100, step=0.05)
    frames = seq.frames()
    for b in range(1015, 1030):
        frames[b] = 128
    _device_run(seq, frames, host="pinned", max_kpts=200, frame_batch=16)


def test_host_streaming_equals_per_frame_calls():
    seq = SceneSequence(nframes=12, step=0.05)
    frames = seq.frames()
    ctx = Context(seq.W, seq.H, K=seq.K, frame_batch=4)
    ctx.set_ground_truth(seq.gt())
    per = [ctx.process_frame(frames[f]) for f in range(6)]
    poses, st, info = ctx.process_frames_host(frames[6:])      # continues the same trajectory
    ctx.reset()
    p2, s2, i2 = ctx.process_frames_host(frames)
    for f in range(6):
        assert s2[f] == per[f][1] and np.array_equal(p2[f], per[f][0])
    assert np.array_equal(p2[6:], poses) and np.array_equal(s2[6:], st)
    ctx.close()


def _write_sequence(d, seq, frames, missing=()):
    os.makedirs(d, exist_ok=True)
    for f in range(len(frames)):
        if f not in missing:
            Image.fromarray(frames[f]).save(os.path.join(d, f"{f:06d}.png"))
    gt = seq.gt()
    with open(os.path.join(d, "poses.txt"), "w") as fh:
        for r in gt:
            fh.write(" ".join("%.17g" % v for v in r) + "\n")


def _csv(rows):
    return "".join(",".join("%.9g" % v for v in np.asarray(r).reshape(12)) + "\n" for r in rows)


@pytest.mark.parametrize("via", ["cli", "python"])
def test_run_png_sequence(tmp_path, via):
    """VisualOdometry::run end to end (main_pipeline.cpp -> VisualOdometry.cpp:38-193): a PNG
    sequence with one missing image, a GT file, the CSV at setprecision(9).  The rows equal the
    oracle's formatted with %.9g."""
    seq = SceneSequence(nframes=14, step=0.05)
    frames = list(seq.frames())
    frames[9] = np.full_like(frames[9], 128)          # a blank frame: < 8 matches (VisualOdometry.cpp:108-115)
    missing = (6,)
    d = str(tmp_path / "seq") + "/"
    _write_sequence(d, seq, frames, missing)
    ref = _oracle_rows(seq, [None if f in missing else frames[f] for f in range(len(frames))], T=4)
    out = str(tmp_path / "out.csv")
    if via == "cli":
        r = subprocess.run([CLI, "4", d, str(len(frames)), d + "poses.txt", out], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        err = r.stderr
        assert "Wrote estimated poses to: " + out in r.stdout
    else:
        import contextlib
        import io
        buf = io.StringIO()
        with contextlib.redirect_stderr(buf):
            VisualOdometry("", 4, seq.W, seq.H, K=seq.K).run(d, len(frames), d + "poses.txt", out)
        err = buf.getvalue()
    assert [r[1] for r in ref][9] == 3
    # the reference's stderr lines, in frame order
    assert err.index("Failed to load image: " + d + "000006.png") < err.index("Too few matches at frame 9")
    assert open(out).read() == _csv([r[0] for r in ref])


def test_run_missing_pose_file(tmp_path):
    r = subprocess.run([CLI, "2", str(tmp_path) + "/", "3", str(tmp_path / "nope.txt"), str(tmp_path / "o.csv")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "Failed to open pose file." in r.stderr
    assert not os.path.exists(tmp_path / "o.csv")


@pytest.mark.parametrize("bits", [32, 512])
def test_config4_full_path_1080p(bits):
    """SURVEY config 4: 1920x1080, N = 4096, the whole path (extract, match, RANSAC, pose,
    trajectory) for 6 frames, with the reference's 32-test matcher and the full 512-test one
    (matching_serial.cpp:24-40)."""
    seq = SceneSequence(1920, 1080, nframes=6, step=0.05)
    frames = seq.frames()
    ref = _device_run(seq, frames, max_kpts=4096, match_bits=bits)
    assert all(r[2][0] == 4096 for r in ref)
    assert all(r[1] == 0 for r in ref[1:])


@pytest.mark.parametrize("bits", [32, 512])
def test_config4_bench_workload(bits):
    """bench.py's own config-4 variant (x1080_32bit / x1080_512bit): 64 frames of sequence 0 at the
    survey's 1.0 m/frame, 1920x1080, N = 4096, the default batch -- every row, status and count
    equal to the oracle's (matching_serial.cpp:42-77 for the 512-test matcher)."""
    seq = SceneSequence(1920, 1080, nframes=64, seq=0, step=1.0)
    frames = seq.frames()
    ref = _device_run(seq, frames, max_kpts=4096, match_bits=bits)
    assert sum(r[1] == 0 for r in ref) >= 32


def test_config1_full_path_640x480():
    """SURVEY config 1 shape: 640x480, N = 2000, 10 frames of the scene generator."""
    seq = SceneSequence(640, 480, nframes=10, step=0.05)
    ref = _device_run(seq, seq.frames())
    assert all(r[1] == 0 for r in ref[1:])


def test_match_512_bit_exact_n4096():
    """The 512-test matcher at N = 4096 (1920x1080 descriptors of two frames)."""
    seq = SceneSequence(1920, 1080, nframes=2, step=0.05)
    frames = seq.frames()
    cfg = O.config(seq.W, seq.H, K=seq.K.reshape(9), max_kpts=4096)
    _, d0, _ = O.extract(frames[0], cfg)
    _, d1, _ = O.extract(frames[1], cfg)
    assert d0.shape[0] == 4096 and d1.shape[0] == 4096
    ctx = Context(seq.W, seq.H, max_kpts=4096, match_bits=512)
    m = ctx.match(d0, d1)
    mr = O.match(d0, d1, match_bits=512)
    assert mr.shape[0] > 100
    assert np.array_equal(m, mr)
    # ragged sizes around the LDS tile edges
    for a, b in [(4096, 1), (1, 4096), (4095, 4093), (1025, 1023), (64, 4096), (2, 2)]:
        assert np.array_equal(ctx.match(d0[:a], d1[:b]), O.match(d0[:a], d1[:b], match_bits=512)), (a, b)
    ctx.close()


def test_config2_batched_extract():
    """SURVEY config 2: extract only, 1241x376, many frames per launch (vo_extract_frames_device,
    frame_batch 64 with a short last batch): keypoints and descriptor bits of every frame equal
    the oracle's; the call leaves the trajectory reset."""
    seq = SceneSequence(nframes=70, step=1.0)
    frames = seq.frames()
    frames[5] = np.random.default_rng(5).integers(0, 256, frames[5].shape, dtype=np.uint8)
    frames[6] = 128
    cfg = O.config(seq.W, seq.H, K=seq.K.reshape(9))
    ctx = Context(seq.W, seq.H, K=seq.K)
    df = ctx.device_frames(frames)
    nk, kps, desc = ctx.extract_frames_device(df, outputs=True)
    for f in range(seq.n):
        kr, dr, _ = O.extract(frames[f], cfg)
        assert nk[f] == kr.shape[0], f
        assert np.array_equal(kps[f], kr) and np.array_equal(desc[f], dr), f
    assert nk[6] == 0
    # the trajectory after it starts from frame 0 again
    ctx.set_ground_truth(seq.gt())
    poses, st, info = ctx.process_frames_device(df)
    assert st[0] == 1 and info[0, 6] == 0
    df.free()
    ctx.close()


@pytest.mark.parametrize("batch,host", [(64, None), (8, None), (16, "pinned")])
def test_sequence_starts(batch, host):
    """Several independent sequences in one frame stream (vo_set_sequence_starts): each
    sequence's rows equal its own oracle run (a fresh VisualOdometry::run), including a sequence
    whose first frames give < 8 inliers (FEW_INLIERS before its first fit: the previous
    sequence's model must not leak into it), a one-frame sequence and a blank frame."""
    parts = []
    a = SceneSequence(nframes=23, step=0.05, seq=1)
    parts.append((a, a.frames()))
    b_seq, b_frames = _leak_sequence()
    parts.append((b_seq, b_frames[:40]))
    c = SceneSequence(nframes=1, step=0.05, seq=2)
    parts.append((c, c.frames()))
    d = SceneSequence(nframes=17, step=0.05, seq=4)
    df_ = d.frames()
    df_[5] = 128
    parts.append((d, df_))
    refs, starts, gts, frames = [], [], [], []
    n = 0
    for sq, fr in parts:
        cfg = O.config(sq.W, sq.H, K=sq.K.reshape(9))
        vo = O.VO(cfg, gt=sq.gt()[:len(fr)])
        refs += [vo.process(fr[f]) for f in range(len(fr))]
        vo.close()
        if n:
            starts.append(n)
        gts.append(sq.gt()[:len(fr)])
        frames.append(fr)
        n += len(fr)
    frames = np.concatenate(frames)
    ctx = Context(a.W, a.H, K=a.K, frame_batch=batch)
    ctx.set_ground_truth(np.concatenate(gts))
    ctx.set_sequence_starts(starts)
    if host:
        hf = ctx.host_frames(frames)
        out = ctx.process_frames_host(hf)
        hf.free()
    else:
        dfr = ctx.device_frames(frames)
        out = ctx.process_frames_device(dfr)
        dfr.free()
    assert [out[1][s] for s in [0] + starts] == [1] * (len(starts) + 1)
    _check(refs, *out)
    ctx.close()


# -- one sequence split over shards (acs_visual_odometry_amd/shard.py) -------------
def _shard_run(seq, frames, G, **ctx_kw):
    ctxs = [Context(seq.W, seq.H, K=seq.K, **ctx_kw) for _ in range(G)]
    try:
        res = shard.run_local([shard.ContextEngine(c, frames, seq.gt()) for c in ctxs], len(frames))
    finally:
        for c in ctxs:
            c.close()
    poses = np.concatenate([r.poses for r in res])
    st = np.concatenate([r.status for r in res])
    info = np.concatenate([r.info for r in res])
    return res, poses, st, info


@pytest.mark.parametrize("G", [2, 3, 7])
def test_sequence_shards_match_unsplit(leak_case, G):
    """Shards of the leak sequence (FEW_INLIERS before the first fit, model leaks next to the
    shard boundaries): halo streams with the sequence's sampler indices, the T_curr chain
    carried over the shards (vo_rechain) -- every row equals the oracle's unsplit run."""
    seq, frames, ref = leak_case
    res, poses, st, info = _shard_run(seq, frames, G, frame_batch=16)
    assert [(r.a, r.b) for r in res] == shard.partition(80, G)
    _check(ref, poses, st, info)


def test_sequence_shard_halo_grows():
    """A blank frame right before the boundary (FEW_MATCHES: desc1 stays on frame 38): a two-frame
    halo holds no frame that reaches the unsplit state, so shard 1's halo grows (4, 8, ...) before
    its own frames continue the stream -- and the rows still equal the oracle's."""
    seq, frames = _leak_sequence()
    frames[39] = 128                      # a blank frame: no keypoints, no matches
    ref = _oracle_rows(seq, frames)
    assert ref[39][1] == 3
    res, poses, st, info = _shard_run(seq, frames, 2)
    assert res[1].start < 38
    _check(ref, poses, st, info)


def _shard_rank(rank, world, port, q, nframes):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seq, frames = _leak_sequence()
    frames = frames[:nframes]
    ctx = Context(seq.W, seq.H, K=seq.K, frame_batch=16)       # every rank on the box's one GPU
    r = shard.run_shard(shard.ContextEngine(ctx, frames, seq.gt()), shard.TorchComm(dist), nframes)
    ctx.close()
    q.put((rank, r.a, r.b, r.poses, r.status, r.info, r.runs))
    dist.destroy_process_group()


def test_sequence_shards_two_processes(leak_case):
    """run_shard in two processes (one context each, gloo carrying the flags and T_curr; RCCL on a
    multi-GPU node): the concatenated rows equal the oracle's unsplit run."""
    import socket
    import torch.multiprocessing as mp
    seq, frames, ref = leak_case
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    procs = [mpc.Process(target=_shard_rank, args=(r, 2, port, q, 80)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(x[1], x[2]) for x in res] == shard.partition(80, 2)
    _check(ref, np.concatenate([x[3] for x in res]), np.concatenate([x[4] for x in res]),
           np.concatenate([x[5] for x in res]))


# -- execution knobs: every measured-and-kept-off alternative still gives the oracle's rows ------
@pytest.mark.parametrize("env", ["VO_PIPELINE=0", "VO_SEL1=0", "VO_RANSAC_Q=0"])
def test_queue_knobs_match_oracle(leak_case, monkeypatch, env):
    """Per-context queue layouts (read by vo_create): every pass on the pose queue without cross-pass
    pipelining (VO_PIPELINE=0), the banded select below its default frame size (VO_SEL1=0), the later
    RANSAC chunks on the fit queue and the trajectory chain on its own queue (VO_RANSAC_Q=0)."""
    seq, frames, ref = leak_case
    k, v = env.split("=")
    monkeypatch.setenv(k, v)
    _device_run(seq, frames, ref=ref, frame_batch=16)


@pytest.mark.parametrize("rq", ["1", "0"])
def test_non_pipelined_passes_follow_the_queues(leak_case, monkeypatch, rq):
    """Round 5's r5final2 failure, isolated: a non-pipelined pass -- the host re-pass rounds after a
    speculation miss (VO_SLACK=0: no slack pass hides them) and a missing frame's pass -- runs its
    trajectory chain on the pose queue, and the commit-point read on the fit / trajectory queue must
    follow it (vo_api.cpp run_chunk: the ev_fin wait).  Under the default layout (the later RANSAC
    chunks on the trajectory queue, the chain on the fit queue) and VO_RANSAC_Q=0 (chunks on the fit
    queue, the chain on its own queue): batched frames 0-29, a missing image at 30 (vo_process_frame
    NULL), batched frames 31-79 -- rows, statuses and counts equal the oracle's run with frame 30
    missing (VisualOdometry.cpp:77-82)."""
    seq, frames, _ = leak_case
    monkeypatch.setenv("VO_SLACK", "0")
    monkeypatch.setenv("VO_RANSAC_Q", rq)
    fr = list(frames)
    fr[30] = None
    ref = _oracle_rows(seq, fr)
    ctx = Context(seq.W, seq.H, K=seq.K, frame_batch=16)
    ctx.set_ground_truth(seq.gt())
    a = ctx.device_frames(np.stack(frames[:30]))
    pa, sa, ia = ctx.process_frames_device(a)
    pm, sm, im = ctx.process_frame(None)
    b = ctx.device_frames(np.stack(frames[31:]))
    pb, sb, ib = ctx.process_frames_device(b)
    a.free(); b.free(); ctx.close()
    poses = np.concatenate([pa, pm[None], pb])
    st = np.concatenate([sa, [sm], sb])
    info = np.concatenate([ia, im[None], ib])
    assert sm == 2                                            # MISSING
    _check(ref, poses, st, info)


_KNOB_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from acs_visual_odometry_amd import Context
d = np.load(sys.argv[2])
ctx = Context(int(d["W"]), int(d["H"]), K=d["K"], frame_batch=int(sys.argv[3]))
ctx.set_ground_truth(d["gt"])
df = ctx.device_frames(d["frames"])
poses, st, info = ctx.process_frames_device(df)
df.free(); ctx.close()
ok = np.array_equal(st, d["st"]) and np.array_equal(poses, d["poses"]) and np.array_equal(info[:, :6], d["info"])
print("KNOB_OK" if ok else "KNOB_DIFF")
"""


@pytest.mark.parametrize("env,batch", [("VO_STSEG=4", 16), ("VO_STSEG=5", 64), ("VO_STSEG=8", 64), ("VO_HYP_CUTS=300:512:1000", 16),
                                       ("VO_TRI_BPF=0", 64), ("VO_RREPS=4", 16), ("VO_XCD=0", 64),
                                       ("VO_EVENT_WAIT=0", 16), ("VO_EVENT_WAIT=0", 8),
                                       ("VO_ST_FLAT=1", 64), ("VO_ST_FLAT=1,VO_STSEG=8", 64), ("VO_ST_FLAT=1", 8),
                                       ("VO_SEL_LDS_KB=48", 64), ("VO_PIPE_FIRST=0", 16), ("VO_RANSAC_SPLIT=0", 16),
                                       ("VO_SEL_SMALL=0", 8), ("VO_STSEG_ADAPT=0", 8), ("VO_TAIL=0", 64),
                                       ("VO_OUT_ZC=0", 16)])
def test_process_knobs_match_oracle(leak_case, tmp_path, env, batch):
    """Knobs the library reads once per process (stencil segment height, RANSAC cut and loop,
    triangulation grid, XCD placement, the branch-free FLAT stencil, the polling wait kernel, the
    80-frame leak sequence as batches of 64 + 16 instead of one batch of 80 (VO_TAIL=0)), each
    in a child process on the leak sequence: rows, statuses and counts equal the oracle's."""
    import sys
    seq, frames, ref = leak_case
    npz = tmp_path / "case.npz"
    np.savez(npz, W=seq.W, H=seq.H, K=seq.K, gt=seq.gt(), frames=frames,
             st=np.array([r[1] for r in ref]), poses=np.stack([r[0] for r in ref]),
             info=np.stack([r[2][:6] for r in ref]))
    kv = dict(e.split("=") for e in env.split(","))
    out = subprocess.run([sys.executable, "-c", _KNOB_SCRIPT, ROOT, str(npz), str(batch)], capture_output=True,
                         text=True, timeout=240, env={**os.environ, **kv})
    assert "KNOB_OK" in out.stdout, (out.stdout[-2000:], out.stderr[-2000:])


_PF_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from acs_visual_odometry_amd import Context
d = np.load(sys.argv[2])
ctx = Context(int(d["W"]), int(d["H"]), K=d["K"])
ctx.set_ground_truth(d["gt"])
import os
hf = ctx.host_frames(d["frames"]) if "VO_PF_PINNED_DIRECT" in os.environ else None
src = hf.array if hf is not None else d["frames"]
rows = [ctx.process_frame(f) for f in src]
if hf is not None:
    hf.free()
ctx.close()
ok = np.array_equal(np.array([r[1] for r in rows]), d["st"]) and \
     np.array_equal(np.stack([r[0] for r in rows]), d["poses"]) and \
     np.array_equal(np.stack([r[2][:6] for r in rows]), d["info"])
print("PF_OK" if ok else "PF_DIFF")
"""


@pytest.mark.parametrize("env", ["VO_PF_ZEROCOPY=0", "VO_DS_LDS_TABLE=1", "VO_DS_PF=0", "VO_RANSAC_FUSED=0",
                                 "VO_SEL_FUSED=0", "VO_SEL_EARLY=0", "VO_PF_OUT_ZC=0", "VO_PF_PINNED_DIRECT=0",
                                 "VO_PF_SEGT=2", "VO_RANSAC_WAVE_HYP=0"])
def test_per_frame_knobs_match_oracle(leak_case, tmp_path, env):
    """Per-frame-call knobs read once per process (the upload kernel instead of the stencil reading
    the frame from the pinned staging buffer, describe's LDS pair table, the one-wave describe instead
    of k_describe_pf, the two RANSAC launches instead of k_ransac_fused, the two-launch select, the fused select emitting
    after its wait with keys from the tiles, the
    output row through a device copy, pinned caller frames staged instead of read in place, stencil
    segments of two tile rows, eight RANSAC hypotheses per wave), in a child process over the leak sequence: one
    vo_process_frame per frame, rows, statuses and counts equal the oracle's."""
    import sys
    seq, frames, ref = leak_case
    npz = tmp_path / "case.npz"
    np.savez(npz, W=seq.W, H=seq.H, K=seq.K, gt=seq.gt(), frames=frames,
             st=np.array([r[1] for r in ref]), poses=np.stack([r[0] for r in ref]),
             info=np.stack([r[2][:6] for r in ref]))
    kv = dict(e.split("=") for e in env.split(","))
    out = subprocess.run([sys.executable, "-c", _PF_SCRIPT, ROOT, str(npz)], capture_output=True,
                         text=True, timeout=240, env={**os.environ, **kv})
    assert "PF_OK" in out.stdout, (out.stdout[-2000:], out.stderr[-2000:])


def test_per_frame_call_from_pinned_frames(leak_case):
    """vo_process_frame on frames that already lie in pinned host memory (vo_host_alloc, one block
    holding the whole sequence, each frame at its offset): the stencil reads each frame in place,
    no staging copy, and every pose row, status and count equals the oracle's."""
    seq, frames, ref = leak_case
    ctx = Context(seq.W, seq.H, K=seq.K)
    ctx.set_ground_truth(seq.gt())
    hf = ctx.host_frames(frames)
    for f in range(len(frames)):
        pose, st, info = ctx.process_frame(hf.array[f])
        assert st == ref[f][1], f
        assert np.array_equal(pose, ref[f][0]), f
        assert np.array_equal(info[:6], ref[f][2][:6]), f
    hf.array[0] = 0                                # the block still belongs to the caller
    hf.free()
    assert ctx.device_errors() == 0
    ctx.close()


def test_per_frame_call_with_row_stride(leak_case):
    """vo_process_frame on frames inside wider rows (a cv::Mat ROI: stride > W): the rows are
    gathered into the pinned staging buffer the stencil reads, and every pose row, status and count
    equals the oracle's (VisualOdometry.cpp:67-190 per frame)."""
    import ctypes as C
    seq, frames, ref = leak_case
    ctx = Context(seq.W, seq.H, K=seq.K)
    ctx.set_ground_truth(seq.gt())
    stride = seq.W + 13
    for f, fr in enumerate(frames):
        buf = np.full((seq.H, stride), 77, np.uint8)
        buf[:, :seq.W] = fr
        pose = np.zeros(12)
        st = C.c_int()
        info = np.zeros(8, np.int32)
        rc = ctx.lib.vo_process_frame(ctx.h, buf.ctypes.data_as(C.c_void_p), stride, pose.ctypes.data_as(C.c_void_p),
                                      C.byref(st), info.ctypes.data_as(C.c_void_p))
        assert rc >= 0 or rc == -10, rc          # VO_ERR_DEGENERATE_E: a row still comes back
        assert st.value == ref[f][1], f
        assert np.array_equal(pose.reshape(3, 4), ref[f][0]), f
        assert np.array_equal(info[:6], ref[f][2][:6]), f
    ctx.close()
