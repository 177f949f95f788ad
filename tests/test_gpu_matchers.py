"""Every matcher form the library can run, against the oracle (feature_matching_parallel.cpp:39-113
for the reference's 32-test matcher, matching_serial.cpp:24-40,58 for the full 512-test one):
k_match<MT_QPL> (batched windows), k_match<1> (the single-frame call, one query per lane) and
k_match512 (LDS candidate tiles), each through
  - the stage API (vo_match) at N = 2000 / 4096 with ragged sizes around the tile edges,
  - the batched path (vo_process_frames_device): the leak sequence (32 tests) and 1920x1080 /
    N = 4096 (512 tests),
  - the single-frame call (vo_process_frame) over the leak sequence.
Matches, rows, statuses and counts must equal the oracle's bit for bit.  (The matrix-core forms of
round 3 are gone: DESIGN.md section 3, tests/test_no_mfma.py.)"""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from acs_visual_odometry_amd.synth import SceneSequence

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from acs_visual_odometry_amd import Context
d = np.load(sys.argv[2])
out = []
def same_rows(p, st, info, tag):
    ok = np.array_equal(st, d[tag + "_st"]) and np.array_equal(p, d[tag + "_poses"]) and \
         np.array_equal(info[:, :6], d[tag + "_info"])
    out.append((tag, ok))
# stage matcher, 32 and 512 tests, ragged sizes
for bits, pre in ((32, "k"), (512, "x")):
    ctx = Context(int(d[pre + "W"]), int(d[pre + "H"]), max_kpts=int(d[pre + "N"]), match_bits=bits)
    d0, d1 = d[pre + "d0"], d[pre + "d1"]
    for i, (a, b) in enumerate(d[pre + "sizes"]):
        out.append((f"match{bits}_{a}x{b}", np.array_equal(ctx.match(d0[:a], d1[:b]), d[f"{pre}m{i}"])))
    ctx.close()
# batched path: the leak sequence (32 tests) and 1080p (512 tests)
for tag, bits, N in (("leak", 32, 2000), ("x1080", 512, 4096)):
    ctx = Context(int(d[tag + "_W"]), int(d[tag + "_H"]), K=d[tag + "_K"], max_kpts=N, match_bits=bits)
    ctx.set_ground_truth(d[tag + "_gt"])
    df = ctx.device_frames(d[tag + "_frames"])
    same_rows(*ctx.process_frames_device(df), tag)
    df.free(); ctx.close()
# single-frame calls (32 tests) over the leak sequence
ctx = Context(int(d["leak_W"]), int(d["leak_H"]), K=d["leak_K"])
ctx.set_ground_truth(d["leak_gt"])
rows = [ctx.process_frame(f) for f in d["leak_frames"]]
ctx.close()
same_rows(np.stack([r[0] for r in rows]), np.array([r[1] for r in rows]), np.stack([r[2] for r in rows]), "leak")
out[-1] = ("single_frame_leak", out[-1][1])
for tag, ok in out:
    print(("MATCH_OK " if ok else "MATCH_DIFF ") + tag)
"""


@pytest.fixture(scope="module")
def cases(tmp_path_factory, leak_case):
    """Inputs and the oracle's answers."""
    arrs = {}
    # stage matcher inputs: KITTI N = 2000 (32 tests), 1920x1080 N = 4096 (512 tests)
    for pre, (W, H, N, bits) in (("k", (1241, 376, 2000, 32)), ("x", (1920, 1080, 4096, 512))):
        seq = SceneSequence(W, H, nframes=2, step=0.05)
        fr = seq.frames()
        cfg = O.config(W, H, K=seq.K.reshape(9), max_kpts=N)
        _, d0, _ = O.extract(fr[0], cfg)
        _, d1, _ = O.extract(fr[1], cfg)
        sizes = [(d0.shape[0], d1.shape[0]), (d0.shape[0], 1), (1, d1.shape[0]), (d0.shape[0] - 1, d1.shape[0] - 3),
                 (1025, 1023), (64, d1.shape[0]), (2, 2)]
        arrs.update({pre + "W": W, pre + "H": H, pre + "N": N, pre + "d0": d0, pre + "d1": d1,
                     pre + "sizes": np.array(sizes)})
        for i, (a, b) in enumerate(sizes):
            arrs[f"{pre}m{i}"] = O.match(d0[:a], d1[:b], match_bits=bits)
    seq, frames, ref = leak_case
    x = SceneSequence(1920, 1080, nframes=6, step=0.05)
    xf = x.frames()
    cfg = O.config(1920, 1080, K=x.K.reshape(9), max_kpts=4096, match_bits=512, ransac_chunk_threads=8)
    vo = O.VO(cfg, gt=x.gt())
    xref = [vo.process(f) for f in xf]
    vo.close()
    for tag, s, fr, rf in (("leak", seq, frames, ref), ("x1080", x, xf, xref)):
        arrs.update({tag + "_W": s.W, tag + "_H": s.H, tag + "_K": s.K, tag + "_gt": s.gt(), tag + "_frames": fr,
                     tag + "_st": np.array([r[1] for r in rf]), tag + "_poses": np.stack([r[0] for r in rf]),
                     tag + "_info": np.stack([r[2][:6] for r in rf])})
    path = tmp_path_factory.mktemp("matchers") / "cases.npz"
    np.savez(path, **arrs)
    return path


def test_matcher_forms_match_oracle(cases):
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, str(cases)], capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("MATCH_")]
    assert r.returncode == 0 and lines, (r.stdout[-2000:], r.stderr[-2000:])
    bad = [ln for ln in lines if ln.startswith("MATCH_DIFF")]
    assert not bad, bad
    assert len(lines) == 2 * 7 + 3


def test_k_match_equals_reference_library():
    """k_match (stage API, 32 tests) against the REFERENCE's own matchCustomBinaryDescriptorsThreadPool
    (feature_matching_parallel.cpp:39-113) compiled from /root/reference into oracle/_ref/libref_matcher.so
    (oracle/ref_matcher.mk): the same pairs, on the factory images and the bench's KITTI-shape frames.
    The library travels with the tree; skipped where it was never built."""
    from acs_visual_odometry_amd import Context
    from test_ref_matcher import LIB, ref_match
    import ctypes as C
    if not os.path.exists(LIB):
        pytest.skip("oracle/_ref/libref_matcher.so not built")
    L = C.CDLL(LIB)
    L.ref_match.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_float, C.c_void_p, C.c_int]
    L.ref_match.restype = C.c_int
    s = SceneSequence(nframes=3, step=1.0)
    cfg = O.config(s.W, s.H, K=s.K.reshape(9))
    desc = [O.extract(f, cfg)[1] for f in s.frames()]
    ctx = Context(s.W, s.H, K=s.K)
    for a, b in zip(desc[:-1], desc[1:]):
        for T in (1, 8):
            assert np.array_equal(ctx.match(a, b), ref_match(L, a, b, T))
    ctx.close()
