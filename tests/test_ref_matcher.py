"""The 32-test matcher pinned against the REFERENCE's own code, compiled here (CPU suite).

oracle/ref_matcher.mk cuts hammingDistance + matchCustomBinaryDescriptorsThreadPool
(feature_matching_parallel.cpp:39-113) out of /root/reference at build time and compiles them with the
reference's own std-only thread pool (feature_extraction_parallel/threadpool.h, ts_queue.h,
join_threads.h) into oracle/_ref/libref_matcher.so -- no stand-in header, nothing copied into the repo.
The reference matcher takes the byte-per-test descriptors (vector<vector<uint8_t>>, 512 bytes) and a
pool of T workers with T chunks of ceil(n1 / T) queries concatenated in task order
(feature_matching_parallel.cpp:59-110), as VisualOdometry::match_descriptors calls it
(VisualOdometry.cpp:34-36).

The oracle's voo_match (oracle/vo_oracle.c) equals it pair for pair on the factory images, on the bench's
KITTI-shape frames at both motion regimes, at T = 1, 3 and 8, and on crafted tie / edge cases; the GPU
tests check k_match against voo_match bit for bit (tests/test_gpu_matchers.py) and, where the .so
travelled, against this library directly.  So a9 and the matcher's chunked concatenation (a13) are pinned.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from acs_visual_odometry_amd.io import read_gray
from acs_visual_odometry_amd.synth import SceneSequence

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libref_matcher.so")
GOLD = os.path.join(ROOT, "tests", "golden")


def ref_lib():
    if os.path.isdir("/root/reference"):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-f", "ref_matcher.mk"])
    if not os.path.exists(LIB):
        pytest.skip("the reference matcher is built only where /root/reference is mounted")
    L = C.CDLL(LIB)
    L.ref_match.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_float, C.c_void_p, C.c_int]
    L.ref_match.restype = C.c_int
    return L


def unpack(words):
    """8 x u64 -> the reference's 512 bytes in {0, 1} (bit t of word t / 64, LSB first)."""
    w = np.ascontiguousarray(words, dtype=np.uint64).reshape(-1, 8)
    return np.unpackbits(w.view(np.uint8).reshape(-1, 64), axis=1, bitorder="little").astype(np.uint8)


def ref_match(L, d1, d2, T, ratio=0.75):
    b1 = np.ascontiguousarray(unpack(d1))
    b2 = np.ascontiguousarray(unpack(d2))
    out = np.zeros((max(len(b1), 1), 2), np.int32)
    m = L.ref_match(b1.ctypes.data, len(b1), b2.ctypes.data, len(b2), 512, T, ratio, out.ctypes.data, len(out))
    return out[:m].copy()


@pytest.fixture(scope="module")
def L():
    return ref_lib()


@pytest.fixture(scope="module")
def factory_desc():
    d = []
    for i in (1, 2):
        img = read_gray(os.path.join(GOLD, f"factory{i}.png"))
        _, desc, _ = O.extract(img, O.config(img.shape[1], img.shape[0]))
        d.append(desc)
    return d


@pytest.mark.parametrize("T", [1, 3, 8])
def test_factory_pairs_equal_reference(L, factory_desc, T):
    d1, d2 = factory_desc
    r = ref_match(L, d1, d2, T)
    assert len(r) > 500
    assert np.array_equal(O.match(d1, d2), r)
    r21 = ref_match(L, d2, d1, T)
    assert np.array_equal(O.match(d2, d1), r21)


@pytest.mark.parametrize("motion,seq", [(1.0, 0), (1.0, 5), (0.12, 0)])
def test_bench_frames_equal_reference(L, motion, seq):
    """Consecutive frames of the bench's sequences (bench.py: SceneSequence(seq=s, step=motion))."""
    s = SceneSequence(nframes=4, seq=seq, step=motion)
    cfg = O.config(s.W, s.H, K=s.K.reshape(9))
    desc = [O.extract(f, cfg)[1] for f in s.frames()]
    for a, b in zip(desc[:-1], desc[1:]):
        for T in (1, 3, 8):
            assert np.array_equal(O.match(a, b), ref_match(L, a, b, T)), T


def test_crafted_edges_equal_reference(L):
    """Ties (equal best distances: the first index wins), equal best and second (ratio rejects),
    distance 0, one or no candidate, more threads than queries; prefixes only differ in tests 0..31,
    and the other 480 tests are random (the matcher must ignore them, quirk 1)."""
    rng = np.random.default_rng(3)

    def desc(prefixes):
        d = rng.integers(0, 2 ** 63, size=(len(prefixes), 8), dtype=np.uint64)
        d[:, 0] = (d[:, 0] & np.uint64(0xFFFFFFFF00000000)) | np.asarray(prefixes, np.uint64)
        return d

    q = desc([0x0, 0xFFFFFFFF, 0x0000FFFF, 0x1, 0x3, 0xF0F0F0F0, 0x7, 0x0])
    cases = [
        desc([0x0, 0x0, 0x1]),                 # two exact ties at distance 0
        desc([0x1, 0x2, 0x4, 0x8]),            # all at distance 1 from query 0
        desc([0xFFFFFFFF]),                    # one candidate: never a match
        desc([0x0000FFFF, 0x0000FFFE, 0x3, 0xF0F0F0F1, 0x0F0F0F0F]),
        desc(rng.integers(0, 2 ** 32, size=64, dtype=np.uint64)),
    ]
    for c in cases:
        for T in (1, 3, 8, 64):
            assert np.array_equal(O.match(q, c), ref_match(L, q, c, T)), (c[:, 0], T)
    empty = np.zeros((0, 8), np.uint64)
    assert len(ref_match(L, q, empty, 3)) == 0 and len(O.match(q, empty)) == 0
