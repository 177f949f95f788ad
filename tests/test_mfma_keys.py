"""The MFMA matcher's key encoding (k_match_mfma, vo_kernels.hip), restated in numpy on CPU: for
32-bit prefixes of candidates (rows) and queries (columns), the bytes the kernel builds --
A' = -64 a and B' = 64 b with a, b = +-1 per bit, the tile index in K = 32, 33 (A = t & 127,
64 (t >> 7); B = 16, 32) and C = 131072 + row -- give D = A'B' + C = 8192 hamming + j for every
pair, so the minimum key is the (smallest distance, first index) pair the reference's loop keeps
(feature_matching_parallel.cpp:72-99).  The operand lane maps are pinned on the GPU by
tests/test_gpu_parity.py::test_mfma_i8_operand_maps."""
import numpy as np


def spread4(n):
    return (n * 0x00204081) & 0x01010101


def a_bytes(p):
    """candidate prefix p -> 32 bytes (bit k -> 0xC0 = -64, clear -> 0x40 = +64), as s_tab"""
    words = [((spread4((p >> (4 * q)) & 15) << 7) | 0x40404040) & 0xFFFFFFFF for q in range(8)]
    return np.frombuffer(np.array(words, np.uint32).tobytes(), np.int8).astype(np.int64)


def b_bytes(p):
    """query prefix p -> 32 bytes (bit k -> 0x40 = +64, clear -> 0xC0 = -64)"""
    words = [(((spread4((p >> (4 * i)) & 15) ^ 0x01010101) << 7) | 0x40404040) & 0xFFFFFFFF for i in range(8)]
    return np.frombuffer(np.array(words, np.uint32).tobytes(), np.int8).astype(np.int64)


def test_keys_are_distance_then_index():
    rng = np.random.default_rng(3)
    nc, nq = 300, 40
    cand = rng.integers(0, 1 << 32, nc, dtype=np.uint64)
    cand[5] = cand[77] = cand[200]                       # ties: equal prefixes
    qry = rng.integers(0, 1 << 32, nq, dtype=np.uint64)
    qry[3] = cand[5]                                     # distance 0
    A = np.zeros((nc, 64), np.int64)
    B = np.zeros((64, nq), np.int64)
    for j, p in enumerate(cand):
        A[j, :32] = a_bytes(int(p))
        t = j // 16
        A[j, 32], A[j, 33] = t & 127, 64 * (t >> 7)
    for q, p in enumerate(qry):
        B[:32, q] = b_bytes(int(p))
        B[32, q], B[33, q] = 16, 32
    assert A.min() >= -128 and A.max() <= 127 and B.min() >= -128 and B.max() <= 127   # int8 operands
    C = 131072 + (np.arange(nc) % 16)[:, None]
    D = A @ B + C
    ham = np.array([[bin(int(c) ^ int(q)).count("1") for q in qry] for c in cand])
    assert np.array_equal(D, 8192 * ham + np.arange(nc)[:, None])
    # top-2 by key = the sequential loop's best (first index among equal distances) and second best
    for q in range(nq):
        order = np.argsort(D[:, q], kind="stable")
        best, second = order[0], order[1]
        d = ham[:, q]
        ref_best = int(np.argmin(d))                     # first index of the minimum
        assert best == ref_best and d[second] == np.partition(d, 1)[1]
