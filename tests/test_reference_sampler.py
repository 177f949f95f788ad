"""VO_RNG_MT19937: the reference's own RANSAC sampler (ransac.cpp:126-142).

The reference draws every hypothesis with std::sample over its match vector from one
std::mt19937 per Ransac::run, seeded by std::random_device (so no two runs agree).  Seeded with a
fixed 32-bit value instead, the draws are a pure function of (seed, M); the library's host sampler
(vo_reference_samples, what VO_RNG_MT19937 uploads for each frame) and the oracle's
(voo_mt_samples) must give the k-th draw of that stream for every hypothesis k.  This test compiles
the reference's statements with g++ -- its Point type (ransac.hpp:14-16), `int sampleSize = 8`
(ransac.cpp:128), `std::mt19937 rng(...)` (:137, the seed injected where random_device stood) and the
std::sample call with back_inserter over a vector<pair<Point, Point>> (:140-142) -- and compares the
element each draw picks (an index carried in Point.x) with both samplers, over 2000 consecutive draws.
libstdc++ is the reference's library (g++ 11 here; the reference names no compiler version)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROGRAM = r"""
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <iterator>
#include <random>
#include <utility>
#include <vector>
struct Point {                                      // ransac.hpp:14-16
    double x, y;
};
int main(int argc, char** argv)
{
    const unsigned seed = (unsigned)std::strtoul(argv[1], nullptr, 10);
    const int M = std::atoi(argv[2]), iters = std::atoi(argv[3]);
    std::vector<std::pair<Point, Point>> data;
    for (int i = 0; i < M; ++i) data.push_back({Point{(double)i, 0.0}, Point{0.0, 0.0}});
    int sampleSize = 8;                              // ransac.cpp:128
    std::mt19937 rng(seed);                          // ransac.cpp:137 (std::random_device{}() injected)
    for (int iter = 0; iter < iters; ++iter) {       // ransac.cpp:139-142
        std::vector<std::pair<Point, Point>> sample;
        std::sample(data.begin(), data.end(), std::back_inserter(sample), sampleSize, rng);
        for (const auto& p : sample) std::printf("%d ", (int)p.first.x);
        std::printf("\n");
    }
    return 0;
}
"""


@pytest.fixture(scope="module")
def ref_prog(tmp_path_factory):
    d = tmp_path_factory.mktemp("sampler")
    src, exe = d / "ref_sample.cpp", d / "ref_sample"
    src.write_text(PROGRAM)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), str(src)], check=True)
    return str(exe)


def ref_draws(exe, seed, m, n):
    out = subprocess.run([exe, str(seed), str(m), str(n)], capture_output=True, text=True, check=True).stdout
    return np.array([[int(v) for v in ln.split()] for ln in out.strip().splitlines()], np.int32)


def lib_draws(seed, m, n):
    from acs_visual_odometry_amd import load
    out = np.zeros((n, 8), np.int32)
    assert load().vo_reference_samples(seed, m, n, out.ctypes.data_as(C.c_void_p)) == 0
    return out


@pytest.mark.parametrize("seed,m", [(5489, 455), (0, 8), (1, 9), (0xDEADBEEF, 2000), (123456789, 1311)])
def test_samplers_equal_the_reference_statements(ref_prog, seed, m):
    ref = ref_draws(ref_prog, seed, m, 2000)
    assert ref.shape == (2000, 8)
    assert (np.diff(ref, axis=1) > 0).all()          # selection sampling keeps data order
    assert np.array_equal(O.mt_samples(seed, m, 2000), ref)
    assert np.array_equal(lib_draws(seed, m, 2000), ref)


def test_oracle_ransac_in_reference_sampler_mode():
    """The oracle's RANSAC with the reference's sampler: hypothesis k fits the k-th draw (its
    count is the count of F fitted to exactly those 8 matches), and mode 0 and mode 1 draw
    differently."""
    rng = np.random.default_rng(4)
    X = np.column_stack([rng.uniform(-20, 20, 300), rng.uniform(-3, 3, 300), rng.uniform(8, 60, 300)])
    K = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1.0]])
    R = np.array([[0.9998, 0, 0.0175], [0, 1, 0], [-0.0175, 0, 0.9998]])
    t = np.array([0.1, 0.0, -1.0])
    x1 = (K @ X.T).T
    x2 = (K @ (R @ X.T + t[:, None])).T
    pts = np.column_stack([x1[:, :2] / x1[:, 2:], x2[:, :2] / x2[:, 2:]])
    pts[::3, 2:] += rng.uniform(-40, 40, (100, 2))    # a third outliers
    r1 = O.ransac(pts, seed=0x1234ABCD, rng_mode=1)
    r0 = O.ransac(pts, seed=0x1234ABCD, rng_mode=0)
    assert r1["fitted"] and r0["fitted"]
    draws = O.mt_samples(0x1234ABCD, len(pts), 2000)
    for k in (0, 1, r1["best_k"]):
        F = O.fit_F8(pts, draws[k])
        assert sum(O.sampson(F, p) < 1.0 for p in pts[: (len(pts) // 8) * 8]) == r1["counts"][k]
    assert not np.array_equal(r1["counts"][:50], r0["counts"][:50])
