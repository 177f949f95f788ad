/* Test infrastructure (the CPU oracle, never linked into the product): the reference's RANSAC sampler
 * for the oracle's VO_RNG_MT19937 mode -- std::mt19937 rng(seed32) once per Ransac::run
 * (ransac.cpp:137), then std::sample(data.begin(), data.end(), std::back_inserter(sample), sampleSize, rng)
 * per hypothesis (ransac.cpp:142) -- over an index vector (random-access iterators and an int
 * sample size, as the reference's vector<pair<Point, Point>> and `int sampleSize = 8`, so libstdc++
 * takes the same path).  The rest of the oracle is plain C. */
#include <algorithm>
#include <cstdint>
#include <iterator>
#include <numeric>
#include <random>
#include <vector>

extern "C" void voo_mt_samples(uint32_t seed32, int m, int nhyp, int32_t* out)
{
    std::mt19937 rng(seed32);
    std::vector<int32_t> idx((size_t)m);
    std::iota(idx.begin(), idx.end(), 0);
    const int sampleSize = 8;
    std::vector<int32_t> smp;
    for (int k = 0; k < nhyp; ++k) {
        smp.clear();
        std::sample(idx.begin(), idx.end(), std::back_inserter(smp), sampleSize, rng);
        for (int i = 0; i < 8; ++i) out[8 * (size_t)k + i] = i < (int)smp.size() ? smp[(size_t)i] : 0;
    }
}
