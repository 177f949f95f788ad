// Test infrastructure (never linked into the product): a C entry point around the REFERENCE's own
// matchCustomBinaryDescriptorsThreadPool (feature_matching_parallel.cpp:49-113) and hammingDistance
// (:39-47), compiled from /root/reference by oracle/ref_matcher.mk with the reference's own thread
// pool (feature_extraction_parallel/threadpool.h:15-62).  Descriptors come in the reference's
// byte-per-test layout (vector<vector<uint8_t>> of 512 bytes, FREAK_feature_descriptor_parallel_GPU.cpp:
// 196-198); the pool has num_threads workers, as VisualOdometry's VO_pool (VisualOdometry.cpp:9-25),
// and the call gets the same numThreads (VisualOdometry.cpp:34-36).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <future>
#include <iterator>
#include <limits>
#include <mutex>
#include <utility>
#include <vector>

#include "threadpool.h"        // /root/reference/feature_extraction_parallel/threadpool.h
#include "matcher_body.inc"    // /root/reference/feature_matching_parallel/feature_matching_parallel.cpp:39-113

extern "C" int ref_match(const uint8_t* d1, int n1, const uint8_t* d2, int n2, int len, int num_threads, float ratio,
                         int32_t* out, int cap)
{
    std::vector<std::vector<uint8_t>> a((size_t)n1), b((size_t)n2);
    for (int i = 0; i < n1; ++i) a[(size_t)i].assign(d1 + (size_t)i * len, d1 + (size_t)(i + 1) * len);
    for (int j = 0; j < n2; ++j) b[(size_t)j].assign(d2 + (size_t)j * len, d2 + (size_t)(j + 1) * len);
    thread_pool pool((unsigned)num_threads);
    const std::vector<std::pair<int, int>> m = matchCustomBinaryDescriptorsThreadPool(a, b, pool, num_threads, ratio);
    const int n = (int)m.size();
    for (int k = 0; k < n && k < cap; ++k) {
        out[2 * k] = m[(size_t)k].first;
        out[2 * k + 1] = m[(size_t)k].second;
    }
    return n;
}
