// facade_test.cpp -- the reference's per-frame stage calls through the C++ facade
// (include/VisualOdometry.hpp), in the order VisualOdometry::run makes them
// (VisualOdometry.cpp:88-172): compute_descriptor_with_key_points on two frames, match_descriptors,
// Ransac::run into a FundamentalMatrix, getInliers / getMatrix, PoseUpdate::getPose; plus a
// standalone FundamentalMatrix::fit on the inliers.  Writes every result as text (doubles at
// %.17g, exact) for tests/test_facade.py, which compares them with the CPU oracle.
//
// usage: vo_facade_test <num_threads> <frame1.pgm|png> <frame2.pgm|png> <out.txt>
#include <cstdio>
#include <vector>

#include "VisualOdometry.hpp"

using namespace vo_mi355x;

static std::vector<uint8_t> load(const char* path, int* w, int* h)
{
    check(vo_imread_gray(path, nullptr, 0, w, h), "vo_imread_gray");
    std::vector<uint8_t> px((size_t)*w * *h);
    check(vo_imread_gray(path, px.data(), px.size(), w, h), "vo_imread_gray");
    return px;
}

int main(int argc, char** argv)
{
    if (argc != 5) {
        std::fprintf(stderr, "usage: %s <num_threads> <frame1> <frame2> <out.txt>\n", argv[0]);
        return 2;
    }
    const int T = std::atoi(argv[1]);
    int w1, h1, w2, h2;
    std::vector<uint8_t> a = load(argv[2], &w1, &h1), b = load(argv[3], &w2, &h2);
    VisualOdometry vo("", (std::size_t)T, w1, h1);
    FILE* f = std::fopen(argv[4], "w");
    if (!f) return 3;
    auto [desc1, kpts1] = vo.compute_descriptor_with_key_points(GrayImage{a.data(), w1, h1, (size_t)w1});
    auto [desc2, kpts2] = vo.compute_descriptor_with_key_points(GrayImage{b.data(), w2, h2, (size_t)w2});
    for (auto* kd : {&kpts1, &kpts2}) {
        std::fprintf(f, "kps %zu", kd->size());
        for (const KeyPoint& k : *kd) std::fprintf(f, " %d %d", (int)k.x, (int)k.y);
        std::fprintf(f, "\n");
    }
    for (auto* dd : {&desc1, &desc2}) {
        std::fprintf(f, "desc %zu", dd->size());
        for (const auto& d : *dd) {
            std::fputc(' ', f);
            for (uint8_t bit : d) std::fputc('0' + bit, f);
        }
        std::fprintf(f, "\n");
    }
    const std::vector<std::pair<int, int>> m = vo.match_descriptors(desc1, desc2);
    std::fprintf(f, "matches %zu", m.size());
    for (auto& p : m) std::fprintf(f, " %d %d", p.first, p.second);
    std::fprintf(f, "\n");
    // VisualOdometry.cpp:117-130
    std::vector<std::pair<Point, Point>> matchedPoints;
    for (const auto& [i1, i2] : m)
        matchedPoints.emplace_back(Point{(double)kpts1[i1].x, (double)kpts1[i1].y},
                                   Point{(double)kpts2[i2].x, (double)kpts2[i2].y});
    FundamentalMatrix model;
    Ransac ransac;
    const int64_t calls0 = vo.pool().calls;
    const uint64_t seed = DevicePool::frame_seed(vo.pool().seed, calls0);
    ransac.run(model, matchedPoints, 0.99, 1.0, T, vo.pool());
    {
        // a pool never bound to a context (built the way the reference builds its thread_pool) runs
        // on the default context: the same draw gives the same model
        DevicePool unbound(nullptr, vo.pool().seed);
        unbound.calls = calls0;
        FundamentalMatrix m2;
        Ransac r2;
        r2.run(m2, matchedPoints, 0.99, 1.0, T, unbound);
        const Matrix3d a = model.getMatrix(), b = m2.getMatrix();
        std::fprintf(f, "unbound_pool_same %d\n",
                     (int)(std::equal(a.a, a.a + 9, b.a) && m2.getInliers().size() == model.getInliers().size()));
    }
    std::fprintf(f, "ransac_seed %llu iterations %d\n", (unsigned long long)seed, ransac.last_iterations);
    const Matrix3d F = model.getMatrix();
    const auto& inliers = model.getInliers();
    std::fprintf(f, "F");
    for (double v : F.a) std::fprintf(f, " %.17g", v);
    std::fprintf(f, "\ninliers %zu", inliers.size());
    for (const auto& p : inliers) std::fprintf(f, " %.17g %.17g %.17g %.17g", p.first.x, p.first.y, p.second.x, p.second.y);
    std::fprintf(f, "\n");
    if (inliers.size() >= 8) {
        FundamentalMatrix refit;                   // FundamentalMatrix::fit on its own
        refit.fit(inliers);
        std::fprintf(f, "fit");
        for (double v : refit.getMatrix().a) std::fprintf(f, " %.17g", v);
        std::fprintf(f, "\n");
        std::vector<Point2f> p1, p2;              // VisualOdometry.cpp:155-159
        for (const auto& p : inliers) {
            p1.push_back(Point2f{(float)p.first.x, (float)p.first.y});
            p2.push_back(Point2f{(float)p.second.x, (float)p.second.y});
        }
        PoseUpdate estimator(vo.pool());
        auto [R, t] = estimator.getPose(F, p1, p2, 1.0);
        std::fprintf(f, "pose");
        for (double v : R.a) std::fprintf(f, " %.17g", v);
        for (double v : t.a) std::fprintf(f, " %.17g", v);
        std::fprintf(f, "\n");
    }
    // the model leak: a second Ransac::run on fewer than 8 points keeps F and the inliers
    std::vector<std::pair<Point, Point>> few(matchedPoints.begin(), matchedPoints.begin() + std::min<size_t>(5, matchedPoints.size()));
    ransac.run(model, few, 0.99, 1.0, T, vo.pool());
    const Matrix3d F2 = model.getMatrix();
    std::fprintf(f, "leak %d %zu\n", (int)std::equal(F.a, F.a + 9, F2.a), model.getInliers().size());
    std::fclose(f);
    return 0;
}
