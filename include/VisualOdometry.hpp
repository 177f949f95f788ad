// VisualOdometry.hpp -- C++ facade with the reference's class interface over the C ABI.
//
// Drop-in for the reference class VisualOdometry (VisualOdometry.h:15-31): same method
// names, same argument meaning, std::runtime_error where the reference throws.  OpenCV
// types are replaced by plain containers at this boundary (GrayImage ~ cv::Mat CV_8UC1,
// KeyPoint ~ cv::KeyPoint's integer pixel position), so the facade builds without OpenCV;
// INTEGRATION.md shows the cv::Mat adapters a reference build would add.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "vo_mi355x.h"

namespace vo_mi355x {

struct GrayImage {                 // row-major 8-bit gray, stride in bytes
    const uint8_t* data = nullptr;
    int width = 0, height = 0;
    size_t stride = 0;
    bool empty() const { return data == nullptr || width <= 0 || height <= 0; }
};

struct KeyPoint { float x, y; };   // cv::KeyPoint::pt (x = column, y = row)

inline void check(int rc, const char* what)
{
    if (rc == VO_ERR_DEGENERATE_E) throw std::runtime_error("Degenerate essential matrix");
    if (rc == VO_ERR_NO_DEVICE) throw std::runtime_error("No HIP devices found for the program.");
    if (rc < 0) throw std::runtime_error(std::string(what) + ": " + vo_strerror(rc));
}

// -- the reference's stage types, OpenCV / Eigen replaced by plain ones -------------------------
struct Point { double x, y; };                     // ransac.hpp:14-16
struct Point2f { float x, y; };                    // cv::Point2f (PoseUpdate::getPose's points)
struct Matrix3d {                                  // Eigen::Matrix3d / cv::Mat 3x3 CV_64F, row-major
    double a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    double& operator()(int r, int c) { return a[3 * r + c]; }
    double operator()(int r, int c) const { return a[3 * r + c]; }
};
struct Vec3d {                                     // cv::Mat 3x1 CV_64F (getPose's t)
    double a[3] = {0, 0, 0};
    double& operator()(int r) { return a[r]; }
    double operator()(int r) const { return a[r]; }
};

// The execution resource of the stage calls: the reference's thread_pool VO_pool
// (VisualOdometry.h:17), which Ransac::run takes, becomes the GPU context.  It also draws the
// RANSAC sampler seed of each Ransac::run call, which replaces std::random_device
// (ransac.cpp:137): call k uses frame_seed(seed, k), the seed frame k of a trajectory uses.
class DevicePool {
public:
    explicit DevicePool(vo_ctx* ctx = nullptr, uint64_t seed = 0xACE0ULL) : seed(seed), ctx_(ctx) {}
    vo_ctx* handle() const { return ctx_; }
    void bind(vo_ctx* ctx) { ctx_ = ctx; }
    uint64_t next_seed() { return frame_seed(seed, calls++); }
    static uint64_t frame_seed(uint64_t s, int64_t k)       // splitmix64 finaliser (oracle voo_frame_seed)
    {
        uint64_t z = s + 0x632BE59BD9B4E019ULL * (uint64_t)(k + 1);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    uint64_t seed;
    int64_t calls = 0;

private:
    vo_ctx* ctx_;
};
using thread_pool = DevicePool;

namespace detail {
// a process-wide context for stage objects built without one (FundamentalMatrix::fit and a
// default-constructed PoseUpdate, as the reference constructs them); created on first use
inline vo_ctx* default_ctx()
{
    static std::mutex mu;
    static vo_ctx* ctx = nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!ctx) {
        vo_config c;
        vo_config_default(&c, 1241, 376);
        c.max_kpts = 4096;
        check(vo_create(&c, &ctx), "vo_create");
    }
    return ctx;
}
inline std::vector<double> xyxy(const std::vector<std::pair<Point, Point>>& d)
{
    std::vector<double> v(d.size() * 4);
    for (size_t i = 0; i < d.size(); ++i) {
        v[4 * i] = d[i].first.x; v[4 * i + 1] = d[i].first.y;
        v[4 * i + 2] = d[i].second.x; v[4 * i + 3] = d[i].second.y;
    }
    return v;
}
}  // namespace detail

// FundamentalMatrix (ransac.hpp:18-34): the model Ransac::run refits; it keeps its F and inliers
// when a fit is refused (< 8 points, ransac.cpp:95-99), which is the reference's model leak across
// frames (quirk 9).
class FundamentalMatrix {
public:
    // ransac.cpp:95-99: computeFundamentalMatrix on all points (normalized least squares, rank 2)
    void fit(const std::vector<std::pair<Point, Point>>& sample)
    {
        if (sample.size() < 8) return;
        const std::vector<double> p = detail::xyxy(sample);
        vo_ctx* ctx = ctx_ ? ctx_ : detail::default_ctx();
        check(vo_fit_F(ctx, p.data(), (int)sample.size(), F_.a), "vo_fit_F");
        inliers_ = sample;
    }
    Matrix3d getMatrix() const { return F_; }
    const std::vector<std::pair<Point, Point>>& getInliers() const { return inliers_; }
    // ransac.cpp:105-114 (unused by the reference's loop): |x2^T F x1| < threshold
    int countInliers(const std::vector<std::pair<Point, Point>>& data, double threshold) const
    {
        int n = 0;
        for (const auto& pr : data) {
            const double x = pr.first.x, y = pr.first.y, xp = pr.second.x, yp = pr.second.y;
            const double e = xp * (F_(0, 0) * x + F_(0, 1) * y + F_(0, 2)) + yp * (F_(1, 0) * x + F_(1, 1) * y + F_(1, 2)) +
                             (F_(2, 0) * x + F_(2, 1) * y + F_(2, 2));
            n += std::abs(e) < threshold;
        }
        return n;
    }
    void bind(vo_ctx* ctx) { ctx_ = ctx; }

private:
    friend class Ransac;
    Matrix3d F_;
    std::vector<std::pair<Point, Point>> inliers_;
    vo_ctx* ctx_ = nullptr;
};

// Ransac::run (ransac.hpp:40-48, ransac.cpp:120-194) on the pool's GPU: every hypothesis, the
// chunk drop of numThreads chunks (quirk 7), the adaptive stop (quirk 8), then model.fit on the best
// hypothesis' inliers (in data order; the reference's order is its mutex's) -- kept from the
// previous call when fewer than 8 (quirk 9).
class Ransac {
public:
    void run(FundamentalMatrix& model, const std::vector<std::pair<Point, Point>>& data, double probability,
             double sampsonThreshold, int numThreads, thread_pool& pool)
    {
        const uint64_t seed = pool.next_seed();
        if (data.size() < 8) return;              // std::sample of < 8 points: fit() refuses every sample
        const std::vector<double> p = detail::xyxy(data);
        std::vector<int32_t> inl(data.size());
        Matrix3d F;
        int fitted = 0, n_inl = 0, n_eval = 0;
        // an unbound pool falls back to the default context, as FundamentalMatrix::fit and getPose do
        vo_ctx* ctx = pool.handle() ? pool.handle() : detail::default_ctx();
        check(vo_ransac_run(ctx, p.data(), (int)data.size(), probability, sampsonThreshold, numThreads, seed,
                            F.a, &fitted, inl.data(), &n_inl, &n_eval),
              "vo_ransac_run");
        last_iterations = n_eval;
        if (!fitted) return;
        model.F_ = F;
        model.inliers_.clear();
        for (int k = 0; k < n_inl; ++k) model.inliers_.push_back(data[(size_t)inl[k]]);
    }
    int last_iterations = 0;                      // hypotheses evaluated by the last run
};

// PoseUpdate::getPose (PoseUpdate.hpp:61-179) on the GPU: E = K^T F K, SVD, the four (R, t)
// candidates by triangulation and cheirality, first maximum, t scaled to GT_pos_norm.  Throws
// std::runtime_error("Degenerate essential matrix") where the reference throws (:71-73), and prints
// its stderr warning when fewer than 100 points have positive depth (:149-152).
class PoseUpdate {
public:
    PoseUpdate() = default;
    explicit PoseUpdate(thread_pool& pool) : ctx_(pool.handle()) {}
    std::pair<Matrix3d, Vec3d> getPose(const Matrix3d& F, const std::vector<Point2f>& points1,
                                       const std::vector<Point2f>& points2, double GT_pos_norm)
    {
        if (points1.size() != points2.size()) throw std::invalid_argument("getPose: point counts differ");
        vo_ctx* ctx = ctx_ ? ctx_ : detail::default_ctx();
        std::vector<float> a(2 * points1.size()), b(2 * points2.size());
        for (size_t i = 0; i < points1.size(); ++i) {
            a[2 * i] = points1[i].x; a[2 * i + 1] = points1[i].y;
            b[2 * i] = points2[i].x; b[2 * i + 1] = points2[i].y;
        }
        std::pair<Matrix3d, Vec3d> out;
        int32_t counts[4] = {0, 0, 0, 0};
        check(vo_pose(ctx, F.a, a.data(), b.data(), (int)points1.size(), GT_pos_norm, out.first.a, out.second.a, counts),
              "vo_pose");
        if (*std::max_element(counts, counts + 4) < 100) std::cerr << "Max positive depth too small\n";
        return out;
    }

private:
    vo_ctx* ctx_ = nullptr;
};

class VisualOdometry {
public:
    // VisualOdometry(kernel_filename, num_threads) (VisualOdometry.h:23).  The HIP code
    // objects are embedded in libvo_mi355x.so, so kernel_filename is not read; num_threads
    // keeps its one effect on results: the RANSAC chunk count (ransac.cpp:152-157).
    VisualOdometry(const std::string& kernel_filename, std::size_t num_threads, int width = 1241,
                   int height = 376, int device = 0)
        : kernel_filename_(kernel_filename), number_of_threads_(num_threads)
    {
        vo_config_default(&cfg_, width, height);
        cfg_.ransac_chunk_threads = (int)std::max<std::size_t>(num_threads, 1);
        cfg_.device = device;
        check(vo_create(&cfg_, &ctx_), "vo_create");
        max_kpts_ = cfg_.max_kpts;
        VO_pool.bind(ctx_);
    }
    ~VisualOdometry() { vo_destroy(ctx_); }
    VisualOdometry(const VisualOdometry&) = delete;
    VisualOdometry& operator=(const VisualOdometry&) = delete;

    // compute_descriptor_with_key_points (VisualOdometry.h:25-26): descriptors as 512
    // bytes in {0,1} per keypoint (the reference layout), keypoints in raster order.
    std::pair<std::vector<std::vector<uint8_t>>, std::vector<KeyPoint>>
    compute_descriptor_with_key_points(const GrayImage& image)
    {
        std::vector<vo_kp> kps(max_kpts_);
        std::vector<uint64_t> words((size_t)max_kpts_ * 8);
        int n = 0;
        check(vo_extract(ctx_, image.data, image.stride, kps.data(), words.data(), &n, nullptr), "vo_extract");
        std::vector<std::vector<uint8_t>> desc(n, std::vector<uint8_t>(512));
        std::vector<KeyPoint> out(n);
        for (int i = 0; i < n; ++i) {
            vo_unpack_descriptor(words.data() + 8 * (size_t)i, desc[i].data());
            out[i] = KeyPoint{(float)kps[i].x, (float)kps[i].y};
        }
        return {desc, out};
    }

    // match_descriptors (VisualOdometry.h:27-29)
    std::vector<std::pair<int, int>> match_descriptors(const std::vector<std::vector<uint8_t>>& desc1,
                                                       const std::vector<std::vector<uint8_t>>& desc2)
    {
        std::vector<std::pair<int, int>> res;
        if (desc1.empty() || desc2.empty()) return res;
        std::vector<uint64_t> a = pack(desc1), b = pack(desc2);
        std::vector<vo_match_t> m(desc1.size());
        int nm = 0;
        check(vo_match(ctx_, a.data(), (int)desc1.size(), b.data(), (int)desc2.size(), m.data(), &nm), "vo_match");
        for (int i = 0; i < nm; ++i) res.emplace_back(m[i].prev, m[i].cur);
        return res;
    }

    // one iteration of run()'s loop; the pose row the reference appends to estimated_poses
    int process_frame(const GrayImage* image, double pose_row[12])
    {
        int status = 0;
        int rc = vo_process_frame(ctx_, image && !image->empty() ? image->data : nullptr,
                                  image ? image->stride : 0, pose_row, &status, nullptr);
        check(rc, "vo_process_frame");
        return status;
    }

    void set_ground_truth(const std::vector<double>& rows12)
    {
        check(vo_set_ground_truth(ctx_, rows12.data(), (int)(rows12.size() / 12)), "vo_set_ground_truth");
    }

    // run (VisualOdometry.h:30, VisualOdometry.cpp:38-193): image_dir + "%06d.png" for frames
    // 0 .. num_images-1 (frame 0 is always read, as the reference reads it before its loop), GT
    // poses from pose_file (one readGTLine per line), the pose rows to output_csv.
    // Present frames are decoded on number_of_threads host threads and streamed to the GPU in
    // batches (vo_process_frames_host: H2D of batch k+1 overlaps the work of batch k); a missing
    // image is one vo_process_frame(NULL) (T_curr pushed, VisualOdometry.cpp:77-82).  The context
    // takes frame 0's size; a later frame of another size throws.
    void run(const std::string image_dir, std::size_t num_images, const std::string pose_file,
             const std::string output_csv)
    {
        std::ifstream infile(pose_file);
        if (!infile.is_open()) {
            std::cerr << "Failed to open pose file.\n";
            return;
        }
        std::vector<double> gt;
        for (std::string line; std::getline(infile, line);) {
            const std::vector<double> T = readGTLine(line);
            gt.insert(gt.end(), T.begin(), T.end());
        }
        infile.close();

        const std::size_t total = std::max<std::size_t>(num_images, 1);
        auto path_of = [&](std::size_t i) {
            std::stringstream ss;
            ss << std::setw(6) << std::setfill('0') << i;
            return image_dir + ss.str() + ".png";
        };
        {   // the context takes frame 0's size
            int w = 0, h = 0;
            if (vo_imread_gray(path_of(0).c_str(), nullptr, 0, &w, &h) == VO_OK &&
                (w != cfg_.width || h != cfg_.height)) {
                vo_config c = cfg_;
                c.width = w;
                c.height = h;
                vo_ctx* nc = nullptr;
                check(vo_create(&c, &nc), "vo_create");
                vo_destroy(ctx_);
                ctx_ = nc;
                cfg_ = c;
                VO_pool.bind(ctx_);
            }
        }
        check(vo_reset(ctx_), "vo_reset");
        set_ground_truth(gt);

        const std::size_t np = (std::size_t)cfg_.width * cfg_.height;
        const std::size_t batch = kRunBatch;
        void* pinned = nullptr;
        check(vo_host_alloc(ctx_, batch * np, &pinned), "vo_host_alloc");
        uint8_t* buf = static_cast<uint8_t*>(pinned);
        std::vector<double> rows;
        rows.reserve(total * 12);
        std::vector<int> ok(batch);
        std::vector<int> status(batch);
        const unsigned nthreads = (unsigned)std::max<std::size_t>(1, std::min<std::size_t>(number_of_threads_, 64));
        try {
            for (std::size_t i0 = 0; i0 < total;) {
                const std::size_t nb = std::min(batch, total - i0);
                // decode frames i0 .. i0+nb-1 (thread t takes every nthreads-th frame)
                std::vector<std::thread> pool;
                for (unsigned t = 0; t < nthreads && t < nb; ++t)
                    pool.emplace_back([&, t] {
                        for (std::size_t z = t; z < nb; z += nthreads) {
                            int w = 0, h = 0;
                            const int rc = vo_imread_gray(path_of(i0 + z).c_str(), buf + z * np, np, &w, &h);
                            const bool same = w == cfg_.width && h == cfg_.height;
                            ok[z] = (rc == VO_OK && same) ? 1 : ((rc == VO_OK || rc == VO_ERR_CAPACITY) ? -1 : 0);
                        }
                    });
                for (std::thread& th : pool) th.join();
                for (std::size_t z = 0; z < nb;) {
                    if (ok[z] < 0) throw std::runtime_error("image size differs from frame 0: " + path_of(i0 + z));
                    if (ok[z] == 0) {   // cv::imread returned an empty Mat
                        if (i0 + z > 0) std::cerr << "Failed to load image: " << path_of(i0 + z) << "\n";
                        double row[12];
                        process_frame(nullptr, row);
                        rows.insert(rows.end(), row, row + 12);
                        ++z;
                        continue;
                    }
                    std::size_t e = z;
                    while (e < nb && ok[e] == 1) ++e;
                    std::vector<double> poses((e - z) * 12);
                    check(vo_process_frames_host(ctx_, buf + z * np, np, (int)(e - z), poses.data(), status.data(),
                                                 nullptr),
                          "vo_process_frames_host");
                    for (std::size_t k = 0; k < e - z; ++k) {
                        if (status[k] == VO_STATUS_FEW_MATCHES)          // VisualOdometry.cpp:108-109
                            std::cerr << "Too few matches at frame " << (i0 + z + k) << "\n";
                        if (status[k] == VO_STATUS_DEGENERATE) throw std::runtime_error("Degenerate essential matrix");
                    }
                    rows.insert(rows.end(), poses.begin(), poses.end());
                    z = e;
                }
                i0 += nb;
            }
        } catch (...) {
            vo_host_free(ctx_, pinned);
            throw;
        }
        vo_host_free(ctx_, pinned);
        writePoseCSV(output_csv, rows);
        std::cout << "Wrote estimated poses to: " << output_csv << "\n";
    }

    // readGTLine (PoseUpdate.cpp:43-50): eye(4), then 12 extractions in row-major order
    static std::vector<double> readGTLine(const std::string& line)
    {
        std::stringstream ss(line);
        std::vector<double> T = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        for (int i = 0; i < 12; ++i) ss >> T[i];
        return T;
    }

    // writePoseCSV (PoseUpdate.cpp:52-69): 12 values per row at setprecision(9)
    static void writePoseCSV(const std::string& filename, const std::vector<double>& rows12)
    {
        std::ofstream file(filename);
        if (!file.is_open()) {
            std::cerr << "Failed to open output CSV file.\n";
            return;
        }
        for (std::size_t r = 0; r + 12 <= rows12.size(); r += 12) {
            for (int k = 0; k < 12; ++k) {
                file << std::setprecision(9) << rows12[r + k];
                if (k != 11) file << ",";
            }
            file << "\n";
        }
    }

    vo_ctx* handle() { return ctx_; }
    // the stage objects' execution resource (the reference's VO_pool, VisualOdometry.h:17)
    thread_pool& pool() { return VO_pool; }
    std::size_t threads() const { return number_of_threads_; }

private:
    static std::vector<uint64_t> pack(const std::vector<std::vector<uint8_t>>& d)
    {
        std::vector<uint64_t> w(d.size() * 8, 0);
        for (size_t i = 0; i < d.size(); ++i)
            for (size_t t = 0; t < d[i].size() && t < 512; ++t)
                if (d[i][t]) w[i * 8 + (t >> 6)] |= 1ull << (t & 63);
        return w;
    }
    static constexpr std::size_t kRunBatch = 256;   // frames decoded and streamed per host batch
    std::string kernel_filename_;
    std::size_t number_of_threads_;
    vo_config cfg_;
    vo_ctx* ctx_ = nullptr;
    int max_kpts_ = 2000;
    thread_pool VO_pool;
};

}  // namespace vo_mi355x
