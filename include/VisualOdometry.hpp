// VisualOdometry.hpp -- C++ facade with the reference's class interface over the C ABI.
//
// Drop-in for the reference class VisualOdometry (VisualOdometry.h:15-31): same method
// names, same argument meaning, std::runtime_error where the reference throws.  OpenCV
// types are replaced by plain containers at this boundary (GrayImage ~ cv::Mat CV_8UC1,
// KeyPoint ~ cv::KeyPoint's integer pixel position), so the facade builds without OpenCV;
// INTEGRATION.md shows the cv::Mat adapters a reference build would add.
#pragma once

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
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

class VisualOdometry {
public:
    // VisualOdometry(kernel_filename, num_threads) (VisualOdometry.h:23).  The HIP code
    // objects are embedded in libvo_mi355x.so, so kernel_filename is not read; num_threads
    // keeps its one effect on results: the RANSAC chunk count (ransac.cpp:152-157).
    VisualOdometry(const std::string& kernel_filename, std::size_t num_threads, int width = 1241,
                   int height = 376, int device = 0)
        : kernel_filename_(kernel_filename), number_of_threads_(num_threads)
    {
        vo_config cfg;
        vo_config_default(&cfg, width, height);
        cfg.ransac_chunk_threads = (int)num_threads;
        cfg.device = device;
        check(vo_create(&cfg, &ctx_), "vo_create");
        max_kpts_ = cfg.max_kpts;
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

    vo_ctx* handle() { return ctx_; }

private:
    static std::vector<uint64_t> pack(const std::vector<std::vector<uint8_t>>& d)
    {
        std::vector<uint64_t> w(d.size() * 8, 0);
        for (size_t i = 0; i < d.size(); ++i)
            for (size_t t = 0; t < d[i].size() && t < 512; ++t)
                if (d[i][t]) w[i * 8 + (t >> 6)] |= 1ull << (t & 63);
        return w;
    }
    std::string kernel_filename_;
    std::size_t number_of_threads_;
    vo_ctx* ctx_ = nullptr;
    int max_kpts_ = 2000;
};

}  // namespace vo_mi355x
