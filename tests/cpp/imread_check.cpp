// Host driver for the PNG / PGM decoder (acs_visual_odometry_amd/csrc/vo_io.cpp, the library's
// cv::imread(path, IMREAD_GRAYSCALE) replacement, VisualOdometry.cpp:65,76), built with
// -fsanitize=address,undefined by tests/test_sanitizers.py and run over the golden PNGs and
// truncated / corrupted copies of them.  Prints "<rc> <width> <height> <checksum>" per file.
#include <cstdio>
#include <cstdint>
#include <vector>
#include "vo_mi355x.h"

int main(int argc, char** argv)
{
    for (int i = 1; i < argc; ++i) {
        int w = 0, h = 0;
        int rc = vo_imread_gray(argv[i], nullptr, 0, &w, &h);        // dimensions only
        uint64_t ck = 0;
        if (rc == VO_OK) {
            if (w <= 0 || h <= 0 || (long long)w * h > (1LL << 28)) { std::printf("bad-dims %d %d\n", w, h); return 2; }
            std::vector<uint8_t> img((size_t)w * h);
            int w2 = 0, h2 = 0;
            rc = vo_imread_gray(argv[i], img.data(), img.size(), &w2, &h2);
            if (rc == VO_OK && (w2 != w || h2 != h)) { std::printf("dims-changed\n"); return 2; }
            // a buffer one byte short must be refused, not overrun
            if (rc == VO_OK && img.size() > 1 && vo_imread_gray(argv[i], img.data(), img.size() - 1, &w2, &h2) != VO_ERR_CAPACITY) {
                std::printf("short-buffer-accepted\n");
                return 2;
            }
            for (size_t k = 0; k < img.size(); ++k) ck = ck * 1315423911u + img[k];
        }
        std::printf("%d %d %d %llu\n", rc, w, h, (unsigned long long)ck);
    }
    return 0;
}
