// vo_cli -- the reference CLI (main_pipeline.cpp:7-43, VisualOdometry::run at
// VisualOdometry.cpp:38-193) on the MI355X path:
//   vo_cli <num_threads> <image_dir> <num_images> <pose_file> <output_csv>
// Images: <image_dir>/%06d.pgm (binary P5) or .png is not decoded here (use the Python
// facade acs_visual_odometry_amd.VisualOdometry.run for PNG sequences).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/VisualOdometry.hpp"

static bool read_pgm(const std::string& path, std::vector<uint8_t>& buf, int& w, int& h)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::string magic;
    int mx = 0;
    f >> magic >> w >> h >> mx;
    if (magic != "P5" || mx > 255 || w <= 0 || h <= 0) return false;
    f.get();
    buf.resize((size_t)w * h);
    f.read((char*)buf.data(), (std::streamsize)buf.size());
    return (bool)f;
}

int main(int argc, char** argv)
{
    if (argc != 6) {
        std::cerr << "Usage: " << argv[0] << " <num_threads> <image_dir> <num_images> <pose_file> <output_csv>"
                  << std::endl;
        return EXIT_FAILURE;
    }
    std::size_t num_threads = 0, num_images = 0;
    try { num_threads = std::stoul(argv[1]); } catch (...) { std::cerr << "Invalid num_threads: " << argv[1] << std::endl; return EXIT_FAILURE; }
    try { num_images = std::stoul(argv[3]); } catch (...) { std::cerr << "Invalid num_images: " << argv[3] << std::endl; return EXIT_FAILURE; }
    std::string dir = argv[2];
    if (!dir.empty() && dir.back() != '/') dir += '/';
    std::ifstream gtf(argv[4]);
    if (!gtf.is_open()) { std::cerr << "Failed to open pose file.\n"; return EXIT_FAILURE; }
    std::vector<double> gt;
    for (std::string line; std::getline(gtf, line);) {          // readGTLine, PoseUpdate.cpp:43-50
        std::stringstream ss(line);
        double v[12] = {0};
        for (int i = 0; i < 12; ++i) ss >> v[i];
        gt.insert(gt.end(), v, v + 12);
    }
    std::vector<uint8_t> img;
    int w = 0, h = 0;
    char name[32];
    snprintf(name, sizeof(name), "%06d.pgm", 0);
    if (!read_pgm(dir + name, img, w, h)) { std::cerr << "Failed to load image: " << dir + name << "\n"; return EXIT_FAILURE; }
    vo_mi355x::VisualOdometry vo("", num_threads, w, h);
    vo.set_ground_truth(gt);
    std::ofstream out(argv[5]);
    if (!out.is_open()) { std::cerr << "Failed to open output CSV file.\n"; return EXIT_FAILURE; }
    for (std::size_t i = 0; i < num_images; ++i) {
        snprintf(name, sizeof(name), "%06lu.pgm", (unsigned long)i);
        int wi = 0, hi = 0;
        bool ok = read_pgm(dir + name, img, wi, hi) && wi == w && hi == h;
        if (!ok && i > 0) std::cerr << "Failed to load image: " << dir + name << "\n";
        vo_mi355x::GrayImage g{img.data(), w, h, (size_t)w};
        double row[12];
        vo.process_frame(ok ? &g : nullptr, row);
        for (int k = 0; k < 12; ++k) out << std::setprecision(9) << row[k] << (k == 11 ? "\n" : ",");   // writePoseCSV
    }
    std::cout << "Wrote estimated poses to: " << argv[5] << "\n";
    return EXIT_SUCCESS;
}
