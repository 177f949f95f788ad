// vo_cli -- the reference CLI (main_pipeline.cpp:7-43) on the MI355X path:
//   vo_cli <num_threads> <image_dir> <num_images> <pose_file> <output_csv>
// VisualOdometry::run reads image_dir + "%06d.png" (the directory string is prefixed as given,
// VisualOdometry.cpp:65,74), the KITTI pose file, and writes the pose CSV.  The reference's
// check for the OpenCL binary (main_pipeline.cpp:32-37) has no counterpart: the HIP code
// objects are embedded in libvo_mi355x.so.
#include <cstdlib>
#include <exception>
#include <iostream>
#include <string>

#include "../../include/VisualOdometry.hpp"

int main(int argc, char** argv)
{
    if (argc != 6) {
        std::cerr << "Usage: " << argv[0] << " <num_threads> <image_dir> <num_images> <pose_file> <output_csv>"
                  << std::endl;
        return EXIT_FAILURE;
    }
    std::size_t num_threads = 0, num_images = 0;
    try {
        num_threads = static_cast<std::size_t>(std::stoul(argv[1]));
    } catch (const std::exception&) {
        std::cerr << "Invalid num_threads: " << argv[1] << std::endl;
        return EXIT_FAILURE;
    }
    const std::string image_dir = argv[2];
    try {
        num_images = static_cast<std::size_t>(std::stoul(argv[3]));
    } catch (const std::exception&) {
        std::cerr << "Invalid num_images: " << argv[3] << std::endl;
        return EXIT_FAILURE;
    }
    vo_mi355x::VisualOdometry vo("", num_threads);
    vo.run(image_dir, num_images, argv[4], argv[5]);
    return EXIT_SUCCESS;
}
