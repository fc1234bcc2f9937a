// panofuse_main -- the reference's command line (Main.cpp:864-895) for the fusion path:
//   panofuse_main 0 <rgb_dir> <gt_dir> <baseline_dir> <result_dir> [--tiles DIR]
//                 [--ext auto|jpg|png] [--width W] [--device D] [--shard R/N]
//                 [--metrics-order tree|sequential]
//   panofuse_main export <rgb_dir> <tile_dir> [--device D]
// "export" is the tile render of mode 0 (Main.cpp:399-430, SaveCubeMap :242-326) on the GPU:
// each RGB panorama becomes the 15 LeReS perspective tiles the depth network consumes.
// Mode 0 = CreateDepthPanoramas (Main.cpp:331-687) minus the OpenGL tile export: the perspective
// depth tiles are read from --tiles (default "test_images", the reference's LeReS folder) named
// <raw>.<a0>_<a1>_<z0>_<z1>.<ext>; "auto" takes .jpg when present, else .png (MiDaS naming).
// --metrics-order: the .aligned.txt means in the reference's row-major float order (sequential,
// the default: the digits Main.cpp prints) or in the fp64-tree order (tree: deterministic, within
// ~1e-3 relative of the reference's float sums).
#include "../../include/pf_depth.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>

int main(int argc, char* argv[])
{
    if (argc < 2) {
        std::cout << "usage: " << argv[0]
                  << " 0 <rgb_dir> <gt_dir> <baseline_dir> <result_dir> [--tiles DIR]"
                     " [--ext auto|jpg|png] [--width W] [--device D] [--shard R/N]"
                     " [--metrics-order tree|sequential]\n       "
                  << argv[0] << " export <rgb_dir> <tile_dir> [--device D]" << std::endl;
        return 0;
    }
    const std::string cmd(argv[1]);
    if (cmd == "export") {
        if (argc < 4) {
            std::cout << "usage: " << argv[0] << " export <rgb_dir> <tile_dir> [--device D]"
                      << std::endl;
            return 1;
        }
        const int dev = argc >= 6 && std::string(argv[4]) == "--device" ? std::atoi(argv[5]) : 0;
        if (hipSetDevice(dev) != hipSuccess) {
            std::cout << "no HIP device " << dev << std::endl;
            return 1;
        }
        return pf_export_rgb_tiles(argv[2], argv[3]);
    }
    if (cmd != "0") return 0;  // Main.cpp:889-893: other commands do nothing
    if (argc < 6) {
        std::cout << "[CreateDepthPanormas] error: need argc>=6" << std::endl;
        return 1;
    }
    std::string tiles = "test_images", ext = "auto";
    int width = 2048, device = 0, shard = 0, nshards = 1;
    for (int i = 6; i + 1 < argc; i += 2) {
        const std::string k(argv[i]), v(argv[i + 1]);
        if (k == "--tiles") tiles = v;
        else if (k == "--ext") ext = v;
        else if (k == "--width") width = std::atoi(v.c_str());
        else if (k == "--device") device = std::atoi(v.c_str());
        else if (k == "--metrics-order") {
            if (v != "tree" && v != "sequential") {
                std::cout << "bad --metrics-order " << v << " (want tree or sequential)" << std::endl;
                return 2;
            }
            setenv("PF_METRICS_ORDER", v.c_str(), 1);  // read when the facade's context is made
        }
        else if (k == "--shard") {  // R/N: one process per GPU over the sorted folder
            if (std::sscanf(v.c_str(), "%d/%d", &shard, &nshards) != 2 || nshards < 1 ||
                shard < 0 || shard >= nshards) {
                std::cout << "bad --shard " << v << " (want R/N, 0 <= R < N)" << std::endl;
                return 2;
            }
        }
        else {
            std::cout << "unknown option " << k << std::endl;
            return 2;
        }
    }
    if (hipSetDevice(device) != hipSuccess) {
        std::cout << "no HIP device " << device << std::endl;
        return 1;
    }
    return pf_create_depth_panoramas(argv[2], argv[3], argv[4], argv[5], tiles, ext, width, shard,
                                     nshards);
}
