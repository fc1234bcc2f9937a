// Mutation fuzzer for the map loaders (csrc/pf_image.cpp, csrc/pf_jpeg.cpp), built host-only
// with AddressSanitizer + UBSan by tests/test_io.py::test_image_decoders_fuzz_sanitized:
//   fuzz_images <iterations> <scratch file> <seed files...>
// Each iteration flips 1-8 random bytes of a seed file (and truncates it one time in four),
// then runs load_image and load_pfm on it; any out-of-bounds access aborts under the sanitizers.
#include "pf_image.hpp"

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

int main(int argc, char** argv)
{
    if (argc < 4) return 2;
    const int iters = std::atoi(argv[1]);
    const std::string scratch = argv[2];
    std::mt19937 rng(1);
    int ok = 0, bad = 0;
    for (int a = 3; a < argc; ++a) {
        std::ifstream f(argv[a], std::ios::binary);
        const std::vector<uint8_t> orig((std::istreambuf_iterator<char>(f)),
                                        std::istreambuf_iterator<char>());
        if (orig.empty()) return 2;
        for (int it = 0; it < iters; ++it) {
            std::vector<uint8_t> d = orig;
            const int nflip = 1 + (int)(rng() % 8);
            for (int k = 0; k < nflip; ++k) d[rng() % d.size()] = (uint8_t)rng();
            if (rng() % 4 == 0) d.resize(rng() % d.size());
            {
                std::ofstream o(scratch, std::ios::binary);
                o.write((const char*)d.data(), (std::streamsize)d.size());
            }
            pfio::Image im;
            std::string err;
            if (pfio::load_image(scratch, im, err)) ok++;
            else bad++;
            int w, h, c;
            float* p = pfio::load_pfm(scratch, &w, &h, &c, err);
            std::free(p);
        }
    }
    std::printf("decoded %d rejected %d\n", ok, bad);
    return 0;
}
