// pf_image.hpp -- file formats either side of the fusion path.
//
// Replaces the reference's third-party image I/O on this path:
//   * stb_image loads (stbi_is_16_bit / stbi_load / stbi_load_16 with req_comp 0,
//     Depth.cpp:56-100 and :304-351): PNG (bit depths 1..16, gray / gray+alpha / RGB / RGBA /
//     palette, interlaced or not, colour-key tRNS) and 8-bit binary PGM/PPM, at the channel count
//     and with the samples stb returns (palette expanded to RGB or RGBA, sub-8-bit gray scaled
//     to 0..255, a colour key adding an alpha channel);
//   * load_pfm (Depth.cpp:376-452): "PF"/"Pf" portable float maps, the reference's endian rule;
//   * Save16BitPNG (Depth.cpp:27-32, cv::imwrite of a CV_16UC1 Mat) and stbi_write_png:
//     16-bit / 8-bit PNG writers on zlib.
//   * stb's JPEG decoding (the LeReS tiles and some baselines) and stbi_write_jpg (the RGB tile
//     export): pf_jpeg.cpp, bit-exact to stb_image v2.23 / stb_image_write v1.15.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace pfio {

struct Image {
    int w = 0, h = 0, c = 0;
    bool is16 = false;               // samples in px16 (else px8)
    std::vector<uint8_t> px8;        // [h][w][c]
    std::vector<uint16_t> px16;      // [h][w][c]
};

// stbi_is_16_bit: a 16-bit PNG or a PGM/PPM with maxval > 255.
// stbi_is_16_bit: a 16-bit PNG.
bool is_16bit(const std::string& fn);
bool load_image(const std::string& fn, Image& out, std::string& err);
// Returns a malloc'd [h][w][c] float buffer (free with std::free) or nullptr.
float* load_pfm(const std::string& fn, int* w, int* h, int* c, std::string& err);
bool save_png16(const std::string& fn, const uint16_t* data, int w, int h, std::string& err);
// JPEG (pf_jpeg.cpp): baseline / extended / progressive Huffman, 8-bit, 1 / 3 / 4 components,
// the samples and channel count of stbi_load(req_comp 0), bit for bit.
bool decode_jpeg(const std::vector<uint8_t>& f, Image& out, std::string& err);
bool save_png8(const std::string& fn, const uint8_t* data, int w, int h, int c,
               std::string& err);
// JPEG writer (pf_jpeg.cpp): the byte stream of stbi_write_jpg (c = 1..4 channels, rows
// top-first; flip = stbi_flip_vertically_on_write), as the reference's tile export calls it
// (Main.cpp:319-320: flipped, quality = width*3, i.e. 100: every quantiser 1, 4:4:4).
bool encode_jpeg(const uint8_t* px, int w, int h, int c, int quality, std::vector<uint8_t>& out,
                 std::string& err, bool flip = false);
bool save_jpeg(const std::string& fn, const uint8_t* px, int w, int h, int c, int quality,
               std::string& err, bool flip = false);

}  // namespace pfio
