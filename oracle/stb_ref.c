/*
 * stb_ref.c -- TEST INFRASTRUCTURE ONLY: the reference's own image codecs, compiled from the
 * reference tree where it lies (/root/reference/stb_image.h v2.23 and stb_image_write.h v1.15,
 * the files Main.cpp:17-20 instantiates) into oracle/_ref/libstbref.so by oracle/Makefile, so the
 * facade's loaders and JPEG writer (csrc/pf_image.cpp, csrc/pf_jpeg.cpp) can be checked byte for
 * byte against what the reference's PerspectiveMap::Load / EquirectangularMap::Load
 * (Depth.cpp:45-109, 277-355) and SaveCubeMap's stbi_write_jpg (Main.cpp:319-320) produce.
 * Nothing here is part of the product, and no reference source is copied: this file only
 * includes the reference's headers by path (-I/root/reference) and wraps three calls.
 */
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"
#define STB_IMAGE_WRITE_IMPLEMENTATION
#include "stb_image_write.h"

#include <string.h>

/* stbi_load / stbi_load_16 with req_comp 0, as the reference's loaders call them; copies the
 * samples (8- or 16-bit) into out (capacity cap bytes).  Returns 0, -1 on a load failure, -2 if
 * out is too small (dims are written either way). */
int sref_load(const char* fn, int want16, void* out, long long cap, int* w, int* h, int* c)
{
    void* px = want16 ? (void*)stbi_load_16(fn, w, h, c, 0) : (void*)stbi_load(fn, w, h, c, 0);
    if (!px) return -1;
    const long long n = (long long)(*w) * (*h) * (*c) * (want16 ? 2 : 1);
    int rc = n > cap ? -2 : 0;
    if (!rc) memcpy(out, px, (size_t)n);
    stbi_image_free(px);
    return rc;
}

int sref_is_16_bit(const char* fn) { return stbi_is_16_bit(fn); }

/* stbi_write_jpg as SaveCubeMap calls it (Main.cpp:319-320: flip on write, quality = stride) */
int sref_write_jpg(const char* fn, int w, int h, int comp, const unsigned char* data, int quality,
                   int flip)
{
    stbi_flip_vertically_on_write(flip);
    return stbi_write_jpg(fn, w, h, comp, data, quality);
}

const char* sref_failure_reason(void) { return stbi_failure_reason(); }
