/* The oracle (oracle/pf_oracle.c, pf_oracle_lm.c) run under AddressSanitizer + UBSan: the E->P
 * depth warp, MergeDepthMaps' registration and fusion, the RGB warp and SolveDepthBySmoothing on
 * inputs written by tests/test_oracle_sanitized.py.  Test infrastructure only (SURVEY.md section 5,
 * "ASan/UBSan on the CPU restatement").  The reference's own hazards -- the seam read of
 * buffer[Y*w + w] and the out-of-tile taps (Depth.cpp:1595-1604) -- are restated in bounds, so any
 * report here is a bug of the restatement.
 *
 *   oracle_asan <dir> : reads dir/{case.bin, tiles.bin, resp.bin, pano.f32, emap.f32, rgb.u8},
 *                       writes dir/{out.u16, abcd.f32, rgb_tiles.u8, smooth.u16}
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pf_oracle.h"

static void* slurp(const char* dir, const char* name, size_t want)
{
    char fn[1024];
    snprintf(fn, sizeof(fn), "%s/%s", dir, name);
    FILE* f = fopen(fn, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", fn); exit(2); }
    void* p = malloc(want ? want : 1);
    if (fread(p, 1, want, f) != want) { fprintf(stderr, "short read %s\n", fn); exit(2); }
    fclose(f);
    return p;
}

static void spill(const char* dir, const char* name, const void* p, size_t n)
{
    char fn[1024];
    snprintf(fn, sizeof(fn), "%s/%s", dir, name);
    FILE* f = fopen(fn, "wb");
    if (!f || fwrite(p, 1, n, f) != n) { fprintf(stderr, "cannot write %s\n", fn); exit(2); }
    fclose(f);
}

int main(int argc, char** argv)
{
    if (argc != 2) { fprintf(stderr, "usage: %s <dir>\n", argv[0]); return 2; }
    const char* dir = argv[1];
    /* case.bin: int32 {ntiles, total, pw, ph, ew, eh, out_w}, float32 {zr0, zr1} */
    int32_t* hdr = (int32_t*)slurp(dir, "case.bin", 7 * 4 + 2 * 4);
    const int ntiles = hdr[0], total = hdr[1], pw = hdr[2], ph = hdr[3], ew = hdr[4], eh = hdr[5];
    const int out_w = hdr[6];
    float zr[2];
    memcpy(zr, hdr + 7, sizeof(zr));
    pfo_tile* tiles = (pfo_tile*)slurp(dir, "tiles.bin", sizeof(pfo_tile) * ntiles);
    pfo_response* resp = (pfo_response*)slurp(dir, "resp.bin", sizeof(pfo_response) * ntiles);
    float* pano = (float*)slurp(dir, "pano.f32", sizeof(float) * pw * ph);
    float* emap = (float*)slurp(dir, "emap.f32", sizeof(float) * ew * eh);
    uint8_t* rgb = (uint8_t*)slurp(dir, "rgb.u8", (size_t)pw * ph * 3);

    float* tile_data = (float*)calloc((size_t)total, sizeof(float));
    pfo_warp_depth(pano, pw, ph, tiles, ntiles, resp, tile_data);
    float* warped = (float*)malloc(sizeof(float) * total);
    memcpy(warped, tile_data, sizeof(float) * total);

    const int out_h = out_w / 2;
    uint16_t* out = (uint16_t*)calloc((size_t)out_w * out_h, sizeof(uint16_t));
    float* abcd = (float*)calloc((size_t)4 * ntiles, sizeof(float));
    int rc = pfo_merge(emap, ew, eh, 1, tiles, ntiles, tile_data, out_w, zr[0], zr[1], 3, 1, out,
                       abcd);
    if (rc != 0) { fprintf(stderr, "pfo_merge rc=%d\n", rc); return 1; }
    spill(dir, "out.u16", out, sizeof(uint16_t) * (size_t)out_w * out_h);
    spill(dir, "abcd.f32", abcd, sizeof(float) * 4 * ntiles);

    /* RGB warp of the same layout (3 bytes per tile pixel, packed in tile order) */
    long long rgb_total = 0;
    for (int i = 0; i < ntiles; i++) rgb_total += (long long)tiles[i].width * tiles[i].height * 3;
    uint8_t* rgb_tiles = (uint8_t*)calloc((size_t)rgb_total, 1);
    pfo_warp_rgb(rgb, pw, ph, tiles, ntiles, rgb_tiles);
    spill(dir, "rgb_tiles.u8", rgb_tiles, (size_t)rgb_total);

    /* SolveDepthBySmoothing on the (untransformed) warped tiles */
    uint16_t* sm = (uint16_t*)calloc((size_t)out_w * out_h, sizeof(uint16_t));
    rc = pfo_solve_smoothing(tiles, ntiles, warped, out_w, out_h, zr[0], zr[1], sm);
    if (rc != 0) { fprintf(stderr, "pfo_solve_smoothing rc=%d\n", rc); return 1; }
    spill(dir, "smooth.u16", sm, sizeof(uint16_t) * (size_t)out_w * out_h);

    free(hdr); free(tiles); free(resp); free(pano); free(emap); free(rgb); free(tile_data);
    free(warped); free(out); free(abcd); free(rgb_tiles); free(sm);
    printf("oracle_asan ok: %d tiles, %dx%d\n", ntiles, out_w, out_h);
    return 0;
}
