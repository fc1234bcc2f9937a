/*
 * pf_depth.h -- the reference's C++ entry points for the fusion path (Depth.h), served by
 * libpanofuse_depth.so on top of the C-ABI of panofuse.h.  A caller of the reference's
 * DepthNamespace (Main.cpp:592, :663) recompiles against this header and links
 * -lpanofuse_depth -lpanofuse; the arithmetic runs in the HIP kernels of libpanofuse.
 *
 * Entry points and the reference interface each one replaces:
 *   EquirectangularMap::{Load, LoadPfm, ValueAtCoord, ValueAtXY, Avg}   Depth.h:9-59
 *   PerspectiveMap::{Load, SetWindow, Value, Depth2DepthTransform}     Depth.h:61-158
 *   Metrics::{Save, Print}                                             Depth.h:161-250
 *   MergeDepthMaps                                                     Depth.h:286-289
 *   SolveDepthToDepth                                                  Depth.h:297-298
 *   SolveDepthAll                                                      Depth.h:306-307
 *   ErrorData / ErrorEmap                                              Depth.h:313-316
 *   Save16BitPNG                                                       Depth.cpp:27-32
 *   g_zenith_range                                                     Depth.cpp:22
 *
 * Ownership follows the reference: the map classes own `data` (new[]), MergeDepthMaps
 * allocates and frees its own u16 output, SolveDepthAll writes a caller buffer of W*H u16.
 * Errors: false returns with a message on std::cout, as the reference prints its diagnostics.
 * Threading: one host thread per device (the facade keeps one pf_ctx per device).
 *
 * Not provided: progressive JPEG, SolveDisparityToDepth / SolveDepthToDepth2 /
 * SolveDepthBySmoothing (dead code in the reference's mode 0), ErrorCompare / ErrorLaplacian.
 */
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#ifndef PF_DEPTH_NO_VEC
/* Minimal stand-ins for the Imath vectors of ILMBase.h (Vec2f / Vec3f / Vec4f), indexable like
 * the reference uses them. */
struct Vec2f {
    float x = 0, y = 0;
    Vec2f() = default;
    explicit Vec2f(float a) : x(a), y(a) {}
    Vec2f(float a, float b) : x(a), y(b) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};
struct Vec3f {
    float x = 0, y = 0, z = 0;
    Vec3f() = default;
    Vec3f(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};
struct Vec4f {
    float v[4] = {0, 0, 0, 0};
    Vec4f() = default;
    Vec4f(float a, float b, float c, float d) : v{a, b, c, d} {}
    float& operator[](int i) { return v[i]; }
    float operator[](int i) const { return v[i]; }
};
#endif

#define PF_MYPI_D 3.14159265359          /* Basic.h:11 */
#define PF_D2R(a) ((a) / 180.0 * PF_MYPI_D) /* Basic.h:14 */

extern Vec2f g_zenith_range; /* Depth.cpp:22 Vec2f(D2R(26), D2R(154)) */

bool Save16BitPNG(unsigned short* data, int width, int height, const char* filename);

namespace DepthNamespace {

class EquirectangularMap {
public:
    int width = 0, height = 0, channels = 0;
    float* data = nullptr; /* [height][width][channels], 0..1 */

    EquirectangularMap() = default;
    ~EquirectangularMap();
    EquirectangularMap(const EquirectangularMap&) = delete;
    EquirectangularMap& operator=(const EquirectangularMap&) = delete;

    bool Load(std::string& filename, bool mono360 = false);
    bool LoadPfm(std::string& filename, bool flip_vertical, bool normalize,
                 const char* save_png_filename = nullptr);
    float ValueAtCoord(float azimuth, float zenith);
    float ValueAtXY(int x, int y);
    double Avg();
};

class PerspectiveMap {
public:
    int width = 0, height = 0, channels = 0;
    float* data = nullptr;
    float az_left = 0, az_right = 0, zen_top = 0, zen_down = 0; /* SetWindow arguments */
    Vec4f ranges;                                               /* valid {aL, aR, zU, zD} */
    bool window_set = false;

    PerspectiveMap() = default;
    ~PerspectiveMap();
    PerspectiveMap(PerspectiveMap&& o) noexcept;
    PerspectiveMap& operator=(PerspectiveMap&& o) noexcept;
    PerspectiveMap(const PerspectiveMap&) = delete;
    PerspectiveMap& operator=(const PerspectiveMap&) = delete;

    bool Load(std::string& filename);
    void SetWindow(float azi_left, float azi_right, float zen_top, float zen_down);
    float Value(float x, float y);
    void Depth2DepthTransform(Vec4f& abcd); /* runs on the GPU (pf_depth_transform) */
};

class Metrics {
public:
    float mse_given = 0, mse_result = 0, mae_given = 0, mae_result = 0, mre_given = 0,
          mre_result = 0, mselog_given = 0, mselog_result = 0, delta1_given = 0,
          delta1_result = 0, delta2_given = 0, delta2_result = 0, delta3_given = 0,
          delta3_result = 0;
    bool Save(const char* filename);
    void Print();
};

bool MergeDepthMaps(std::string& equirectangular_map_filename,
                    std::vector<std::string>& perspective_map_filenames,
                    std::string& out_filename, std::vector<Vec4f>& perspective_map_FOVs,
                    std::vector<Vec4f>& perspective_map_ranges, int out_width,
                    Vec2f& zenith_range, std::string* equirectangular_map_groundtruth = nullptr,
                    Metrics* metrics = nullptr, int* time_Reg = nullptr,
                    int* time_Laplacian = nullptr);

bool SolveDepthToDepth(EquirectangularMap& emap, std::vector<PerspectiveMap>& pmaps,
                       std::vector<bool>& pmaps_actives, Vec2f& zenith_range, Vec4f& abcd);

bool SolveDepthAll(EquirectangularMap& emap, std::vector<PerspectiveMap>& pmaps,
                   unsigned short* data, int& out_width, int& out_height, Vec2f& zenith_range,
                   const char* Laplacian_filename = nullptr);

bool ErrorData(EquirectangularMap& emap_gt, unsigned short* data, int data_width,
               int data_height, float& mse, float& mae, float& mre, float& mse_log,
               float& delta1, float& delta2, float& delta3, int align_way, bool cap_depth,
               Vec2f* least_square_shift = nullptr, float* median_shift_factor = nullptr);
bool ErrorEmap(EquirectangularMap& emap_gt, EquirectangularMap& emap_given, float& mse,
               float& mae, float& mre, float& mse_log, float& delta1, float& delta2,
               float& delta3, int align_way, bool cap_depth,
               Vec2f* least_square_shift = nullptr, float* median_shift_factor = nullptr);

}  // namespace DepthNamespace

/* The mode-0 driver (Main.cpp:331-687 CreateDepthPanoramas) over std::filesystem; tile_ext is
 * "png" (MiDaS naming, Main.cpp:570-573), "jpg" (LeReS naming, :576-578) or "auto"; the LeReS
 * layout of Main.cpp:788-843 is used.  shard / nshards: this process takes the panoramas
 * shard, shard + nshards, ... of the sorted folder (one process per GPU, no communication).
 * Returns the process exit code. */
int pf_create_depth_panoramas(const std::string& rgb_folder, const std::string& gt_folder,
                              const std::string& baseline_folder,
                              const std::string& result_folder, const std::string& tile_dir,
                              const std::string& tile_ext, int out_width, int shard = 0,
                              int nshards = 1);
/* The RGB tile export of mode 0 (Main.cpp:399-430 + SaveCubeMap :242-326): every panorama of
 * rgb_folder (8/16-bit PNG, PGM/PPM) warped on the GPU (pf_warp_rgb) into the 15 LeReS tiles
 * of 1024 x round(1024/aspect) px, written as <tile_dir>/<raw>.<a0>_<a1>_<z0>_<z1>.png (rows
 * top-first, like the reference's flipped JPEG write; PNG instead of JPEG q=100). */
int pf_export_rgb_tiles(const std::string& rgb_folder, const std::string& tile_dir);
/* The active LeReS layout (Main.cpp:788-843): 15 FOVs and ranges. */
void pf_leres_layout(std::vector<Vec4f>& fovs, std::vector<Vec4f>& ranges);

/* C-ABI helpers (ctypes bindings, tests): load a map as EquirectangularMap::Load (is_emap = 1)
 * or PerspectiveMap::Load (0) into out (float, capacity `cap`; dims always written; returns -1
 * on a load failure); write a 16-bit gray PNG as Save16BitPNG; the LeReS layout as 15x4
 * floats each. */
extern "C" int pfd_load_map(const char* fn, int is_emap, float* out, long long cap, int* w,
                            int* h, int* c);
extern "C" int pfd_save_png16(const char* fn, const uint16_t* data, int w, int h);
extern "C" void pfd_leres_layout(float* fovs, float* ranges);
