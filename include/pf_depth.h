/*
 * pf_depth.h -- the reference's C++ entry points for the fusion path (Depth.h), served by
 * libpanofuse_depth.so on top of the C-ABI of panofuse.h.  A caller of the reference's
 * DepthNamespace (Main.cpp:592, :663) recompiles against this header and links
 * -lpanofuse_depth -lpanofuse; the arithmetic runs in the HIP kernels of libpanofuse.
 *
 * Entry points and the reference interface each one replaces:
 *   EquirectangularMap::{Load, LoadPfm, ValueAtCoord, ValueAtXY, Avg}   Depth.h:9-59
 *   PerspectiveMap::{Load, SetWindow, Value, ValueAtXY, ToSphericalCoord, SphericalTo2D,
 *                    Contain, Azimuth/ZenithMin/Max, Depth2DepthTransform} and the cached
 *                    window members middle/hedge/vedge/corner0-3    Depth.h:61-158
 *   Metrics::{Save, Print}                                             Depth.h:161-250
 *   MergeDepthMaps                                                     Depth.h:286-289
 *   SolveDepthToDepth                                                  Depth.h:297-298
 *   SolveDepthAll                                                      Depth.h:306-307
 *   SolveDepthBySmoothing                                              Depth.h:309
 *   ErrorData / ErrorEmap                                              Depth.h:313-316
 *   SphericalToWorld / WorldToSpherical                                Depth.h:326-329
 *   Save16BitPNG                                                       Depth.cpp:27-32
 *   g_zenith_range                                                     Depth.cpp:22
 *
 * Ownership follows the reference: the map classes own `data` (new[]), MergeDepthMaps
 * allocates and frees its own u16 output, SolveDepthAll writes a caller buffer of W*H u16.
 * Errors: false returns with a message on std::cout, as the reference prints its diagnostics.
 * Threading: one host thread per device (the facade keeps one pf_ctx per device).
 *
 * The window geometry and projections (SetWindow, ToSphericalCoord, SphericalTo2D, Contain,
 * SphericalToWorld, WorldToSpherical) are host fp32 code with the reference's Imath semantics
 * and glibc calls (csrc/pf_geom.hpp), bit-identical to it; the per-pixel path runs on the GPU.
 *
 * Not provided: SolveDisparityToDepth (declared, never defined: Depth.h:293) and
 * SolveDepthToDepth2 (never called), ErrorCompare / ErrorLaplacian, the triangulation/subdivision
 * members (vertices, faces, subd_*: never used on the path).
 */
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#ifndef PF_DEPTH_NO_VEC
/* The vector types of the reference's ILMBase.h:14-16 (`typedef Imath::Vec4<float> Vec4f`, ...)
 * for callers that do not include Imath.  They are declared as class templates in namespace
 * Imath with Imath's layout (public x, y[, z[, w]] of T, ImathVec.h:63-66, 259-262, 563-566),
 * so the entry points below mangle exactly as the reference's do
 * (`DepthNamespace::MergeDepthMaps(..., std::vector<Imath::Vec4<float>>&, ..., Imath::Vec2<float>&,
 * ...)`): libpanofuse_depth.so is built with these, and a caller that includes the real
 * ILMBase.h first and then this header with -DPF_DEPTH_NO_VEC (as Main.cpp:13-15 includes
 * ILMBase.h before Depth.h) links against the same symbols.  Like Imath's, the copy
 * constructors are user-provided (ImathVec.h:96, 294, 507), which makes the types non-trivial for
 * calls: a Vec2f returned by value travels through a hidden pointer in both builds, so the
 * calling convention matches as well as the names.  Every member is inline (and hidden
 * in the library: -fvisibility-inlines-hidden), so nothing here competes with the real Imath.
 * The operations are the ones a caller of the window members uses, with Imath's arithmetic
 * (ImathVec.h:1467-1486 dot/cross, :1631-1700 length with lengthTiny, normalize by division). */
#include <cmath>
#include <limits>
namespace Imath {
template <class T>
class Vec2 {
public:
    T x, y;
    Vec2() : x(0), y(0) {}
    explicit Vec2(T a) : x(a), y(a) {}
    Vec2(T a, T b) : x(a), y(b) {}
    Vec2(const Vec2& v) : x(v.x), y(v.y) {}
    const Vec2& operator=(const Vec2& v) { x = v.x; y = v.y; return *this; }
    T& operator[](int i) { return (&x)[i]; }
    const T& operator[](int i) const { return (&x)[i]; }
    T dot(const Vec2& v) const { return x * v.x + y * v.y; }
    T length() const
    {
        const T l2 = dot(*this);
        if (l2 < T(2) * std::numeric_limits<T>::min()) {  // lengthTiny
            T ax = x >= T(0) ? x : -x, ay = y >= T(0) ? y : -y;
            const T mx = ax < ay ? ay : ax;
            if (mx == T(0)) return T(0);
            ax /= mx;
            ay /= mx;
            return mx * std::sqrt(ax * ax + ay * ay);
        }
        return std::sqrt(l2);
    }
};
template <class T>
class Vec3 {
public:
    T x, y, z;
    Vec3() : x(0), y(0), z(0) {}
    explicit Vec3(T a) : x(a), y(a), z(a) {}
    Vec3(T a, T b, T c) : x(a), y(b), z(c) {}
    Vec3(const Vec3& v) : x(v.x), y(v.y), z(v.z) {}
    const Vec3& operator=(const Vec3& v) { x = v.x; y = v.y; z = v.z; return *this; }
    T& operator[](int i) { return (&x)[i]; }
    const T& operator[](int i) const { return (&x)[i]; }
    Vec3 operator+(const Vec3& v) const { return Vec3(x + v.x, y + v.y, z + v.z); }
    Vec3 operator-(const Vec3& v) const { return Vec3(x - v.x, y - v.y, z - v.z); }
    Vec3 operator*(T s) const { return Vec3(x * s, y * s, z * s); }
    T dot(const Vec3& v) const { return x * v.x + y * v.y + z * v.z; }
    Vec3 cross(const Vec3& v) const
    {
        return Vec3(y * v.z - z * v.y, z * v.x - x * v.z, x * v.y - y * v.x);
    }
    T length() const
    {
        const T l2 = dot(*this);
        if (l2 < T(2) * std::numeric_limits<T>::min()) {  // lengthTiny
            T ax = x >= T(0) ? x : -x, ay = y >= T(0) ? y : -y, az = z >= T(0) ? z : -z;
            T mx = ax;
            if (mx < ay) mx = ay;
            if (mx < az) mx = az;
            if (mx == T(0)) return T(0);
            ax /= mx;
            ay /= mx;
            az /= mx;
            return mx * std::sqrt(ax * ax + ay * ay + az * az);
        }
        return std::sqrt(l2);
    }
    const Vec3& normalize()  /* in place, returns *this */
    {
        const T l = length();
        if (l != T(0)) {
            x /= l;
            y /= l;
            z /= l;
        }
        return *this;
    }
};
template <class T>
inline Vec3<T> operator*(T s, const Vec3<T>& v) { return Vec3<T>(s * v.x, s * v.y, s * v.z); }
template <class T>
class Vec4 {
public:
    T x, y, z, w;
    Vec4() : x(0), y(0), z(0), w(0) {}
    explicit Vec4(T a) : x(a), y(a), z(a), w(a) {}
    Vec4(T a, T b, T c, T d) : x(a), y(b), z(c), w(d) {}
    Vec4(const Vec4& v) : x(v.x), y(v.y), z(v.z), w(v.w) {}
    const Vec4& operator=(const Vec4& v) { x = v.x; y = v.y; z = v.z; w = v.w; return *this; }
    T& operator[](int i) { return (&x)[i]; }
    const T& operator[](int i) const { return (&x)[i]; }
};
}  // namespace Imath
typedef Imath::Vec2<float> Vec2f;
typedef Imath::Vec3<float> Vec3f;
typedef Imath::Vec4<float> Vec4f;
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
    /* the FOVs of the viewing window (SetWindow arguments, Depth.h:70-73) */
    float azimuth_left = 0, azimuth_right = 0, zenith_top = 0, zenith_down = 0;
    Vec4f ranges; /* valid {azi_left, azi_right, zen_up, zen_down} (Depth.h:76) */
    /* the cached quadrilateral window of SetWindow (Depth.h:87-93) */
    Vec3f middle, hedge, vedge;
    Vec3f corner0, corner1, corner2, corner3;
    bool window_set = false;

    PerspectiveMap() = default;
    ~PerspectiveMap();
    PerspectiveMap(PerspectiveMap&& o) noexcept;
    PerspectiveMap& operator=(PerspectiveMap&& o) noexcept;
    PerspectiveMap(const PerspectiveMap&) = delete;
    PerspectiveMap& operator=(const PerspectiveMap&) = delete;

    bool Load(std::string& filename);
    void SetWindow(float AzimuthLeft, float AzimuthRight, float ZenithTop, float ZenithDown);
    float Value(float x, float y);
    Vec2f ToSphericalCoord(float x, float y);       /* Depth.cpp:157-166 */
    Vec2f SphericalTo2D(float azimuth, float zenith); /* Depth.cpp:168-182 */
    bool Contain(float azimuth, float zenith);        /* Depth.cpp:184-207 */
    float AzimuthMin() { return azimuth_left < azimuth_right ? azimuth_left : azimuth_right; }
    float AzimuthMax() { return azimuth_left > azimuth_right ? azimuth_left : azimuth_right; }
    float ZenithMin() { return zenith_top < zenith_down ? zenith_top : zenith_down; }
    float ZenithMax() { return zenith_top > zenith_down ? zenith_top : zenith_down; }
    float ValueAtXY(int x, int y);                    /* Depth.cpp:209-212 */
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
// Depth.h:309, Depth.cpp:1773-1878: the reference's alternate solver (tiles written into the
// grid, 500 Gauss-Seidel smoothing iterations near the tile-box edges), on the GPU, bit-exact.
bool SolveDepthBySmoothing(std::vector<PerspectiveMap>& pmaps, unsigned short* data,
                           int& out_width, int& out_height, Vec2f& zenith_range);

bool ErrorData(EquirectangularMap& emap_gt, unsigned short* data, int data_width,
               int data_height, float& mse, float& mae, float& mre, float& mse_log,
               float& delta1, float& delta2, float& delta3, int align_way, bool cap_depth,
               Vec2f* least_square_shift = nullptr, float* median_shift_factor = nullptr);
bool ErrorEmap(EquirectangularMap& emap_gt, EquirectangularMap& emap_given, float& mse,
               float& mae, float& mre, float& mse_log, float& delta1, float& delta2,
               float& delta3, int align_way, bool cap_depth,
               Vec2f* least_square_shift = nullptr, float* median_shift_factor = nullptr);

/* spherical coord. (radians) to 3d position (Depth.cpp:2955-2958) */
Vec3f SphericalToWorld(float azimuth, float zenith);
/* 3d position to spherical coord.; p is normalized in place (Depth.cpp:2960-2971) */
Vec2f WorldToSpherical(Vec3f& p);

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
 * of 1024 x round(1024/aspect) px, written as <tile_dir>/<raw>.<a0>_<a1>_<z0>_<z1>.jpg (rows
 * top-first, like the reference's flipped write; baseline JPEG at quality 100, 4:4:4, as the
 * reference's stbi_write_jpg call ends up, Main.cpp:319-320). */
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
/* the tile writer of the RGB export: the bytes of stbi_write_jpg(fn, w, h, c, px, quality) with
 * stbi_flip_vertically_on_write(flip) (Main.cpp:319-320), c = 1..4 channels, rows top-first */
extern "C" int pfd_save_jpeg(const char* fn, const uint8_t* px, int w, int h, int c, int quality,
                             int flip);
/* the image decoders behind Load (stbi_load / stbi_load_16 with req_comp 0, Depth.cpp:56-100):
 * native samples (u8, or u16 when *is16) into out (capacity cap bytes); -1 load failure, -2 out
 * too small (dims written either way).  pfd_is_16_bit = stbi_is_16_bit. */
extern "C" int pfd_decode_image(const char* fn, void* out, long long cap, int* w, int* h, int* c,
                                int* is16);
extern "C" int pfd_is_16_bit(const char* fn);
extern "C" void pfd_leres_layout(float* fovs, float* ranges);
