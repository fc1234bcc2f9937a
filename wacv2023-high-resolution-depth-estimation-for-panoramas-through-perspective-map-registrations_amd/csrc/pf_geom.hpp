// pf_geom.hpp -- host fp32 geometry of the reference's projection, with Imath Vec2/Vec3<float>
// semantics (ImathVec.h:1145-1180 Vec2 length, :1467-1486 dot/cross, :1631-1700 length/lengthTiny
// and normalize-by-division).  Shared by the library's layout setup (pf_api.hip) and the
// DepthNamespace facade (pf_depth.cpp) so both produce the reference's bits; compiled with
// -ffp-contract=off (no fused multiply-adds), glibc sincosf/tanf/atan2f as the g++ build of
// Depth.cpp calls them.
#pragma once

#include <cfloat>
#include <cmath>

namespace pfgeom {

constexpr double MYPI = 3.14159265359;  // Basic.h:11

struct V3 {
    float x, y, z;
};
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b)
{
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline float length(V3 a)
{
    float l2 = dot(a, a);
    if (l2 < 2.0f * FLT_MIN) {  // lengthTiny
        float ax = a.x >= 0.0f ? a.x : -a.x, ay = a.y >= 0.0f ? a.y : -a.y,
              az = a.z >= 0.0f ? a.z : -a.z;
        float mx = ax;
        if (mx < ay) mx = ay;
        if (mx < az) mx = az;
        if (mx == 0.0f) return 0.0f;
        ax /= mx; ay /= mx; az /= mx;
        return mx * sqrtf(ax * ax + ay * ay + az * az);
    }
    return sqrtf(l2);
}
inline float length2(float x, float y)
{
    float l2 = x * x + y * y;
    if (l2 < 2.0f * FLT_MIN) {
        float ax = x >= 0.0f ? x : -x, ay = y >= 0.0f ? y : -y;
        float mx = ax < ay ? ay : ax;
        if (mx == 0.0f) return 0.0f;
        ax /= mx; ay /= mx;
        return mx * sqrtf(ax * ax + ay * ay);
    }
    return sqrtf(l2);
}
inline V3 normalized(V3 a)
{
    float l = length(a);
    if (l != 0.0f) { a.x /= l; a.y /= l; a.z /= l; }
    return a;
}

// SphericalToWorld (Depth.cpp:2955-2958; g++ emits sincosf for each sin/cos pair)
inline V3 sph_to_world(float az, float zen)
{
    float sz, cz, sa, ca;
    sincosf(zen, &sz, &cz);
    sincosf(az, &sa, &ca);
    return {sz * ca, sz * sa, cz};
}

// WorldToSpherical (Depth.cpp:2960-2971): normalize, fmod(atan2f, 2*MYPI) in double, +2*MYPI
// below 0, zenith = atan2f(|(x, y)|, z).  `p` is normalized in place, as the reference's
// Vec3f& argument is.
inline void world_to_sph(V3& p, float& az, float& zen)
{
    p = normalized(p);
    float a = (float)std::fmod((double)atan2f(p.y, p.x), 2 * MYPI);
    if (a < 0) a = (float)((double)a + 2 * MYPI);
    az = a;
    zen = atan2f(length2(p.x, p.y), p.z);
}

// PerspectiveMap::SetWindow (Depth.cpp:120-155), in its operation order.
struct Window {
    V3 middle, hedge, vedge, corner0, corner1, corner2, corner3;
};
inline Window set_window(float aL, float aR, float zT, float zD)
{
    Window w;
    w.middle = sph_to_world((aL + aR) / 2, (zT + zD) / 2);
    const V3 left = normalized(cross(V3{0, 0, 1}, w.middle));
    const V3 up = normalized(cross(left, w.middle));
    const float ta = tanf(fabsf(aR - aL) / 2), tz = tanf(fabsf(zT - zD) / 2);
    const V3 left_middle = add(w.middle, mul(left, ta));
    const V3 right_middle = sub(w.middle, mul(left, ta));
    const V3 up_middle = sub(w.middle, mul(up, tz));
    const V3 down_middle = add(w.middle, mul(up, tz));
    w.corner0 = add(add(w.middle, sub(left_middle, w.middle)), sub(up_middle, w.middle));
    w.corner1 = add(add(w.middle, sub(left_middle, w.middle)), sub(down_middle, w.middle));
    w.corner2 = add(add(w.middle, sub(right_middle, w.middle)), sub(down_middle, w.middle));
    w.corner3 = add(add(w.middle, sub(right_middle, w.middle)), sub(up_middle, w.middle));
    w.hedge = sub(right_middle, left_middle);
    w.vedge = sub(down_middle, up_middle);
    return w;
}

// PerspectiveMap::SphericalTo2D (Depth.cpp:168-182) with LinePlaneIntersection (:34-42) for
// p = 0, p0 = normal = middle.
inline void sph_to_2d(const Window& w, float az, float zen, float& x, float& y)
{
    const V3 dir = sph_to_world(az, zen);
    const V3 p0mp = {w.middle.x - 0.0f, w.middle.y - 0.0f, w.middle.z - 0.0f};
    const float t = dot(p0mp, w.middle) / dot(dir, w.middle);
    const V3 pos = {0.0f + t * dir.x, 0.0f + t * dir.y, 0.0f + t * dir.z};
    const V3 e = sub(pos, w.corner0);
    x = (dot(e, w.hedge) / length(w.hedge)) / length(w.hedge);
    y = (dot(e, w.vedge) / length(w.vedge)) / length(w.vedge);
}

// PerspectiveMap::ToSphericalCoord (Depth.cpp:157-166)
inline void to_spherical_coord(const Window& w, float x, float y, float& az, float& zen)
{
    V3 pos = add(add(w.corner0, mul(w.hedge, x)), mul(w.vedge, y));
    world_to_sph(pos, az, zen);
}

}  // namespace pfgeom
