// facade_check.cpp -- a reference-style caller of the DepthNamespace facade (include/pf_depth.h),
// written the way Main.cpp / MergeDepthMaps use Depth.h, for the parity tests
// (tests/test_facade.py): it includes pf_depth.h, links -lpanofuse_depth -lpanofuse, and dumps
// what the reference's entry points return so the tests can compare it with the oracle.
//
//   facade_check geom  IN OUT   window members, ToSphericalCoord, SphericalTo2D, Contain,
//                               SphericalToWorld, WorldToSpherical (host only, no GPU)
//   facade_check solve IN OUT   per tile SolveDepthToDepth (one active map) +
//                               Depth2DepthTransform (Depth.cpp:794-805), then SolveDepthAll
//                               (:913), then SolveDepthToDepth with several active maps, then
//                               SolveDepthBySmoothing (:1773-1878) on the transformed maps
//   facade_check merge IN OUT   MergeDepthMaps on files, called as Main.cpp:592-594 calls it
//                               (global FOV/range vectors, g_zenith_range, timing outputs)
//
// IN/OUT are flat little-endian binaries written/read by tests/test_facade.py.
//
// Built twice: with the header's own Imath-layout vectors (bin/pf_facade_check), and with
// -DPF_FACADE_IMATH against the reference's ILMBase.h + IlmBase 2.2 headers
// (oracle/_ref/pf_facade_check_imath, only where /root/reference exists): that build includes
// ILMBase.h first and pf_depth.h with PF_DEPTH_NO_VEC, exactly as Main.cpp:13-15 includes
// ILMBase.h before Depth.h, so it only links if the library's exported signatures carry
// Imath::Vec2<float> / Imath::Vec4<float>.
#ifdef PF_FACADE_IMATH
#include "ILMBase.h"
#define PF_DEPTH_NO_VEC
#endif
#include "../../include/pf_depth.h"

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace DepthNamespace;

namespace {
struct Reader {
    FILE* f;
    template <class T>
    T get()
    {
        T v;
        if (fread(&v, sizeof(T), 1, f) != 1) throw std::string("short input");
        return v;
    }
    template <class T>
    void get(T* p, size_t n)
    {
        if (fread(p, sizeof(T), n, f) != n) throw std::string("short input");
    }
};
struct Writer {
    FILE* f;
    template <class T>
    void put(const T& v) { fwrite(&v, sizeof(T), 1, f); }
    template <class T>
    void put(const T* p, size_t n) { fwrite(p, sizeof(T), n, f); }
    void put3(const Vec3f& v) { put(v.x); put(v.y); put(v.z); }
};

void read_layout(Reader& r, std::vector<PerspectiveMap>& pmaps, int tw, int th)
{
    for (auto& p : pmaps) {
        float fov[4], rng[4];
        r.get(fov, 4);
        r.get(rng, 4);
        p.width = tw;
        p.height = th;
        p.channels = 1;
        p.SetWindow(fov[0], fov[1], fov[2], fov[3]);  // MergeDepthMaps :780
        p.ranges = Vec4f(rng[0], rng[1], rng[2], rng[3]);
    }
}

int geom(Reader& r, Writer& w)
{
    const int n = r.get<int>();
    std::vector<PerspectiveMap> pmaps(n);
    read_layout(r, pmaps, 2, 2);
    const int nxy = r.get<int>();
    std::vector<float> xy(2 * nxy);
    r.get(xy.data(), xy.size());
    const int nsp = r.get<int>();
    std::vector<float> sp(2 * nsp);
    r.get(sp.data(), sp.size());
    for (auto& p : pmaps) {
        w.put3(p.middle); w.put3(p.hedge); w.put3(p.vedge);
        w.put3(p.corner0); w.put3(p.corner1); w.put3(p.corner2); w.put3(p.corner3);
        for (int k = 0; k < nxy; k++) {
            const Vec2f c = p.ToSphericalCoord(xy[2 * k], xy[2 * k + 1]);
            w.put(c.x); w.put(c.y);
        }
        for (int k = 0; k < nsp; k++) {
            const Vec2f c = p.SphericalTo2D(sp[2 * k], sp[2 * k + 1]);
            w.put(c.x); w.put(c.y);
            w.put(p.Contain(sp[2 * k], sp[2 * k + 1]) ? 1.0f : 0.0f);
        }
    }
    for (int k = 0; k < nsp; k++) {
        Vec3f d = SphericalToWorld(sp[2 * k], sp[2 * k + 1]);
        w.put3(d);
        Vec3f q = d * 3.5f;  // a non-unit vector: WorldToSpherical normalizes it in place
        const Vec2f c = WorldToSpherical(q);
        w.put(c.x); w.put(c.y);
        w.put3(q);
    }
    return 0;
}

int solve(Reader& r, Writer& w)
{
    const int n = r.get<int>(), tw = r.get<int>(), th = r.get<int>();
    std::vector<PerspectiveMap> pmaps(n);
    read_layout(r, pmaps, tw, th);
    EquirectangularMap emap;
    emap.width = r.get<int>();
    emap.height = r.get<int>();
    emap.channels = 1;
    emap.data = new float[(size_t)emap.width * emap.height];
    r.get(emap.data, (size_t)emap.width * emap.height);
    for (auto& p : pmaps) {
        p.data = new float[(size_t)tw * th];
        r.get(p.data, (size_t)tw * th);
    }
    int out_w = r.get<int>();
    Vec2f zr;
    zr.x = r.get<float>();
    zr.y = r.get<float>();
    const int nact = r.get<int>();
    std::vector<int> act(nact);
    r.get(act.data(), act.size());
    // MergeDepthMaps' registration loop (Depth.cpp:794-805)
    for (int p = 0; p < n; p++) {
        std::vector<bool> actives(n, false);
        actives[p] = true;
        Vec4f abcd;
        if (!SolveDepthToDepth(emap, pmaps, actives, zr, abcd)) return 2;
        pmaps[p].Depth2DepthTransform(abcd);
        w.put(abcd.x); w.put(abcd.y); w.put(abcd.z); w.put(abcd.w);
    }
    for (auto& p : pmaps) w.put(p.data, (size_t)tw * th);
    int out_h = out_w / 2;
    std::vector<unsigned short> out((size_t)out_w * out_h);
    if (!SolveDepthAll(emap, pmaps, out.data(), out_w, out_h, zr)) return 3;
    w.put(out.data(), out.size());
    // several active maps in one problem (on the transformed maps, as a caller would)
    std::vector<bool> actives(n, false);
    for (int a : act) actives[a] = true;
    Vec4f joint;
    if (!SolveDepthToDepth(emap, pmaps, actives, zr, joint)) return 4;
    w.put(joint.x); w.put(joint.y); w.put(joint.z); w.put(joint.w);
    // the alternate solver on the same (transformed) maps (Depth.h:309)
    if (!SolveDepthBySmoothing(pmaps, out.data(), out_w, out_h, zr)) return 5;
    w.put(out.data(), out.size());
    return 0;
}

// Main.cpp:32-33 keeps the layout in globals and passes them by reference (:592-594)
std::vector<Vec4f> g_cubemap_FOVs;
std::vector<Vec4f> g_cubemap_ranges;

std::string get_str(Reader& r)
{
    const int n = r.get<int>();
    std::string s(n, '\0');
    r.get(&s[0], n);
    return s;
}

int merge(Reader& r, Writer& w)
{
    const int n = r.get<int>();
    for (int i = 0; i < n; i++) {
        float fov[4], rng[4];
        r.get(fov, 4);
        r.get(rng, 4);
        g_cubemap_FOVs.push_back(Vec4f(fov[0], fov[1], fov[2], fov[3]));
        g_cubemap_ranges.push_back(Vec4f(rng[0], rng[1], rng[2], rng[3]));
    }
    const int out_width = r.get<int>();
    std::string fn_baseline = get_str(r), output_filename = get_str(r), fn_gt = get_str(r);
    std::vector<std::string> pmap_fns;
    for (int i = 0; i < n; i++) pmap_fns.push_back(get_str(r));
    DepthNamespace::Metrics metrics_aligned;
    int time_Reg = 0, time_Laplacian = 0;
    if (!DepthNamespace::MergeDepthMaps(fn_baseline, pmap_fns, output_filename, g_cubemap_FOVs,
                                        g_cubemap_ranges, out_width, g_zenith_range, &fn_gt,
                                        &metrics_aligned, &time_Reg, &time_Laplacian))
        return 6;
    const float m[14] = {metrics_aligned.mse_given,    metrics_aligned.mse_result,
                         metrics_aligned.mae_given,    metrics_aligned.mae_result,
                         metrics_aligned.mre_given,    metrics_aligned.mre_result,
                         metrics_aligned.mselog_given, metrics_aligned.mselog_result,
                         metrics_aligned.delta1_given, metrics_aligned.delta1_result,
                         metrics_aligned.delta2_given, metrics_aligned.delta2_result,
                         metrics_aligned.delta3_given, metrics_aligned.delta3_result};
    w.put(m, 14);
    w.put(time_Reg);
    w.put(time_Laplacian);
    return 0;
}
}  // namespace

int main(int argc, char** argv)
{
    if (argc != 4) {
        fprintf(stderr, "usage: %s geom|solve|merge IN OUT\n", argv[0]);
        return 1;
    }
    FILE* fi = fopen(argv[2], "rb");
    FILE* fo = fopen(argv[3], "wb");
    if (!fi || !fo) return 1;
    Reader r{fi};
    Writer w{fo};
    int rc = 1;
    try {
        const std::string mode = argv[1];
        rc = mode == "geom" ? geom(r, w) : mode == "merge" ? merge(r, w) : solve(r, w);
    } catch (const std::string& e) {
        fprintf(stderr, "%s\n", e.c_str());
        rc = 1;
    }
    fclose(fi);
    fclose(fo);
    return rc;
}
