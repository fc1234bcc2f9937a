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
//
// IN/OUT are flat little-endian binaries written/read by tests/test_facade.py.
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
        w.put(abcd.v, 4);
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
    w.put(joint.v, 4);
    // the alternate solver on the same (transformed) maps (Depth.h:309)
    if (!SolveDepthBySmoothing(pmaps, out.data(), out_w, out_h, zr)) return 5;
    w.put(out.data(), out.size());
    return 0;
}
}  // namespace

int main(int argc, char** argv)
{
    if (argc != 4) {
        fprintf(stderr, "usage: %s geom|solve IN OUT\n", argv[0]);
        return 1;
    }
    FILE* fi = fopen(argv[2], "rb");
    FILE* fo = fopen(argv[3], "wb");
    if (!fi || !fo) return 1;
    Reader r{fi};
    Writer w{fo};
    int rc = 1;
    try {
        rc = std::string(argv[1]) == "geom" ? geom(r, w) : solve(r, w);
    } catch (const std::string& e) {
        fprintf(stderr, "%s\n", e.c_str());
        rc = 1;
    }
    fclose(fi);
    fclose(fo);
    return rc;
}
