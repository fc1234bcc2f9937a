// Exhaustive check of cubic_map's float clamp thresholds (csrc/pf_internal.hpp) against the
// reference's form, which compares the float X with the double constants 1e-4 and 1 - 1e-4
// (Depth2DepthTransform, Depth.cpp:245-274): with a = b = d = 0 and c = 1 cubic_map returns the
// clamped X itself, so the two must agree bit for bit on all 2^32 float bit patterns.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "pf_internal.hpp"

static float reference_form(float X)
{
    if (X < 1e-4) X = (float)1e-4;
    else if (X > (1 - 1e-4)) X = (float)(1 - 1e-4);
    float Y = 0.0f * X * X * X + 0.0f * X * X + 1.0f * X + 0.0f;
    if (Y < 0) Y = 0;
    else if (Y > 1) Y = 1;
    return Y;
}

int main()
{
    uint64_t bad = 0;
    for (uint64_t u = 0; u <= 0xFFFFFFFFull; u++) {
        const uint32_t b = (uint32_t)u;
        float X;
        std::memcpy(&X, &b, 4);
        const float r = reference_form(X), g = pf::cubic_map(X, 0.0f, 0.0f, 1.0f, 0.0f);
        if (std::memcmp(&r, &g, 4) != 0) {
            if (bad < 5) std::printf("mismatch at 0x%08x\n", b);
            bad++;
        }
    }
    std::printf("cubic thresholds: %llu mismatches over 2^32 floats\n", (unsigned long long)bad);
    return bad != 0;
}
