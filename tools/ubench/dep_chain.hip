// Dependent-VALU latency probe: one wave per block runs a chain of N dependent fp32 fma (or
// fp32 add, or the cvt/add-f64/cvt step); hipEvent time / N = cycles per dependent step at
// the measured clock.  Used to size the sequential-order metrics chain (metrics).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k_chain(const float* in, float* out, int n)
{
    float acc = in[threadIdx.x], v = in[64 + threadIdx.x];
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (MODE == 0) acc = __builtin_fmaf(v, v, acc);
            else if (MODE == 1) acc = acc + v;
            else { const double t = (double)v; acc = (float)((double)acc + t * t); }
        }
    }
    out[threadIdx.x] = acc;
}

int main()
{
    float *in, *out;
    (void)hipMalloc(&in, 128 * 4);
    (void)hipMalloc(&out, 64 * 4);
    (void)hipMemset(in, 0, 128 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int n = 1 << 22;
    for (int mode = 0; mode < 3; ++mode)
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(a);
            if (mode == 0) hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, in, out, n);
            if (mode == 1) hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, in, out, n);
            if (mode == 2) hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, in, out, n);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("mode %d (%s): %.3f ns per dependent step\n", mode,
                   mode == 0 ? "fma f32" : mode == 1 ? "add f32" : "cvt/add f64/cvt", ms * 1e6 / n);
        }
    return 0;
}
