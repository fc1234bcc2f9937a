// HBM ceiling for the depth warp's access mix on MI355X: the C3 launch of
// k_warp_depth reads 64 panoramas of 2048x1024 fp32 (536,870,912 B) and writes 64 x 20 tiles of
// 512^2 fp32 (1,342,177,280 B).  These kernels move exactly those bytes with plain streaming
// accesses -- no gather, no LDS -- so their time is the floor for any warp kernel of this shape.
//
//   mix16   out[o] = in[o*2/5] * s  (every input float4 read once from HBM, 2.5 outputs each)
//   mix4    the same with one float per lane (the warp kernel's 4-B stores)
//   write16 the 1.34 GB of writes alone;  read16 the 0.54 GB of reads alone;  copy16 R = W = 0.54 GB
//   write4 / read4  one float per lane;  mix_r16w4  16-B reads, 4-B writes (2.5 writes per float read)
//
// hipcc --offload-arch=gfx950 -O3 -o stream_mix stream_mix.hip && ./stream_mix
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__global__ void __launch_bounds__(256) k_mix16(const float4* __restrict__ in, float4* __restrict__ out,
                                               long long nout, float s)
{
    for (unsigned o = blockIdx.x * 256 + threadIdx.x; o < (unsigned)nout; o += gridDim.x * 256) {
        float4 v = in[o * 2u / 5u];
        v.x *= s; v.y *= s; v.z *= s; v.w *= s;
        out[o] = v;
    }
}

__global__ void __launch_bounds__(256) k_mix4(const float* __restrict__ in, float* __restrict__ out,
                                              long long nout, float s)
{
    for (unsigned o = blockIdx.x * 256 + threadIdx.x; o < (unsigned)nout; o += gridDim.x * 256)
        out[o] = in[o * 2u / 5u] * s;
}

__global__ void __launch_bounds__(256) k_write4(float* __restrict__ out, long long nout, float s)
{
    for (unsigned o = blockIdx.x * 256 + threadIdx.x; o < (unsigned)nout; o += gridDim.x * 256)
        out[o] = s;
}

__global__ void __launch_bounds__(256) k_read4(const float* __restrict__ in, float* __restrict__ out,
                                               long long nin)
{
    float a = 0;
    for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < (unsigned)nin; i += gridDim.x * 256)
        a += in[i];
    if (a == 1234.5f) out[threadIdx.x] = a;
}

// 16-B reads, 4-B writes: each lane reads one float4 of the panorama stream and writes 2.5
// floats' worth of output as 4-B stores over a contiguous 640-B-per-wave span (lane-interleaved)
__global__ void __launch_bounds__(256) k_mix_r16w4(const float4* __restrict__ in,
                                                   float* __restrict__ out, long long nin, float s)
{
    for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < (unsigned)nin; i += gridDim.x * 256) {
        const float4 v = in[i];
        const float q = (v.x + v.y + v.z + v.w) * s;
        const unsigned wbase = (i & ~63u) * 10u, l = i & 63u;  // 10 floats per input float4
#pragma unroll
        for (int k = 0; k < 10; k++) out[wbase + k * 64 + l] = q;
    }
}

__global__ void __launch_bounds__(256) k_write16(float4* __restrict__ out, long long nout, float s)
{
    for (long long o = (long long)blockIdx.x * 256 + threadIdx.x; o < nout;
         o += (long long)gridDim.x * 256)
        out[o] = make_float4(s, s, s, s);
}

__global__ void __launch_bounds__(256) k_read16(const float4* __restrict__ in, float* __restrict__ out,
                                                long long nin)
{
    float a = 0;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nin;
         i += (long long)gridDim.x * 256) {
        const float4 v = in[i];
        a += v.x + v.y + v.z + v.w;
    }
    if (a == 1234.5f) out[threadIdx.x] = a;
}

__global__ void __launch_bounds__(256) k_copy16(const float4* __restrict__ in, float4* __restrict__ out,
                                                long long n)
{
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (long long)gridDim.x * 256)
        out[i] = in[i];
}

int main()
{
    const long long R = 536870912LL, W = 1342177280LL;
    float *in, *out;
    CK(hipMalloc(&in, R));
    CK(hipMalloc(&out, W));
    CK(hipMemset(in, 0, R));
    CK(hipMemset(out, 0, W));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    struct Case {
        const char* name;
        double bytes;
        int kind;
    };
    const Case cases[] = {{"mix16", double(R + W), 0}, {"mix4", double(R + W), 1},
                          {"write16", double(W), 2},   {"read16", double(R), 3},
                          {"copy16", double(2 * R), 4}, {"write4", double(W), 5},
                          {"read4", double(R), 6},     {"mix_r16w4", double(R + W), 7}};
    for (int blocks_per_cu : {4, 8, 16, 32}) {
        const int grid = cus * blocks_per_cu;
        for (const Case& c : cases) {
            std::vector<float> ms;
            for (int rep = 0; rep < 12; rep++) {
                CK(hipEventRecord(e0));
                switch (c.kind) {
                case 0: k_mix16<<<grid, 256>>>((const float4*)in, (float4*)out, W / 16, 1.0001f); break;
                case 1: k_mix4<<<grid, 256>>>(in, out, W / 4, 1.0001f); break;
                case 2: k_write16<<<grid, 256>>>((float4*)out, W / 16, 0.5f); break;
                case 3: k_read16<<<grid, 256>>>((const float4*)in, out, R / 16); break;
                case 4: k_copy16<<<grid, 256>>>((const float4*)in, (float4*)out, R / 16); break;
                case 5: k_write4<<<grid, 256>>>(out, W / 4, 0.5f); break;
                case 6: k_read4<<<grid, 256>>>(in, out, R / 4); break;
                case 7: k_mix_r16w4<<<grid, 256>>>((const float4*)in, out, R / 16, 1.0001f); break;
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (rep >= 2) ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2], best = ms[0];
            printf("%-8s grid=%5d  best %.4f ms (%.2f TB/s)  median %.4f ms (%.2f TB/s)\n", c.name,
                   grid, best, c.bytes / best / 1e9, med, c.bytes / med / 1e9);
        }
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
