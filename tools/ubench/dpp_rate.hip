// Issue-rate probe for gfx950: DPP folded into a VOP2 arithmetic op vs the separate mov_dpp,
// plain VOP2 and packed fp32 ops, at 1..8 waves per SIMD (16 independent chains per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 4096
#define CH 16

#define KERNEL(name, body)                                                              \
  __global__ void __launch_bounds__(256) name(float* out, float a, float b)             \
  {                                                                                     \
    float x[CH];                                                                        \
    float y = threadIdx.x * 1e-3f + a;                                                  \
    for (int i = 0; i < CH; i++) x[i] = threadIdx.x * 1e-3f + i;                        \
    for (int it = 0; it < ITER; it++) {                                                 \
      _Pragma("unroll") for (int i = 0; i < CH; i++) { body; }                          \
    }                                                                                   \
    float s = 0;                                                                        \
    for (int i = 0; i < CH; i++) s += x[i];                                             \
    if (s == 1234.5f) out[threadIdx.x] = s + y;                                         \
  }

KERNEL(k_add_vv, asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[i]) : "v"(y)))
KERNEL(k_add_dpp, asm volatile("v_add_f32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                               : "+v"(x[i]) : "v"(y)))
KERNEL(k_fmac_dpp, asm volatile("v_fmac_f32_dpp %0, %1, %2 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                                : "+v"(x[i]) : "v"(y), "v"(y)))
KERNEL(k_mov_dpp, asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                               : "=v"(x[i]) : "v"(x[(i + 1) % CH])))
KERNEL(k_mov, asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 1) % CH])))

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) k_pk_add(float* out, float a, float b)
{
  f2 x[CH / 2];
  f2 y = {threadIdx.x * 1e-3f + a, b};
  for (int i = 0; i < CH / 2; i++) x[i] = f2{threadIdx.x * 1e-3f + i, (float)i};
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH / 2; i++) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(x[i]) : "v"(y));
  }
  float s = 0;
  for (int i = 0; i < CH / 2; i++) s += x[i].x + x[i].y;
  if (s == 1234.5f) out[threadIdx.x] = s;
}

typedef void (*K)(float*, float, float);
int main()
{
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int ncu = p.multiProcessorCount;
  float* out;
  hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct { const char* name; K k; double instr_per_iter; } ks[] = {
      {"v_add_f32 (vv)", k_add_vv, CH},     {"v_add_f32_dpp", k_add_dpp, CH},
      {"v_fmac_f32_dpp", k_fmac_dpp, CH},   {"v_mov_b32_dpp", k_mov_dpp, CH},
      {"v_mov_b32", k_mov, CH},             {"v_pk_add_f32", k_pk_add, CH / 2}};
  for (auto& kk : ks) {
    for (int wps : {1, 2, 3, 4, 8}) {
      int blocks = ncu * wps;
      hipLaunchKernelGGL(kk.k, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f);
      hipEventRecord(e0);
      hipLaunchKernelGGL(kk.k, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double winstr = (double)ITER * kk.instr_per_iter * wps;
      printf("%-18s waves/SIMD %d : %.3f ms  %.2f cyc/wave-instr/SIMD @2.4GHz\n", kk.name, wps, ms,
             ms * 1e6 / winstr * 2.4);
    }
  }
  return 0;
}
