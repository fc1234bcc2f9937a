// VALU issue-rate probe for gfx950: cycles per wave-instruction of a few instruction kinds at
// 1..8 waves per SIMD.  Every kernel runs ITER iterations of 16 independent chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define ITER 4096
#define CH 16

__global__ void __launch_bounds__(256) k_fma(float* out, float a, float b) {
  float x[CH];
  for (int i = 0; i < CH; i++) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) x[i] = __builtin_fmaf(x[i], a, b);
  }
  float s = 0; for (int i = 0; i < CH; i++) s += x[i];
  if (s == 1234.5f) out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_add(float* out, float a, float b) {
  float x[CH];
  for (int i = 0; i < CH; i++) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) x[i] = x[i] + a;
  }
  float s = 0; for (int i = 0; i < CH; i++) s += x[i];
  if (s == 1234.5f) out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_pkfma(float* out, float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 x[CH / 2];
  for (int i = 0; i < CH / 2; i++) x[i] = f2{threadIdx.x * 1e-3f + i, (float)i};
  f2 av = {a, a}, bv = {b, b};
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH / 2; i++) x[i] = __builtin_elementwise_fma(x[i], av, bv);
  }
  float s = 0; for (int i = 0; i < CH / 2; i++) s += x[i].x + x[i].y;
  if (s == 1234.5f) out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_dpp(float* out, float a, float b) {
  float x[CH];
  for (int i = 0; i < CH; i++) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++)
      x[i] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x[i]), 0x138, 0xF, 0xF, true));
  }
  float s = 0; for (int i = 0; i < CH; i++) s += x[i];
  if (s == 1234.5f) out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_adddpp(float* out, float a, float b) {
  float x[CH];
  for (int i = 0; i < CH; i++) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++)
      x[i] = b + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x[i]), 0x138, 0xF, 0xF, true));
  }
  float s = 0; for (int i = 0; i < CH; i++) s += x[i];
  if (s == 1234.5f) out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_cnd(float* out, float a, float b) {
  float x[CH];
  for (int i = 0; i < CH; i++) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      uint32_t m = __float_as_uint(x[i]) == 0x7FBADBADu ? 0u : 0xFFFFFFFFu;
      x[i] = __uint_as_float(__float_as_uint(x[i] + a) & m);
    }
  }
  float s = 0; for (int i = 0; i < CH; i++) s += x[i];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

typedef void (*K)(float*, float, float);
int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  int ncu = p.multiProcessorCount;
  float* out; hipMalloc(&out, 4096);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  struct { const char* name; K k; double instr_per_iter; } ks[] = {
    {"v_fma_f32", k_fma, CH}, {"v_add_f32", k_add, CH}, {"v_pk_fma_f32", k_pkfma, CH / 2},
    {"v_mov_b32_dpp", k_dpp, CH}, {"v_add_f32_dpp", k_adddpp, CH}, {"add+cmp+cndmask", k_cnd, 3 * CH}};
  printf("CUs %d clock %d kHz\n", ncu, p.clockRate);
  for (auto& kk : ks) {
    for (int wps : {1, 2, 3, 4, 8}) {
      int blocks = ncu * wps;  // 256-thread blocks: 4 waves = 1 per SIMD per block
      hipLaunchKernelGGL(kk.k, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f);
      hipEventRecord(e0);
      hipLaunchKernelGGL(kk.k, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double winstr = (double)ITER * kk.instr_per_iter * wps;  // per SIMD
      double ghz = 2.4;  // nominal; report ns per wave-instr too
      printf("%-18s waves/SIMD %d : %.3f ms  %.2f ns/wave-instr/SIMD  (%.2f cyc @2.4GHz)\n", kk.name,
             wps, ms, ms * 1e6 / winstr, ms * 1e6 / winstr * ghz);
    }
  }
  return 0;
}
