// Microbenchmark: per-instruction VALU issue cost on gfx950 (wave64), for the
// op types of the k-NN inner loop. 8 independent chains per lane so latency
// never binds; many waves per SIMD. Calibration for DESIGN.md only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t *out, int iters, uint32_t seed) {
  uint32_t a[8], b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
  f2 fa[8], fb = {(float)b, 1.5f}, fc = {0.25f, (float)c};
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = b + j; fa[j] = f2{(float)j, (float)(j + b)}; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (OP == 0) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (OP == 2) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (OP == 3) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(fa[j]) : "v"(fb), "v"(fc));
      if (OP == 4) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(fa[j]) : "v"(fb));
      if (OP == 5) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (OP == 6) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(fa[j].x) : "v"(fb.x), "v"(fc.x));
      if (OP == 7) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(*(double *)&fa[j]) : "v"(*(double *)&fb), "v"(*(double *)&fc));
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc ^= a[j] ^ __float_as_uint(fa[j].x) ^ __float_as_uint(fa[j].y);
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const int blocks = 4096, iters = 2048;
  uint32_t *d;
  CHK(hipMalloc(&d, blocks * 256 * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  int clk_khz = 0;
  CHK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  const char *names[] = {"v_med3_u32", "v_add_u32", "v_and_or_b32", "v_pk_fma_f32", "v_pk_add_f32",
                         "v_min_u32", "v_fma_f32", "v_fma_f64"};
  for (int op = 0; op < 8; ++op) {
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
      CHK(hipEventRecord(e0));
      switch (op) {
        case 0: hipLaunchKernelGGL(k_op<0>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u); break;
        case 1: hipLaunchKernelGGL(k_op<1>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u); break;
        case 2: hipLaunchKernelGGL(k_op<2>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u); break;
        case 3: hipLaunchKernelGGL(k_op<3>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u); break;
        case 4: hipLaunchKernelGGL(k_op<4>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u); break;
        case 5: hipLaunchKernelGGL(k_op<5>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u); break;
        case 6: hipLaunchKernelGGL(k_op<6>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u); break;
        case 7: hipLaunchKernelGGL(k_op<7>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u); break;
      }
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms, e0, e1));
    }
    const double wave_ops = (double)blocks * 4 * iters * 8;  // wave-instructions
    const double per_simd = wave_ops / 1024.0;
    const double ghz = clk_khz / 1e6;
    printf("%-14s %8.3f ms  %.2f cycles per wave64 op per SIMD (at %.2f GHz)\n", names[op], ms,
           ms * 1e-3 * ghz * 1e9 / per_simd, ghz);
  }
  return 0;
}
