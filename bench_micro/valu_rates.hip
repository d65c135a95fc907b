// Microbenchmark: wave64 VALU issue cost per SIMD on gfx950 for the k-NN
// scan's instruction types, at 1..8 waves per SIMD and 12 independent chains
// per lane (so dependent latency never binds). Calibration for DESIGN.md only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int NC = 12;

template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t *out, int iters, uint32_t seed) {
  uint32_t a[NC], b = seed ^ threadIdx.x, c = seed * 3u + blockIdx.x;
  f2 fa[NC], fb = {(float)b, 1.5f}, fc = {0.25f, (float)c};
#pragma unroll
  for (int j = 0; j < NC; ++j) { a[j] = b + j; fa[j] = f2{(float)j, (float)(j + b)}; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (OP == 0) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(b));
      if (OP == 1) asm volatile("v_min_u32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(b));
      if (OP == 2) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (OP == 3) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (OP == 4) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(fa[j].x) : "v"(fb.x));
      if (OP == 5) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(fa[j].x) : "v"(fb.x), "v"(fc.x));
      if (OP == 6) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(fa[j]) : "v"(fb), "v"(fc));
      if (OP == 7) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(fa[j]) : "v"(fb));
      if (OP == 8) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (OP == 9) asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(b));
      if (OP == 10) asm volatile("v_max_u32_e32 %0, %1, %0" : "+v"(a[j]) : "v"(b));
      if (OP == 11) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(fa[j].x) : "v"(fb.x));
      if (OP == 12) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(fa[j]) : "v"(fb));
      if (OP == 13) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(fa[j].x) : "v"(fb.x), "v"(fc.x));
      if (OP == 14) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b));
      if (OP == 15) asm volatile("v_sub_f32_e32 %0, %1, %0" : "+v"(fa[j].x) : "v"(fb.x));
      if (OP == 16) asm volatile("v_min_f32_e32 %0, %1, %0" : "+v"(fa[j].x) : "v"(fb.x));
      if (OP == 17) asm volatile("v_max_f32_e32 %0, %1, %0" : "+v"(fa[j].x) : "v"(fb.x));
      if (OP == 18) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(fa[j].x) : "v"(fb.x), "v"(fc.x));
      if (OP == 19) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (OP == 20) asm volatile("v_cndmask_b32_e32 %0, %1, %0, vcc" : "+v"(a[j]) : "v"(b));
      if (OP == 21) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
      if (OP == 22) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a[j]) : "v"(b));
      if (OP == 23) asm volatile("v_max_f32_e64 %0, %1, %0" : "+v"(fa[j].x) : "v"(fb.x));
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < NC; ++j) acc ^= a[j] ^ __float_as_uint(fa[j].x) ^ __float_as_uint(fa[j].y);
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int OP>
float run(uint32_t *d, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms;
}

int main() {
  const int iters = 4096;
  uint32_t *d;
  CHK(hipMalloc(&d, 8192 * 256 * 4));
  int clk_khz = 0;
  CHK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  const char *names[] = {"v_add_u32_e32", "v_min_u32_e32", "v_med3_u32", "v_min3_u32", "v_add_f32_e32",
                         "v_fma_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_and_or_b32", "v_xor_b32_e32",
                         "v_max_u32_e32", "v_mul_f32_e32", "v_pk_mul_f32", "v_med3_f32", "v_pk_max_u16",
                         "v_sub_f32_e32", "v_min_f32_e32", "v_max_f32_e32", "v_min3_f32",
                         "v_perm_b32", "v_cndmask_b32", "v_med3_i32", "v_lshl_or_b32",
                         "v_max_f32_e64"};
  // waves per SIMD: 256 CUs x 4 SIMDs; a 256-thread block = one wave per SIMD
  for (int wps : {4, 8}) {
    const int blocks = 256 * wps;
    float (*fns[24])(uint32_t *, int, int) = {
        run<0>,  run<1>,  run<2>,  run<3>,  run<4>,  run<5>,  run<6>,  run<7>,
        run<8>,  run<9>,  run<10>, run<11>, run<12>, run<13>, run<14>, run<15>,
        run<16>, run<17>, run<18>, run<19>, run<20>, run<21>, run<22>, run<23>};
    for (int op = 0; op < 24; ++op) {
      const float ms = fns[op](d, blocks, iters);
      const double wave_ops_per_simd = (double)wps * iters * NC;
      printf("wps=%d %-15s %.2f cycles/op/SIMD (clock attr %.2f GHz)\n", wps, names[op],
             ms * 1e-3 * clk_khz * 1e3 / wave_ops_per_simd, clk_khz / 1e6);
    }
  }
  return 0;
}
