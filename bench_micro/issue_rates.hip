// Microbenchmark: issue throughput of the k-NN inner-loop building blocks on
// gfx950 (calibration for DESIGN.md; not part of the product).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  return max(min(a, b), min(max(a, b), c));
}

// 9-slot insertion per step, keys from an xorshift stream
template <int MODE>
__global__ __launch_bounds__(256) void k_ins(uint32_t *out, int iters) {
  uint32_t key[9];
  for (int s = 0; s < 9; ++s) key[s] = 0xffffffffu;
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  for (int it = 0; it < iters; ++it) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const uint32_t kk = x;
    if (MODE == 0) {  // full med3 insertion
#pragma unroll
      for (int s = 8; s > 0; --s) key[s] = umed3(key[s - 1], key[s], kk);
      key[0] = min(key[0], kk);
    } else {  // min only
      key[0] = min(key[0], kk);
    }
  }
  uint32_t acc = 0;
  for (int s = 0; s < 9; ++s) acc ^= key[s];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// LDS read b96 (xyz) + f32 distance per step, lane-varying addresses
__global__ __launch_bounds__(256) void k_lds(float *out, int iters) {
  __shared__ float4 buf[2048];
  for (int i = threadIdx.x; i < 2048; i += 256) buf[i] = make_float4(i, i * 0.5f, i * 0.25f, 0);
  __syncthreads();
  float acc = 0.f;
  int p = threadIdx.x * 7;
  for (int it = 0; it < iters; ++it) {
    const float4 r = buf[p & 2047];
    p += 5;
    const float dx = r.x - 1.f, dy = r.y - 2.f, dz = r.z - 3.f;
    acc += __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const int blocks = 2048, iters = 4096;
  uint32_t *d;
  CHK(hipMalloc(&d, blocks * 256 * 4));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  float ms;
  const double waves = blocks * 4.0;
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CHK(hipEventRecord(a));
      if (mode == 0) hipLaunchKernelGGL(k_ins<0>, dim3(blocks), dim3(256), 0, 0, d, iters);
      if (mode == 1) hipLaunchKernelGGL(k_ins<1>, dim3(blocks), dim3(256), 0, 0, d, iters);
      if (mode == 2) hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(256), 0, 0, (float *)d, iters);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      CHK(hipEventElapsedTime(&ms, a, b));
    }
    // wave-steps per SIMD per microsecond
    const double steps = waves * iters / 1024.0;  // per SIMD
    printf("mode %d (%s): %.3f ms  -> %.2f wave-steps/SIMD/us, %.1f cycles/step/SIMD @2.1GHz\n",
           mode, mode == 0 ? "9-slot med3 insert + xorshift" : mode == 1 ? "min + xorshift" : "ds_read_b128 + f32 dist",
           ms, steps / (ms * 1e3), ms * 1e-3 * 2.1e9 / steps);
  }
  return 0;
}
