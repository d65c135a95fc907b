// Microbenchmark: scattered counter increments (the grid cell count) by
// atomic scope, and XCD-private counter copies keyed on HW_REG_XCC_ID.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ int xcc_id() {
  // s_getreg_b32 HW_REG_XCC_ID (id 20), bits [3:0]
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
}

__device__ __forceinline__ uint32_t hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ void k_count(int *cnt, int *slot, int n, int ncells) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = hash(i) % ncells;
  int s;
  if (MODE == 0) s = atomicAdd(&cnt[c], 1);
  if (MODE == 1) s = __hip_atomic_fetch_add(&cnt[c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (MODE == 2) s = __hip_atomic_fetch_add(&cnt[c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (MODE == 3) s = __hip_atomic_fetch_add(&cnt[xcc_id() * ncells + c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (MODE == 4) { __hip_atomic_fetch_add(&cnt[c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); s = 0; }
  if (MODE == 5) { __hip_atomic_fetch_add(&cnt[xcc_id() * ncells + c], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); s = 0; }
  slot[i] = s;
}

__global__ void k_xcc(int *out) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

int main() {
  const int n = 1 << 20, ncells = 400000;
  int *cnt, *slot, *xo;
  CHK(hipMalloc(&cnt, 8ull * ncells * 4));
  CHK(hipMalloc(&slot, n * 4));
  CHK(hipMalloc(&xo, 4096 * 4));
  hipLaunchKernelGGL(k_xcc, dim3(4096), dim3(64), 0, 0, xo);
  std::vector<int> h(4096);
  CHK(hipMemcpy(h.data(), xo, 4096 * 4, hipMemcpyDeviceToHost));
  int match = 0, hist[16] = {0};
  for (int b = 0; b < 4096; ++b) { match += (h[b] == b % 8); if (h[b] >= 0 && h[b] < 16) hist[h[b]]++; }
  printf("xcc_id == blockIdx %% 8 for %d of 4096 blocks; hist:", match);
  for (int x = 0; x < 16; ++x) printf(" %d", hist[x]);
  printf("\n");
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  const char *names[] = {"atomicAdd (default scope)", "agent scope", "workgroup scope, shared array",
                         "workgroup scope, per-XCC copies", "agent scope, no return", "workgroup, per-XCC, no return"};
  for (int mode = 0; mode < 6; ++mode) {
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      CHK(hipMemset(cnt, 0, 8ull * ncells * 4));
      CHK(hipEventRecord(a));
      switch (mode) {
        case 0: hipLaunchKernelGGL(k_count<0>, dim3(n / 256), dim3(256), 0, 0, cnt, slot, n, ncells); break;
        case 1: hipLaunchKernelGGL(k_count<1>, dim3(n / 256), dim3(256), 0, 0, cnt, slot, n, ncells); break;
        case 2: hipLaunchKernelGGL(k_count<2>, dim3(n / 256), dim3(256), 0, 0, cnt, slot, n, ncells); break;
        case 3: hipLaunchKernelGGL(k_count<3>, dim3(n / 256), dim3(256), 0, 0, cnt, slot, n, ncells); break;
        case 4: hipLaunchKernelGGL(k_count<4>, dim3(n / 256), dim3(256), 0, 0, cnt, slot, n, ncells); break;
        case 5: hipLaunchKernelGGL(k_count<5>, dim3(n / 256), dim3(256), 0, 0, cnt, slot, n, ncells); break;
      }
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms; CHK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    // correctness: total of all counters == n
    std::vector<int> hc(8ull * ncells);
    CHK(hipMemcpy(hc.data(), cnt, 8ull * ncells * 4, hipMemcpyDeviceToHost));
    long long tot = 0; for (int v : hc) tot += v;
    printf("mode %d %-34s %8.1f us  total=%lld (expect %d)\n", mode, names[mode], best * 1e3, tot, n);
  }
  return 0;
}
