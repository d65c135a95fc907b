// Microbenchmark: where do the workgroups of a CU-masked stream run?
// For a few masks (hipExtStreamCreateWithCUMask) a kernel records, per
// workgroup, HW_REG_XCC_ID and HW_REG_HW_ID (SE, SH, CU), and the host prints
// the distinct CUs per XCD. Checks the bit order the split pipeline assumes
// (bit i -> XCD i % nxcd, CU i / nxcd within it), then times a VALU-bound
// kernel on masks of 4..32 CUs per XCD.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <set>
#include <vector>

#define CHK(x)                                                         \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("%s: %s\n", #x, hipGetErrorString(e));                    \
      return 1;                                                        \
    }                                                                  \
  } while (0)

__device__ __forceinline__ uint32_t xcc_id() {
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
}
__device__ __forceinline__ uint32_t hw_id() {
  return __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
}

__global__ void k_where(uint32_t *out, int spin) {
  if (threadIdx.x == 0) out[blockIdx.x] = (xcc_id() << 16) | (hw_id() & 0xffff);
  // keep the workgroup resident a while so later ones spread over the CUs
  float v = threadIdx.x;
  for (int i = 0; i < spin; ++i) v = v * 1.0000001f + 0.5f;
  if (v == -1.f) out[0] = 0;
}

__global__ void k_valu(float *out, int iters) {
  float a = threadIdx.x, b = blockIdx.x;
  for (int i = 0; i < iters; ++i) {
    a = fmaf(a, 1.0000001f, b);
    b = fmaf(b, 0.9999999f, a);
  }
  if (a + b == -1.f) out[blockIdx.x] = a;
}

static std::vector<uint32_t> mask_of(int ncu, int nx, int c0, int c1) {
  std::vector<uint32_t> m((ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i) {
    const int c = i / nx;
    if (c >= c0 && c < c1) m[i / 32] |= 1u << (i % 32);
  }
  return m;
}

static int run_where(const char *name, const std::vector<uint32_t> &m, int nx,
                     std::vector<int> *counts = nullptr) {
  hipStream_t s;
  CHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
  const int nb = 8192;
  uint32_t *d;
  CHK(hipMalloc(&d, nb * 4));
  hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d, 20000);
  CHK(hipStreamSynchronize(s));
  std::vector<uint32_t> h(nb);
  CHK(hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost));
  std::vector<std::set<uint32_t>> per(nx);
  for (uint32_t v : h) {
    const uint32_t x = v >> 16, hw = v & 0xffff;
    // gfx9 HW_ID: CU [11:8], SH [12], SE [15:13]
    const uint32_t cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    if (x < (uint32_t)nx) per[x].insert(se * 32 + sh * 16 + cu);
  }
  printf("%-22s", name);
  int tot = 0;
  for (int x = 0; x < nx; ++x) {
    printf(" x%d:%zu", x, per[x].size());
    tot += (int)per[x].size();
  }
  printf("  total %d\n", tot);
  if (counts)
    for (int x = 0; x < nx; ++x) counts->push_back((int)per[x].size());
  if (tot <= 16)
    for (int x = 0; x < nx; ++x)
      for (uint32_t c : per[x]) printf("    xcd %d se %u sh %u cu %u\n", x, c / 32, (c / 16) & 1, c & 15);
  CHK(hipFree(d));
  CHK(hipStreamDestroy(s));
  return 0;
}

// Safe first probe (argv[1] == "probe"): every bit set except bits 0..3.
// Under either bit order (interleaved: bit i -> XCD i % 8; contiguous: bit i
// -> XCD i / 32) no XCD loses all its CUs (a queue with an XCD left without
// CUs never finishes its dispatch). Exit 0 only if the order is interleaved:
// XCDs 0..3 lose one CU each.
int main(int argc, char **argv) {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const int nx = ncu >= 256 ? 8 : 1;
  printf("%s: %d CUs, assuming %d XCDs\n", p.gcnArchName, ncu, nx);
  if (argc > 1 && argv[1][0] == 'p') {
    std::vector<uint32_t> m((ncu + 31) / 32, 0xffffffffu);
    m[0] &= ~0xfu;
    std::vector<int> per;
    if (run_where("all but bits 0..3", m, nx, &per)) return 1;
    const int cus_x = ncu / nx;
    bool inter = nx == 8;
    for (int x = 0; x < nx; ++x) inter = inter && per[x] == (x < 4 ? cus_x - 1 : cus_x);
    printf("bit order: %s\n", inter ? "interleaved (bit i -> XCD i %% 8)" : "NOT interleaved");
    return inter ? 0 : 3;
  }
  if (run_where("c 0..1 per xcd", mask_of(ncu, nx, 0, 1), nx)) return 1;
  if (run_where("c 0..4 per xcd", mask_of(ncu, nx, 0, 4), nx)) return 1;
  if (run_where("c 4..32 per xcd", mask_of(ncu, nx, 4, 32), nx)) return 1;
  if (run_where("all", mask_of(ncu, nx, 0, 32), nx)) return 1;
  // VALU-bound kernel time by CUs per XCD
  float *o;
  CHK(hipMalloc(&o, 1 << 20));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int cus_x = ncu / nx;
  for (int c : {4, 8, 16, 24, 28, 32}) {
    if (c > cus_x) continue;
    auto m = mask_of(ncu, nx, cus_x - c, cus_x);
    hipStream_t s;
    CHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    hipLaunchKernelGGL(k_valu, dim3(ncu * 8), dim3(256), 0, s, o, 20000);
    CHK(hipEventRecord(a, s));
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_valu, dim3(ncu * 8), dim3(256), 0, s, o, 20000);
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    printf("valu kernel on %2d CUs/xcd: %.3f ms per launch\n", c, ms / 3);
    CHK(hipStreamDestroy(s));
  }
  return 0;
}
