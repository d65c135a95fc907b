// navgpu_common.h — what the two translation units of libnavgpu.so share:
// navgpu.hip (per-row mode, curvature, KD build, host plumbing) and knn.hip
// (global-mode grid index and exact k-NN). Internal: never installed.
#pragma once

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "navgpu.h"

#pragma clang fp contract(off)

constexpr int kWave = 64;
constexpr int kKnnMaxSx = 8;  // x cells per h of the global-mode grid (knn.hip)

// Diagnostic phase stamps (build with -DNAVGPU_STAMPS; never in the product
// build): lane 0 of each wave adds s_memtime deltas per phase into g_stamps.
#ifdef NAVGPU_STAMPS
// one copy per translation unit (no relocatable device code): navgpu.hip's
// navgpu_debug_stamps adds knn.hip's through nv::knn_stamps_take
static __device__ unsigned long long g_stamps[16];
#define NV_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define NV_STAMP_ADD(slot, a, b) \
  if ((threadIdx.x & 63) == 0) atomicAdd(&g_stamps[slot], (b) - (a))
#define NV_STAMP_ADD0(slot, a, b) \
  if (threadIdx.x == 0) atomicAdd(&g_stamps[slot], (b) - (a))
#define NV_COUNT0(slot) \
  if (threadIdx.x == 0) atomicAdd(&g_stamps[slot], 1ull)
// per-wave accumulators, flushed with one atomic per slot at the kernel's end
// (atomics inside a hot loop would distort what they time)
#define NV_ACC_DECL unsigned long long nv_acc[16] = {}
#define NV_ACC(slot, a, b) nv_acc[slot] += (b) - (a)
#define NV_ACC_FLUSH                                              \
  if ((threadIdx.x & 63) == 0) {                                  \
    _Pragma("unroll") for (int s_ = 1; s_ < 16; ++s_)             \
      if (nv_acc[s_]) atomicAdd(&g_stamps[s_], nv_acc[s_]);       \
  }
#else
#define NV_ACC_DECL
#define NV_ACC(slot, a, b)
#define NV_ACC_FLUSH
#define NV_COUNT0(slot)
#define NV_STAMP(v)
#define NV_STAMP_ADD(slot, a, b)
#define NV_STAMP_ADD0(slot, a, b)
#endif

namespace nv {
void set_err(const char *fmt, ...);
}

#define HIP_TRY(expr)                                                          \
  do {                                                                         \
    hipError_t e_ = (expr);                                                    \
    if (e_ != hipSuccess) {                                                    \
      nv::set_err("%s:%d %s: %s", __FILE__, __LINE__, #expr,                  \
                  hipGetErrorString(e_));                                      \
      return NAVGPU_EHIP;                                                      \
    }                                                                          \
  } while (0)

#define CHECK_LAUNCH(name)                                                     \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess) {                                                    \
      nv::set_err("launch %s: %s", name, hipGetErrorString(e_));              \
      return NAVGPU_EHIP;                                                      \
    }                                                                          \
  } while (0)

#define ARG_CHECK(cond)                                                        \
  do {                                                                         \
    if (!(cond)) {                                                             \
      nv::set_err("invalid argument: %s", #cond);                             \
      return NAVGPU_EINVAL;                                                    \
    }                                                                          \
  } while (0)

#define RC(x)                         \
  do {                                \
    int rc_ = (x);                    \
    if (rc_ != NAVGPU_OK) return rc_; \
  } while (0)

// ------------------------------------------------------------ device helpers
namespace {

// utils/kdtree.c:14-17 (euclideanDistance; gcc folds pow(v,2) to v*v) and
// src/slam.c:28-33,47-50: sqrt((dx*dx + dy*dy) + dz*dz), no contraction.
__device__ __forceinline__ double ref_dist(double ax, double ay, double az,
                                           double bx, double by, double bz) {
  const double dx = ax - bx, dy = ay - by, dz = az - bz;
  return __builtin_sqrt(dx * dx + dy * dy + dz * dz);
}

__device__ __forceinline__ int lanes_below(unsigned long long bal) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                   __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
}

__device__ __forceinline__ void wave_sync_mem() {
  // Cross-lane hand-off through memory inside one wavefront (LDS, or global
  // scratch of the large-n build): workgroup-scope release/acquire makes the
  // other lanes' stores visible; wave_barrier stops code motion across it.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// inclusive prefix sum over the 64 lanes by DPP (row shifts, then the row
// broadcasts 15 and 31): no LDS, a few cycles per step
__device__ __forceinline__ int wave_scan_add(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return x;
}


// Block-wide exclusive scan of one int per thread. scratch: >= nwaves+1 ints.
__device__ __forceinline__ int block_excl_scan(int v, int *scratch, int *total) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int nw = blockDim.x / kWave;
  int incl = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    int t = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += t;
  }
  if (lane == kWave - 1) scratch[wid] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < nw; ++w) {
      int t = scratch[w];
      scratch[w] = acc;
      acc += t;
    }
    scratch[nw] = acc;
  }
  __syncthreads();
  const int res = scratch[wid] + incl - v;
  *total = scratch[nw];
  __syncthreads();
  return res;
}

// ---- packed-f32 screens with an f64 certificate (knn.hip k_knnw, the row
// screen k_rows_screen32) ----
typedef float f2 __attribute__((ext_vector_type(2)));

// sqrt(v) rounded up by more than v_sqrt_f32's 1-ulp error: an upper bound
// for the error terms below (they only need to bound, not be exact)
__device__ __forceinline__ double sqrt_up(double v) {
  return (double)__builtin_amdgcn_sqrtf((float)v) * (1.0 + 0x1p-20);
}

// Error of the packed-f32 squared distance: each coordinate is rounded to f32
// once relative to the tile origin (<= 2^-24 |v|) and subtracted once in f32,
// so each difference is within dl = Dq 2^-22 of the exact one (Dq bounds the
// magnitudes); then |d2_f32 - d2| <= err(d2_f32-ish) below.
__device__ __forceinline__ double f32_err(double V, double dl) {
  return V * 0x1p-20 + 4.0 * dl * sqrt_up(V) + 4.0 * dl * dl;
}

// f32 admission bound for an f64 dsq bound T: every candidate whose exact
// dsq is <= T has an f32 dsq <= the returned value.
__device__ __forceinline__ float f32_bound(double T, double dl) {
  if (!(T < INFINITY)) return INFINITY;
  const double E = T * 0x1p-20 + 4.0 * dl * sqrt_up(T) + 4.0 * dl * dl;
  return (float)((T + E) * (1.0 + 0x1p-20));
}

// the converse: an upper bound on the exact dsq of a candidate whose f32 dsq
// is <= V (each coordinate difference within dl of the exact one)
__device__ __forceinline__ double f32_upper(double V, double dl) {
  return (V + f32_err(V, dl)) * (1.0 + 0x1p-20);
}

constexpr uint32_t kNoKey32 = 0xffffffffu;  // an empty key slot

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  return max(min(a, b), min(max(a, b), c));  // one v_med3_u32
}

// key = (f32 distance bits with the low kKeyBits cleared) | local id, as ONE
// v_and_or_b32 (the mask in a VGPR, the id in an SGPR). lid MUST be
// wave-uniform: a divergent value would be read from the first lane only.
__device__ __forceinline__ uint32_t knn_key(float d, uint32_t vmask, uint32_t lid) {
  uint32_t k;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(k) : "v"(__float_as_uint(d)), "v"(vmask), "s"(lid));
  return k;
}

}  // namespace

// ------------------------------------------------------------------ host
struct navgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::map<int, std::pair<void *, size_t>> bufs;  // grow-only workspace
  bool timing = false;
  std::string timing_only;  // navgpu_timing_select: record only this region ("" = all)
  std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> ev;
  std::vector<hipEvent_t> free_ev;
  std::vector<double> tan_c, tan_r;
  int tan_R = -1, tan_C = -1;
  hipStream_t aux = nullptr;                 // side stream (pair path: curvature)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  double knn_occ = 5.0;  // target points per h^3 grid cell (NAVGPU_KNN_OCC)
  int knn_sx = 3;        // x cells per h (NAVGPU_KNN_SX; r4: 3 -> build -5 us, query same)
  int knn_mode = 2;      // query pass: 2 = k_knng (row lists, r5), 1 = k_knnw (NAVGPU_KNN_MODE)
  bool knn_stats = false;
  bool pair_side = true;  // pair curvature on the side stream (NAVGPU_PAIR_SIDE=0: on this one)
  // the lazy K5 query's tie flags (kRowTieLazy): zeroed once, then cleared by
  // k_rows_retree as it reads them, so no memset per call
  int32_t *lazy_tie = nullptr;
  int lazy_tie_rows = 0;  // rows the tie buffer was zeroed for
  int screen_rows = 0, screen_S = 0;  // last screened rows_match call (tie diagnostic)
};

namespace nv {

// workspace slots (grow-only buffers of a context)
enum Slot {
  kBBox = 1, kParams, kCnt, kStart, kBSum, kCellId, kSlotBuf, kRec, kTan,
  kKdFc, kKdP, kKdT, kQStart, kQCell, kQSlot, kQPerm, kStats, kOvf, kSlowQ,
  kSlowThr, kTSort, kRowMaskS, kRowMaskT, kRowTie, kCorrEnt, kCorrN, kCorrSums, kKdPtmp, kKdSel,
  kQSort, kCellId2, kSRec, kNpg, kGl, kRowTieLazy,
  kH0 = 100, kH1, kH2, kH3, kH4, kH5,
};

int ws_get(navgpu_ctx *ctx, int slot, size_t bytes, void **out);

template <class T>
int ws(navgpu_ctx *ctx, int slot, size_t count, T **out) {
  void *p;
  int rc = ws_get(ctx, slot, count * sizeof(T), &p);
  *out = (T *)p;
  return rc;
}

// HIP events around a span of launches on one stream (navgpu_timing_*)
struct TimedRegion {
  navgpu_ctx *ctx;
  const char *name;
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t st;
  hipEvent_t take() {
    if (!ctx->free_ev.empty()) {
      hipEvent_t e = ctx->free_ev.back();
      ctx->free_ev.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  TimedRegion(navgpu_ctx *c, const char *n, hipStream_t on = nullptr)
      : ctx(c), name(n), st(on ? on : c->stream) {
    if (!ctx->timing || (!ctx->timing_only.empty() && ctx->timing_only != name)) return;
    a = take();
    b = take();
    if (a && b) (void)hipEventRecord(a, st);
  }
  ~TimedRegion() {
    if (!a || !b) return;
    (void)hipEventRecord(b, st);
    ctx->ev[name].push_back({a, b});
  }
};

inline unsigned grid1d(size_t n, int block) {
  return (unsigned)((n + block - 1) / block);
}

// diagnostic builds (-DNAVGPU_STAMPS): knn.hip's phase stamps, read and
// cleared; NAVGPU_EINVAL otherwise
int knn_stamps_take(unsigned long long *out16);

// side stream of a context, created on first use
int ensure_aux(navgpu_ctx *ctx);

// R1 curvature of up to two clouds (both R x C, row-major Points) in one
// launch on `stream` (src/slam.c:11-61); navgpu.hip
int launch_curvature(const double *pts0, int32_t *mask0, double *curv0,
                     const double *pts1, int32_t *mask1, double *curv1, int R, int C,
                     hipStream_t stream);

}  // namespace nv
