// navgpu.hip — MI355X (gfx950) kernels and C ABI of the NAV-SLAM scan-matching
// front end (include/navgpu.h). Built with `-ffp-contract=off`, no fast-math:
// every floating-point expression keeps the reference's association order so
// masks, tree permutations, neighbours and distances are bit-identical to the
// reference C path (wuHakureReimu/NAV-SLAM src/slam.c, utils/kdtree.c,
// utils/pointcloud.c).
//
// Kernels (DESIGN.md has the HBM layout and the roofline of each):
//   k_curvature      R1  row tiles + 2-point halo staged in LDS
//   k_project        R2  depth grid -> xyz with host-computed tan tables
//   k_transform      R3  t + R*p (and - tr), elementwise
//   k_rows_match     R1+R4+R5+R6 fused per row: target-row features, exact
//                    reference KD permutation built in LDS, source-row
//                    feature queries against it, one workgroup per row
//   k_rows_build / k_rows_query  the same split in two (slam.c keeps the
//                    target trees across frames)
//   k_bbox_partial, k_grid_params, k_bin_hist, k_scan_*, k_bin_scatter,
//   k_bin_fine       global mode index: uniform grid over the target cloud,
//                    both clouds counting-sorted by cell without global atomics
//   k_knn<K>, k_knn_slow<K>
//                    exact k-NN over that grid, (distance, index) ordering
#include <hip/hip_runtime.h>

#include <type_traits>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "navgpu.h"

#pragma clang fp contract(off)

#define NAVGPU_VERSION "navgpu 0.1 (gfx950)"

namespace {

constexpr int kWave = 64;
constexpr int kRowsBlock = 512;     // 8 waves per row workgroup
#ifndef NAVGPU_ROWS_BUILD_BLOCK
#define NAVGPU_ROWS_BUILD_BLOCK 512
#endif
constexpr int kRowsBuildBlock = NAVGPU_ROWS_BUILD_BLOCK;  // k_rows_build (trees only)
constexpr int kStackDepth = 14;     // implicit-tree height bound, n < 8192
constexpr int kMaxRowCols = 8191;   // 13-bit stack-entry fields
constexpr int kCurvTile = 256;

// Diagnostic phase stamps (build with -DNAVGPU_STAMPS; never in the product
// build): lane 0 of each wave adds s_memtime deltas per phase into g_stamps.
#ifdef NAVGPU_STAMPS
__device__ unsigned long long g_stamps[16];
#define NV_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define NV_STAMP_ADD(slot, a, b) \
  if ((threadIdx.x & 63) == 0) atomicAdd(&g_stamps[slot], (b) - (a))
#define NV_STAMP_ADD0(slot, a, b) \
  if (threadIdx.x == 0) atomicAdd(&g_stamps[slot], (b) - (a))
#define NV_COUNT0(slot) \
  if (threadIdx.x == 0) atomicAdd(&g_stamps[slot], 1ull)
#else
#define NV_COUNT0(slot)
#define NV_STAMP(v)
#define NV_STAMP_ADD(slot, a, b)
#define NV_STAMP_ADD0(slot, a, b)
#endif

// ------------------------------------------------------------------ errors
char g_err[1024] = "";

void set_err(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

#define HIP_TRY(expr)                                                          \
  do {                                                                         \
    hipError_t e_ = (expr);                                                    \
    if (e_ != hipSuccess) {                                                    \
      set_err("%s:%d %s: %s", __FILE__, __LINE__, #expr,                      \
              hipGetErrorString(e_));                                          \
      return NAVGPU_EHIP;                                                      \
    }                                                                          \
  } while (0)

#define CHECK_LAUNCH(name)                                                     \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess) {                                                    \
      set_err("launch %s: %s", name, hipGetErrorString(e_));                  \
      return NAVGPU_EHIP;                                                      \
    }                                                                          \
  } while (0)

#define ARG_CHECK(cond)                                                        \
  do {                                                                         \
    if (!(cond)) {                                                             \
      set_err("invalid argument: %s", #cond);                                 \
      return NAVGPU_EINVAL;                                                    \
    }                                                                          \
  } while (0)

// ============================================================ device helpers

// utils/kdtree.c:14-17 (euclideanDistance; gcc folds pow(v,2) to v*v) and
// src/slam.c:28-33,47-50: sqrt((dx*dx + dy*dy) + dz*dz), no contraction.
__device__ __forceinline__ double ref_dist(double ax, double ay, double az,
                                           double bx, double by, double bz) {
  const double dx = ax - bx, dy = ay - by, dz = az - bz;
  return __builtin_sqrt(dx * dx + dy * dy + dz * dz);
}

// src/slam.c:15-58 for one point with its four same-row neighbours
// (k = -2, -1, +1, +2 in that order). The four distances are computed once
// and reused for the variance: sqrt is deterministic, so this is the
// reference's second loop bit for bit.
__device__ __forceinline__ double curvature_of(double d0, double d1, double d2, double d3) {
  double sum = 0.0;
  sum += d0;
  sum += d1;
  sum += d2;
  sum += d3;
  const int count = 4;
  const double avg = sum / count;
  double curv = 0.0;
  if (avg > 0) {
    double var = 0.0;
    var += (d0 - avg) * (d0 - avg);
    var += (d1 - avg) * (d1 - avg);
    var += (d2 - avg) * (d2 - avg);
    var += (d3 - avg) * (d3 - avg);
    curv = var / count / (avg * avg + 1e-6f);
  }
  return curv;
}

__device__ __forceinline__ double curvature5(const double *c, const double *m2,
                                             const double *m1, const double *p1,
                                             const double *p2) {
  return curvature_of(ref_dist(c[0], c[1], c[2], m2[0], m2[1], m2[2]),
                      ref_dist(c[0], c[1], c[2], m1[0], m1[1], m1[2]),
                      ref_dist(c[0], c[1], c[2], p1[0], p1[1], p1[2]),
                      ref_dist(c[0], c[1], c[2], p2[0], p2[1], p2[2]));
}

// curvature of column j of a row held AoS in LDS (raw[3*j..]); 0 outside the
// reference's window 2 <= j < C-2 (src/slam.c:16).
__device__ __forceinline__ double row_curv_lds(const double *raw, int C, int j) {
  if (j < 2 || j >= C - 2) return 0.0;
  return curvature5(raw + 3 * j, raw + 3 * (j - 2), raw + 3 * (j - 1),
                    raw + 3 * (j + 1), raw + 3 * (j + 2));
}

// Coalesced copy of n doubles global -> LDS by the whole block.
__device__ __forceinline__ void block_copy(double *dst, const double *src,
                                           int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
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

// Block-wide exclusive scan of one int per thread. scratch: >= nwaves+1 ints.
__device__ int block_excl_scan(int v, int *scratch, int *total) {
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

// Stable compaction of [0, C): flag(j) -> write(j, rank). Each thread owns a
// contiguous chunk so ranks follow column order (flattenPoints order,
// src/slam.c:64-72). Returns the count.
template <class Flag, class Write>
__device__ int block_compact(int C, int *scratch, Flag flag, Write write) {
  const int per = (C + blockDim.x - 1) / blockDim.x;
  const int j0 = threadIdx.x * per;
  const int j1 = min(C, j0 + per);
  int cnt = 0;
  for (int j = j0; j < j1; ++j) cnt += flag(j) ? 1 : 0;
  int total;
  int off = block_excl_scan(cnt, scratch, &total);
  for (int j = j0; j < j1; ++j)
    if (flag(j)) write(j, off++);
  __syncthreads();
  return total;
}

// ------------------------------------------------------------------------
// Exact reference KD build (utils/kdtree.c:20-82) in LDS.
//
// The build permutes the row's feature array in place; that permuted array
// IS the tree (node of [lo,hi) at lo+(hi-lo)/2). P[pos] = feature id at tree
// position pos; key coordinates in FC[axis*NS + id].
//
// nth_element is a Lomuto quickselect (pivot = last, `cmp <= 0` goes left).
// One wave runs one nth_element; a partition pass walks the window in 64-event
// chunks: small events are stable-compacted to the front (ballot + mbcnt);
// the large ones follow the "tape" rule that reproduces Lomuto's swaps
// exactly: tape[p] = large ? elem(p) : tape[#smalls before p], resolved within
// a chunk by pointer jumping over lanes (DESIGN.md §KD build). The final
// layout is smalls | pivot | tape[S+1..m) with tape[S] moved to `last`.
// ------------------------------------------------------------------------
// Where the tape chain of a small position p leads (tape[x] = tape[x - L]
// while x is small with L larges before it): every position of p's run of
// smalls [s, p] has the same L = p - sp, so the chain jumps by multiples of L
// to the first position below s. s = one past the last large below p in this
// wave (lbelow = the wave's large ballot masked to lanes below p), else the
// wave's first position (the run then continues into earlier positions,
// still of the same L). One hop per run of smalls instead of one per L.
__device__ __forceinline__ int tape_jump(int p, int sp, unsigned long long lbelow,
                                         int wave_p0) {
  const int k = p - sp;  // >= 1
  const int s = lbelow ? wave_p0 + kWave - __clzll(lbelow) : wave_p0;
  return p - k * ((p - s + k) / k);
}

template <class IdxT, bool GMEM = false>
__device__ void wave_nth_element(const double *key, IdxT *P, IdxT *T,
                                 int first, int last, int nth, int lane) {
  // One wave owns [first, last]. In LDS its accesses execute in program
  // order, so no fence is needed between chunks; P/T in global memory
  // (GMEM, the large-n build) need one after each chunk's writes. The next
  // chunk's P/key reads are issued before the current chunk resolves (this
  // chunk only writes positions below the next chunk).
  while (first < last) {
    const int pe = (int)P[last];
    const double pk = key[pe];
    const int m = last - first;
    int S = 0;
    int e_n = lane < m ? (int)P[first + lane] : 0;
    double k_n = key[e_n];
    for (int cs = 0; cs < m; cs += kWave) {
      const int p = cs + lane;
      const bool act = p < m;
      const int e = e_n;
      const bool small = act && ((k_n - pk) <= 0.0);  // kdtree.c:31-43
      if (cs + kWave < m) {  // read ahead
        const int pn = p + kWave;
        e_n = pn < m ? (int)P[first + pn] : 0;
        k_n = key[e_n];
      }
      const unsigned long long bal = __ballot(small);
      const unsigned long long lbal = __ballot(act && !small);
      const int sp = S + lanes_below(bal);
      // tape value of position p: bit 31 = resolved, low bits = the value, or
      // (unresolved) the chunk lane whose value it equals
      unsigned w = 0x80000000u | (unsigned)e;
      if (small && sp != p) {
        const int y = tape_jump(p, sp, lbal & ((1ull << lane) - 1ull), cs);
        if (y < cs)
          w = 0x80000000u | (unsigned)T[first + y];
        else
          w = (unsigned)(y - cs);
      }
      // pointer jumping: one shuffle per round (taking the pointee's word is
      // right both when it is resolved and when it is a further pointer)
      while (__ballot(!(w >> 31))) {
        const unsigned o = __shfl(w, (w >> 31) ? lane : (int)(w & (kWave - 1)), kWave);
        if (!(w >> 31)) w = o;
      }
      if (act) T[first + p] = (IdxT)(w & 0x7fffffffu);
      if (small) P[first + sp] = (IdxT)e;
      S += __popcll(bal);
      if (GMEM) wave_sync_mem();
    }
    for (int q = S + lane; q < m; q += kWave) {
      const int v = (int)T[first + q];
      P[q == S ? last : first + q] = (IdxT)v;
    }
    if (lane == 0) P[first + S] = (IdxT)pe;
    wave_sync_mem();  // the pass's writes before the next pass reads P
    const int i = first + S;
    if (i == nth) break;
    if (i < nth)
      first = i + 1;
    else
      last = i - 1;
  }
}

// The reference nth_element for ONE subarray by the whole block (the top of
// the tree, where a single wave would leave the rest of the block idle): the
// same tape rule as wave_nth_element, one block-wide chunk of blockDim
// positions per step. Small counts are prefix-summed across the waves. Tape
// chains are first followed inside each wave with shuffles (a pointer always
// leads to a lower position, so what is left points into an earlier wave),
// then across waves by pointer jumping through LDS, one barrier per round
// (double-buffered words, a rotating any-unresolved flag); the common chunk
// with no cross-wave chain costs two barriers. Requires blockDim.x <=
// kBlockNthMax; P/T in LDS, or in global memory (k_kd_level: the barriers
// order the waves' global writes at workgroup scope).
constexpr int kBlockNthMax = 1024;
#ifndef NAVGPU_BLOCK_TO_WAVE
#define NAVGPU_BLOCK_TO_WAVE 256
#endif
// windows this short finish on wave 0 alone (a block pass costs ~4 barriers
// whatever its length; a wave pass over a few 64-position chunks needs none)
constexpr int kBlockToWave = NAVGPU_BLOCK_TO_WAVE;
template <class IdxT, bool GMEM = false>
__device__ void block_nth_element(const double *key, IdxT *P, IdxT *T, int first,
                                  int last, int nth) {
  __shared__ unsigned bw[2 * kBlockNthMax];
  __shared__ int bcnt[2][kBlockNthMax / kWave];
  __shared__ int bany[3];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const int bd = blockDim.x, nw = bd / kWave, wbase = wid * kWave;
  if (tid < 3) bany[tid] = 0;
  __syncthreads();
  int rnd = 0, chunk = 0;  // running counters (buffer and flag rotation)
  while (first < last) {
    if (last - first < kBlockToWave) {
      if (wid == 0) wave_nth_element<IdxT, GMEM>(key, P, T, first, last, nth, lane);
      if (GMEM) __threadfence_block();
      __syncthreads();
      return;
    }
    const int pe = (int)P[last];
    const double pk = key[pe];
    const int m = last - first;
    int S = 0;
    NV_COUNT0(13);
    for (int cs = 0; cs < m; cs += bd, ++chunk) {
      NV_COUNT0(14);
      const int p = cs + tid;
      const bool act = p < m;
      const int e = act ? (int)P[first + p] : 0;
      const bool small = act && ((key[e] - pk) <= 0.0);  // kdtree.c:31-43
      const unsigned long long bal = __ballot(small);
      const unsigned long long lbal = __ballot(act && !small);
      int *cnt = bcnt[chunk & 1];
      if (lane == 0) cnt[wid] = __popcll(bal);
      // also orders the previous chunk's T writes before this chunk's reads
      __syncthreads();
      int before = 0, tot = 0;
      for (int w = 0; w < nw; ++w) {
        const int c = cnt[w];
        before += w < wid ? c : 0;
        tot += c;
      }
      const int sp = S + before + lanes_below(bal);
      // bit 31 = resolved value, else the chunk position it equals
      unsigned w = 0x80000000u | (unsigned)e;
      if (small && sp != p) {
        const int y = tape_jump(p, sp, lbal & ((1ull << lane) - 1ull), cs + wbase);
        if (y < cs)
          w = 0x80000000u | (unsigned)T[first + y];
        else
          w = (unsigned)(y - cs);
      }
      // inside the wave: shuffles, no barrier
      for (;;) {
        const bool loc = !(w >> 31) && (int)w >= wbase;
        if (!__ballot(loc)) break;
        const unsigned o = __shfl(w, loc ? (int)w - wbase : lane, kWave);
        if (loc) w = o;
      }
      // across waves: publish, barrier, follow; until no word is unresolved
      for (;;) {
        unsigned *cur = bw + (rnd & 1) * kBlockNthMax;
        const int f = rnd % 3;
        cur[tid] = w;
        if (!(w >> 31)) bany[f] = 1;
        if (tid == 0) bany[(rnd + 1) % 3] = 0;  // last read two rounds ago
        __syncthreads();
        const bool more = bany[f] != 0;
        ++rnd;
        if (!more) break;
        NV_COUNT0(15);
        if (!(w >> 31)) w = cur[w & (kBlockNthMax - 1)];
      }
      if (act) T[first + p] = (IdxT)(w & 0x7fffffffu);
      if (small) P[first + sp] = (IdxT)e;
      S += tot;
    }
    __syncthreads();  // the last chunk's T and P before the tape copy
    for (int q = S + tid; q < m; q += bd) {
      const int v = (int)T[first + q];
      P[q == S ? last : first + q] = (IdxT)v;
    }
    if (tid == 0) P[first + S] = (IdxT)pe;
    __syncthreads();
    const int i = first + S;
    if (i == nth) break;
    if (i < nth)
      first = i + 1;
    else
      last = i - 1;
  }
}

// The reference nth_element (utils/kdtree.c:20-52) run serially by one lane:
// Lomuto partition, pivot = last, `cmp <= 0` goes left.
template <class IdxT>
__device__ void lane_nth_element(const double *key, IdxT *P, int first, int last,
                                 int nth) {
  while (first < last) {
    const IdxT pe = P[last];
    const double pk = key[pe];
    int i = first;
    for (int j = first; j < last; ++j) {
      const IdxT ej = P[j];
      if ((key[ej] - pk) <= 0.0) {
        P[j] = P[i];
        P[i] = ej;
        ++i;
      }
    }
    P[last] = P[i];
    P[i] = pe;
    if (i == nth) return;
    if (i < nth)
      first = i + 1;
    else
      last = i - 1;
  }
}

// [lo, hi) = node range k at `depth` below a root range [0, n): walk the
// bits of k down from the root (node of [lo, hi) at lo + (hi - lo) / 2).
__device__ __forceinline__ void kd_node_range(int n, int depth, int k, int &lo, int &hi) {
  lo = 0;
  hi = n;
  for (int b = depth - 1; b >= 0; --b) {
    const int mid = lo + (hi - lo) / 2;
    if ((k >> b) & 1)
      lo = mid + 1;
    else
      hi = mid;
  }
}

constexpr int kLaneSubtree = 32;  // subarrays this short: one lane per subtree
#ifndef NAVGPU_BLOCK_NTH_MIN
#define NAVGPU_BLOCK_NTH_MIN 256
#endif
constexpr int kBlockNthMin = NAVGPU_BLOCK_NTH_MIN;  // root partition by the block from here
#ifndef NAVGPU_BLOCK_LEVEL_MIN
#define NAVGPU_BLOCK_LEVEL_MIN 512
#endif
constexpr int kBlockLevelMin = NAVGPU_BLOCK_LEVEL_MIN;  // deeper levels by the block from here

// buildKDTree over n points, level by level: every subarray of one depth is
// independent. Long subarrays: waves take them round-robin (wave-parallel
// partition passes). Once every subarray at a depth is at most kLaneSubtree
// long, each lane builds whole subtrees serially, level by level inside the
// subtree (subtrees are independent, so the order of their levels is free).
// Root axis = depth0 % 3 (kdtree.c:70, getAxis(depth)).
template <class IdxT, bool GMEM = false, bool LEVELS = true>
__device__ void block_build_kdtree(const double *FC, size_t NS, int n,
                                   IdxT *P, IdxT *T, int depth0) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int nw = blockDim.x / kWave;
  for (int i = threadIdx.x; i < n; i += blockDim.x) P[i] = (IdxT)i;
  __syncthreads();
  int depth = 0;
  NV_STAMP(kb0);
  if (!GMEM && n >= kBlockNthMin && blockDim.x <= kBlockNthMax) {
    // the root partition by the whole block
    block_nth_element<IdxT>(FC + (depth0 % 3) * NS, P, T, 0, n - 1, n / 2);
    depth = 1;
    // levels whose subarrays are still long: each subarray by the whole
    // block in turn (a level of w subarrays would otherwise keep only w
    // waves busy, and its pass chain would be the longest of the build)
    // (512+ thread blocks only; the lean 256-thread K4 kernel shares its CU
    // with a second row and is compiled without this loop, LEVELS = false:
    // with it, 54.2 -> 56.3 ms per 256 pairs)
    for (; LEVELS && (n >> depth) >= kBlockLevelMin && blockDim.x >= 512; ++depth) {
      const double *key = FC + ((depth0 + depth) % 3) * NS;
      for (int k = 0; k < (1 << depth); ++k) {
        int lo, hi;
        kd_node_range(n, depth, k, lo, hi);
        if (hi - lo >= 2) block_nth_element<IdxT>(key, P, T, lo, hi - 1, lo + (hi - lo) / 2);
      }
    }
  }
  NV_STAMP(kb1);
  NV_STAMP_ADD0(9, kb0, kb1);
  for (; (n >> depth) >= 2; ++depth) {
    if ((n >> depth) < kLaneSubtree) break;  // every range at this depth is <= n >> depth
    const double *key = FC + ((depth0 + depth) % 3) * NS;
    const int nodes = 1 << depth;
    for (int k = wid; k < nodes; k += nw) {
      int lo, hi;
      kd_node_range(n, depth, k, lo, hi);
      const int len = hi - lo;
      if (len >= 2) wave_nth_element<IdxT, GMEM>(key, P, T, lo, hi - 1, lo + len / 2, lane);
    }
    __syncthreads();
  }
  NV_STAMP(kb2);
  NV_STAMP_ADD0(10, kb1, kb2);
  if (n >= 2) {
    const int roots = 1 << depth;
    for (int k = threadIdx.x; k < roots; k += blockDim.x) {
      int lo0, hi0;
      kd_node_range(n, depth, k, lo0, hi0);
      const int m = hi0 - lo0;
      for (int d = 0; (m >> d) >= 2; ++d) {
        const double *key = FC + ((depth0 + depth + d) % 3) * NS;
        for (int j = 0; j < (1 << d); ++j) {
          int lo, hi;
          kd_node_range(m, d, j, lo, hi);
          if (hi - lo >= 2)
            lane_nth_element<IdxT>(key, P, lo0 + lo, lo0 + hi - 1, lo0 + lo + (hi - lo) / 2);
        }
      }
    }
    if (GMEM) __threadfence_block();
    __syncthreads();
  }
  NV_STAMP(kb3);
  NV_STAMP_ADD0(11, kb2, kb3);
  NV_STAMP_ADD0(12, 0ull, 1ull);
}

// Stack entry of the far subtree still to visit: [flo, fhi) at depth d; the
// parent node is flo-1 when the far side is the right child, fhi otherwise.
__device__ __forceinline__ uint32_t stk_enc(int flo, int fhi, int right, int d) {
  return (uint32_t)flo | ((uint32_t)fhi << 13) | ((uint32_t)right << 26) |
         ((uint32_t)d << 27);
}

// utils/kdtree.c:110-152 over the implicit tree TX/TY/TZ[0..n): the
// recursion's visit order (node, near subtree, then far subtree iff
// |q[axis]-node[axis]| < best at that moment) with an explicit LIFO stack.
__device__ __forceinline__ void kd_query(const double *TX, const double *TY,
                                         const double *TZ, int n, double qx,
                                         double qy, double qz, uint32_t *stk,
                                         int stride, int *best_pos,
                                         double *best_dist) {
  double best = INFINITY;
  int bpos = -1;
  int lo = 0, hi = n, depth = 0, sp = 0;
  while (true) {
    while (lo < hi) {
      const int mid = lo + ((hi - lo) >> 1);
      const double nx = TX[mid], ny = TY[mid], nz = TZ[mid];
      const double d = ref_dist(nx, ny, nz, qx, qy, qz);
      if (d < best) {
        best = d;
        bpos = mid;
      }
      const int axis = depth % 3;
      const double qa = axis == 0 ? qx : (axis == 1 ? qy : qz);
      const double na = axis == 0 ? nx : (axis == 1 ? ny : nz);
      const bool left = qa < na;
      const int flo = left ? mid + 1 : lo;
      const int fhi = left ? hi : mid;
      if (flo < fhi) stk[(sp++) * stride] = stk_enc(flo, fhi, left ? 1 : 0, depth + 1);
      if (left)
        hi = mid;
      else
        lo = mid + 1;
      ++depth;
    }
    bool resume = false;
    while (sp > 0) {
      const uint32_t e = stk[(--sp) * stride];
      const int flo = e & 0x1fff, fhi = (e >> 13) & 0x1fff;
      const int right = (e >> 26) & 1, d1 = (int)(e >> 27);
      const int parent = right ? flo - 1 : fhi;
      const int axis = (d1 - 1) % 3;
      const double qa = axis == 0 ? qx : (axis == 1 ? qy : qz);
      const double na =
          axis == 0 ? TX[parent] : (axis == 1 ? TY[parent] : TZ[parent]);
      if (fabs(qa - na) < best) {  // kdtree.c:147-151
        lo = flo;
        hi = fhi;
        depth = d1;
        resume = true;
        break;
      }
    }
    if (!resume) break;
  }
  *best_pos = bpos;
  *best_dist = best;
}

// LDS carve-up of the row kernels (byte offsets, 16-B aligned).
struct RowsLds {
  int raw, fc, fcol, p, t, stk, scan, total;
};

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

__host__ __device__ inline RowsLds rows_lds(int C, int nthreads, bool stack) {
  RowsLds L;
  int o = 0;
  L.raw = o;  o += align16(24 * C);
  L.fc = o;   o += align16(24 * C);
  L.fcol = o; o += align16(2 * C);
  L.p = o;    o += align16(2 * C);
  L.t = o;    o += align16(2 * C);
  L.stk = o;  o += stack ? align16(4 * nthreads * kStackDepth) : 0;
  L.scan = o; o += align16(4 * 40);
  L.total = o;
  return L;
}

extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

// Target row r of `coords` (features from `feat_src`): mask -> LDS + global,
// compact features into FC/FCOL, build the exact KD permutation P.
// On return the block is synchronised; returns n.
__device__ int row_stage_and_build(const double *feat_src, const double *coords,
                                   int r, int C, const RowsLds &L,
                                   int32_t *mask_out) {
  double *raw = (double *)(smem + L.raw);
  double *FC = (double *)(smem + L.fc);
  uint16_t *FCOL = (uint16_t *)(smem + L.fcol);
  uint16_t *P = (uint16_t *)(smem + L.p);
  uint16_t *MK = (uint16_t *)(smem + L.t);
  int *scan = (int *)(smem + L.scan);
  const size_t rowoff = (size_t)r * C;
  NV_STAMP(rs0);
  block_copy(raw, feat_src + 3 * rowoff, 3 * C);
  __syncthreads();
  for (int j = threadIdx.x; j < C; j += blockDim.x) {
    const int f = row_curv_lds(raw, C, j) > 0.1 ? 1 : 0;  // src/slam.c:58
    MK[j] = (uint16_t)f;
    if (mask_out) mask_out[rowoff + j] = f;
  }
  __syncthreads();
  const bool same = coords == feat_src;
  const int NS = C;
  const int n = block_compact(
      C, scan, [&](int j) { return MK[j] != 0; },
      [&](int j, int pos) {
        const double *s = same ? raw + 3 * j : coords + 3 * (rowoff + j);
        FC[pos] = s[0];
        FC[NS + pos] = s[1];
        FC[2 * NS + pos] = s[2];
        FCOL[pos] = (uint16_t)j;
      });
  NV_STAMP(rs1);
  NV_STAMP_ADD0(8, rs0, rs1);
#ifdef NAVGPU_DBG_ROWS_NOBUILD  // timing-only ablation: identity "tree"
  for (int i = threadIdx.x; i < n; i += blockDim.x) P[i] = (uint16_t)i;
  __syncthreads();
#else
  block_build_kdtree<uint16_t>(FC, NS, n, P, (uint16_t *)(smem + L.t), 0);
#endif
  return n;
}

// -------------------------------------------------------------- R1 kernel
// up to two clouds per launch (blockIdx.z)
struct CurvJob {
  const double *pts[2];
  int32_t *mask[2];
  double *curv[2];
};

// Each neighbour distance serves two points: d(i, i+1) is point i's p1
// distance and point i+1's m1 distance, d(i, i+2) point i's p2 and point
// i+2's m2 (|a - b| squares to the same bits as |b - a|), so the tile
// computes the two forward distances of every staged point once, in LDS,
// and each point reads its four: two sqrt per point instead of four.
__global__ __launch_bounds__(kCurvTile) void k_curvature(CurvJob J, int R, int C) {
  __shared__ double tile[3 * (kCurvTile + 4)];
  __shared__ double dA[kCurvTile + 4], dB[kCurvTile + 4];  // d(i, i+1), d(i, i+2)
  const int z = blockIdx.z;
  const double *pts = J.pts[z];
  const int r = blockIdx.y;
  const int c0 = blockIdx.x * kCurvTile;
  const int lo = max(0, c0 - 2), hi = min(C, c0 + kCurvTile + 2);
  const size_t rowoff = (size_t)r * C;
  const double *src = pts + 3 * (rowoff + lo);
  const int n = hi - lo, nd = 3 * n;
  for (int i = threadIdx.x; i < nd; i += kCurvTile) tile[i] = src[i];
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += kCurvTile) {
    const double *a = tile + 3 * i;
    if (i + 1 < n) dA[i] = ref_dist(a[0], a[1], a[2], a[3], a[4], a[5]);
    if (i + 2 < n) dB[i] = ref_dist(a[0], a[1], a[2], a[6], a[7], a[8]);
  }
  __syncthreads();
  const int j = c0 + threadIdx.x;
  if (j >= C) return;
  double cv = 0.0;
  if (j >= 2 && j < C - 2) {  // src/slam.c:16-58: k = -2, -1, +1, +2
    const int i = j - lo;
    cv = curvature_of(dB[i - 2], dA[i - 1], dA[i], dB[i]);
  }
  J.mask[z][rowoff + j] = cv > 0.1 ? 1 : 0;
  if (J.curv[z]) J.curv[z][rowoff + j] = cv;
}

// -------------------------------------------------------------- R2 kernel
// utils/pointcloud.c:17-46; tan tables are computed on the host with libm.
__global__ void k_project(const int32_t *__restrict__ depth, int R, int C,
                          const double *__restrict__ tan_col,
                          const double *__restrict__ tan_row,
                          double *__restrict__ pts) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)R * C) return;
  const int row = (int)(i / C), col = (int)(i % C);
  const double d = depth[i];
  double x = 0.0, y = 0.0, z = 0.0;
  if (!(d <= 0)) {
    x = d;
    y = -(d)*tan_col[col];
    z = -(d)*tan_row[row];
  }
  pts[3 * i] = x;
  pts[3 * i + 1] = y;
  pts[3 * i + 2] = z;
}

// -------------------------------------------------------------- R3 kernel
struct Rigid {
  double R[9], t[3], tr[3];
};

__global__ void k_transform(const double *__restrict__ pts, size_t n, Rigid g,
                            double *__restrict__ out,
                            double *__restrict__ out_last) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double lx = pts[3 * i], ly = pts[3 * i + 1], lz = pts[3 * i + 2];
  const double rx = g.R[0] * lx + g.R[1] * ly + g.R[2] * lz;
  const double ry = g.R[3] * lx + g.R[4] * ly + g.R[5] * lz;
  const double rz = g.R[6] * lx + g.R[7] * ly + g.R[8] * lz;
  const double ox = g.t[0] + rx, oy = g.t[1] + ry, oz = g.t[2] + rz;
  out[3 * i] = ox;
  out[3 * i + 1] = oy;
  out[3 * i + 2] = oz;
  if (out_last) {  // src/slam.c:126-128
    out_last[3 * i] = ox - g.tr[0];
    out_last[3 * i + 1] = oy - g.tr[1];
    out_last[3 * i + 2] = oz - g.tr[2];
  }
}

// ------------------------------------------------- fused per-row K2 kernel
// Block = one row of a batch of pairs laid out [pair][R][C]; nn_idx is the
// target's linear index r*C+c within its own pair.
// tie != nullptr: the tie pass after k_rows_screen. Rows none of whose S
// screen splits flagged a tie exit at once; the others build the tree and
// query only the columns the screen left at kTiePending (masks and the other
// columns are already written).
constexpr int32_t kTiePending = -2;

__device__ __forceinline__ bool row_has_tie(const int32_t *tie, int r, int S) {
  int any = 0;
  for (int s = 0; s < S; ++s) any |= tie[(size_t)r * S + s];
  return any != 0;
}

// nn_idx names the reference's answer, a Point (utils/kdtree.c:110-152 returns
// coordinates): the lowest column among the row's target features
// bit-identical to the tree node found at position pos (duplicates, e.g.
// no-return points at the origin, are otherwise told apart by visit order).
__device__ __forceinline__ int canon_col(const double *TX, const double *TY, const double *TZ,
                                         const uint16_t *T, int n, int pos) {
  const long long rx = __double_as_longlong(TX[pos]), ry = __double_as_longlong(TY[pos]),
                  rz = __double_as_longlong(TZ[pos]);
  int best = T[pos];
  for (int p = 0; p < n; ++p)
    if (__double_as_longlong(TX[p]) == rx && __double_as_longlong(TY[p]) == ry &&
        __double_as_longlong(TZ[p]) == rz)
      best = min(best, (int)T[p]);
  return best;
}

__global__ __launch_bounds__(kRowsBlock) void k_rows_match(
    const double *__restrict__ src, const double *__restrict__ tgt, int R,
    int C, int32_t *__restrict__ src_mask, int32_t *__restrict__ tgt_mask,
    int32_t *__restrict__ nn_idx, double *__restrict__ nn_dist,
    const int32_t *__restrict__ tie, int S) {
  const RowsLds L = rows_lds(C, kRowsBlock, true);
  const int r = blockIdx.x;
  if (tie && !row_has_tie(tie, r, S)) return;  // uniform
  const size_t rowoff = (size_t)r * C;
  const int pair_row0 = (r % R) * C;  // this row's offset within its pair
  const int n = row_stage_and_build(tgt, tgt, r, C, L, tgt_mask);
  double *raw = (double *)(smem + L.raw);
  double *FC = (double *)(smem + L.fc);
  uint16_t *FCOL = (uint16_t *)(smem + L.fcol);
  uint16_t *P = (uint16_t *)(smem + L.p);
  uint16_t *T = (uint16_t *)(smem + L.t);
  uint32_t *stk = (uint32_t *)(smem + L.stk);
  int *scan = (int *)(smem + L.scan);
  // materialise the tree in position order: raw <- SoA tree, T <- columns
  double *TX = raw, *TY = raw + C, *TZ = raw + 2 * C;
  for (int pos = threadIdx.x; pos < n; pos += blockDim.x) {
    const int e = P[pos];
    TX[pos] = FC[e];
    TY[pos] = FC[C + e];
    TZ[pos] = FC[2 * C + e];
    T[pos] = FCOL[e];
  }
  __syncthreads();
  // source row (AoS) -> FC region; its mask -> P region; query list -> FCOL
  double *sraw = FC;
  uint16_t *SM = P;
  block_copy(sraw, src + 3 * rowoff, 3 * C);
  __syncthreads();
  for (int j = threadIdx.x; j < C; j += blockDim.x) {
    const int f = row_curv_lds(sraw, C, j) > 0.1 ? 1 : 0;
    SM[j] = (uint16_t)(f && (!tie || nn_idx[rowoff + j] == kTiePending));
    if (src_mask) src_mask[rowoff + j] = f;
    if (!f && !tie) {
      nn_idx[rowoff + j] = -1;
      nn_dist[rowoff + j] = INFINITY;
    }
  }
  __syncthreads();
  uint16_t *QL = FCOL;
  const int nq = block_compact(
      C, scan, [&](int j) { return SM[j] != 0; },
      [&](int j, int pos) { QL[pos] = (uint16_t)j; });
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {
    const int c = QL[i];
    int bpos;
    double bd;
#ifdef NAVGPU_DBG_ROWS_NOQUERY  // timing-only ablation
    bpos = n ? (int)(i % n) : -1;
    bd = sraw[3 * c];
#else
    kd_query(TX, TY, TZ, n, sraw[3 * c], sraw[3 * c + 1], sraw[3 * c + 2],
             stk + threadIdx.x, blockDim.x, &bpos, &bd);
#endif
    nn_idx[rowoff + c] = bpos >= 0 ? pair_row0 + canon_col(TX, TY, TZ, T, n, bpos) : -1;
    nn_dist[rowoff + c] = bd;
  }
}

// K4 batches: the same fused row step with a lean LDS footprint, so that
// several rows share a CU. A row's step is a latency chain (the reference's
// Lomuto passes, then dependent tree walks), so a batch's throughput is set
// by how many rows run on a CU at once. The resident k_rows_match (512
// threads, ~136 KB) fits one per CU. This variant fits two: NT = 256
// threads, the curvature reads the rows straight from global memory (L2)
// instead of staging them, and the tree is permuted in place. Its LDS is the
// SoA features (24 C), FCOL/P/T (6 C) and the walk stacks (4 NT x 14).
// Results are identical to k_rows_match.
constexpr int kLeanMaxC = 2048;  // in-place permutation: <= kLeanMaxC / NT per thread

__host__ __device__ inline int rows_lean_lds(int C, int nt) {
  return align16(24 * C) + 3 * align16(2 * C) + align16(4 * nt * kStackDepth) + align16(4 * 40);
}

// src/slam.c:16-58 for column j of a row read from global memory
__device__ __forceinline__ int row_feature_global(const double *row, int C, int j) {
  if (j < 2 || j >= C - 2) return 0;
  const double *c = row + 3 * j;
  return curvature5(c, c - 6, c - 3, c + 3, c + 6) > 0.1 ? 1 : 0;
}

template <int NT>
__global__ __launch_bounds__(NT) void k_rows_match_lean(
    const double *__restrict__ src, const double *__restrict__ tgt, int R,
    int C, int32_t *__restrict__ src_mask, int32_t *__restrict__ tgt_mask,
    int32_t *__restrict__ nn_idx, double *__restrict__ nn_dist,
    const int32_t *__restrict__ tie, int S) {
  constexpr int kHold = kLeanMaxC / NT;
  const int r = blockIdx.x;
  if (tie && !row_has_tie(tie, r, S)) return;  // uniform
  const size_t rowoff = (size_t)r * C;
  const int pair_row0 = (r % R) * C;
  double *FC = (double *)smem;
  uint16_t *FCOL = (uint16_t *)(smem + align16(24 * C));
  uint16_t *P = (uint16_t *)(smem + align16(24 * C) + align16(2 * C));
  uint16_t *T = (uint16_t *)(smem + align16(24 * C) + 2 * align16(2 * C));
  uint32_t *stk = (uint32_t *)(smem + align16(24 * C) + 3 * align16(2 * C));
  int *scan = (int *)(smem + align16(24 * C) + 3 * align16(2 * C) +
                      align16(4 * NT * kStackDepth));
  // target row: features (flag in T), compacted SoA in column order
  const double *tg = tgt + 3 * rowoff;
  for (int j = threadIdx.x; j < C; j += NT) {
    const int f = row_feature_global(tg, C, j);
    T[j] = (uint16_t)f;
    if (tgt_mask) tgt_mask[rowoff + j] = f;
  }
  __syncthreads();
  const int n = block_compact(
      C, scan, [&](int j) { return T[j] != 0; },
      [&](int j, int pos) {
        FC[pos] = tg[3 * j];
        FC[C + pos] = tg[3 * j + 1];
        FC[2 * C + pos] = tg[3 * j + 2];
        FCOL[pos] = (uint16_t)j;
      });
  block_build_kdtree<uint16_t, false, false>(FC, C, n, P, T, 0);
  // the tree in position order, in place: every old value is read into
  // registers before the barrier, then written to its position
  {
    double hx[kHold], hy[kHold], hz[kHold];
    uint16_t hc[kHold];
#pragma unroll
    for (int u = 0; u < kHold; ++u) {
      const int pos = (int)threadIdx.x + u * NT;
      if (pos < n) {
        const int e = P[pos];
        hx[u] = FC[e];
        hy[u] = FC[C + e];
        hz[u] = FC[2 * C + e];
        hc[u] = FCOL[e];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kHold; ++u) {
      const int pos = (int)threadIdx.x + u * NT;
      if (pos < n) {
        FC[pos] = hx[u];
        FC[C + pos] = hy[u];
        FC[2 * C + pos] = hz[u];
        T[pos] = hc[u];
      }
    }
  }
  // source row: feature flags in P, query list in FCOL
  const double *sg = src + 3 * rowoff;
  for (int j = threadIdx.x; j < C; j += NT) {
    const int f = row_feature_global(sg, C, j);
    P[j] = (uint16_t)(f && (!tie || nn_idx[rowoff + j] == kTiePending));
    if (src_mask) src_mask[rowoff + j] = f;
    if (!f && !tie) {
      nn_idx[rowoff + j] = -1;
      nn_dist[rowoff + j] = INFINITY;
    }
  }
  __syncthreads();
  uint16_t *QL = FCOL;
  const int nq = block_compact(
      C, scan, [&](int j) { return P[j] != 0; },
      [&](int j, int pos) { QL[pos] = (uint16_t)j; });
  const double *TX = FC, *TY = FC + C, *TZ = FC + 2 * C;
  for (int i = threadIdx.x; i < nq; i += NT) {
    const int c = QL[i];
    int bpos;
    double bd;
    kd_query(TX, TY, TZ, n, sg[3 * c], sg[3 * c + 1], sg[3 * c + 2], stk + threadIdx.x, NT,
             &bpos, &bd);
    nn_idx[rowoff + c] = bpos >= 0 ? pair_row0 + canon_col(TX, TY, TZ, T, n, bpos) : -1;
    nn_dist[rowoff + c] = bd;
  }
}

// ------------------------------------------ per-row screen (K2/K4 batches)
// nearestNeighborSearch (utils/kdtree.c:110-152) returns a point of minimum
// reference distance: it skips a far subtree only when |q[a] - node[a]| >=
// best (kdtree.c:147), and every point beyond the node's plane has a computed
// distance >= that difference (rounding is monotone, and sqrt(RN(d*d)) = |d|
// while d*d does not underflow). So when ONE point attains the minimum (no
// other at the same distance as the reference compares them, after sqrt), the
// answer does not depend on the tree at all: it is the argmin.
// The screen finds the minimum and the runner-up of the reference dsq by an
// exact f64 scan over the row's target features, in 32-point chunks with
// bounding boxes: a wave skips a chunk when no lane's runner-up could change.
// A query whose runner-up has the minimum's sqrt (a tie the tree would break
// by visit order), or whose minimum is a positive distance below 1e-150
// (d*d underflows there and the argument above fails), is left at
// kTiePending and its split flags the row; the tie pass (k_rows_match /
// k_rows_match_lean with `tie`) builds the reference tree for those rows only.
// Masks come from k_curvature; tie[r*S + split] is written by every split.
#ifndef NAVGPU_SCREEN_CHUNK
#define NAVGPU_SCREEN_CHUNK 32
#endif
constexpr int kScreenChunk = NAVGPU_SCREEN_CHUNK;

__host__ __device__ inline int rows_screen_lds(int C, int w) {
  const int cp = (C + kScreenChunk - 1) / kScreenChunk * kScreenChunk;
  return 3 * align16(8 * cp) + 2 * align16(2 * C) + align16(48 * (cp / kScreenChunk)) +
         align16(2 * w) + align16(4 * 160);
}

// Stable compaction of columns [c0, c1) with mask[j] != 0, coalesced: thread
// t takes columns j0 + u NT + t, a wave's ranks come from its ballot, and the
// (pass, wave) counts are scanned in LDS, so ranks follow column order
// (flattenPoints, src/slam.c:64-72). U passes are loaded before any is
// ranked. Writes put(j, rank, load(j)) for each kept column and, when rank_at != null,
// rank_at[j] = the number of kept columns before j (every j in [c0, c1)).
// cnt: LDS, >= U * NT / 64 + 1 ints. Returns the count; synchronises.
template <int NT, class Load, class Put>
__device__ int compact_cols(int c0, int c1, const int32_t *__restrict__ mask, Load load,
                            Put put, uint16_t *rank_at, int *cnt) {
  using Val = decltype(load(0));
  constexpr int NW = NT / kWave, U = 4;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  int base = 0;
  for (int j0 = c0; j0 < c1; j0 += U * NT) {
    bool f[U];
    unsigned long long bal[U];
    Val v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * NT + (int)threadIdx.x;
      f[u] = j < c1 && mask[j] != 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // the kept columns' loads, all in flight
      const int j = j0 + u * NT + (int)threadIdx.x;
      if (f[u]) v[u] = load(j);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bal[u] = __ballot(f[u]);
      if (lane == 0) cnt[u * NW + wid] = __popcll(bal[u]);
    }
    __syncthreads();
    if (threadIdx.x < kWave) {  // one wave scans the U * NW counts
      int a = base;
      for (int i0 = 0; i0 < U * NW; i0 += kWave) {
        const int i = i0 + lane;
        const int v = i < U * NW ? cnt[i] : 0;
        int incl = v;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
          const int t = __shfl_up(incl, o, kWave);
          if (lane >= o) incl += t;
        }
        if (i < U * NW) cnt[i] = a + incl - v;
        a += __shfl(incl, kWave - 1, kWave);
      }
      if (lane == 0) cnt[U * NW] = a;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u * NT + (int)threadIdx.x;
      const int rk = cnt[u * NW + wid] + lanes_below(bal[u]);
      if (rank_at && j < c1) rank_at[j] = (uint16_t)rk;
      if (f[u]) put(j, rk, v[u]);
    }
    base = cnt[U * NW];
    __syncthreads();
  }
  return base;
}

// One row's target points in LDS for the exact screen: SoA, padded with
// +inf to whole chunks, with the chunks' bounding boxes.
struct ScreenSet {
  const double *TX, *TY, *TZ, *BOX;
  int nch;
};

// lower bound of the computed dsq between any point of box bx and any query
// of [qlo, qhi] (one query: qlo = qhi): each |fl(p - q)| >= fl(gap) by
// monotone rounding, the same association
__device__ __forceinline__ double screen_box_lb(const double *bx, double qlx, double qhx,
                                                double qly, double qhy, double qlz,
                                                double qhz) {
  const double gx = fmax(fmax(bx[0] - qhx, qlx - bx[1]), 0.0);
  const double gy = fmax(fmax(bx[2] - qhy, qly - bx[3]), 0.0);
  const double gz = fmax(fmax(bx[4] - qhz, qlz - bx[5]), 0.0);
  return gx * gx + gy * gy + gz * gz;
}

// Chunk boxes of TX/TY/TZ[0, n) (NaN coordinates left out: such a point's
// distance is NaN and never taken); 64 / kScreenChunk chunks per wave per
// pass. The caller synchronises before the boxes are read.
template <int NT>
__device__ void screen_boxes(const double *TX, const double *TY, const double *TZ,
                             double *BOX, int n, int nch) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  constexpr int NW = NT / kWave, CPW = kWave / kScreenChunk;
  static_assert(kWave % kScreenChunk == 0, "chunks tile a wave");
  for (int b0 = CPW * wid; b0 < nch; b0 += CPW * NW) {
    const int b = b0 + lane / kScreenChunk, e = b * kScreenChunk + lane % kScreenChunk;
    const bool in = b < nch && e < n;
    double lo[3], hi[3];
    const double v[3] = {in ? TX[e] : NAN, in ? TY[e] : NAN, in ? TZ[e] : NAN};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const bool ok = v[a] == v[a];
      lo[a] = ok ? v[a] : INFINITY;
      hi[a] = ok ? v[a] : -INFINITY;
    }
#pragma unroll
    for (int o = kScreenChunk / 2; o > 0; o >>= 1) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        lo[a] = fmin(lo[a], __shfl_xor(lo[a], o, kWave));
        hi[a] = fmax(hi[a], __shfl_xor(hi[a], o, kWave));
      }
    }
    if (b < nch && lane % kScreenChunk == 0) {
      double *bx = BOX + 6 * b;
      bx[0] = lo[0];
      bx[1] = hi[0];
      bx[2] = lo[1];
      bx[3] = hi[1];
      bx[4] = lo[2];
      bx[5] = hi[2];
    }
  }
}

// The exact screen of one query per lane (called by whole waves): the
// minimum d1 at position j1 and the runner-up d2 of the reference dsq over
// the set. bound2 >= the final runner-up (e.g. the second smallest dsq of
// any subset) prunes chunks before the scan has found two. Chunks s0
// and s1 (wave-uniform, -1: none) are scanned first; then a lane per chunk
// tests the chunk's box against the box of the wave's queries and the
// largest runner-up of its lanes, and only chunks that pass get the
// per-query test and the scan.
__device__ void screen_query(const ScreenSet &T, bool act, double qx, double qy, double qz,
                             int s0, int s1, double &d1, double &d2, int &j1,
                             double bound2 = INFINITY) {
  const int lane = threadIdx.x & (kWave - 1);
  auto scan_chunk = [&](int k) {
    NV_STAMP_ADD(13, 0ull, 1ull);
    const int e0 = k * kScreenChunk;
#pragma unroll 8
    for (int u = 0; u < kScreenChunk; ++u) {
      const int e = e0 + u;
      const double dx = T.TX[e] - qx, dy = T.TY[e] - qy, dz = T.TZ[e] - qz;
      const double d = dx * dx + dy * dy + dz * dz;  // utils/kdtree.c:16
      j1 = d < d1 ? e : j1;
      d2 = fmin(d2, fmax(d1, d));  // a NaN d makes d2 = d1: a (safe) tie
      d1 = fmin(d1, d);
    }
  };
  if (s0 >= 0) scan_chunk(s0);
  if (s1 >= 0 && s1 != s0) scan_chunk(s1);
  const bool qok = act && qx == qx && qy == qy && qz == qz;  // NaN: never matches
  double wl[3] = {qok ? qx : INFINITY, qok ? qy : INFINITY, qok ? qz : INFINITY};
  double wh[3] = {qok ? qx : -INFINITY, qok ? qy : -INFINITY, qok ? qz : -INFINITY};
  double wd2 = qok ? fmin(d2, bound2) : -INFINITY;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      wl[a] = fmin(wl[a], __shfl_xor(wl[a], o, kWave));
      wh[a] = fmax(wh[a], __shfl_xor(wh[a], o, kWave));
    }
    wd2 = fmax(wd2, __shfl_xor(wd2, o, kWave));
  }
  for (int k0 = 0; k0 < T.nch; k0 += kWave) {
    const int kl = k0 + lane;
    bool pass = false;
    if (kl < T.nch && kl != s0 && kl != s1)
      pass = screen_box_lb(T.BOX + 6 * kl, wl[0], wh[0], wl[1], wh[1], wl[2], wh[2]) <= wd2;
    unsigned long long m = __ballot(pass);
    while (m) {
      const int k = k0 + __builtin_ctzll(m);
      m &= m - 1;
      const double lb = screen_box_lb(T.BOX + 6 * k, qx, qx, qy, qy, qz, qz);
      if (__any(act && lb <= fmin(d2, bound2))) scan_chunk(k);
    }
  }
}

// A runner-up at the minimum's distance (after sqrt, as the reference
// compares) is a real tie only if some point in that distance band has
// other coordinates: the reference returns a Point, so bit-identical
// duplicates give the same answer whichever the tree visits first. Rare
// (duplicated no-return points at the origin, integer data), so it is a
// second pass over the chunks that can hold the band. Returns genuine (a
// tie the tree must break) and emin, the lowest position of the duplicates.
__device__ void screen_verify(const ScreenSet &T, bool act, double qx, double qy, double qz,
                              double d1, double d2, int j1, bool &genuine, int &emin) {
  const double dist = __builtin_sqrt(d1);
  const bool suspect = act && d1 < INFINITY && __builtin_sqrt(d2) == dist;
  genuine = false;
  emin = j1;
  if (!__any(suspect)) return;
  const int jr = j1 >= 0 ? j1 : 0;
  const long long rx = __double_as_longlong(T.TX[jr]), ry = __double_as_longlong(T.TY[jr]),
                  rz = __double_as_longlong(T.TZ[jr]);
  for (int k = 0; k < T.nch; ++k) {
    const double lb = screen_box_lb(T.BOX + 6 * k, qx, qx, qy, qy, qz, qz);
    if (!__any(suspect && __builtin_sqrt(lb) <= dist)) continue;
    for (int u = 0; u < kScreenChunk; ++u) {
      const int e = k * kScreenChunk + u;
      const double dx = T.TX[e] - qx, dy = T.TY[e] - qy, dz = T.TZ[e] - qz;
      const double d = dx * dx + dy * dy + dz * dz;
      if (suspect && __builtin_sqrt(d) == dist) {
        const bool same = __double_as_longlong(T.TX[e]) == rx &&
                          __double_as_longlong(T.TY[e]) == ry &&
                          __double_as_longlong(T.TZ[e]) == rz;
        genuine |= !same;
        emin = same ? min(emin, e) : emin;
      }
    }
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_rows_screen(
    const double *__restrict__ src, const double *__restrict__ tgt, int R, int C,
    const int32_t *__restrict__ src_mask, const int32_t *__restrict__ tgt_mask,
    int32_t *__restrict__ nn_idx, double *__restrict__ nn_dist, int32_t *__restrict__ tie) {
  const int r = blockIdx.x, S = gridDim.y, sp = blockIdx.y;
  const int w = (C + S - 1) / S;
  const int c0 = sp * w, c1 = min(C, c0 + w);
  const size_t rowoff = (size_t)r * C;
  const int pair_row0 = (r % R) * C;
  const int cp = (C + kScreenChunk - 1) / kScreenChunk * kScreenChunk;
  double *TX = (double *)smem;
  double *TY = (double *)(smem + align16(8 * cp));
  double *TZ = (double *)(smem + 2 * align16(8 * cp));
  uint16_t *FCOL = (uint16_t *)(smem + 3 * align16(8 * cp));
  uint16_t *RANK = (uint16_t *)(smem + 3 * align16(8 * cp) + align16(2 * C));
  double *BOX = (double *)(smem + 3 * align16(8 * cp) + 2 * align16(2 * C));
  uint16_t *QL = (uint16_t *)((unsigned char *)BOX + align16(48 * (cp / kScreenChunk)));
  int *scan = (int *)((unsigned char *)QL + align16(2 * w));
  NV_STAMP(ss0);
  // target row features, compacted in column order (flattenPoints);
  // RANK[j] = features before column j
  const double *tg = tgt + 3 * rowoff;
  const int n = compact_cols<NT>(
      0, C, tgt_mask + rowoff, [&](int j) { return double3{tg[3 * j], tg[3 * j + 1], tg[3 * j + 2]}; },
      [&](int j, int pos, const double3 &p) {
        TX[pos] = p.x;
        TY[pos] = p.y;
        TZ[pos] = p.z;
        FCOL[pos] = (uint16_t)j;
      },
      RANK, scan);
  NV_STAMP(ss1);
  NV_STAMP_ADD(0, ss0, ss1);
  const int nch = (n + kScreenChunk - 1) / kScreenChunk;
  // the last chunk's tail: +inf coordinates, dsq = inf is never taken
  for (int e = n + (int)threadIdx.x; e < nch * kScreenChunk; e += NT)
    TX[e] = TY[e] = TZ[e] = INFINITY;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  screen_boxes<NT>(TX, TY, TZ, BOX, n, nch);
  NV_STAMP(ss2);
  NV_STAMP_ADD(1, ss1, ss2);
  // this split's source features (block_compact synchronises, so the boxes
  // and the padded tail are visible after it)
  const int32_t *sm = src_mask + rowoff;
  const int nq = compact_cols<NT>(
      c0, c1, sm, [&](int) { return 0; }, [&](int j, int pos, int) { QL[pos] = (uint16_t)j; },
      nullptr, scan);
  for (int j = c0 + (int)threadIdx.x; j < c1; j += NT)
    if (!sm[j]) {
      nn_idx[rowoff + j] = -1;
      nn_dist[rowoff + j] = INFINITY;
    }
  int mytie = 0;
  NV_STAMP(ss3);
  NV_STAMP_ADD(2, ss2, ss3);
  for (int i0 = wid * kWave; i0 < nq; i0 += NT) {  // wave-uniform trip count
    const int i = i0 + lane;
    const bool act = i < nq;
    NV_STAMP_ADD(14, 0ull, 1ull);
    const int c = QL[act ? i : i0];
    const double *qp = src + 3 * (rowoff + c);
    const double qx = qp[0], qy = qp[1], qz = qp[2];
    // start at the chunk holding the first target feature at or after the
    // wave's first query column (scan rows are azimuth sweeps: the nearest
    // point is usually a few columns away)
    const int s = min((int)RANK[QL[i0]] / kScreenChunk, max(nch - 1, 0));
    double d1 = INFINITY, d2 = INFINITY;
    int j1 = -1;
    const ScreenSet T = {TX, TY, TZ, BOX, nch};
    // the two chunks where the wave's columns start, unconditionally
    screen_query(T, act, qx, qy, qz, nch > 0 ? s : -1, nch > 0 ? min(s + 1, nch - 1) : -1,
                 d1, d2, j1);
    const double dist = __builtin_sqrt(d1);
    bool genuine;
    int emin;
    screen_verify(T, act, qx, qy, qz, d1, d2, j1, genuine, emin);
    if (act) {
      const bool t = genuine || (d1 < INFINITY && dist > 0.0 && dist < 1e-150);
      if (t) {
        nn_idx[rowoff + c] = kTiePending;
        mytie = 1;
      } else {
        nn_idx[rowoff + c] = j1 >= 0 ? pair_row0 + (int)FCOL[emin] : -1;
        nn_dist[rowoff + c] = j1 >= 0 ? dist : INFINITY;
      }
    }
  }
  NV_STAMP(ss4);
  NV_STAMP_ADD(3, ss3, ss4);
  const int any = __syncthreads_or(mytie);
  if (threadIdx.x == 0) tie[(size_t)r * S + sp] = any;
}

// ------------------------------------------- split per-row build / query
__global__ __launch_bounds__(kRowsBuildBlock) void k_rows_build(
    const double *__restrict__ feat_src, const double *__restrict__ coords,
    int R, int C, double *__restrict__ tree_pts, int32_t *__restrict__ tree_col,
    int32_t *__restrict__ tree_n, int32_t *__restrict__ mask_out) {
  const RowsLds L = rows_lds(C, kRowsBlock, false);
  const int r = blockIdx.x;
  const size_t rowoff = (size_t)r * C;
  const int n = row_stage_and_build(feat_src, coords, r, C, L, mask_out);
  const double *FC = (const double *)(smem + L.fc);
  const uint16_t *FCOL = (const uint16_t *)(smem + L.fcol);
  const uint16_t *P = (const uint16_t *)(smem + L.p);
  for (int pos = threadIdx.x; pos < n; pos += blockDim.x) {
    const int e = P[pos];
    double *o = tree_pts + 3 * (rowoff + pos);
    o[0] = FC[e];
    o[1] = FC[C + e];
    o[2] = FC[2 * C + e];
    tree_col[rowoff + pos] = FCOL[e];
  }
  if (threadIdx.x == 0) tree_n[r] = n;
}

// Host KDNode images of the per-row trees (navgpu_kd_rows_nodes_dev).
// off[r] = tree_n[0] + ... + tree_n[r-1], off[R] = total: one workgroup,
// each thread a contiguous run of rows, then a scan of the run sums.
constexpr int kOffBlock = 1024;
__global__ __launch_bounds__(kOffBlock) void k_rows_offsets(
    const int32_t *__restrict__ tree_n, int R, int32_t *__restrict__ off) {
  __shared__ int32_t part[kOffBlock];
  const int per = (R + kOffBlock - 1) / kOffBlock;
  const int r0 = min(R, (int)threadIdx.x * per), r1 = min(R, r0 + per);
  int32_t s = 0;
  for (int r = r0; r < r1; ++r) s += tree_n[r];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < kOffBlock; d <<= 1) {  // Hillis-Steele inclusive scan
    const int32_t v = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int32_t acc = part[threadIdx.x] - s;
  for (int r = r0; r < r1; ++r) {
    off[r] = acc;
    acc += tree_n[r];
  }
  if (threadIdx.x == kOffBlock - 1) off[R] = part[kOffBlock - 1];
}

// One thread per tree position: the node of position p in the implicit
// layout (node of [lo,hi) at lo+(hi-lo)/2, utils/kdtree.c:65-82) found by
// descending from the root, its children's host addresses written beside the
// Point so that the image downloads straight into a KDNode array at host_base
// (utils/kdtree.h:7-11: Point point; KDNode *left, *right — 40 bytes).
__global__ __launch_bounds__(256) void k_rows_nodes(
    const double *__restrict__ tree_pts, const int32_t *__restrict__ tree_n,
    const int32_t *__restrict__ off, int C, uint64_t host_base,
    uint64_t *__restrict__ nodes) {
  const int r = blockIdx.y;
  const int p = (int)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = tree_n[r];
  if (p >= n) return;
  int lo = 0, hi = n, mid = n >> 1;
  while (mid != p) {
    if (p < mid)
      hi = mid;
    else
      lo = mid + 1;
    mid = lo + ((hi - lo) >> 1);
  }
  const long long o = off[r];
  const int left = lo < mid ? lo + ((mid - lo) >> 1) : -1;
  const int right = mid + 1 < hi ? mid + 1 + ((hi - mid - 1) >> 1) : -1;
  const double *t = tree_pts + 3 * ((size_t)r * C + p);
  uint64_t *nd = nodes + 5 * (o + p);
  nd[0] = __double_as_longlong(t[0]);
  nd[1] = __double_as_longlong(t[1]);
  nd[2] = __double_as_longlong(t[2]);
  nd[3] = left < 0 ? 0 : host_base + 40ull * (uint64_t)(o + left);
  nd[4] = right < 0 ? 0 : host_base + 40ull * (uint64_t)(o + right);
}

// Per-row 1-NN, each row's columns split over gridDim.y workgroups so a
// frame of R rows fills the chip (R = 128 rows alone would occupy half the
// CUs): every split loads the row's whole tree into LDS (SoA) and its own
// column slice of the query row plus the 2-column curvature halo.
constexpr int kRowsQBlock = 256;

__host__ __device__ inline int rows_query_lds(int C, int w) {
  return align16(24 * C) + align16(24 * (w + 4)) + 4 * kRowsQBlock * kStackDepth;
}

__global__ __launch_bounds__(kRowsQBlock) void k_rows_query(
    const double *__restrict__ tree_pts, const int32_t *__restrict__ tree_n,
    const double *__restrict__ feat_src, const double *__restrict__ queries,
    int R, int C, int32_t *__restrict__ nn_pos, double *__restrict__ nn_dist,
    int32_t *__restrict__ mask_out) {
  const int r = blockIdx.x;
  const int w = (C + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c0 = (int)blockIdx.y * w, c1 = min(C, c0 + w);
  if (c0 >= c1) return;
  const size_t rowoff = (size_t)r * C;
  double *TX = (double *)smem, *TY = TX + C, *TZ = TX + 2 * C;
  double *rs = (double *)(smem + align16(24 * C));
  uint32_t *stk = (uint32_t *)(smem + align16(24 * C) + align16(24 * (w + 4)));
  const int n = tree_n[r];
  for (int pos = threadIdx.x; pos < n; pos += blockDim.x) {
    const double *t = tree_pts + 3 * (rowoff + pos);
    TX[pos] = t[0];
    TY[pos] = t[1];
    TZ[pos] = t[2];
  }
  const int lo = max(c0 - 2, 0), hi = min(c1 + 2, C);  // slice + curvature halo
  block_copy(rs, feat_src + 3 * (rowoff + lo), 3 * (hi - lo));
  __syncthreads();
  for (int j = c0 + (int)threadIdx.x; j < c1; j += blockDim.x) {
    int f = 0;
    if (j >= 2 && j < C - 2) {  // src/slam.c:16 window
      const double *cj = rs + 3 * (j - lo);
      f = curvature5(cj, cj - 6, cj - 3, cj + 3, cj + 6) > 0.1 ? 1 : 0;
    }
    if (mask_out) mask_out[rowoff + j] = f;
    int bpos = -1;
    double bd = INFINITY;
    if (f) {
      const double *q = queries + 3 * (rowoff + j);
      kd_query(TX, TY, TZ, n, q[0], q[1], q[2], stk + threadIdx.x, blockDim.x,
               &bpos, &bd);
    }
    nn_pos[rowoff + j] = bpos;
    nn_dist[rowoff + j] = bd;
  }
}

// k_rows_query without the tree walk (default): the same answers from the
// exact screen over the row's tree points (a set; the tree order only
// decides duplicates, which give the same Point). Each lane first descends
// the implicit tree without backtracking (the nodes on its path are real
// candidates and seed the minimum and runner-up), then screen_query scans
// the chunks that can still matter. Genuine ties (distinct points at the
// minimum distance) and underflowing distances take kd_query, the
// reference walk, on the same LDS tree. nn_pos is a position holding the
// reference's answer (for bit-identical duplicates, the lowest such one).
template <int NT>
__global__ __launch_bounds__(NT) void k_rows_query_screen(
    const double *__restrict__ tree_pts, const int32_t *__restrict__ tree_n,
    const double *__restrict__ feat_src, const double *__restrict__ queries, int R, int C,
    int32_t *__restrict__ nn_pos, double *__restrict__ nn_dist, int32_t *__restrict__ mask_out) {
  const int r = blockIdx.x;
  const int w = (C + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c0 = (int)blockIdx.y * w, c1 = min(C, c0 + w);
  if (c0 >= c1) return;
  const size_t rowoff = (size_t)r * C;
  const int cp = (C + kScreenChunk - 1) / kScreenChunk * kScreenChunk;
  double *TX = (double *)smem;
  double *TY = (double *)(smem + align16(8 * cp));
  double *TZ = (double *)(smem + 2 * align16(8 * cp));
  double *BOX = (double *)(smem + 3 * align16(8 * cp));
  double *rs = (double *)((unsigned char *)BOX + align16(48 * (cp / kScreenChunk)));
  uint16_t *QL = (uint16_t *)((unsigned char *)rs + align16(24 * (w + 4)));
  uint16_t *FL = QL + align16(2 * w) / 2;
  int *scan = (int *)((unsigned char *)FL + align16(2 * w));
  uint32_t *stk = (uint32_t *)((unsigned char *)scan + align16(4 * 40));
  const int n = tree_n[r];
  const int nch = (n + kScreenChunk - 1) / kScreenChunk;
  for (int pos = threadIdx.x; pos < nch * kScreenChunk; pos += NT) {
    if (pos < n) {
      const double *t = tree_pts + 3 * (rowoff + pos);
      TX[pos] = t[0];
      TY[pos] = t[1];
      TZ[pos] = t[2];
    } else {
      TX[pos] = TY[pos] = TZ[pos] = INFINITY;  // dsq = inf: never taken
    }
  }
  const int lo = max(c0 - 2, 0), hi = min(c1 + 2, C);  // slice + curvature halo
  block_copy(rs, feat_src + 3 * (rowoff + lo), 3 * (hi - lo));
  __syncthreads();
  screen_boxes<NT>(TX, TY, TZ, BOX, n, nch);
  for (int j = c0 + (int)threadIdx.x; j < c1; j += NT) {
    int f = 0;
    if (j >= 2 && j < C - 2) {  // src/slam.c:16 window
      const double *cj = rs + 3 * (j - lo);
      f = curvature5(cj, cj - 6, cj - 3, cj + 3, cj + 6) > 0.1 ? 1 : 0;
    }
    FL[j - c0] = (uint16_t)f;
    if (mask_out) mask_out[rowoff + j] = f;
    if (!f) {
      nn_pos[rowoff + j] = -1;
      nn_dist[rowoff + j] = INFINITY;
    }
  }
  __syncthreads();  // flags and boxes visible
  const int nq = block_compact(
      c1 - c0, scan, [&](int j) { return FL[j] != 0; },
      [&](int j, int pos) { QL[pos] = (uint16_t)(c0 + j); });
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const ScreenSet T = {TX, TY, TZ, BOX, nch};
  for (int i0 = wid * kWave; i0 < nq; i0 += NT) {  // wave-uniform trip count
    const int i = i0 + lane;
    const bool act = i < nq;
    const int c = QL[act ? i : i0];
    const double *qp = queries + 3 * (rowoff + c);
    const double qx = qp[0], qy = qp[1], qz = qp[2];
    // bound: the two smallest dsq on the path of a descent without
    // backtracking (utils/kdtree.c:132-145's near branch at every node); the
    // final runner-up can only be smaller. They are a bound only: the scan
    // starts empty, so no point is counted twice (a point counted twice would
    // look like a runner-up at the minimum's distance).
    double e1 = INFINITY, e2 = INFINITY;
    {
      int a0 = 0, a1 = n, depth = 0;
      while (a0 < a1) {
        const int mid = a0 + ((a1 - a0) >> 1);
        const double nx = TX[mid], ny = TY[mid], nz = TZ[mid];
        const double dx = nx - qx, dy = ny - qy, dz = nz - qz;
        const double d = dx * dx + dy * dy + dz * dz;
        // explicit compares: a NaN d changes nothing (e2 must stay >= the
        // true runner-up to be a safe pruning bound)
        if (d < e1) {
          e2 = e1;
          e1 = d;
        } else if (d < e2) {
          e2 = d;
        }
        const int axis = depth % 3;
        const double qa = axis == 0 ? qx : (axis == 1 ? qy : qz);
        const double na = axis == 0 ? nx : (axis == 1 ? ny : nz);
        if (qa < na)
          a1 = mid;
        else
          a0 = mid + 1;
        ++depth;
      }
    }
    double d1 = INFINITY, d2 = INFINITY;
    int j1 = -1;
    screen_query(T, act, qx, qy, qz, -1, -1, d1, d2, j1, e2);
    const double dist = __builtin_sqrt(d1);
    bool genuine;
    int emin;
    screen_verify(T, act, qx, qy, qz, d1, d2, j1, genuine, emin);
    if (act) {
      int bpos = j1 >= 0 ? emin : -1;
      double bd = j1 >= 0 ? dist : INFINITY;
      if (genuine || (d1 < INFINITY && dist > 0.0 && dist < 1e-150))
        kd_query(TX, TY, TZ, n, qx, qy, qz, stk + threadIdx.x, NT, &bpos, &bd);
      nn_pos[rowoff + c] = bpos;
      nn_dist[rowoff + c] = bd;
    }
  }
}

// ---------------------------------------- R5 for one arbitrary array
// kdtree.h buildKDTree: n points, in place, root axis depth0 % 3.
__global__ __launch_bounds__(1024) void k_kd_build_lds(double *__restrict__ pts,
                                                       int n, int depth0) {
  double *FC = (double *)smem;
  uint16_t *P = (uint16_t *)(smem + align16(24 * n));
  uint16_t *T = P + ((align16(2 * n)) / 2);
  for (int i = threadIdx.x; i < 3 * n; i += blockDim.x) {
    const int e = i / 3, a = i % 3;
    FC[a * n + e] = pts[i];
  }
  __syncthreads();
  // without the block-level loop below the root: on arbitrary point sets it
  // costs more than it saves (n = 3000 / 5000: 306 / 546 us with it, 211 /
  // 303 us without, scripts/kd_lds_time.py); it pays on scan rows only
  // (k_rows_build)
#ifdef NAVGPU_KD_LDS_LEVELS  // timing variant: with the loop
  block_build_kdtree<uint16_t>(FC, n, n, P, T, depth0);
#else
  block_build_kdtree<uint16_t, false, false>(FC, n, n, P, T, depth0);
#endif
  for (int i = threadIdx.x; i < 3 * n; i += blockDim.x) {
    const int pos = i / 3, a = i % 3;
    pts[i] = FC[a * n + P[pos]];
  }
}

__global__ __launch_bounds__(1024) void k_kd_build_global(
    double *__restrict__ pts, int n, int depth0, double *__restrict__ FC,
    uint32_t *__restrict__ P, uint32_t *__restrict__ T) {
  for (size_t i = threadIdx.x; i < 3 * (size_t)n; i += blockDim.x) {
    const size_t e = i / 3, a = i % 3;
    FC[a * n + e] = pts[i];
  }
  __syncthreads();
  block_build_kdtree<uint32_t, true>(FC, (size_t)n, n, P, T, depth0);
  for (size_t i = threadIdx.x; i < 3 * (size_t)n; i += blockDim.x) {
    const size_t pos = i / 3, a = i % 3;
    pts[i] = FC[a * (size_t)n + P[pos]];
  }
}

inline int kd_build_lds_bytes(int n) {
  return align16(24 * n) + 2 * align16(2 * n);
}

// ---- buildKDTree for arrays beyond one workgroup's LDS: level-parallel.
// k_kd_prep: SoA key copy + identity permutation. k_kd_level: the
// nth_element of every subarray of one depth, one single-wave workgroup per
// subarray (2^d of them; the reference's Lomuto passes on global P/T).
// k_kd_leaves: once every subarray fits the LDS build, one workgroup builds
// each whole subtree in LDS (root axis = its depth) and writes its points.
__global__ __launch_bounds__(256) void k_kd_prep(const double *__restrict__ pts, int n,
                                                 double *__restrict__ FC,
                                                 uint32_t *__restrict__ P) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)n) return;
  FC[i] = pts[3 * i];
  FC[(size_t)n + i] = pts[3 * i + 1];
  FC[2 * (size_t)n + i] = pts[3 * i + 2];
  P[i] = (uint32_t)i;
}

// ---- Grid-wide Lomuto passes for the top levels of a large build.
// One pass of the reference nth_element (utils/kdtree.c:20-52) over a window
// [first, last] (pivot = P[last], m = last - first positions before it) is
// a stable compaction of the smalls plus the "tape" of the larges: with
// c(p) = smalls before p, tape[p] = elem(p) for a large p and tape[c(p)]
// for a small one; the window becomes smalls | pivot | tape[S+1..m) and
// tape[S] moves to last (the same rule wave_nth_element resolves within a
// wave). Here every window of a level runs at once, each over many
// workgroups: k_sel_count (smalls per chunk), k_sel_rank (ranks from the
// chunk prefix, smalls compacted into Ptmp, tape words into W: bit 31 =
// resolved element, else the position it copies), k_sel_jump (tape chains
// followed kSelHops hops per round, in place: a chain of length M resolves in
// log_kSelHops(M) rounds; a round starts only if the last left work),
// k_sel_scatter (the new window contents), k_sel_update (quickselect's next
// window: i = first + S; done at nth).
constexpr int kSelThreads = 256, kSelPer = 16, kSelChunk = kSelThreads * kSelPer;
constexpr int kSelHops = 64;
constexpr int kSelFinishMax = 8192;  // windows this short finish in one workgroup's LDS
constexpr uint32_t kSelRes = 0x80000000u;

struct SelState {
  int *first, *last, *nth, *act, *S, *pivot, *cnt;  // per window (cnt: [nW][nb])
  int *unres;                                       // per jump round
  int *nact;                                        // active windows after update
  int nb, nW;
};

__global__ __launch_bounds__(256) void k_sel_init(SelState st, int n, int d) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= st.nW) return;
  int lo, hi;
  kd_node_range(n, d, k, lo, hi);
  st.first[k] = lo;
  st.last[k] = hi - 1;
  st.nth[k] = lo + (hi - lo) / 2;
  st.act[k] = hi - lo < 2 ? 0 : (hi - lo <= kSelFinishMax ? 2 : 1);
}

__global__ __launch_bounds__(kSelThreads) void k_sel_count(SelState st,
                                                           const double *__restrict__ key,
                                                           const uint32_t *__restrict__ P) {
  __shared__ int red[kSelThreads / kWave];
  const int k = blockIdx.y, b = blockIdx.x;
  if (st.act[k] != 1) return;
  const int first = st.first[k], last = st.last[k], m = last - first;
  const int p0 = b * kSelChunk;
  if (p0 >= m) return;
  const uint32_t pe = P[last];
  const double pk = key[pe];
  int c = 0;
#pragma unroll 4
  for (int i = 0; i < kSelPer; ++i) {
    const int p = p0 + i * kSelThreads + (int)threadIdx.x;
    if (p < m) c += (key[P[first + p]] - pk) <= 0.0;  // kdtree.c:31-43
  }
  for (int o = kWave / 2; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kSelThreads / kWave; ++w) t += red[w];
    st.cnt[k * st.nb + b] = t;
    if (b == 0) st.pivot[k] = (int)pe;
  }
}

__global__ __launch_bounds__(kSelThreads) void k_sel_rank(SelState st,
                                                          const double *__restrict__ key,
                                                          const uint32_t *__restrict__ P,
                                                          uint32_t *__restrict__ Ptmp,
                                                          uint32_t *__restrict__ W) {
  __shared__ int wc[kSelThreads / kWave + 1];
  __shared__ int sbefore, stotal;
  const int k = blockIdx.y, b = blockIdx.x;
  if (st.act[k] != 1) return;
  const int first = st.first[k], last = st.last[k], m = last - first;
  const int p0 = b * kSelChunk;
  if (p0 >= m) return;
  const int nbk = (m + kSelChunk - 1) / kSelChunk;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (wid == 0) {  // smalls before this chunk, and the window's total
    int bef = 0, tot = 0;
    for (int j = lane; j < nbk; j += kWave) {
      const int c = st.cnt[k * st.nb + j];
      tot += c;
      bef += j < b ? c : 0;
    }
    for (int o = kWave / 2; o > 0; o >>= 1) {
      bef += __shfl_xor(bef, o, kWave);
      tot += __shfl_xor(tot, o, kWave);
    }
    if (lane == 0) {
      sbefore = bef;
      stotal = tot;
    }
  }
  const double pk = key[P[last]];
  __syncthreads();
  int base = sbefore;
  if (b == 0 && threadIdx.x == 0) st.S[k] = stotal;
  for (int i = 0; i < kSelPer; ++i) {
    const int p = p0 + i * kSelThreads + (int)threadIdx.x;
    const bool in = p < m;
    const uint32_t e = in ? P[first + p] : 0u;
    const bool small = in && (key[e] - pk) <= 0.0;
    const unsigned long long bal = __ballot(small);
    if (lane == 0) wc[wid] = __popcll(bal);
    __syncthreads();
    int before = base, tot = 0;
    for (int w = 0; w < kSelThreads / kWave; ++w) {
      before += w < wid ? wc[w] : 0;
      tot += wc[w];
    }
    const int sp = before + lanes_below(bal);
    if (small) Ptmp[first + sp] = e;
    if (in) W[first + p] = (small && sp != p) ? (uint32_t)sp : (kSelRes | e);
    base += tot;
    __syncthreads();
  }
}

// The tape values the window needs are those of [S, m): one position per
// thread follows its chain up to kSelHops hops and stores how far it got.
__global__ __launch_bounds__(kSelThreads) void k_sel_jump0(SelState st, uint32_t *W) {
  const int k = blockIdx.y;
  if (st.act[k] != 1) return;
  const int first = st.first[k], m = st.last[k] - first;
  const int q = st.S[k] + (int)(blockIdx.x * kSelThreads + threadIdx.x);
  int left = 0;
  if (q < m) {
    uint32_t w = W[first + q];
    if (!(w & kSelRes)) {
      for (int h = 0; h < kSelHops && !(w & kSelRes); ++h) w = W[first + (int)w];
      W[first + q] = w;
      left = !(w & kSelRes);
    }
  }
  left = __syncthreads_count(left);
  if (threadIdx.x == 0 && left) atomicAdd(&st.unres[0], left);
}

// Chains k_sel_jump0 left unresolved (long ones only): every position of the
// window jumps kSelHops hops in place, shortening all chains that many
// times; runs only when round - 1 left work.
__global__ __launch_bounds__(kSelThreads) void k_sel_jump(SelState st, uint32_t *W, int round) {
  const int k = blockIdx.y, b = blockIdx.x;
  if (st.act[k] != 1 || (round > 0 && st.unres[round - 1] == 0)) return;
  const int first = st.first[k], m = st.last[k] - first;
  const int p0 = b * kSelChunk;
  if (p0 >= m) return;
  int left = 0;
  for (int i = 0; i < kSelPer; ++i) {
    const int p = p0 + i * kSelThreads + (int)threadIdx.x;
    if (p >= m) break;
    uint32_t w = W[first + p];
    if (w & kSelRes) continue;
    for (int h = 0; h < kSelHops && !(w & kSelRes); ++h) w = W[first + (int)w];
    W[first + p] = w;
    left += !(w & kSelRes);
  }
  left = __syncthreads_count(left > 0);
  if (threadIdx.x == 0 && left) atomicAdd(&st.unres[round], left);
}

__global__ __launch_bounds__(kSelThreads) void k_sel_scatter(SelState st,
                                                             uint32_t *__restrict__ P,
                                                             const uint32_t *__restrict__ Ptmp,
                                                             const uint32_t *__restrict__ W) {
  const int k = blockIdx.y, b = blockIdx.x;
  if (st.act[k] != 1) return;
  const int first = st.first[k], last = st.last[k], m = last - first;
  const int p0 = b * kSelChunk;
  if (p0 >= m) return;
  const int S = st.S[k];  // S == m: no tape, the pivot stays at last
  // a chain the jump rounds left unresolved (only past both rounds' 64^2
  // hops): followed to its end here; W is read-only in this kernel
  auto tape = [&](int q) {
    uint32_t w = W[first + q];
    while (!(w & kSelRes)) w = W[first + (int)w];
    return w & ~kSelRes;
  };
  for (int i = 0; i < kSelPer; ++i) {
    const int p = p0 + i * kSelThreads + (int)threadIdx.x;
    if (p >= m) break;
    if (p < S)
      P[first + p] = Ptmp[first + p];
    else if (p == S) {
      P[first + S] = (uint32_t)st.pivot[k];
      if (S < m) P[last] = tape(S);
    } else
      P[first + p] = tape(p);
  }
}

__global__ __launch_bounds__(256) void k_sel_update(SelState st, int rounds) {
  __shared__ int cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  for (int k = threadIdx.x; k < st.nW; k += blockDim.x) {
    if (st.act[k] != 1) continue;
    const int i = st.first[k] + st.S[k], nth = st.nth[k];
    int a = 1;
    if (i == nth)
      a = 0;
    else if (i < nth)
      st.first[k] = i + 1;
    else
      st.last[k] = i - 1;
    if (st.first[k] >= st.last[k]) a = 0;
    if (a && st.last[k] - st.first[k] + 1 <= kSelFinishMax) a = 2;
    st.act[k] = a;
    if (a == 1) atomicAdd(&cnt, 1);
  }
  if (threadIdx.x < rounds) st.unres[threadIdx.x] = 0;
  __syncthreads();
  if (threadIdx.x == 0) *st.nact = cnt;
}

// The rest of a window's nth_element once it holds <= kSelFinishMax
// positions: the window's ids and keys in LDS, block_nth_element there
// (local indices), the permuted ids written back.
__global__ __launch_bounds__(1024) void k_sel_finish(SelState st, const double *__restrict__ key,
                                                     uint32_t *__restrict__ P) {
  const int k = blockIdx.x;
  if (st.act[k] != 2) return;
  const int first = st.first[k], m = st.last[k] - first + 1;
  double *kl = (double *)smem;
  uint32_t *gid = (uint32_t *)(smem + 8 * kSelFinishMax);
  uint16_t *pl = (uint16_t *)(gid + kSelFinishMax);
  uint16_t *tl = pl + kSelFinishMax;
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    const uint32_t e = P[first + i];
    gid[i] = e;
    kl[i] = key[e];
    pl[i] = (uint16_t)i;
  }
  __syncthreads();
  block_nth_element<uint16_t>(kl, pl, tl, 0, m - 1, st.nth[k] - first);
  for (int i = threadIdx.x; i < m; i += blockDim.x) P[first + i] = gid[pl[i]];
}

// pts[i] = point P[i]: places the upper levels' nodes (the leaves kernel
// then overwrites every leaf subarray with its built subtree)
__global__ __launch_bounds__(256) void k_kd_gather(double *__restrict__ pts,
                                                   const double *__restrict__ FC, int n,
                                                   const uint32_t *__restrict__ P) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)n) return;
  const uint32_t e = P[i];
  pts[3 * i] = FC[e];
  pts[3 * i + 1] = FC[(size_t)n + e];
  pts[3 * i + 2] = FC[2 * (size_t)n + e];
}

__global__ __launch_bounds__(1024) void k_kd_level(const double *__restrict__ FC, int n,
                                                   int depth0, int d, uint32_t *P,
                                                   uint32_t *T) {
  int lo, hi;
  kd_node_range(n, d, (int)blockIdx.x, lo, hi);
  if (hi - lo < 2) return;
  const double *key = FC + (size_t)((depth0 + d) % 3) * n;
  // the block-wide tape pass on global P/T: 1024 positions per step (the
  // barriers order the waves' global writes at workgroup scope)
  block_nth_element<uint32_t, true>(key, P, T, lo, hi - 1, lo + (hi - lo) / 2);
}

__global__ __launch_bounds__(1024) void k_kd_leaves(double *__restrict__ pts,
                                                    const double *__restrict__ FC, int n,
                                                    int depth0, int L,
                                                    const uint32_t *__restrict__ P) {
  int lo, hi;
  kd_node_range(n, L, (int)blockIdx.x, lo, hi);
  const int m = hi - lo;
  if (m <= 0) return;
  double *lf = (double *)smem;  // SoA, m points
  uint16_t *Pl = (uint16_t *)(smem + align16(24 * m));
  uint16_t *Tl = Pl + ((align16(2 * m)) / 2);
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    const uint32_t e = P[lo + i];
    lf[i] = FC[e];
    lf[m + i] = FC[(size_t)n + e];
    lf[2 * m + i] = FC[2 * (size_t)n + e];
  }
  __syncthreads();
  block_build_kdtree<uint16_t, false, false>(lf, m, m, Pl, Tl, (depth0 + L) % 3);  // as k_kd_build_lds
  for (int i = threadIdx.x; i < 3 * m; i += blockDim.x) {
    const int pos = i / 3, a = i % 3;
    pts[3 * (size_t)lo + i] = lf[a * m + Pl[pos]];
  }
}

// ------------------------------------------------- R7: correspondence dedup
// src/slam.c:247-284, one workgroup per row: of the row's feature queries
// that found the same nearest point (coordinate equality, -0.0 == 0.0), the
// kept one is the first (lowest column) at the smallest distance -- what the
// reference's "replace only if strictly closer" list update leaves. Nearest
// points are canonicalised through an LDS hash of the row tree's
// coordinates (first-come owner per distinct coordinate triple), the
// per-point minimum is two LDS atomicMin passes (distance bits, then
// column). Outputs: keep[r*C+c] (1 = kept correspondence; nullable) and the
// row's residual sums over kept pairs, d = ori - near:
//   sums[r*6 + {0,1,2}] = sum d.x, d.y, d.z; [3] = sum |d - mean d|^2 (the
//   centred second moment, mean over the row's kept pairs); [4] = count;
//   [5] = queries of the row that found a nearest point (before the dedup).
// Order-free: the sums are what a closed-form Adam step needs (the
// reference's own sequential sum order is kept by the host path instead).
// A nearest point with a NaN coordinate never matches another (== is false)
// and stays its own correspondence, as in the reference.
constexpr int kCorrBlock = 512;

__device__ __forceinline__ uint64_t corr_key_bits(double v) {
  return (uint64_t)__double_as_longlong(v == 0.0 ? 0.0 : v);
}

__global__ __launch_bounds__(kCorrBlock) void k_rows_corr(
    const double *__restrict__ tree_pts, const int32_t *__restrict__ tree_n,
    const int32_t *__restrict__ nn_pos, const double *__restrict__ nn_dist,
    const double *__restrict__ ori, int C, int HS, int32_t *__restrict__ keep,
    double *__restrict__ sums, double *__restrict__ ent, int32_t *__restrict__ ent_n) {
  extern __shared__ __attribute__((aligned(8))) unsigned char corr_lds[];
  unsigned long long *bdist = (unsigned long long *)corr_lds;  // [HS]
  int *owner = (int *)(bdist + HS);                            // [HS]
  int *bcol = owner + HS;                                      // [HS]
  int *fcol = bcol + HS;                                       // [HS] (ent only)
  int *canon = fcol + HS;                                      // [C]
  __shared__ double red[kCorrBlock / kWave][6];
  __shared__ int cscan[kCorrBlock / kWave + 1];
  const int row = blockIdx.x;
  const size_t base = (size_t)row * C;
  const int n = tree_n[row];
  for (int h = threadIdx.x; h < HS; h += blockDim.x) {
    owner[h] = -1;
    bdist[h] = ~0ull;
    bcol[h] = INT_MAX;
    fcol[h] = INT_MAX;
  }
  __syncthreads();
  // canonical slot of every tree point (-1: a NaN coordinate)
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    const double *tp = tree_pts + 3 * (base + p);
    const double x = tp[0], y = tp[1], z = tp[2];
    if (x != x || y != y || z != z) {
      canon[p] = -1;
      continue;
    }
    uint64_t hh = corr_key_bits(x) * 0x9E3779B97F4A7C15ull;
    hh ^= corr_key_bits(y) + 0x632BE59BD9B4E019ull + (hh << 6) + (hh >> 2);
    hh ^= corr_key_bits(z) + 0x85EBCA77C2B2AE63ull + (hh << 6) + (hh >> 2);
    int h = (int)((hh ^ (hh >> 29)) & (uint64_t)(HS - 1));
    // HS >= 2C > n: the probe always finds a free or matching slot
    for (;;) {
      const int o = atomicCAS(&owner[h], -1, p);
      if (o < 0) break;
      const double *op = tree_pts + 3 * (base + o);
      if (op[0] == x && op[1] == y && op[2] == z) break;
      h = (h + 1) & (HS - 1);
    }
    canon[p] = h;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int pos = nn_pos[base + c];
    if (pos < 0 || pos >= n) continue;
    const int h = canon[pos];
    if (h >= 0) {
      atomicMin(&bdist[h], (unsigned long long)__double_as_longlong(nn_dist[base + c]));
      if (ent) atomicMin(&fcol[h], c);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int pos = nn_pos[base + c];
    if (pos < 0 || pos >= n) continue;
    const int h = canon[pos];
    if (h >= 0 && (unsigned long long)__double_as_longlong(nn_dist[base + c]) == bdist[h])
      atomicMin(&bcol[h], c);
  }
  __syncthreads();
  double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int pos = nn_pos[base + c];
    bool kept = false;
    if (pos >= 0 && pos < n) {
      const int h = canon[pos];
      kept = h < 0 || bcol[h] == c;
      acc[5] += 1.0;
    }
    if (keep) keep[base + c] = kept ? 1 : 0;
    if (kept) {
      const double *a = ori + 3 * (base + c), *b = tree_pts + 3 * (base + pos);
      acc[0] += a[0] - b[0];
      acc[1] += a[1] - b[1];
      acc[2] += a[2] - b[2];
      acc[4] += 1.0;
    }
  }
  auto block_sum = [&](double *v, int nv) {  // every thread gets the block totals
#pragma unroll 1
    for (int k = 0; k < nv; ++k)
      for (int o = kWave / 2; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, kWave);
    __syncthreads();
    if ((threadIdx.x & (kWave - 1)) == 0)
      for (int k = 0; k < nv; ++k) red[threadIdx.x / kWave][k] = v[k];
    __syncthreads();
    for (int k = 0; k < nv; ++k) {
      double t = 0.0;
      for (int w = 0; w < kCorrBlock / kWave; ++w) t += red[w][k];
      v[k] = t;
    }
  };
  block_sum(acc, 6);
  // second pass: the centred second moment sum |d - mean|^2. E(t) =
  // M2 + n |mean - t|^2 then keeps its significant digits when the residuals
  // are small against d itself (the uncentred sum |d|^2 - 2 t.S1 + n|t|^2
  // cancels catastrophically, and can even go negative).
  const double cnt = acc[4];
  const double mx = cnt > 0 ? acc[0] / cnt : 0.0, my = cnt > 0 ? acc[1] / cnt : 0.0,
               mz = cnt > 0 ? acc[2] / cnt : 0.0;
  double m2 = 0.0;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int pos = nn_pos[base + c];
    if (pos < 0 || pos >= n) continue;
    const int h = canon[pos];
    if (!(h < 0 || bcol[h] == c)) continue;
    const double *a = ori + 3 * (base + c), *b = tree_pts + 3 * (base + pos);
    const double ex = (a[0] - b[0]) - mx, ey = (a[1] - b[1]) - my, ez = (a[2] - b[2]) - mz;
    m2 += ex * ex + ey * ey + ez * ez;
  }
  block_sum(&m2, 1);
  if (sums && threadIdx.x < 6)
    sums[(size_t)row * 6 + threadIdx.x] = threadIdx.x == 3 ? m2 : acc[threadIdx.x];
  if (!ent) return;
  // the row's correspondence list in the reference's order: an entry per
  // distinct nearest point at its FIRST query's column (src/slam.c:247-281
  // appends there), holding the KEPT query (smallest distance, then first
  // column: the in-place replacements leave that one). A NaN point is an
  // entry of its own. ent[(row*C + rank)*7]: oriPoint, nearestPoint, distance
  // (the NeighborResult layout, utils/kdtree.h); ent_n[row] = the count.
  const int ne = block_compact(
      C, cscan,
      [&](int c) {
        const int pos = nn_pos[base + c];
        if (pos < 0 || pos >= n) return false;
        const int h = canon[pos];
        return h < 0 || fcol[h] == c;
      },
      [&](int c, int rank) {
        const int h = canon[nn_pos[base + c]];
        const int kc = h < 0 ? c : bcol[h];
        const int kp = nn_pos[base + kc];
        const double *a = ori + 3 * (base + kc), *b = tree_pts + 3 * (base + kp);
        double *e = ent + 7 * (base + rank);
        e[0] = a[0];
        e[1] = a[1];
        e[2] = a[2];
        e[3] = b[0];
        e[4] = b[1];
        e[5] = b[2];
        e[6] = nn_dist[base + kc];
      });
  if (threadIdx.x == 0) ent_n[row] = ne;
}

// Concatenates the rows' lists of k_rows_corr (row order) into list[7 * i];
// count[0] = entries, count[1] = queries that found a nearest point.
__global__ __launch_bounds__(256) void k_corr_pack(const double *__restrict__ ent,
                                                   const int32_t *__restrict__ ent_n,
                                                   const double *__restrict__ sums, int R,
                                                   int C, double *__restrict__ list,
                                                   int32_t *__restrict__ count) {
  __shared__ int part[256 / kWave + 1];
  const int row = blockIdx.x;
  int off = 0;
  for (int r = threadIdx.x; r < row; r += blockDim.x) off += ent_n[r];
  int total;
  (void)block_excl_scan(off, part, &total);
  off = total;
  const int n = ent_n[row];
  const double *src = ent + 7 * (size_t)row * C;
  double *dst = list + 7 * (size_t)off;
  for (int i = threadIdx.x; i < 7 * n; i += blockDim.x) dst[i] = src[i];
  if (row == R - 1 && threadIdx.x == 0) {
    count[0] = off + n;
    double q = 0.0;
    for (int r = 0; r < R; ++r) q += sums[6 * (size_t)r + 5];
    count[1] = (int32_t)q;
  }
}

// ============================================================ global mode
// Uniform grid over the target cloud. Cells are numbered x-fastest, so the
// cells x-1..x+1 of one (y,z) row are contiguous in the cell-sorted target
// array: a query's 3x3x3 neighbourhood is 9 contiguous "runs".
struct GridParams {
  double o[3];      // origin = target bbox min
  double e[3], inv_e[3];  // cell edge per axis: x h / sx, y and z h
  double h;         // the coarse edge
  double delta;     // slack on cell boxes (cell assignment is f64 arithmetic)
  double emax;      // largest bbox extent
  int g[3];
  int ncells;
  int sx;           // x cells per h: a query's block is cells x-sx .. x+sx,
                    // y-1 .. y+1, z-1 .. z+1 (the reach is >= h on every axis)
  int tile_w;       // cells per k_knn tile along x
};

// soff entries per staged row of a k_knn tile (W + 2 sx + 1 <= kTileCols)
#ifndef NAVGPU_TILE_COLS
#define NAVGPU_TILE_COLS 136
#endif
constexpr int kTileCols = NAVGPU_TILE_COLS;
constexpr int kMaxSx = 8;
#ifndef NAVGPU_KNN_SX
#define NAVGPU_KNN_SX 1  // sx = 2: query stage 183 -> 177 us, build 99 -> 109 us (K3)
#endif
#ifndef NAVGPU_TILE_QUERIES
#define NAVGPU_TILE_QUERIES 165.0  // target queries per k_knn tile
#endif
#ifndef NAVGPU_TILE_REC
#define NAVGPU_TILE_REC 1600
#endif

struct __align__(16) Rec16 {  // cell-sorted target: (coords - origin) in f32
  float x, y, z;
  int cx;  // x index of its grid cell (the f64 binning's, exact)
};
struct __align__(16) TRec {  // cell-sorted target, exact: the reference f64 point + its index
  double x, y, z;
  int idx, pad;
};

constexpr int kBBoxBlocks = 1024;
constexpr int kKeyBits = 10;  // local id in the low bits of a key: run (4) | offset (6)
constexpr uint32_t kKeyMask = (1u << kKeyBits) - 1;
constexpr uint32_t kNoKey = 0xffffffffu;

// per-block min/max of the finite coordinates -> part[block][6]
__global__ __launch_bounds__(256) void k_bbox_partial(const double *__restrict__ p,
                                                      size_t n, double *__restrict__ part) {
  __shared__ double s[4][6];
  double v6[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  // batches of 4 points per thread, all loads of a batch in flight together
  // (flat 16-B loads of the 3n doubles measured the same, r2)
  constexpr int U = 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t ib = (size_t)blockIdx.x * blockDim.x + threadIdx.x; ib < n; ib += U * stride) {
    double v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = ib + u * stride;
#pragma unroll
      for (int a = 0; a < 3; ++a) v[u][a] = i < n ? p[3 * i + a] : INFINITY;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int a = 0; a < 3; ++a)
        if (fabs(v[u][a]) < INFINITY) {
          v6[a] = fmin(v6[a], v[u][a]);
          v6[3 + a] = fmax(v6[3 + a], v[u][a]);
        }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a)
    for (int o = kWave / 2; o > 0; o >>= 1) {
      v6[a] = fmin(v6[a], __shfl_xor(v6[a], o, kWave));
      v6[3 + a] = fmax(v6[3 + a], __shfl_xor(v6[3 + a], o, kWave));
    }
  const int wid = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0)
    for (int a = 0; a < 6; ++a) s[wid][a] = v6[a];
  __syncthreads();
  if (threadIdx.x < 6) {
    const int a = threadIdx.x;
    double r = s[0][a];
    for (int w = 1; w < 4; ++w) r = a < 3 ? fmin(r, s[w][a]) : fmax(r, s[w][a]);
    part[blockIdx.x * 6 + a] = r;
  }
}

// bbox from the partials, then the grid: h for ~occ points per cell, capped
// at `cap` cells.
__global__ __launch_bounds__(256) void k_grid_params(const double *__restrict__ part,
                                                     int nparts, size_t n, int cap,
                                                     double occ, int sx, size_t nq,
                                                     GridParams *gp, int *counters) {
  // also resets the call's k-NN counters (overflow tiles, slow queries): one
  // launch fewer than a memset
  if (threadIdx.x < 4) counters[threadIdx.x] = 0;
  __shared__ double s[4][6];
  double v6[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int b = threadIdx.x; b < nparts; b += blockDim.x)
    for (int a = 0; a < 6; ++a)
      v6[a] = a < 3 ? fmin(v6[a], part[b * 6 + a]) : fmax(v6[a], part[b * 6 + a]);
#pragma unroll
  for (int a = 0; a < 3; ++a)
    for (int o = kWave / 2; o > 0; o >>= 1) {
      v6[a] = fmin(v6[a], __shfl_xor(v6[a], o, kWave));
      v6[3 + a] = fmax(v6[3 + a], __shfl_xor(v6[3 + a], o, kWave));
    }
  if ((threadIdx.x & (kWave - 1)) == 0)
    for (int a = 0; a < 6; ++a) s[threadIdx.x / kWave][a] = v6[a];
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int w = 1; w < (int)blockDim.x / kWave; ++w)
    for (int a = 0; a < 6; ++a)
      v6[a] = a < 3 ? fmin(v6[a], s[w][a]) : fmax(v6[a], s[w][a]);
  GridParams G;
  double lo[3], ext[3];
  bool any = n > 0;
  for (int a = 0; a < 3; ++a) {
    if (!(v6[a] <= v6[3 + a])) any = false;
    lo[a] = v6[a];
    ext[a] = v6[3 + a] - v6[a];
  }
  if (!any) {
    for (int a = 0; a < 3; ++a) {
      G.o[a] = 0.0;
      G.g[a] = 1;
      G.e[a] = G.inv_e[a] = 1.0;
    }
    G.h = G.delta = 1.0;
    G.sx = 1;
    G.emax = 0.0;
    G.ncells = 1;
    G.tile_w = 1;
    *gp = G;
    return;
  }
  const double emax = fmax(ext[0], fmax(ext[1], ext[2]));
  const double floor_e = fmax(emax * 1e-3, 1e-9);
  double vol = 1.0;
  for (int a = 0; a < 3; ++a) vol *= fmax(ext[a], floor_e);
  double h = cbrt(vol * occ / (double)n);
  if (!(h > 0) || !(h < INFINITY)) h = fmax(emax, 1.0);
  int g[3];
  for (int it = 0; it < 200; ++it) {
    long long tot = 1;
    for (int a = 0; a < 3; ++a) {
      const double ea = a == 0 ? h / sx : h;
      double ga = floor(ext[a] / ea) + 1.0;  // covers [lo, lo + ext] inclusive
      if (ga > 2048) ga = 2048;
      g[a] = (int)ga;
      tot *= g[a];
    }
    if (tot <= cap) break;
    h *= 1.1;
  }
  for (int a = 0; a < 3; ++a) G.o[a] = lo[a];
  G.h = h;
  G.sx = sx;
  for (int a = 0; a < 3; ++a) {
    G.e[a] = a == 0 ? h / sx : h;
    G.inv_e[a] = 1.0 / G.e[a];
  }
  G.delta = 1e-7 * (emax + h);
  G.emax = emax;
  G.g[0] = g[0];
  G.g[1] = g[1];
  G.g[2] = g[2];
  G.ncells = g[0] * g[1] * g[2];
  // tile width: ~165 queries per 192-thread tile, and its 9 staged row
  // segments of W + 2 sx cells within ~90 % of the LDS record budget
  const double occ_q = (double)nq / G.ncells, occ_t = (double)n / G.ncells;
  double w = fmin(NAVGPU_TILE_QUERIES / fmax(occ_q, 1e-9),
                  0.9 * NAVGPU_TILE_REC / (9.0 * fmax(occ_t, 1e-9)) - 2.0 * sx);
  // balanced: the fewest tiles per grid row at that width, then equal widths
  // (a ragged last tile would pay a full staging + barrier cycle for a few
  // cells)
  const int wmax = (int)fmax(1.0, fmin((double)(kTileCols - 1 - 2 * sx), floor(w)));
  const int tpr = (G.g[0] + wmax - 1) / wmax;
  G.tile_w = (G.g[0] + tpr - 1) / tpr;
  *gp = G;
}

__device__ __forceinline__ int cell_axis(double v, const GridParams &G, int a) {
  const double t = (v - G.o[a]) * G.inv_e[a];
  if (!(t >= 0.0)) return 0;  // below the grid, or NaN
  if (t >= (double)G.g[a]) return G.g[a] - 1;
  return (int)t;
}

__device__ __forceinline__ int cell_of(const double *p, const GridParams &G) {
  return (cell_axis(p[2], G, 2) * G.g[1] + cell_axis(p[1], G, 1)) * G.g[0] +
         cell_axis(p[0], G, 0);
}

constexpr int kScanBlock = 1024, kScanPer = 4,
              kScanTile = kScanBlock * kScanPer;

__global__ __launch_bounds__(kScanBlock) void k_scan_sums(
    const int *__restrict__ in, int n, int *__restrict__ bsum) {
  __shared__ int scratch[40];
  const int base = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
  int s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k)
    if (base + k < n) s += in[base + k];
  int total;
  block_excl_scan(s, scratch, &total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanBlock) void k_scan_apply(
    const int *__restrict__ in, int n, const int *__restrict__ bsum,
    int *__restrict__ out) {
  __shared__ int scratch[40];
  const int base = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
  int v[kScanPer];
  int s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    v[k] = base + k < n ? in[base + k] : 0;
    s += v[k];
  }
  // this block's offset: the sum of the block totals before it, read straight
  // from bsum (at most kScanTile of them; a separate top-level scan launch
  // costs more than these few reads)
  int pre = 0;
  for (int i = threadIdx.x; i < (int)blockIdx.x; i += blockDim.x) pre += bsum[i];
  int total, ptot;
  block_excl_scan(pre, scratch, &ptot);
  __syncthreads();  // scratch is reused by the next scan
  int off = block_excl_scan(s, scratch, &total) + ptot;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (base + k < n) out[base + k] = off;
    off += v[k];
  }
}

// ---- cell binning: counting sort of both clouds by grid cell --------------
// Scattered global atomics run at the memory side on this part (~24 G/s
// whatever their scope), so the sort uses none: LDS histograms and LDS ranks
// only.
//  k_bin_hist    each block takes a contiguous chunk of points and counts
//                their coarse bucket (cell >> shift) in LDS; counts land in a
//                bucket-major table[b * nblk + block], so ONE exclusive scan
//                of the table gives every (bucket, block) its output offset.
//  k_bin_scatter same chunks: each point gets an LDS rank within its
//                (bucket, block) and moves to the coarse-bucketed array.
//  k_bin_fine    one block per bucket: LDS counting sort over the bucket's
//                2^shift cells, writes start[] for them and every point at its
//                final cell-sorted position (target: Rec16 + TRec;
//                query: its index). Order inside a cell is unspecified: the
//                k-NN result does not depend on it (ties are resolved by
//                (distance, index) in the exact stage).
// Side 0 = targets, side 1 = queries; both are handled by the same launches
// (block ranges), and their tables are concatenated so one scan covers both.
struct BinPt {
  double x, y, z;
  int idx, cell;
};
struct BinSide {
  const double *p;
  int n, P, nblk;
  int tab;  // offset of this side's table in the concatenated table
  int sub;  // subtracted from scanned offsets (targets' total, for side 1)
  int *start;
};
struct BinJob {
  BinSide s[2];
  int shift, nb;  // buckets per side
  BinPt *bin_t;
  int2 *bin_q;    // (idx, cell)
  Rec16 *rec;
  TRec *tsort;
  int *qperm;
};
constexpr int kBinMaxBuckets = 4096;
constexpr int kBinMaxShift = 15;

__device__ __forceinline__ int bin_side(const BinJob &J, int &blk) {
  const int side = blk >= J.s[0].nblk ? 1 : 0;
  if (side) blk -= J.s[0].nblk;
  return side;
}

#ifndef NAVGPU_BIN_UNROLL
#define NAVGPU_BIN_UNROLL 8
#endif
// points per thread with loads in flight (r2 sweep: 4 / 8 / 16 -> isolated
// build 97 / 98 / 96 us, but the two-in-flight bench step 0.2805 ms with 16
// against 0.2767 with 8: the build shares the chip with a query stage there)
constexpr int kBinUnroll = NAVGPU_BIN_UNROLL;

struct P3 {
  double x, y, z;
};

// the block's chunk in batches of kBinUnroll points per thread: every load of
// a batch is issued before any of its cells is used, so a wave keeps
// kBinUnroll x 24 B per lane in flight instead of one point's worth
template <class F>
__device__ __forceinline__ void bin_chunk(const BinSide &S, int blk, const GridParams &G, F f) {
  const int i0 = blk * S.P, i1 = min(S.n, (blk + 1) * S.P);
  const int bd = (int)blockDim.x;
  for (int ib = i0; ib < i1; ib += kBinUnroll * bd) {
    P3 v[kBinUnroll];
#pragma unroll
    for (int u = 0; u < kBinUnroll; ++u) {
      const int i = ib + u * bd + (int)threadIdx.x;
      if (i < i1) v[u] = *(const P3 *)(S.p + 3 * (size_t)i);
    }
#pragma unroll
    for (int u = 0; u < kBinUnroll; ++u) {
      const int i = ib + u * bd + (int)threadIdx.x;
      if (i < i1) f(i, v[u], cell_of(&v[u].x, G));
    }
  }
}

__global__ __launch_bounds__(256) void k_bin_hist(BinJob J,
                                                  const GridParams *__restrict__ gp,
                                                  int *__restrict__ table) {
  __shared__ int hist[kBinMaxBuckets];
  int blk = blockIdx.x;
  const BinSide S = J.s[bin_side(J, blk)];
  const GridParams G = *gp;
  for (int b = threadIdx.x; b < J.nb; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  bin_chunk(S, blk, G, [&](int, const P3 &, int c) { atomicAdd(&hist[c >> J.shift], 1); });
  __syncthreads();
  for (int b = threadIdx.x; b < J.nb; b += blockDim.x)
    table[S.tab + b * S.nblk + blk] = hist[b];
  if (blk == 0 && threadIdx.x == 0) table[S.tab + J.nb * S.nblk] = 0;  // sentinel
}

__global__ __launch_bounds__(256) void k_bin_scatter(BinJob J,
                                                     const GridParams *__restrict__ gp,
                                                     const int *__restrict__ offs) {
  __shared__ int cur[kBinMaxBuckets];
  int blk = blockIdx.x;
  const int side = bin_side(J, blk);
  const BinSide S = J.s[side];
  const GridParams G = *gp;
  for (int b = threadIdx.x; b < J.nb; b += blockDim.x)
    cur[b] = offs[S.tab + b * S.nblk + blk] - S.sub;
  __syncthreads();
  bin_chunk(S, blk, G, [&](int i, const P3 &v, int c) {
    const int pos = atomicAdd(&cur[c >> J.shift], 1);
    if (side == 0) {
      BinPt t;
      t.x = v.x;
      t.y = v.y;
      t.z = v.z;
      t.idx = i;
      t.cell = c;
      J.bin_t[pos] = t;
    } else {
      J.bin_q[pos] = make_int2(i, c);
    }
  });
}

#ifndef NAVGPU_BIN_P
#define NAVGPU_BIN_P 4096  // minimum points per k_bin_hist / k_bin_scatter block
#endif
#ifndef NAVGPU_BIN_FINE_THREADS
#define NAVGPU_BIN_FINE_THREADS 512
#endif
#ifndef NAVGPU_BIN_MIN_SHIFT
// coarse buckets of 2^10 cells (r2 two-in-flight bench A/B, two sessions of
// 3 interleaved runs: 9 -> 0.2745 / 0.2744 ms, 10 -> 0.2716 / 0.2733, 11 ->
// 0.2942; profiles/r2/bench_ab_r2l.txt)
#define NAVGPU_BIN_MIN_SHIFT 10
#endif
constexpr int kBinFineThreads = NAVGPU_BIN_FINE_THREADS;

constexpr int kBinFineHold = 4096 / kBinFineThreads;  // points per thread held in registers

// One bucket: count its points per cell (LDS), scan, write the cell starts,
// then place every point. The first kBinFineHold * blockDim points stay in
// registers between the count and the placement (one global read, not two);
// a larger bucket re-reads the rest.
template <bool QSIDE>
__device__ void bin_fine_bucket(const BinJob &J, const BinSide &S, const GridParams *gp,
                                int lo, int hi, int base, int ncell, int nscan, int *cnt,
                                int *scratch) {
  typedef typename std::conditional<QSIDE, int2, BinPt>::type E;
  const E *src = QSIDE ? (const E *)J.bin_q : (const E *)J.bin_t;
  auto cell_of_e = [](const E &e) {
    if constexpr (QSIDE) return e.y; else return e.cell;
  };
  for (int j = threadIdx.x; j < ncell; j += blockDim.x) cnt[j] = 0;
  __syncthreads();
  E hold[kBinFineHold];
  const int bd = (int)blockDim.x, held_end = min(hi, lo + kBinFineHold * bd);
#pragma unroll
  for (int u = 0; u < kBinFineHold; ++u) {
    const int i = lo + u * bd + (int)threadIdx.x;
    if (i < held_end) hold[u] = src[i];
  }
#pragma unroll
  for (int u = 0; u < kBinFineHold; ++u) {
    const int i = lo + u * bd + (int)threadIdx.x;
    if (i < held_end) atomicAdd(&cnt[cell_of_e(hold[u]) - base], 1);
  }
  for (int i = held_end + (int)threadIdx.x; i < hi; i += bd)
    atomicAdd(&cnt[cell_of_e(src[i]) - base], 1);
  __syncthreads();
  // exclusive scan over the bucket's cells: each thread owns a contiguous run
  const int per = ncell / bd;  // ncell is a multiple of the block size
  const int j0 = (int)threadIdx.x * per;
  int sum = 0;
  for (int u = 0; u < per; ++u) sum += cnt[j0 + u];
  int total;
  int acc = lo + block_excl_scan(sum, scratch, &total);
  for (int u = 0; u < per; ++u) {
    const int v = cnt[j0 + u];
    cnt[j0 + u] = acc;
    if (base + j0 + u < nscan) S.start[base + j0 + u] = acc;
    acc += v;
  }
  __syncthreads();
  const GridParams G = *gp;
  auto place = [&](const E &e) {
    if constexpr (QSIDE) {
      J.qperm[atomicAdd(&cnt[e.y - base], 1)] = e.x;
    } else {
      const int pos = atomicAdd(&cnt[e.cell - base], 1);
      TRec t;
      t.x = e.x;
      t.y = e.y;
      t.z = e.z;
      t.idx = e.idx;
      t.pad = 0;
      J.tsort[pos] = t;
      Rec16 r;
      r.x = (float)(e.x - G.o[0]);
      r.y = (float)(e.y - G.o[1]);
      r.z = (float)(e.z - G.o[2]);
      r.cx = e.cell % G.g[0];
      J.rec[pos] = r;
    }
  };
#pragma unroll
  for (int u = 0; u < kBinFineHold; ++u) {
    const int i = lo + u * bd + (int)threadIdx.x;
    if (i < held_end) place(hold[u]);
  }
  for (int i = held_end + (int)threadIdx.x; i < hi; i += bd) place(src[i]);
}

__global__ __launch_bounds__(kBinFineThreads) void k_bin_fine(
    BinJob J, const GridParams *__restrict__ gp, const int *__restrict__ offs,
    int nscan) {
  extern __shared__ int cnt[];  // 2^shift
  __shared__ int scratch[40];
  const int side = blockIdx.x >= J.nb ? 1 : 0;
  const int b = blockIdx.x - (side ? J.nb : 0);
  const BinSide S = J.s[side];
  const int ncell = 1 << J.shift, base = b << J.shift;
  const int lo = offs[S.tab + b * S.nblk] - S.sub;
  const int hi = offs[S.tab + (b + 1) * S.nblk] - S.sub;
  if (side)
    bin_fine_bucket<true>(J, S, gp, lo, hi, base, ncell, nscan, cnt, scratch);
  else
    bin_fine_bucket<false>(J, S, gp, lo, hi, base, ncell, nscan, cnt, scratch);
}

// (d, i) < (kd, ki): distance first, then index. Never true for d = inf/NaN.
__device__ __forceinline__ bool knn_less(double d, int i, double kd, int ki) {
  return d < kd || (d == kd && i < ki);
}

// squared distance from q to the box of cells [x0..x1] x [y0..y1] x [z0..z1]
// grown by delta: a lower bound on the reference dsq of any point binned there
__device__ __forceinline__ double box_d2(const GridParams &G, const double *qv,
                                         int x0, int x1, int y0, int y1, int z0,
                                         int z1) {
  const int lo[3] = {x0, y0, z0}, hi[3] = {x1, y1, z1};
  double s = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double bl = G.o[a] + lo[a] * G.e[a] - G.delta;
    const double bh = G.o[a] + (hi[a] + 1) * G.e[a] + G.delta;
    // boundary cells also hold everything clamped into them
    const double e = fmax(0.0, fmax(lo[a] > 0 ? bl - qv[a] : 0.0,
                                     hi[a] < G.g[a] - 1 ? qv[a] - bh : 0.0));
    s += e * e;
  }
  return s;
}

// Distance from q (in cell c) to the outside of its block of radius r: cells
// x - r sx .. x + r sx, y - r .. y + r, z - r .. z + r. A block face on the
// grid boundary does not count (the boundary cells hold everything clamped
// into them); INFINITY when every face is.
__device__ __forceinline__ double block_reach(const GridParams &G, const double *qv,
                                              const int c[3], int r) {
  double L = INFINITY;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int ra = a == 0 ? r * G.sx : r;
    if (c[a] - ra > 0) L = fmin(L, qv[a] - (G.o[a] + (c[a] - ra) * G.e[a]));
    if (c[a] + ra < G.g[a] - 1) L = fmin(L, (G.o[a] + (c[a] + ra + 1) * G.e[a]) - qv[a]);
  }
  return L;
}

// f32 admission bound for an f64 dsq bound T: every candidate whose exact
// dsq is <= T has an f32 dsq (coordinates relative to the grid origin, each
// f32 difference within dl of the exact one) <= the returned value.
__device__ __forceinline__ float f32_bound(double T, double dl) {
  if (!(T < INFINITY)) return INFINITY;
  const double E = T * 0x1p-20 + 4.0 * dl * __builtin_sqrt(T) + 4.0 * dl * dl;
  return (float)((T + E) * (1.0 + 0x1p-20));
}

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  return max(min(a, b), min(max(a, b), c));
}

// (dy, dz) of the 9 runs of a 3x3x3 neighbourhood: centre, faces, corners
__device__ __forceinline__ void run_dydz(int r, int &dy, int &dz) {
  dy = r == 0 ? 0 : (r == 1 ? -1 : (r == 2 ? 1 : (r <= 4 ? 0 : (r & 1 ? -1 : 1))));
  dz = r <= 2 ? 0 : (r == 3 ? -1 : (r == 4 ? 1 : (r <= 6 ? -1 : 1)));
}

// One query of the global-mode k-NN.
// Fast path over the query's 3x3x3 cell neighbourhood, taken as 9 runs: the
// three cells x-1..x+1 of one (y, z) row are contiguous in the cell-sorted
// arrays, so each run is one record range (own row first, then faces, then
// corners). Each candidate gets an f32 distance (coordinates relative to the
// grid origin) packed with its local id (run | offset) into a 32-bit key; a
// sorted list of the K+1 smallest keys is kept by branch-free median-of-3
// insertion. The K+1 survivors are then re-evaluated with the reference f64
// formula and ordered by (distance, index); the result is certified exact when
// every candidate left out (visited but not kept, or outside the block) is
// provably farther than the K-th, using the f32 error bound. Otherwise (near
// ties, a neighbourhood reaching past the block, overfull runs) the query is
// queued for k_knn_slow with the K-th distance found as its starting bound.
// runs(r, t0, t1, g0): record range [t0, t1) of run r in the index space of
// the fetches and g0 = the global (cell-sorted) position of record t0.
// pair(t): packed coordinates of records t, t+1 (t even); idx(p): index of
// record p. A run is walked in even-aligned pairs from t0 & ~1, lanes outside
// [t0, t1) masked, so the key's local id (run | position from t0 & ~1) is the
// wave-uniform loop counter.
constexpr int kRunOffBits = 6;  // candidates per run addressable by a key

struct KnnLists {
  int *ovf_tiles, *n_ovf;  // tiles whose segments overflow the LDS budget
  int *slow_q, *n_slow;    // queries the fast path could not certify
  double *slow_thr;        // their starting bound (K-th dsq upper bound)
  int vec_out;             // outputs 16-B aligned: k_knn may store them as vectors
};

typedef float f2 __attribute__((ext_vector_type(2)));
struct Pair3 {
  f2 x, y, z;
};
// record cursors for knn_one: load() = packed coordinates of the current
// pair of records, next() = the following pair
// The k_knn LDS tile, pair-interleaved in two planes of 16 B per pair of
// records: XY (x0 x1 y0 y1) and, kZgOff floats further, ZG (z0 z1 g0 g1).
// A 16-B stride spreads the lanes' b128 reads over all bank quads (one 32-B
// pair stride used only every other quad: a 2-way conflict floor).
#ifndef NAVGPU_TILE_REC
#define NAVGPU_TILE_REC 1600
#endif
constexpr int kTilePairs = NAVGPU_TILE_REC / 2 + 2;  // two spare pairs: read-ahead
constexpr int kZgOff = 4 * kTilePairs;
struct LdsPairCursor {
  const float *p;  // XY plane, pair P at p = XY + 4 P
  __device__ Pair3 load() const {
    const float4 xy = *(const float4 *)p;
    const float2 zz = *(const float2 *)(p + kZgOff);
    Pair3 P;
    P.x = f2{xy.x, xy.y};
    P.y = f2{xy.z, xy.w};
    P.z = f2{zz.x, zz.y};
    return P;
  }
  __device__ void next() { p += 4; }
};
struct RecPairCursor {  // global Rec16 array (two records of padding at its end)
  const Rec16 *p;
  __device__ Pair3 load() const {
    const Rec16 a = p[0], b = p[1];
    Pair3 P;
    P.x = f2{a.x, b.x};
    P.y = f2{a.y, b.y};
    P.z = f2{a.z, b.z};
    return P;
  }
  __device__ void next() { p += 2; }
};

// key = (f32 distance bits with the low kKeyBits cleared) | local id, as ONE
// v_and_or_b32 (the mask held in a VGPR, the id in an SGPR: the compiler
// otherwise emits and + or / or3). lid MUST be wave-uniform: a divergent
// value would be read from the first lane only.
__device__ __forceinline__ uint32_t knn_key(float d, uint32_t vmask, uint32_t lid) {
#ifdef NAVGPU_NO_ASM_KEY
  return (__float_as_uint(d) & vmask) | lid;
#else
  uint32_t k;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(k) : "v"(__float_as_uint(d)), "v"(vmask), "s"(lid));
  return k;
#endif
}

template <int K, int NR, class Runs, class CurF, class GposF>
__device__ __forceinline__ void knn_one(
    const GridParams &G, const TRec *__restrict__ tsort, const double qv[3],
    const int c[3], size_t q, Runs runs, CurF cursor, GposF fgpos,
    int32_t *__restrict__ oidx, double *__restrict__ odist, const KnnLists &L_) {
  // NR = 9: the block as 9 runs (run | offset ids); NR = 1: one contiguous
  // range (the column-major tile), the whole key id is the offset
  constexpr int kOffBits = NR == 1 ? kKeyBits : kRunOffBits;
  static_assert(NR == 1 || NR == 9, "a 3x3x3 block is 1 or 9 ranges");
  NV_STAMP(ts0);
  const double qr[3] = {qv[0] - G.o[0], qv[1] - G.o[1], qv[2] - G.o[2]};
  const float qf[3] = {(float)qr[0], (float)qr[1], (float)qr[2]};
  // |f32 difference - exact difference| <= dl: each operand rounded to f32
  // once (<= 2^-24 |v| each), one f32 subtraction (<= 2^-24 |difference|)
  const double Dq = fmax(G.emax + G.h,
                         fmax(fabs(qr[0]), fmax(fabs(qr[1]), fabs(qr[2]))));
  const double dl = Dq * 0x1p-22;
  constexpr int KL = K + 1;
  uint32_t key[KL];
#pragma unroll
  for (int s = 0; s < KL; ++s) key[s] = kNoKey;
  bool overflow = false;  // a run longer than the key's offset field
  const f2 qx2 = {qf[0], qf[0]}, qy2 = {qf[1], qf[1]}, qz2 = {qf[2], qf[2]};
  auto dist2 = [&](const Pair3 &a) {  // packed f32 squared distances
    const f2 fx2 = a.x - qx2, fy2 = a.y - qy2, fz2 = a.z - qz2;
    return __builtin_elementwise_fma(fz2, fz2, __builtin_elementwise_fma(fy2, fy2, fx2 * fx2));
  };
  auto ins = [&](uint32_t kk) {  // keep the K+1 smallest keys sorted
#ifndef NAVGPU_DBG_NOINSERT
#pragma unroll
    for (int s = K; s > 0; --s) key[s] = umed3(key[s - 1], key[s], kk);
#endif
    key[0] = min(key[0], kk);
  };
  constexpr uint32_t kOffMask = (1u << kOffBits) - 1;
  const uint32_t vmask = ~kKeyMask;
#pragma unroll 1
  for (int r = 0; r < NR; ++r) {
    int t0, t1;
    runs(r, t0, t1);
    const int ta = t0 & ~1;
    const int np = (t1 - ta + 1) >> 1;  // pairs the run touches
    overflow |= (t1 - ta) > (1 << kOffBits);
    const uint32_t rid = (uint32_t)r << kOffBits;
    auto cur = cursor(ta);
    if (np > 0) {  // first pair: may start before the run (odd t0) or end past it
      const f2 d = dist2(cur.load());
      uint32_t k0 = knn_key(d[0], vmask, rid);
      uint32_t k1 = knn_key(d[1], vmask, rid + 1);
      if (ta < t0) k0 = kNoKey;
      if (ta + 1 >= t1) k1 = kNoKey;
      ins(k0);
      ins(k1);
      cur.next();
    }
    // interior pairs: both records inside the run, no masks; the key's local
    // id is the wave-uniform pair counter
    // exit on the per-lane cursor reaching the last pair (one compare on the
    // address the loop advances anyway, no separate per-lane trip counter).
    // Only entered with np >= 3, so `last` lies past `cur`: LDS addresses
    // start at 0, and a cursor before the run's start would wrap around.
    if (np > 2) {
      const auto last = cursor(ta + 2 * (np - 1));
      uint32_t v2 = 2;
#ifndef NAVGPU_KNN_UNROLL
#define NAVGPU_KNN_UNROLL 1
#endif
#pragma unroll NAVGPU_KNN_UNROLL
      do {
        const f2 d = dist2(cur.load());
        const uint32_t lid = rid | (v2 & kOffMask);
        ins(knn_key(d[0], vmask, lid));
        ins(knn_key(d[1], vmask, lid + 1));
        cur.next();
        v2 += 2;
      } while (cur.p < last.p);
    }
    if (np > 1) {  // last pair: may end past the run
      const f2 d = dist2(cur.load());
      const uint32_t lid = rid | ((uint32_t)(2 * (np - 1)) & kOffMask);
      // lid depends on the lane's np here: divergent, so the plain and + or
      // (knn_key wants a wave-uniform id in an SGPR)
      uint32_t k1 = (__float_as_uint(d[1]) & vmask) | (lid + 1);
      if (ta + 2 * (np - 1) + 1 >= t1) k1 = kNoKey;
      ins((__float_as_uint(d[0]) & vmask) | lid);
      ins(k1);
    }
  }
  NV_STAMP(ts1);
  NV_STAMP_ADD(3, ts0, ts1);
  // anything outside the block (x +- sx, y +- 1, z +- 1 cells) is at least L away
  const double L = block_reach(G, qv, c, 1);
  double B = INFINITY;  // lower bound on the exact dsq of every excluded point
  if (L < INFINITY) {
    const double Lg = L - 2.0 * G.delta;
    B = Lg > 0.0 ? Lg * Lg : 0.0;
  }
  if (key[K] != kNoKey) {
    const double V = (double)__uint_as_float(key[K] & ~kKeyMask);
    const double err = V * 0x1p-20 + 4.0 * dl * __builtin_sqrt(V) + 4.0 * dl * dl;
    B = fmin(B, V - err);
  }
  bool ok = !overflow && Dq < 1e17;
  // exact f64 re-evaluation of the K best keys. All loads are issued
  // unconditionally (an empty slot re-reads slot 0) so their latencies
  // overlap; coordinates come from the cell-sorted copy (L2-local). The
  // (K+1)-th key V is the smallest of every candidate left out, so B above
  // bounds them all: a left-out candidate nearer than the K-th cannot pass
  // the certificate, and V's own exact distance is never needed.
  double ed[K];
  int ei[K];
#ifdef NAVGPU_DBG_NOEXACT
  if (false) {
#else
  if (key[0] != kNoKey) {
#endif
    int gpos[K];
    bool val[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
      val[s] = key[s] != kNoKey;
      const int l = (int)((val[s] ? key[s] : key[0]) & kKeyMask);
#ifdef NAVGPU_DBG_NODECODE  // timing-only ablation: every slot decodes in run 0
      const int r = 0, off = l & (int)kOffMask;
#else
      const int r = NR == 1 ? 0 : min(l >> kOffBits, NR - 1), off = l & (int)kOffMask;
#endif
      int t0, t1;
      runs(r, t0, t1);
      // record, in the fetch index space; clamped into the run so that a
      // corrupt id can never address outside the staged/sorted arrays
      const int p = min(max((t0 & ~1) + off, t0), max(t1 - 1, t0));
      gpos[s] = fgpos(p);
    }
#pragma unroll
    for (int s = 0; s < K; ++s) {
#ifdef NAVGPU_DBG_NOF64  // timing-only ablation: f32 key as the distance
      const double dsq = (double)__uint_as_float(key[s] & ~kKeyMask) + gpos[s] * 1e-30;
      ei[s] = val[s] ? gpos[s] : -1;
#else
      // x, y as one 16-B load, z + idx as one 12-B load (the pad is never read)
      const TRec *tp = tsort + gpos[s];
      const double2 xy = *(const double2 *)&tp->x;
      const double pz = tp->z;
      const int pid = tp->idx;
      const double ddx = xy.x - qv[0], ddy = xy.y - qv[1], ddz = pz - qv[2];
      const double dsq = ddx * ddx + ddy * ddy + ddz * ddz;  // utils/kdtree.c:16
      ei[s] = val[s] ? pid : -1;
#endif
      ed[s] = ei[s] >= 0 ? __builtin_sqrt(dsq) : INFINITY;
      // an inf/NaN distance is never a neighbour (kdtree.c:117)
      if (ei[s] >= 0 && !(ed[s] < INFINITY)) {
        ed[s] = INFINITY;
        ei[s] = -1;
        ok = false;
      }
    }

  } else {
#pragma unroll
    for (int s = 0; s < K; ++s) {
      ed[s] = INFINITY;
      ei[s] = -1;
    }
  }
  // order by (distance, index): the truncated-key order is almost always
  // right, and a misordered survivor sits next to its place. Bubble passes
  // run until no lane of the wave is out of order, usually one: some lane of
  // a wave is misordered about every other batch, so a fixed K-1 passes
  // cost a large share of the scan (NAVGPU_SORT_FIXED restores them).
  bool sorted = true;
#pragma unroll
  for (int s = 1; s < K; ++s) sorted &= !knn_less(ed[s], ei[s], ed[s - 1], ei[s - 1]);
#if defined(NAVGPU_DBG_NOSORT)  // timing-only ablation: no ordering pass
  if (false) {
#pragma unroll 1
    for (int pass = 0; pass < K - 1; ++pass) {
#elif defined(NAVGPU_SORT_FIXED)
  if (!sorted) {
#pragma unroll 1
    for (int pass = 0; pass < K - 1; ++pass) {
#else
  {
#pragma unroll 1
    for (int pass = 0; pass < K - 1 && __any(!sorted); ++pass) {
#endif
#pragma unroll
      for (int u = 1; u < K; ++u) {
        const bool sw = knn_less(ed[u], ei[u], ed[u - 1], ei[u - 1]);
        const double td = ed[u];
        const int ti = ei[u];
        ed[u] = sw ? ed[u - 1] : ed[u];
        ei[u] = sw ? ei[u - 1] : ei[u];
        ed[u - 1] = sw ? td : ed[u - 1];
        ei[u - 1] = sw ? ti : ei[u - 1];
      }
#ifndef NAVGPU_SORT_FIXED
      sorted = true;
#pragma unroll
      for (int s = 1; s < K; ++s) sorted &= !knn_less(ed[s], ei[s], ed[s - 1], ei[s - 1]);
#endif
    }
  }
  const double dk = ed[K - 1];
  const double dk2 = dk * dk;  // >= the exact K-th dsq (sqrt rounds to nearest)
  if (dk < INFINITY)
    ok = ok && B > dk2 * (1.0 + 0x1p-46);
  else
    ok = ok && B == INFINITY;  // fewer than K neighbours: only if all was seen
#if defined(NAVGPU_DBG_NOINSERT) || defined(NAVGPU_DBG_NOEXACT) || \
    defined(NAVGPU_DBG_NOF64) || defined(NAVGPU_DBG_NOSTAGE) || \
    defined(NAVGPU_DBG_NODECODE) || defined(NAVGPU_DBG_NOSORT) || \
    defined(NAVGPU_DBG_STAGE_ONCE)
  ok = true;  // timing-only ablation builds: never take the slow path
#endif
  if (ok) {
#ifdef NAVGPU_DBG_NOOUT  // timing-only ablation: one store per query, data kept live
    double acc = 0.0;
    int iacc = 0;
#pragma unroll
    for (int s = 0; s < K; ++s) {
      acc += ed[s];
      iacc ^= ei[s];
    }
    oidx[q * K] = iacc + (int)acc;
#else
    // a query's K results are contiguous: 16-B stores when K allows and the
    // host found both outputs 16-B aligned (L_.vec_out)
    if constexpr (K % 4 == 0) {
      if (L_.vec_out) {
#pragma unroll
        for (int s = 0; s < K; s += 4)
          *(int4 *)(oidx + q * K + s) = make_int4(ei[s], ei[s + 1], ei[s + 2], ei[s + 3]);
#pragma unroll
        for (int s = 0; s < K; s += 2)
          *(double2 *)(odist + q * K + s) = make_double2(ed[s], ed[s + 1]);
        return;
      }
    }
#pragma unroll
    for (int s = 0; s < K; ++s) {
      oidx[q * K + s] = ei[s];
      odist[q * K + s] = ed[s];
    }
#endif
  } else {
    // K listed points have dsq <= dk2: a valid starting bound for the slow
    // path, which runs in its own launch (k_knn_slow). Not after an overfull
    // run: its keys' offsets wrapped, so two slots can decode to the same
    // record and the list may hold fewer than K distinct points (a bound
    // from it can exclude a true neighbour); the slow path then starts from
    // an infinite bound (the ring search).
    const int e = atomicAdd(L_.n_slow, 1);
    L_.slow_q[e] = (int)q;
    L_.slow_thr[e] = (dk < INFINITY && !overflow) ? dk2 * (1.0 + 0x1p-46) : INFINITY;
  }
  NV_STAMP(ts2);
  NV_STAMP_ADD(4, ts1, ts2);
  NV_STAMP_ADD(5, 0ull, 1ull);
}

#ifndef NAVGPU_TILE_THREADS
#define NAVGPU_TILE_THREADS 192  // 3 waves: a ~150-query tile fills them
#endif
constexpr int kTileThreads = NAVGPU_TILE_THREADS;
constexpr int kTileRec = NAVGPU_TILE_REC;  // records staged per tile (16 B each)
#ifndef NAVGPU_STAGE_U
#define NAVGPU_STAGE_U 2  // records per thread per staging batch (4: 188.8 us, 8: 140 VGPRs, one block fewer per CU)
#endif

// Global-mode exact k-NN over tiles of W consecutive cells of one grid row.
// A tile stages the 9 neighbouring row segments (cells xa-1 .. xb+1) of the
// cell-sorted target records into LDS with coalesced loads, then its threads
// run the tile's (cell-sorted) queries against LDS. Tiles are dealt to the
// 8 XCDs in contiguous ranges (block b runs on XCD b % 8 under the observed
// round-robin placement; a different placement only costs L2 hits), so each
// XCD's L2 holds only its slab of the cloud.
// The LDS tile is COLUMN-major: for each x cell j of the segment, the records
// of its 9 (y, z) rows follow one another. A query's 3x3x3 block (columns
// x-1 .. x+1, all 9 rows) is then one contiguous record range, walked as one
// loop: a wave's trip count is the longest block among its lanes (neighbouring
// blocks share 18 of 27 cells), not the sum over 9 runs of each run's longest,
// and there is one run setup and one masked pair per query instead of 9.
// GLOBAL = false: the tile pass; a tile whose segments exceed the LDS budget
// is appended to the overflow list. GLOBAL = true: the overflow tiles, read
// straight from the global record array as 9 runs.
template <int K, bool GLOBAL>
#ifndef NAVGPU_KNN_MINW
#define NAVGPU_KNN_MINW 1
#endif
#ifdef NAVGPU_KNN_WPE
#define NAVGPU_KNN_ATTR __attribute__((amdgpu_waves_per_eu(NAVGPU_KNN_WPE)))
#else
#define NAVGPU_KNN_ATTR
#endif
__global__ __launch_bounds__(kTileThreads, NAVGPU_KNN_MINW) NAVGPU_KNN_ATTR void k_knn(
    const GridParams *__restrict__ gp, const int *__restrict__ start,
    const Rec16 *__restrict__ rec, const TRec *__restrict__ tsort,
    const double *__restrict__ qs, const int *__restrict__ qstart,
    const int *__restrict__ qperm, int32_t *__restrict__ oidx,
    double *__restrict__ odist, KnnLists L_) {
  // pair-interleaved records: pair P = LDS slots 2P, 2P+1 as x0 x1 y0 y1 z0 z1
  // g0 g1 (32 B; g = the record's cell-sorted position), so one b128 + one
  // b64 read gives packed operands; two spare pairs absorb the read-ahead
  // past a range's end
  __shared__ __attribute__((aligned(16))) float spair[GLOBAL ? 8 : 2 * kZgOff];
  // soff[r][i] = first record of cell xa - sx + i of row r; then, in place
  // (tile pass), cbase[r][j]: the LDS slot of the record at cell-sorted
  // position g of cell (row r, column j) is cbase[r][j] + g
  __shared__ int soff[9][kTileCols];
  __shared__ int colst[GLOBAL ? 1 : kTileCols];  // first slot of column j (j = 0: cell xa - sx)
  __shared__ int scratch[kTileThreads / kWave + 1];
  const GridParams G = *gp;
  const int W = G.tile_w, sx = G.sx;
  const int tpr = (G.g[0] + W - 1) / W;
  long long t_hi, step, first;
  if (GLOBAL) {
    t_hi = *L_.n_ovf;
    first = blockIdx.x;
    step = gridDim.x;
  } else {
    const long long ntiles = (long long)tpr * G.g[1] * G.g[2];
    const int xcd = blockIdx.x & 7;
    t_hi = ntiles * (xcd + 1) / 8;
    first = ntiles * xcd / 8 + (blockIdx.x >> 3);
    step = gridDim.x >> 3;
  }
  for (long long it = first; it < t_hi; it += step) {
    NV_STAMP(tb0);
    const long long tile = GLOBAL ? (long long)L_.ovf_tiles[it] : it;
    const int row = (int)(tile / tpr), chunk = (int)(tile % tpr);
    const int y = row % G.g[1], z = row / G.g[1];
    const int xa = chunk * W, xb = min(xa + W, G.g[0]) - 1;
    const int ncell = xb - xa + 2 + 2 * sx;  // soff entries per row: cells xa-sx .. xb+sx+1
#ifdef NAVGPU_DBG_STAGE_ONCE  // timing-only ablation: the first tile's staging serves all
    if (it == first) {
#endif
    // staging is latency-bound: every thread issues all its global loads
    // before it writes any of them to LDS
    // soff: the 9 rows (uniform loop, no index division), all loads first
    for (int i0 = 0; i0 < ncell; i0 += (int)blockDim.x) {
      const int i = i0 + (int)threadIdx.x;
      int v[9];
#pragma unroll
      for (int r = 0; r < 9; ++r) {
        int dy, dz;
        run_dydz(r, dy, dz);
        const int yy = y + dy, zz = z + dz;
        v[r] = 0;
        if (i < ncell && yy >= 0 && yy < G.g[1] && zz >= 0 && zz < G.g[2]) {
          const int x = min(max(xa - sx + i, 0), G.g[0]);  // x = gx: row end
          v[r] = start[(zz * G.g[1] + yy) * G.g[0] + x];
        }
      }
      if (i < ncell) {
#pragma unroll
        for (int r = 0; r < 9; ++r) soff[r][i] = v[r];
      }
    }
    __syncthreads();
    int sb[10], s0[9];  // row segment bases (staging index) and global offsets
    if (!GLOBAL) {
      // the copy's source order: the 9 row segments one after another
      sb[0] = 0;
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        const int lo = soff[u][0];
        sb[u + 1] = sb[u] + (soff[u][ncell - 1] - lo);
        s0[u] = lo - sb[u];  // global = e + s0[r]
      }
      // the column-major layout: thread j owns column j of the W + 2 sx
      const int ncol = ncell - 1, j = (int)threadIdx.x;
      int n[9], sv[9], cs = 0;
#pragma unroll
      for (int r = 0; r < 9; ++r) {
        sv[r] = j < ncol ? soff[r][j] : 0;
        n[r] = j < ncol ? soff[r][j + 1] - sv[r] : 0;
        cs += n[r];
      }
      int total;
      const int cex = block_excl_scan(cs, scratch, &total);  // barriers: soff reads done
      if (total > kTileRec) {  // uniform: defer the tile to the global pass
        if (threadIdx.x == 0) L_.ovf_tiles[atomicAdd(L_.n_ovf, 1)] = (int)tile;
        __syncthreads();
        continue;
      }
      if (j <= ncol) colst[j] = cex;  // colst[ncol] = the total
      if (j < ncol) {
        int a = cex;
#pragma unroll
        for (int r = 0; r < 9; ++r) {
          soff[r][j] = a - sv[r];  // cbase
          a += n[r];
        }
      }
      __syncthreads();
      const int jmax = ncol - 1;
      // each wave copies whole row segments (r = wave, wave + nwaves, ...):
      // r is wave-uniform, so a record's global position is e + s0[r] with
      // no per-record segment decode (that decode was most of the staging
      // VALU); a batch's loads are all issued before any LDS write
      const int lane = (int)threadIdx.x & (kWave - 1);
      const int nwv = (int)blockDim.x / kWave;
      constexpr int U = NAVGPU_STAGE_U;  // records per lane per batch
      for (int r = (int)threadIdx.x / kWave; r < 9; r += nwv) {
        const int g0 = sb[r] + s0[r], nr = sb[r + 1] - sb[r];
        const int *cb = &soff[r][0];
        for (int k0 = 0; k0 < nr; k0 += U * kWave) {
          Rec16 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int k = k0 + u * kWave + lane;
            if (k < nr) {
#ifdef NAVGPU_DBG_NOSTAGE  // timing-only ablation: no record loads
              v[u].x = v[u].y = v[u].z = (float)k;
              v[u].cx = xa;
#else
              v[u] = rec[g0 + k];
#endif
            }
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int k = k0 + u * kWave + lane;
            if (k < nr) {
              // the record's column (its cell lies in xa-sx .. xb+sx; clamped
              // so that a corrupt value cannot address outside the tile)
              const int g = g0 + k;
              const int jj = min(max(v[u].cx - xa + sx, 0), jmax);
              const int slot = cb[jj] + g;
              float *d = spair + (slot >> 1) * 4 + (slot & 1);
              d[0] = v[u].x;
              d[2] = v[u].y;
              d[kZgOff] = v[u].z;
              d[kZgOff + 2] = __int_as_float(g);
            }
          }
        }
      }
      __syncthreads();
    }
#ifdef NAVGPU_DBG_STAGE_ONCE
    }
#endif
    NV_STAMP(tb1);
    NV_STAMP_ADD(1, tb0, tb1);
    NV_STAMP_ADD(6, 0ull, 1ull);
    const int cell0 = (z * G.g[1] + y) * G.g[0];
    const int q0 = qstart[cell0 + xa], q1 = qstart[cell0 + xb + 1];
#ifdef NAVGPU_DBG_NOQUERY  // timing-only ablation: staging and barriers only
    if (q1 < 0)
#endif
    for (int qi = q0 + threadIdx.x; qi < q1; qi += blockDim.x) {
      const size_t q = (size_t)qperm[qi];
      const double qv[3] = {qs[3 * q], qs[3 * q + 1], qs[3 * q + 2]};
      const int c[3] = {cell_axis(qv[0], G, 0), y, z};
      const int i = c[0] - xa;  // columns i .. i + 2 sx = cells c - sx .. c + sx
      if (!GLOBAL) {
        knn_one<K, 1>(G, tsort, qv, c, q,
                      [&](int, int &t0, int &t1) {
                        t0 = colst[i];
                        t1 = colst[i + 2 * sx + 1];
                      },
                      [&](int t) { return LdsPairCursor{spair + (t >> 1) * 4}; },
                      [&](int p) { return __float_as_int(spair[kZgOff + (p >> 1) * 4 + 2 + (p & 1)]); },
                      oidx, odist, L_);
      } else {
        knn_one<K, 9>(G, tsort, qv, c, q,
                      [&](int r, int &t0, int &t1) {
                        t0 = soff[r][i];
                        t1 = soff[r][i + 2 * sx + 1];
                      },
                      [&](int t) { return RecPairCursor{rec + t}; },
                      [&](int p) { return p; }, oidx, odist, L_);
      }
    }
    NV_STAMP(tb2);
    NV_STAMP_ADD(2, tb1, tb2);
    __syncthreads();
    NV_STAMP(tb3);
    NV_STAMP_ADD(7, tb2, tb3);
  }
}

// insert (d, id) into the sorted exact list kd/ki if it ranks among the K
template <int K>
__device__ __forceinline__ void knn_insert(double *kd, int *ki, double d, int id) {
  if (!knn_less(d, id, kd[K - 1], ki[K - 1])) return;
  bool placed = false;
#pragma unroll
  for (int s = K - 1; s >= 0; --s) {
    if (!placed) {
      if (s > 0 && knn_less(d, id, kd[s - 1], ki[s - 1])) {
        kd[s] = kd[s - 1];
        ki[s] = ki[s - 1];
      } else {
        kd[s] = d;
        ki[s] = id;
        placed = true;
      }
    }
  }
}

// merge the 64 lane lists kd/ki (each sorted) into md/mi: K rounds of a
// wave (distance, index) argmin on the list heads
template <int K>
__device__ __forceinline__ void knn_wave_merge(double *kd, int *ki, double *md, int *mi,
                                               int lane) {
#pragma unroll
  for (int s = 0; s < K; ++s) {
    double bd = kd[0];
    int bi = ki[0], bl = lane;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const double od = __shfl_xor(bd, o, kWave);
      const int oi = __shfl_xor(bi, o, kWave), ol = __shfl_xor(bl, o, kWave);
      const bool take = knn_less(od, oi, bd, bi) ||
                        (!knn_less(bd, bi, od, oi) && ol < bl);
      bd = take ? od : bd;
      bi = take ? oi : bi;
      bl = take ? ol : bl;
    }
    md[s] = bd;
    mi[s] = bi;
    if (lane == bl) {  // pop the winner's head
#pragma unroll
      for (int u = 0; u < K - 1; ++u) {
        kd[u] = kd[u + 1];
        ki[u] = ki[u + 1];
      }
      kd[K - 1] = INFINITY;
      ki[K - 1] = -1;
    }
  }
}

// f32 screen + exact f64 distance of record t against the query; inserts
// into the lane's sorted list when within thr
template <int K>
__device__ __forceinline__ void knn_visit(const Rec16 &rr, size_t t,
                                          const TRec *__restrict__ tsort,
                                          const double qv[3], const float qf[3],
                                          double thr, float thr_f, double *kd, int *ki) {
  const float fx = rr.x - qf[0], fy = rr.y - qf[1], fz = rr.z - qf[2];
  const float d2f = __builtin_fmaf(fz, fz, __builtin_fmaf(fy, fy, fx * fx));
  if (!(d2f <= thr_f)) return;
  const TRec tp = tsort[t];
  const double ddx = tp.x - qv[0], ddy = tp.y - qv[1], ddz = tp.z - qv[2];
  const double dsq = ddx * ddx + ddy * ddy + ddz * ddz;  // utils/kdtree.c:16
  if (!(dsq <= thr)) return;
  knn_insert<K>(kd, ki, __builtin_sqrt(dsq), tp.idx);
}

constexpr int kSlowMaxR = 3;  // one-shot cube: at most (2R+1)^2 = 49 rows

// The queries k_knn could not certify, one WAVE per query, from the recorded
// starting bound thr (K real points lie within it, so every neighbour does).
// One-shot cube: the smallest cube of cells around the query whose outside is
// provably beyond thr; its (y, z) rows are contiguous record ranges, counted
// and prefix-summed across the wave so the records are dealt evenly over the
// 64 lanes. Each lane keeps a sorted list (f32 screen, then the reference f64
// distance); one wave merge gives the answer. An infinite bound, or a cube
// beyond kSlowMaxR, takes the ring search: rings of cells split over the
// lanes, merged after every ring, the merged K-th bounding the next ring.
template <int K>
__global__ __launch_bounds__(256) void k_knn_slow(
    const GridParams *__restrict__ gp, const int *__restrict__ start,
    const Rec16 *__restrict__ rec, const TRec *__restrict__ tsort,
    const double *__restrict__ qs, int32_t *__restrict__ oidx,
    double *__restrict__ odist, KnnLists L_) {
  __shared__ double sd[4][kWave];  // per-wave survivor buffers (256 threads)
  __shared__ int si[4][kWave];
  const GridParams G = *gp;
  const int n = *L_.n_slow;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) / kWave);
  const int nwaves = (int)(gridDim.x * blockDim.x / kWave);
  const int gmax = max((G.g[0] + G.sx - 1) / G.sx, max(G.g[1], G.g[2]));
  for (int e = wave; e < n; e += nwaves) {
    const size_t q = (size_t)L_.slow_q[e];
    double thr = L_.slow_thr[e];
    const double qv[3] = {qs[3 * q], qs[3 * q + 1], qs[3 * q + 2]};
    const double qr[3] = {qv[0] - G.o[0], qv[1] - G.o[1], qv[2] - G.o[2]};
    const float qf[3] = {(float)qr[0], (float)qr[1], (float)qr[2]};
    const double Dq = fmax(G.emax + G.h,
                           fmax(fabs(qr[0]), fmax(fabs(qr[1]), fabs(qr[2]))));
    const double dl = Dq * 0x1p-22;
    float thr_f = f32_bound(thr, dl);
    const int c[3] = {cell_axis(qv[0], G, 0), cell_axis(qv[1], G, 1),
                      cell_axis(qv[2], G, 2)};
    double kd[K], md[K];
    int ki[K], mi[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
      kd[s] = INFINITY;
      ki[s] = -1;
    }
    // cube radius: everything outside cube R is at least L_R away
    int R = -1;
    if (thr < INFINITY) {
      for (int r = 1; r <= kSlowMaxR; ++r) {
        const double L = block_reach(G, qv, c, r);
        const double Lg = L - 2.0 * G.delta;
        if (L == INFINITY || (Lg > 0.0 && thr < Lg * Lg)) {
          R = r;
          break;
        }
      }
    }
    if (R > 0) {
      const int xl = max(c[0] - R * G.sx, 0), xh = min(c[0] + R * G.sx, G.g[0] - 1);
      const int yl = max(c[1] - R, 0), yh = min(c[1] + R, G.g[1] - 1);
      const int zl = max(c[2] - R, 0), zh = min(c[2] + R, G.g[2] - 1);
      const int ny = yh - yl + 1, nrows = ny * (zh - zl + 1);  // <= 49
      int cnt = 0, b = 0;
      if (lane < nrows) {
        const int y = yl + lane % ny, z = zl + lane / ny;
        if (!(box_d2(G, qv, xl, xh, y, y, z, z) > thr)) {
          const int row = (z * G.g[1] + y) * G.g[0];
          b = start[row + xl];
          cnt = start[row + xh + 1] - b;
        }
      }
      int pre = cnt;  // inclusive wave scan of the row counts
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const int t = __shfl_up(pre, o, kWave);
        if (lane >= o) pre += t;
      }
      const int total = __shfl(pre, kWave - 1, kWave);
      pre -= cnt;  // exclusive
      for (int j0 = 0; j0 < total; j0 += kWave) {
        const int j = j0 + lane;
        // row of flattened record j: the last row whose prefix is <= j
        int lo = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
          const int cand = lo + step;
          const int pc = __shfl(pre, cand < nrows ? cand : 0, kWave);
          if (cand < nrows && pc <= j) lo = cand;
        }
        const int pb = __shfl(b, lo, kWave), pp = __shfl(pre, lo, kWave);
        if (j < total) {
          const size_t t = (size_t)(pb + (j - pp));
          knn_visit<K>(rec[t], t, tsort, qv, qf, thr, thr_f, kd, ki);
        }
      }
      // the lanes' survivors (usually ~K in all): compact them into LDS and
      // rank each by counting smaller ones; more than 64 take the merge
      int nsv = 0;
#pragma unroll
      for (int u = 0; u < K; ++u) nsv += kd[u] < INFINITY ? 1 : 0;
      int off = nsv;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const int t = __shfl_up(off, o, kWave);
        if (lane >= o) off += t;
      }
      const int tot = __shfl(off, kWave - 1, kWave);
      off -= nsv;
      if (tot <= kWave) {
        double *bd = sd[threadIdx.x / kWave];
        int *bi = si[threadIdx.x / kWave];
#pragma unroll
        for (int u = 0; u < K; ++u)
          if (u < nsv) {
            bd[off + u] = kd[u];
            bi[off + u] = ki[u];
          }
        wave_sync_mem();
        if (lane < tot) {
          const double d = bd[lane];
          const int id = bi[lane];
          int rank = 0;
          for (int t = 0; t < tot; ++t) rank += knn_less(bd[t], bi[t], d, id) ? 1 : 0;
          if (rank < K) {
            oidx[q * K + rank] = id;
            odist[q * K + rank] = d;
          }
        } else if (lane < K) {  // fewer than K survivors: empty slots
          oidx[q * K + lane] = -1;
          odist[q * K + lane] = INFINITY;
        }
        wave_sync_mem();  // the buffer is reused by this wave's next query
        continue;
      }
      knn_wave_merge<K>(kd, ki, md, mi, lane);
    }
    for (int r = 0; R < 0 && r <= gmax; ++r) {
      // the ring's cube clipped to the grid (a degenerate axis stays 1 thick);
      // x reaches r * sx cells
      const int xl = max(c[0] - r * G.sx, 0), xh = min(c[0] + r * G.sx, G.g[0] - 1);
      const int yl = max(c[1] - r, 0), yh = min(c[1] + r, G.g[1] - 1);
      const int zl = max(c[2] - r, 0), zh = min(c[2] + r, G.g[2] - 1);
      const int bx = xh - xl + 1, by = yh - yl + 1, bz = zh - zl + 1;
      const int nbox = bx * by * bz;
      for (int u = lane; u < nbox; u += kWave) {
        const int x = xl + u % bx, y = yl + (u / bx) % by, z = zl + u / (bx * by);
        if (max((abs(x - c[0]) + G.sx - 1) / G.sx, max(abs(y - c[1]), abs(z - c[2]))) != r)
          continue;
        if (box_d2(G, qv, x, x, y, y, z, z) > thr) continue;
        const int cell = (z * G.g[1] + y) * G.g[0] + x;
        const int b = start[cell], en = start[cell + 1];
        for (int t = b; t < en; ++t)
          knn_visit<K>(rec[t], (size_t)t, tsort, qv, qf, thr, thr_f, kd, ki);
      }
      knn_wave_merge<K>(kd, ki, md, mi, lane);
      // lane 0 carries the merged list into the next ring
#pragma unroll
      for (int s = 0; s < K; ++s) {
        kd[s] = lane == 0 ? md[s] : INFINITY;
        ki[s] = lane == 0 ? mi[s] : -1;
      }
      if (md[K - 1] < INFINITY) {
        thr = fmin(thr, md[K - 1] * md[K - 1] * (1.0 + 0x1p-46));
        thr_f = f32_bound(thr, dl);
      }
      const double L = block_reach(G, qv, c, r);
      if (L == INFINITY) break;
      const double Lg = L - 2.0 * G.delta;
      if (Lg > 0.0 && thr < Lg * Lg) break;  // all points with dsq <= thr seen
    }
    if (lane == 0) {
#pragma unroll
      for (int s = 0; s < K; ++s) {
        oidx[q * K + s] = mi[s];
        odist[q * K + s] = md[s];
      }
    }
  }
}

}  // namespace

// =================================================================== host
struct navgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::map<int, std::pair<void *, size_t>> bufs;  // grow-only workspace
  bool timing = false;
  std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> ev;
  std::vector<hipEvent_t> free_ev;
  std::vector<double> tan_c, tan_r;
  int tan_R = -1, tan_C = -1;
  hipStream_t aux = nullptr;                 // side stream (pair path: curvature)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  double knn_occ = 5.0;  // target points per h^3 grid cell (NAVGPU_KNN_OCC)
  int knn_sx = NAVGPU_KNN_SX;  // x cells per h (NAVGPU_KNN_SX)
  int knn_blocks = 0;    // k_knn blocks per XCD, 0 = auto (NAVGPU_KNN_BLOCKS)
  bool knn_stats = false;
  int screen_rows = 0, screen_S = 0;  // last screened rows_match call (tie diagnostic)
};

namespace {

enum Slot {
  kBBox = 1, kParams, kCnt, kStart, kBSum, kCellId, kSlotBuf, kRec, kTan,
  kKdFc, kKdP, kKdT, kQStart, kQCell, kQSlot, kQPerm, kStats, kOvf, kSlowQ,
  kSlowThr, kTSort, kRowMaskS, kRowMaskT, kRowTie, kCorrEnt, kCorrN, kCorrSums, kKdPtmp, kKdSel,
  kH0 = 100, kH1, kH2, kH3, kH4, kH5,
};

int ws_get(navgpu_ctx *ctx, int slot, size_t bytes, void **out) {
  auto &b = ctx->bufs[slot];
  if (b.second < bytes || !b.first) {
    if (b.first) {
      HIP_TRY(hipStreamSynchronize(ctx->stream));
      HIP_TRY(hipFree(b.first));
      b.first = nullptr;
      b.second = 0;
    }
    size_t want = bytes < 256 ? 256 : bytes;
    hipError_t e = hipMalloc(&b.first, want);
    if (e != hipSuccess) {
      set_err("hipMalloc(%zu): %s", want, hipGetErrorString(e));
      b.first = nullptr;
      return NAVGPU_ENOMEM;
    }
    b.second = want;
  }
  *out = b.first;
  return NAVGPU_OK;
}

template <class T>
int ws(navgpu_ctx *ctx, int slot, size_t count, T **out) {
  void *p;
  int rc = ws_get(ctx, slot, count * sizeof(T), &p);
  *out = (T *)p;
  return rc;
}

#define RC(x)                    \
  do {                           \
    int rc_ = (x);               \
    if (rc_ != NAVGPU_OK) return rc_; \
  } while (0)

struct TimedRegion {
  navgpu_ctx *ctx;
  const char *name;
  hipEvent_t a = nullptr, b = nullptr;
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
  hipStream_t st;
  TimedRegion(navgpu_ctx *c, const char *n, hipStream_t on = nullptr)
      : ctx(c), name(n), st(on ? on : c->stream) {
    if (!ctx->timing) return;
    a = take();
    b = take();
    if (a && b) (void)hipEventRecord(a, st);
  }
  ~TimedRegion() {
    if (!ctx->timing || !a || !b) return;
    (void)hipEventRecord(b, st);
    ctx->ev[name].push_back({a, b});
  }
};

// dynamic LDS a tree-building kernel may request: the device limit minus
// the static LDS of block_nth_element (pointer-jumping words + counts)
int lds_limit() {
  constexpr int kStaticLds = 8 * kBlockNthMax + 8 * (kBlockNthMax / kWave) + 16 + 256;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 65536 - kStaticLds;
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock,
                            dev) != hipSuccess || v <= 0)
    return 65536 - kStaticLds;
  return v - kStaticLds;
}

int check_rows_shape(int R, int C, bool stack) {
  ARG_CHECK(R >= 0 && C >= 0);
  if (C > kMaxRowCols) {
    set_err("rows kernels: C=%d exceeds %d", C, kMaxRowCols);
    return NAVGPU_ERANGE;
  }
  const RowsLds L = rows_lds(C, kRowsBlock, stack);
  if (L.total > lds_limit()) {
    set_err("rows kernels: C=%d needs %d B of LDS (device limit %d)", C,
            L.total, lds_limit());
    return NAVGPU_ERANGE;
  }
  return NAVGPU_OK;
}

template <class Kern>
int set_lds(Kern k, int bytes) {
  HIP_TRY(hipFuncSetAttribute((const void *)k,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              bytes));
  return NAVGPU_OK;
}

unsigned grid1d(size_t n, int block) {
  return (unsigned)((n + block - 1) / block);
}

}  // namespace

// ------------------------------------------------------------------ C ABI
extern "C" {

const char *navgpu_last_error(void) { return g_err; }
const char *navgpu_version(void) { return NAVGPU_VERSION; }

int navgpu_create(int device, void *stream, navgpu_ctx **out) {
  ARG_CHECK(out);
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    set_err("device %d not present (%d visible)", device, ndev);
    return NAVGPU_EHIP;
  }
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_err("device %d is %s; libnavgpu is built for gfx950 (MI355X) only",
            device, prop.gcnArchName);
    return NAVGPU_EHIP;
  }
  HIP_TRY(hipSetDevice(device));
  navgpu_ctx *c = new navgpu_ctx();
  c->device = device;
  if (const char *st = getenv("NAVGPU_KNN_STATS")) c->knn_stats = *st && *st != '0';
  if (const char *o = getenv("NAVGPU_KNN_BLOCKS")) c->knn_blocks = atoi(o);
  if (const char *o = getenv("NAVGPU_KNN_SX")) {
    const int v = atoi(o);
    if (v >= 1 && v <= kMaxSx) c->knn_sx = v;
  }
  if (const char *o = getenv("NAVGPU_KNN_OCC")) {
    const double v = atof(o);
    if (v > 0.05 && v < 1000) c->knn_occ = v;
  }
  if (stream) {
    c->stream = (hipStream_t)stream;
  } else {
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete c;
      set_err("hipStreamCreate: %s", hipGetErrorString(e));
      return NAVGPU_EHIP;
    }
    c->own_stream = true;
  }
  *out = c;
  return NAVGPU_OK;
}

void navgpu_destroy(navgpu_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto &kv : ctx->bufs)
    if (kv.second.first) (void)hipFree(kv.second.first);
  for (auto &kv : ctx->ev)
    for (auto &pr : kv.second) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  for (auto e : ctx->free_ev) (void)hipEventDestroy(e);
  if (ctx->aux) {
    (void)hipStreamSynchronize(ctx->aux);
    (void)hipStreamDestroy(ctx->aux);
  }
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int navgpu_set_stream(navgpu_ctx *ctx, void *stream) {
  ARG_CHECK(ctx && stream);
  if (ctx->own_stream) {
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipStreamDestroy(ctx->stream));
    ctx->own_stream = false;
  }
  ctx->stream = (hipStream_t)stream;
  return NAVGPU_OK;
}

void *navgpu_stream(navgpu_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int navgpu_sync(navgpu_ctx *ctx) {
  ARG_CHECK(ctx);
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (ctx->aux) HIP_TRY(hipStreamSynchronize(ctx->aux));
  return NAVGPU_OK;
}

static int ensure_aux(navgpu_ctx *ctx) {
  if (!ctx->aux) {
    HIP_TRY(hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
  }
  return NAVGPU_OK;
}

int navgpu_side_mark(navgpu_ctx *ctx) {
  ARG_CHECK(ctx);
  RC(ensure_aux(ctx));
  HIP_TRY(hipEventRecord(ctx->ev_fork, ctx->stream));
  return NAVGPU_OK;
}

int navgpu_side_download(navgpu_ctx *ctx, void *dst, const void *src, size_t bytes) {
  ARG_CHECK(ctx);
  if (!bytes) return NAVGPU_OK;
  ARG_CHECK(dst && src);
  RC(ensure_aux(ctx));
  HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->aux));
  return NAVGPU_OK;
}

int navgpu_rows_max_cols(void) {
  const int lim = lds_limit();
  int lo = 0, hi = kMaxRowCols;
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if (rows_lds(mid, kRowsBlock, true).total <= lim)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

void navgpu_timing_enable(navgpu_ctx *ctx, int on) {
  if (ctx) ctx->timing = on != 0;
}

double navgpu_timing_read(navgpu_ctx *ctx, const char *name, int reset) {
  if (!ctx || !name) return -1.0;
  auto it = ctx->ev.find(name);
  if (it == ctx->ev.end()) return -1.0;
  double ms = 0.0;
  for (auto &pr : it->second) {
    if (hipEventSynchronize(pr.second) != hipSuccess) return -1.0;
    float t = 0.f;
    if (hipEventElapsedTime(&t, pr.first, pr.second) != hipSuccess) return -1.0;
    ms += t;
  }
  if (reset) {
    for (auto &pr : it->second) {
      ctx->free_ev.push_back(pr.first);
      ctx->free_ev.push_back(pr.second);
    }
    it->second.clear();
  }
  return ms;
}

// diagnostic builds only (-DNAVGPU_STAMPS): read and clear the phase stamps
int navgpu_debug_stamps(unsigned long long *out16) {
#ifdef NAVGPU_STAMPS
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_stamps), 16 * 8));
  unsigned long long z[16] = {0};
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, 16 * 8));
  return NAVGPU_OK;
#else
  (void)out16;
  return NAVGPU_EINVAL;
#endif
}

long long navgpu_knn_fallbacks(navgpu_ctx *ctx) {
  if (!ctx) return -1;
  auto it = ctx->bufs.find(kStats);
  if (it == ctx->bufs.end() || !it->second.first) return -1;
  int v[2] = {0, 0};
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return -1;
  if (hipMemcpy(v, it->second.first, 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (long long)v[1];
}

long long navgpu_knn_overflows(navgpu_ctx *ctx) {
  if (!ctx) return -1;
  auto it = ctx->bufs.find(kStats);
  if (it == ctx->bufs.end() || !it->second.first) return -1;
  int v[2] = {0, 0};
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return -1;
  if (hipMemcpy(v, it->second.first, 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (long long)v[0];
}

long long navgpu_rows_tie_rows(navgpu_ctx *ctx) {
  if (!ctx || ctx->screen_rows <= 0) return -1;
  auto it = ctx->bufs.find(kRowTie);
  if (it == ctx->bufs.end() || !it->second.first) return -1;
  std::vector<int32_t> v((size_t)ctx->screen_rows * ctx->screen_S);
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return -1;
  if (hipMemcpy(v.data(), it->second.first, 4 * v.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  long long n = 0;
  for (int r = 0; r < ctx->screen_rows; ++r) {
    int any = 0;
    for (int s = 0; s < ctx->screen_S; ++s) any |= v[(size_t)r * ctx->screen_S + s];
    n += any != 0;
  }
  return n;
}

int navgpu_timing_count(navgpu_ctx *ctx, const char *name) {
  if (!ctx || !name) return -1;
  auto it = ctx->ev.find(name);
  return it == ctx->ev.end() ? 0 : (int)it->second.size();
}

// ---------------------------------------------------------------- R1
int navgpu_curvature_dev(navgpu_ctx *ctx, const double *pts, int R, int C,
                         int32_t *mask, double *curv) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  if ((size_t)R * C == 0) return NAVGPU_OK;
  ARG_CHECK(pts && mask);
  TimedRegion tr(ctx, "curvature");
  CurvJob J = {{pts, nullptr}, {mask, nullptr}, {curv, nullptr}};
  dim3 grid((C + kCurvTile - 1) / kCurvTile, R, 1);
  hipLaunchKernelGGL(k_curvature, grid, dim3(kCurvTile), 0, ctx->stream, J, R, C);
  CHECK_LAUNCH("k_curvature");
  return NAVGPU_OK;
}

int navgpu_curvature_host(navgpu_ctx *ctx, const double *pts, int R, int C,
                          int32_t *mask, double *curv) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  const size_t N = (size_t)R * C;
  if (!N) return NAVGPU_OK;
  ARG_CHECK(pts && mask);
  double *dp, *dc = nullptr;
  int32_t *dm;
  RC(ws(ctx, kH0, 3 * N, &dp));
  RC(ws(ctx, kH1, N, &dm));
  if (curv) RC(ws(ctx, kH2, N, &dc));
  HIP_TRY(hipMemcpyAsync(dp, pts, 24 * N, hipMemcpyHostToDevice, ctx->stream));
  RC(navgpu_curvature_dev(ctx, dp, R, C, dm, dc));
  HIP_TRY(hipMemcpyAsync(mask, dm, 4 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (curv)
    HIP_TRY(hipMemcpyAsync(curv, dc, 8 * N, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return NAVGPU_OK;
}

// ---------------------------------------------------------------- R2
int navgpu_project_dev(navgpu_ctx *ctx, const int32_t *depth, int R, int C,
                       double *pts) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  const size_t N = (size_t)R * C;
  if (!N) return NAVGPU_OK;
  ARG_CHECK(depth && pts);
  double *dt;
  RC(ws(ctx, kTan, (size_t)R + C, &dt));
  if (ctx->tan_R != R || ctx->tan_C != C) {
    // utils/pointcloud.c:10-36, the angle tables with the host's libm tan
    const double fov_h = 45.0, fov_v = 45.0;
    const double theta_step_deg = fov_h / (C - 1);
    const double phi_step_deg = fov_v / (R - 1);
    ctx->tan_c.resize(C);
    ctx->tan_r.resize(R);
    for (int i = 0; i < C; ++i) {
      double theta = -fov_h / 2.0 + i * theta_step_deg;
      theta = theta * M_PI / 180.0;
      ctx->tan_c[i] = tan(theta);
    }
    for (int j = 0; j < R; ++j) {
      double phi = -fov_v / 2.0 + j * phi_step_deg;
      phi = phi * M_PI / 180.0;
      ctx->tan_r[j] = tan(phi);
    }
    HIP_TRY(hipMemcpyAsync(dt, ctx->tan_c.data(), 8 * (size_t)C,
                           hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(dt + C, ctx->tan_r.data(), 8 * (size_t)R,
                           hipMemcpyHostToDevice, ctx->stream));
    ctx->tan_R = R;
    ctx->tan_C = C;
  }
  hipLaunchKernelGGL(k_project, dim3(grid1d(N, 256)), dim3(256), 0,
                     ctx->stream, depth, R, C, dt, dt + C, pts);
  CHECK_LAUNCH("k_project");
  return NAVGPU_OK;
}

int navgpu_project_host(navgpu_ctx *ctx, const int32_t *depth, int R, int C,
                        double *pts) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  const size_t N = (size_t)R * C;
  if (!N) return NAVGPU_OK;
  ARG_CHECK(depth && pts);
  int32_t *dd;
  double *dp;
  RC(ws(ctx, kH0, N, &dd));
  RC(ws(ctx, kH1, 3 * N, &dp));
  HIP_TRY(hipMemcpyAsync(dd, depth, 4 * N, hipMemcpyHostToDevice, ctx->stream));
  RC(navgpu_project_dev(ctx, dd, R, C, dp));
  HIP_TRY(hipMemcpyAsync(pts, dp, 24 * N, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return NAVGPU_OK;
}

// ---------------------------------------------------------------- R3
int navgpu_transform_dev(navgpu_ctx *ctx, const double *pts, size_t n,
                         const double Rm[9], const double t[3],
                         const double tr[3], double *out, double *out_last) {
  ARG_CHECK(ctx);
  if (!n) return NAVGPU_OK;
  ARG_CHECK(pts && Rm && t && out);
  ARG_CHECK(!out_last || tr);
  Rigid g;
  memcpy(g.R, Rm, sizeof(g.R));
  memcpy(g.t, t, sizeof(g.t));
  if (tr)
    memcpy(g.tr, tr, sizeof(g.tr));
  else
    memset(g.tr, 0, sizeof(g.tr));
  hipLaunchKernelGGL(k_transform, dim3(grid1d(n, 256)), dim3(256), 0,
                     ctx->stream, pts, n, g, out, out_last);
  CHECK_LAUNCH("k_transform");
  return NAVGPU_OK;
}

// ------------------------------------------------------------ R4-R6 rows
int navgpu_kd_build_rows_dev(navgpu_ctx *ctx, const double *feat_src,
                             const double *coords, int R, int C,
                             double *tree_pts, int32_t *tree_col,
                             int32_t *tree_n, int32_t *mask_out) {
  ARG_CHECK(ctx);
  RC(check_rows_shape(R, C, false));
  if (R == 0) return NAVGPU_OK;
  ARG_CHECK(tree_n);
  if (C == 0) {
    HIP_TRY(hipMemsetAsync(tree_n, 0, 4 * (size_t)R, ctx->stream));
    return NAVGPU_OK;
  }
  ARG_CHECK(feat_src && coords && tree_pts && tree_col);
  const RowsLds L = rows_lds(C, kRowsBlock, false);
  RC(set_lds(k_rows_build, L.total));
  TimedRegion tr(ctx, "rows_build");
  hipLaunchKernelGGL(k_rows_build, dim3(R), dim3(kRowsBuildBlock), L.total,
                     ctx->stream, feat_src, coords, R, C, tree_pts, tree_col,
                     tree_n, mask_out);
  CHECK_LAUNCH("k_rows_build");
  return NAVGPU_OK;
}

int navgpu_kd_rows_nodes_dev(navgpu_ctx *ctx, const double *tree_pts,
                             const int32_t *tree_n, int R, int C,
                             uint64_t host_base, void *nodes, int32_t *row_off) {
  ARG_CHECK(ctx);
  RC(check_rows_shape(R, C, false));
  ARG_CHECK(row_off);
  if (R == 0) {
    HIP_TRY(hipMemsetAsync(row_off, 0, 4, ctx->stream));
    return NAVGPU_OK;
  }
  ARG_CHECK(tree_n && (C == 0 || (tree_pts && nodes)));
  ARG_CHECK(R <= 65535);  // grid.y of k_rows_nodes
  hipLaunchKernelGGL(k_rows_offsets, dim3(1), dim3(kOffBlock), 0, ctx->stream,
                     tree_n, R, row_off);
  CHECK_LAUNCH("k_rows_offsets");
  if (C == 0) return NAVGPU_OK;
  hipLaunchKernelGGL(k_rows_nodes, dim3((C + 255) / 256, R), dim3(256), 0,
                     ctx->stream, tree_pts, tree_n, row_off, C, host_base,
                     (uint64_t *)nodes);
  CHECK_LAUNCH("k_rows_nodes");
  return NAVGPU_OK;
}

int navgpu_host_alloc(navgpu_ctx *ctx, size_t bytes, void **hptr) {
  ARG_CHECK(ctx && hptr);
  *hptr = nullptr;
  hipError_t e = hipHostMalloc(hptr, bytes ? bytes : 16, hipHostMallocDefault);
  if (e != hipSuccess) {
    set_err("hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
    *hptr = nullptr;
    return NAVGPU_ENOMEM;
  }
  return NAVGPU_OK;
}

void navgpu_host_free(navgpu_ctx *ctx, void *hptr) {
  if (!ctx || !hptr) return;
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->aux) (void)hipStreamSynchronize(ctx->aux);
  (void)hipHostFree(hptr);
}

int navgpu_kd_query_rows_dev(navgpu_ctx *ctx, const double *tree_pts,
                             const int32_t *tree_n, const double *feat_src,
                             const double *queries, int R, int C,
                             int32_t *nn_pos, double *nn_dist,
                             int32_t *mask_out) {
  ARG_CHECK(ctx);
  RC(check_rows_shape(R, C, true));
  if ((size_t)R * C == 0) return NAVGPU_OK;
  ARG_CHECK(tree_pts && tree_n && feat_src && queries && nn_pos && nn_dist);
  const char *qt = getenv("NAVGPU_ROWS_QUERY_TREE");
  if (!(qt && *qt && *qt != '0')) {
    // the screen (default): >= 1024 workgroups, >= 128 columns each (two
    // ~74 KB workgroups per CU at C = 2048)
    int S = 1;
    while (S < 16 && (long long)R * S < 1024 && C / (2 * S) >= 128) S <<= 1;
    const int w = (C + S - 1) / S;
    const int cp = (C + kScreenChunk - 1) / kScreenChunk * kScreenChunk;
    const int lds = 3 * align16(8 * cp) + align16(48 * (cp / kScreenChunk)) +
                    align16(24 * (w + 4)) + 2 * align16(2 * w) + align16(4 * 40) +
                    4 * kRowsQBlock * kStackDepth;
    if (lds > lds_limit()) {
      set_err("rows_query: C=%d needs %d B of LDS (device limit %d)", C, lds, lds_limit());
      return NAVGPU_ERANGE;
    }
    RC(set_lds(k_rows_query_screen<kRowsQBlock>, lds));
    TimedRegion tr(ctx, "rows_query");
    hipLaunchKernelGGL(k_rows_query_screen<kRowsQBlock>, dim3(R, S), dim3(kRowsQBlock), lds,
                       ctx->stream, tree_pts, tree_n, feat_src, queries, R, C, nn_pos, nn_dist,
                       mask_out);
    CHECK_LAUNCH("k_rows_query_screen");
    return NAVGPU_OK;
  }
  // NAVGPU_ROWS_QUERY_TREE=1: the reference walk for every query. Column
  // splits per row: >= 512 workgroups in all (2 per CU), slices of at least
  // 256 columns (one per thread)
  int S = 1;
  while (S < 8 && (long long)R * S < 512 && C / (2 * S) >= kRowsQBlock) S <<= 1;
  const int w = (C + S - 1) / S;
  const int lds = rows_query_lds(C, w);
  if (lds > lds_limit()) {
    set_err("rows_query: C=%d needs %d B of LDS (device limit %d)", C, lds, lds_limit());
    return NAVGPU_ERANGE;
  }
  RC(set_lds(k_rows_query, lds));
  TimedRegion tr(ctx, "rows_query");
  hipLaunchKernelGGL(k_rows_query, dim3(R, S), dim3(kRowsQBlock), lds, ctx->stream,
                     tree_pts, tree_n, feat_src, queries, R, C, nn_pos, nn_dist, mask_out);
  CHECK_LAUNCH("k_rows_query");
  return NAVGPU_OK;
}

int navgpu_rows_corr_dev(navgpu_ctx *ctx, const double *tree_pts,
                         const int32_t *tree_n, const int32_t *nn_pos,
                         const double *nn_dist, const double *ori, int R, int C,
                         int32_t *keep, double *sums) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  if (C > kMaxRowCols) {
    set_err("rows_corr: C=%d exceeds %d", C, kMaxRowCols);
    return NAVGPU_ERANGE;
  }
  if ((size_t)R * C == 0) return NAVGPU_OK;
  ARG_CHECK(tree_pts && tree_n && nn_pos && nn_dist && ori && sums);
  int HS = 64;
  while (HS < 2 * C) HS <<= 1;
  const int lds = HS * (8 + 4 + 4 + 4) + 4 * C;
  RC(set_lds(k_rows_corr, lds));
  TimedRegion tr(ctx, "rows_corr");
  hipLaunchKernelGGL(k_rows_corr, dim3(R), dim3(kCorrBlock), lds, ctx->stream, tree_pts,
                     tree_n, nn_pos, nn_dist, ori, C, HS, keep, sums, nullptr, nullptr);
  CHECK_LAUNCH("k_rows_corr");
  return NAVGPU_OK;
}

int navgpu_rows_corr_list_dev(navgpu_ctx *ctx, const double *tree_pts,
                              const int32_t *tree_n, const int32_t *nn_pos,
                              const double *nn_dist, const double *ori, int R, int C,
                              double *list, int32_t *count) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  if (C > kMaxRowCols) {
    set_err("rows_corr_list: C=%d exceeds %d", C, kMaxRowCols);
    return NAVGPU_ERANGE;
  }
  ARG_CHECK(count);
  if ((size_t)R * C == 0) {
    HIP_TRY(hipMemsetAsync(count, 0, 8, ctx->stream));
    return NAVGPU_OK;
  }
  ARG_CHECK(tree_pts && tree_n && nn_pos && nn_dist && ori && list);
  int HS = 64;
  while (HS < 2 * C) HS <<= 1;
  const int lds = HS * (8 + 4 + 4 + 4) + 4 * C;
  double *ent, *sums;
  int32_t *ent_n;
  RC(ws(ctx, kCorrEnt, 7 * (size_t)R * C, &ent));
  RC(ws(ctx, kCorrN, (size_t)R, &ent_n));
  RC(ws(ctx, kCorrSums, 6 * (size_t)R, &sums));
  RC(set_lds(k_rows_corr, lds));
  TimedRegion tr(ctx, "rows_corr");
  hipLaunchKernelGGL(k_rows_corr, dim3(R), dim3(kCorrBlock), lds, ctx->stream, tree_pts,
                     tree_n, nn_pos, nn_dist, ori, C, HS, nullptr, sums, ent, ent_n);
  CHECK_LAUNCH("k_rows_corr");
  hipLaunchKernelGGL(k_corr_pack, dim3(R), dim3(256), 0, ctx->stream, ent, ent_n, sums, R, C,
                     list, count);
  CHECK_LAUNCH("k_corr_pack");
  return NAVGPU_OK;
}

namespace {

// The per-row scan-pair step over `rows` rows ([pair][R][C], R | rows).
// Default: k_curvature (both masks) -> k_rows_screen (exact argmin per query,
// ties flagged) -> the tree kernel for flagged rows only. NAVGPU_ROWS_SCREEN=0
// runs the tree kernel on every row (the r1 path; same results).
int rows_match_launch(navgpu_ctx *ctx, const double *src, const double *tgt, int rows,
                      int R, int C, int32_t *src_mask, int32_t *tgt_mask, int32_t *nn_idx,
                      double *nn_dist) {
  const char *sc = getenv("NAVGPU_ROWS_SCREEN");
  const bool screen = !(sc && *sc == '0');
  // enough rows to fill the chip several times over: the lean tree kernel
  // (two rows per CU); a short batch keeps the 512-thread one (lower latency)
  const bool lean = C <= kLeanMaxC && rows >= 1024 && !getenv("NAVGPU_ROWS_NO_LEAN");
  const int32_t *tie = nullptr;
  int S = 1;
  TimedRegion tr(ctx, "rows_match");
  if (screen) {
    const size_t N = (size_t)rows * C;
    if (!src_mask) RC(ws(ctx, kRowMaskS, N, &src_mask));
    if (!tgt_mask) RC(ws(ctx, kRowMaskT, N, &tgt_mask));
    // column splits: >= 512 workgroups in all (two per CU: ~64 KB of LDS
    // each), >= 128 columns each; 512 threads once a split holds >= 512
    // columns (measured: K2 83 us at S = 4 x 512 threads, 102 us at S = 8 x
    // 256; a K4 batch is fastest unsplit at 512 threads)
    while (S < 8 && (long long)rows * S < 512 && C / (2 * S) >= 128) S <<= 1;
    if (const char *e = getenv("NAVGPU_SCREEN_S")) S = std::max(1, std::min(64, atoi(e)));
    const int w = (C + S - 1) / S;
    int32_t *tf;
    RC(ws(ctx, kRowTie, (size_t)rows * S, &tf));
    tie = tf;
    ctx->screen_rows = rows;
    ctx->screen_S = S;
    // R1 on both clouds, <= 65535 rows per launch (grid y)
    for (int r0 = 0; r0 < rows; r0 += 65535) {
      const int nr = std::min(rows - r0, 65535);
      const size_t o = (size_t)r0 * C;
      CurvJob J = {{src + 3 * o, tgt + 3 * o}, {src_mask + o, tgt_mask + o}, {nullptr, nullptr}};
      hipLaunchKernelGGL(k_curvature, dim3((C + kCurvTile - 1) / kCurvTile, nr, 2),
                         dim3(kCurvTile), 0, ctx->stream, J, nr, C);
      CHECK_LAUNCH("k_curvature");
    }
    const int lds = rows_screen_lds(C, w);
    if (lds > lds_limit()) {
      set_err("rows_screen: C=%d needs %d B of LDS (device limit %d)", C, lds, lds_limit());
      return NAVGPU_ERANGE;
    }
    const char *nte = getenv("NAVGPU_SCREEN_NT");
    if (nte ? atoi(nte) == 512 : w >= 512) {
      RC(set_lds(k_rows_screen<512>, lds));
      hipLaunchKernelGGL(k_rows_screen<512>, dim3(rows, S), dim3(512), lds, ctx->stream, src,
                         tgt, R, C, src_mask, tgt_mask, nn_idx, nn_dist, tf);
    } else {
      RC(set_lds(k_rows_screen<256>, lds));
      hipLaunchKernelGGL(k_rows_screen<256>, dim3(rows, S), dim3(256), lds, ctx->stream, src,
                         tgt, R, C, src_mask, tgt_mask, nn_idx, nn_dist, tf);
    }
    CHECK_LAUNCH("k_rows_screen");
    // the tie pass writes no masks (already written)
    src_mask = nullptr;
    tgt_mask = nullptr;
  }
  if (lean) {
    const int lds = rows_lean_lds(C, 256);
    RC(set_lds(k_rows_match_lean<256>, lds));
    hipLaunchKernelGGL(k_rows_match_lean<256>, dim3(rows), dim3(256), lds, ctx->stream, src,
                       tgt, R, C, src_mask, tgt_mask, nn_idx, nn_dist, tie, S);
    CHECK_LAUNCH("k_rows_match_lean");
    return NAVGPU_OK;
  }
  const RowsLds L = rows_lds(C, kRowsBlock, true);
  RC(set_lds(k_rows_match, L.total));
  hipLaunchKernelGGL(k_rows_match, dim3(rows), dim3(kRowsBlock), L.total, ctx->stream, src,
                     tgt, R, C, src_mask, tgt_mask, nn_idx, nn_dist, tie, S);
  CHECK_LAUNCH("k_rows_match");
  return NAVGPU_OK;
}

}  // namespace

int navgpu_rows_match_dev(navgpu_ctx *ctx, const double *src,
                          const double *tgt, int R, int C, int32_t *src_mask,
                          int32_t *tgt_mask, int32_t *nn_idx, double *nn_dist) {
  ARG_CHECK(ctx);
  RC(check_rows_shape(R, C, true));
  if ((size_t)R * C == 0) return NAVGPU_OK;
  ARG_CHECK(src && tgt && nn_idx && nn_dist);
  return rows_match_launch(ctx, src, tgt, R, R, C, src_mask, tgt_mask, nn_idx, nn_dist);
}

int navgpu_rows_match_batch_dev(navgpu_ctx *ctx, const double *src,
                                const double *tgt, int npairs, int R, int C,
                                int32_t *src_mask, int32_t *tgt_mask,
                                int32_t *nn_idx, double *nn_dist) {
  ARG_CHECK(ctx && npairs >= 0);
  RC(check_rows_shape(R, C, true));
  ARG_CHECK((long long)npairs * R <= INT32_MAX && (long long)npairs * R * C < INT32_MAX);
  if ((size_t)npairs * R * C == 0) return NAVGPU_OK;
  ARG_CHECK(src && tgt && nn_idx && nn_dist);
  return rows_match_launch(ctx, src, tgt, npairs * R, R, C, src_mask, tgt_mask, nn_idx,
                           nn_dist);
}

int navgpu_rows_match_host(navgpu_ctx *ctx, const double *src,
                           const double *tgt, int R, int C, int32_t *src_mask,
                           int32_t *tgt_mask, int32_t *nn_idx,
                           double *nn_dist) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  const size_t N = (size_t)R * C;
  if (!N) return NAVGPU_OK;
  ARG_CHECK(src && tgt && nn_idx && nn_dist);
  double *ds, *dt, *dd;
  int32_t *dsm, *dtm, *di;
  RC(ws(ctx, kH0, 3 * N, &ds));
  RC(ws(ctx, kH1, 3 * N, &dt));
  RC(ws(ctx, kH2, N, &dsm));
  RC(ws(ctx, kH3, N, &dtm));
  RC(ws(ctx, kH4, N, &di));
  RC(ws(ctx, kH5, N, &dd));
  HIP_TRY(hipMemcpyAsync(ds, src, 24 * N, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dt, tgt, 24 * N, hipMemcpyHostToDevice, ctx->stream));
  RC(navgpu_rows_match_dev(ctx, ds, dt, R, C, dsm, dtm, di, dd));
  HIP_TRY(hipMemcpyAsync(nn_idx, di, 4 * N, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipMemcpyAsync(nn_dist, dd, 8 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (src_mask)
    HIP_TRY(hipMemcpyAsync(src_mask, dsm, 4 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (tgt_mask)
    HIP_TRY(hipMemcpyAsync(tgt_mask, dtm, 4 * N, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return NAVGPU_OK;
}

// ------------------------------------------------- kdtree.h buildKDTree
int navgpu_kd_build_dev(navgpu_ctx *ctx, double *pts, size_t n, int depth0) {
  ARG_CHECK(ctx && depth0 >= 0);
  ARG_CHECK(n < ((size_t)1 << 30));
  if (n < 2) return NAVGPU_OK;  // kdtree.c:22: nothing to permute
  ARG_CHECK(pts);
  const int ni = (int)n;
  TimedRegion tr(ctx, "kd_build");
  if (n <= 65535 && kd_build_lds_bytes(ni) <= lds_limit()) {
    const int lds = kd_build_lds_bytes(ni);
    RC(set_lds(k_kd_build_lds, lds));
    hipLaunchKernelGGL(k_kd_build_lds, dim3(1), dim3(1024), lds, ctx->stream,
                       pts, ni, depth0 % 3);
    CHECK_LAUNCH("k_kd_build_lds");
    return NAVGPU_OK;
  }
  double *fc;
  uint32_t *P, *T;
  RC(ws(ctx, kKdFc, 3 * n, &fc));
  RC(ws(ctx, kKdP, n, &P));
  RC(ws(ctx, kKdT, n, &T));
  // levels above the leaves: until every subarray (<= ceil(n / 2^L)) fits
  // the LDS build of k_kd_leaves
  int L = 0;
  while (L < 30 && !(((n + ((size_t)1 << L) - 1) >> L) <= 65535 &&
                     kd_build_lds_bytes((int)((n + ((size_t)1 << L) - 1) >> L)) <= lds_limit()))
    ++L;
  if (getenv("NAVGPU_KD_ONE_WG") || L >= 24) {  // the single-workgroup build (reference for tests)
    hipLaunchKernelGGL(k_kd_build_global, dim3(1), dim3(1024), 0, ctx->stream,
                       pts, ni, depth0 % 3, fc, P, T);
    CHECK_LAUNCH("k_kd_build_global");
    return NAVGPU_OK;
  }
  hipLaunchKernelGGL(k_kd_prep, dim3(grid1d(n, 256)), dim3(256), 0, ctx->stream, pts, ni, fc, P);
  CHECK_LAUNCH("k_kd_prep");
  // levels whose subarrays exceed kSelMinLen: grid-wide passes over all of
  // a level's windows at once; below: a workgroup per subarray
  constexpr int kSelMinLen = 0;  // NAVGPU_KD_NO_SEL=1: a workgroup per subarray at every level
  uint32_t *Ptmp;
  RC(ws(ctx, kKdPtmp, n, &Ptmp));
  const int kRounds = 2;  // 64 hops, then 64 more of the compressed chains;
                          // scatter follows whatever is left
  int32_t *stbuf;
  const int nWmax = 1 << std::max(0, L - 1);
  const int nbmax = (int)((n + kSelChunk - 1) / kSelChunk);
  RC(ws(ctx, kKdSel, (size_t)7 * nWmax + (size_t)nWmax * nbmax + kRounds + 1, &stbuf));
  for (int d = 0; d < L; ++d) {
    const int nW = 1 << d;
    const int maxlen = (int)(n >> d);
    if (maxlen < kSelMinLen || getenv("NAVGPU_KD_NO_SEL")) {
      hipLaunchKernelGGL(k_kd_level, dim3(nW), dim3(1024), 0, ctx->stream, fc, ni,
                         depth0 % 3, d, P, T);
      CHECK_LAUNCH("k_kd_level");
      continue;
    }
    SelState st;
    st.nW = nW;
    st.nb = (maxlen + kSelChunk - 1) / kSelChunk;
    int32_t *q = stbuf;
    st.first = q; q += nW;
    st.last = q; q += nW;
    st.nth = q; q += nW;
    st.act = q; q += nW;
    st.S = q; q += nW;
    st.pivot = q; q += nW;
    st.nact = q; q += nW;
    st.unres = q; q += kRounds + 1;
    st.cnt = q;
    const double *key = fc + (size_t)((depth0 % 3 + d) % 3) * n;
    hipLaunchKernelGGL(k_sel_init, dim3((nW + 255) / 256), dim3(256), 0, ctx->stream, st, ni, d);
    CHECK_LAUNCH("k_sel_init");
    HIP_TRY(hipMemsetAsync(st.unres, 0, 4 * (kRounds + 1), ctx->stream));
    const dim3 grid(st.nb, nW);
    // quickselect iterations until every window found its median; the
    // active count is read back every few iterations
    for (int it = 0; maxlen > kSelFinishMax; ++it) {
      hipLaunchKernelGGL(k_sel_count, grid, dim3(kSelThreads), 0, ctx->stream, st, key, P);
      hipLaunchKernelGGL(k_sel_rank, grid, dim3(kSelThreads), 0, ctx->stream, st, key, P, Ptmp,
                         T);
      hipLaunchKernelGGL(k_sel_jump0, dim3(st.nb * kSelPer, nW), dim3(kSelThreads), 0,
                         ctx->stream, st, T);
      for (int r = 1; r < kRounds; ++r)  // only if the round before left chains
        hipLaunchKernelGGL(k_sel_jump, grid, dim3(kSelThreads), 0, ctx->stream, st, T, r);
      hipLaunchKernelGGL(k_sel_scatter, grid, dim3(kSelThreads), 0, ctx->stream, st, P, Ptmp, T);
      hipLaunchKernelGGL(k_sel_update, dim3(1), dim3(256), 0, ctx->stream, st, kRounds);
      CHECK_LAUNCH("k_sel");
      if (it > 4 * ni + 64) {  // quickselect shrinks its window every iteration
        set_err("kd_build: selection did not converge (level %d)", d);
        return NAVGPU_EHIP;
      }
      if (it % 4 == 3) {
        int32_t nact = 0;
        HIP_TRY(hipMemcpyAsync(&nact, st.nact, 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        if (getenv("NAVGPU_KD_TRACE"))
          fprintf(stderr, "kd_build level %d (%d windows, %d max): it %d active %d\n", d, nW,
                  maxlen, it, nact);
        if (nact == 0) break;
      }
    }
    const int flds = kSelFinishMax * (8 + 4 + 2 + 2);
    RC(set_lds(k_sel_finish, flds));
    hipLaunchKernelGGL(k_sel_finish, dim3(nW), dim3(1024), flds, ctx->stream, st, key, P);
    CHECK_LAUNCH("k_sel_finish");
  }
  hipLaunchKernelGGL(k_kd_gather, dim3(grid1d(n, 256)), dim3(256), 0, ctx->stream, pts, fc, ni, P);
  CHECK_LAUNCH("k_kd_gather");
  const int leaf = (int)((n + ((size_t)1 << L) - 1) >> L);
  const int lds = kd_build_lds_bytes(leaf);
  RC(set_lds(k_kd_leaves, lds));
  hipLaunchKernelGGL(k_kd_leaves, dim3(1u << L), dim3(1024), lds, ctx->stream, pts, fc, ni,
                     depth0 % 3, L, P);
  CHECK_LAUNCH("k_kd_leaves");
  return NAVGPU_OK;
}

int navgpu_kd_build_host(navgpu_ctx *ctx, double *pts, size_t n, int depth0) {
  ARG_CHECK(ctx);
  if (n < 2) return NAVGPU_OK;
  ARG_CHECK(pts);
  double *dp;
  RC(ws(ctx, kH0, 3 * n, &dp));
  HIP_TRY(hipMemcpyAsync(dp, pts, 24 * n, hipMemcpyHostToDevice, ctx->stream));
  RC(navgpu_kd_build_dev(ctx, dp, n, depth0));
  HIP_TRY(hipMemcpyAsync(pts, dp, 24 * n, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return NAVGPU_OK;
}

// ------------------------------------------------------ memory helpers
int navgpu_malloc(navgpu_ctx *ctx, size_t bytes, void **dptr) {
  ARG_CHECK(ctx && dptr);
  *dptr = nullptr;
  hipError_t e = hipMalloc(dptr, bytes ? bytes : 16);
  if (e != hipSuccess) {
    set_err("hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    *dptr = nullptr;
    return NAVGPU_ENOMEM;
  }
  return NAVGPU_OK;
}

void navgpu_free(navgpu_ctx *ctx, void *dptr) {
  if (!ctx || !dptr) return;
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipFree(dptr);
}

int navgpu_upload(navgpu_ctx *ctx, void *dst, const void *src, size_t bytes) {
  ARG_CHECK(ctx);
  if (!bytes) return NAVGPU_OK;
  ARG_CHECK(dst && src);
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return NAVGPU_OK;
}

int navgpu_download(navgpu_ctx *ctx, void *dst, const void *src, size_t bytes) {
  ARG_CHECK(ctx);
  if (!bytes) return NAVGPU_OK;
  ARG_CHECK(dst && src);
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return NAVGPU_OK;
}

// ------------------------------------------------------------ global k-NN
}  // extern "C"

// The k-NN call (navgpu_knn_dev).
static int knn_run(navgpu_ctx *ctx, const double *tgt, size_t nt, const double *queries,
                   size_t nq, int k, int32_t *idx, double *dist) {
  ARG_CHECK(ctx && k >= 1 && k <= 16);
  ARG_CHECK(nt < (size_t)INT32_MAX / 2 && nq < (size_t)INT32_MAX);
  if (!nq) return NAVGPU_OK;
  ARG_CHECK(queries && idx && dist && (tgt || nt == 0));
  const double occ = ctx->knn_occ;
  const int sx = ctx->knn_sx;
  const long long capl = (long long)((double)nt / occ) * 2 * sx + 1024;
  ARG_CHECK(capl < INT32_MAX / 2);
  const int cap = (int)capl;
  const int nscan = cap + 1;  // start[] has one entry past the last cell
  // binning geometry (k_bin_*): coarse buckets of 2^shift cells, at most
  // kBinMaxBuckets of them; chunks of P points per histogram block
  // at least one cell per fine-pass thread (the fine scan gives each thread a
  // contiguous run of 2^shift / threads cells)
  int shift = NAVGPU_BIN_MIN_SHIFT;
  while ((1 << shift) < kBinFineThreads) ++shift;
  while (((long long)nscan + (1 << shift) - 1) >> shift > kBinMaxBuckets) ++shift;
  if (shift > kBinMaxShift) {
    set_err("knn: %zu targets exceed the binning capacity", nt);
    return NAVGPU_ERANGE;
  }
  BinJob J;
  J.shift = shift;
  J.nb = (int)(((long long)nscan + (1 << shift) - 1) >> shift);
  const size_t ns[2] = {nt, nq};
  long long ntab = 0;
  for (int side = 0; side < 2; ++side) {
    BinSide &S = J.s[side];
    S.n = (int)ns[side];
    S.P = (int)std::max<size_t>(NAVGPU_BIN_P, (ns[side] / 2000 + 256) / 256 * 256);
    S.nblk = (int)std::max<size_t>(1, (ns[side] + S.P - 1) / S.P);
    S.tab = (int)ntab;
    S.sub = side ? (int)nt : 0;
    ntab += (long long)J.nb * S.nblk + 1;
  }
  const int nbs = (int)((ntab + kScanTile - 1) / kScanTile);
  if (nbs > kScanTile) {
    set_err("knn: binning table of %lld entries exceeds the scan capacity", ntab);
    return NAVGPU_ERANGE;
  }
  const int nparts = (int)std::min<size_t>(kBBoxBlocks, std::max<size_t>(1, grid1d(nt, 256)));
  double *part;
  GridParams *gp;
  int *tab, *offs, *tstart, *qstart, *bsum, *qperm;
  Rec16 *rec = nullptr;
  TRec *tsort = nullptr;
  BinPt *bin_t = nullptr;
  int2 *bin_q;
  RC(ws(ctx, kBBox, (size_t)kBBoxBlocks * 6, &part));
  RC(ws(ctx, kParams, 1, &gp));
  RC(ws(ctx, kCnt, (size_t)ntab, &tab));
  RC(ws(ctx, kCellId, (size_t)ntab, &offs));
  RC(ws(ctx, kStart, nscan, &tstart));
  RC(ws(ctx, kQStart, nscan, &qstart));
  RC(ws(ctx, kBSum, nbs, &bsum));
  int *counters;
  RC(ws(ctx, kStats, 4, &counters));  // [n_ovf, n_slow, pad, pad], zeroed by k_grid_params
  if (nt) {
    RC(ws(ctx, kSlotBuf, nt, &bin_t));
    RC(ws(ctx, kRec, nt + 2, &rec));  // + 2: a last pair may read one past the end
    RC(ws(ctx, kTSort, nt, &tsort));
  }
  RC(ws(ctx, kQCell, nq, &bin_q));
  RC(ws(ctx, kQPerm, nq, &qperm));
  J.s[0].p = tgt;
  J.s[1].p = queries;
  J.s[0].start = tstart;
  J.s[1].start = qstart;
  J.bin_t = bin_t;
  J.bin_q = bin_q;
  J.rec = rec;
  J.tsort = tsort;
  J.qperm = qperm;
  hipStream_t s = ctx->stream;
  {
    TimedRegion tb(ctx, "knn_build");
    if (nt) {
      hipLaunchKernelGGL(k_bbox_partial, dim3(nparts), dim3(256), 0, s, tgt, nt, part);
      CHECK_LAUNCH("k_bbox_partial");
    }
    hipLaunchKernelGGL(k_grid_params, dim3(1), dim3(256), 0, s, part, nt ? nparts : 0, nt,
                       cap, occ, sx, nq, gp, counters);
    CHECK_LAUNCH("k_grid_params");
    const dim3 gb(J.s[0].nblk + J.s[1].nblk);
    hipLaunchKernelGGL(k_bin_hist, gb, dim3(256), 0, s, J, gp, tab);
    CHECK_LAUNCH("k_bin_hist");
    const int ntabi = (int)ntab;
    hipLaunchKernelGGL(k_scan_sums, dim3(nbs), dim3(kScanBlock), 0, s, tab, ntabi, bsum);
    CHECK_LAUNCH("k_scan_sums");
    hipLaunchKernelGGL(k_scan_apply, dim3(nbs), dim3(kScanBlock), 0, s, tab, ntabi, bsum,
                       offs);
    CHECK_LAUNCH("k_scan_apply");
    hipLaunchKernelGGL(k_bin_scatter, gb, dim3(256), 0, s, J, gp, (const int *)offs);
    CHECK_LAUNCH("k_bin_scatter");
    const size_t lds = (size_t)4 << shift;
    if (lds > 48 * 1024)
      HIP_TRY(hipFuncSetAttribute((const void *)k_bin_fine,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_bin_fine, dim3(2 * J.nb), dim3(kBinFineThreads), lds, s, J, gp,
                       (const int *)offs, nscan);
    CHECK_LAUNCH("k_bin_fine");
  }
  KnnLists lists;
  RC(ws(ctx, kOvf, (size_t)cap + 1, &lists.ovf_tiles));
  RC(ws(ctx, kSlowQ, nq, &lists.slow_q));
  RC(ws(ctx, kSlowThr, nq, &lists.slow_thr));
  lists.n_ovf = counters;
  lists.n_slow = counters + 1;
  lists.vec_out = ((uintptr_t)idx % 16 == 0 && (uintptr_t)dist % 16 == 0) ? 1 : 0;
#ifdef NAVGPU_SCALAR_OUT
  lists.vec_out = 0;
#endif
  TimedRegion tr(ctx, "knn_query");
  // tiles are walked by a grid of 8 x nbx blocks (block b -> XCD b % 8, the
  // placement HW_REG_XCC_ID reports); more blocks than resident slots
  // balance the uneven tiles (measured plateau from ~512 per XCD at 1M)
  const int nbx = ctx->knn_blocks > 0
                      ? ctx->knn_blocks
                      : (int)std::min<size_t>(768, std::max<size_t>(1, nq / 1300 + 1));
  const dim3 g(8 * nbx), b(kTileThreads);
  const dim3 go(8 * std::min(nbx, 4));  // overflow tiles: rare, few blocks (an empty pass is launch cost only)
  const dim3 gs(std::max<unsigned>(1, std::min<unsigned>(2048, grid1d(nq, 256))));
#define KNN_CASE(KK)                                                              \
  case KK:                                                                        \
    hipLaunchKernelGGL((k_knn<KK, false>), g, b, 0, s, gp, tstart, rec, tsort,   \
                       queries, qstart, qperm, idx, dist, lists);                 \
    hipLaunchKernelGGL((k_knn<KK, true>), go, b, 0, s, gp, tstart, rec, tsort,   \
                       queries, qstart, qperm, idx, dist, lists);                 \
    hipLaunchKernelGGL((k_knn_slow<KK>), gs, dim3(256), 0, s, gp, tstart, rec,    \
                       tsort, queries, idx, dist, lists);                         \
    break;
  switch (k) {
    KNN_CASE(1)
    KNN_CASE(2)
    KNN_CASE(3)
    KNN_CASE(4)
    KNN_CASE(5)
    KNN_CASE(6)
    KNN_CASE(7)
    KNN_CASE(8)
    KNN_CASE(9)
    KNN_CASE(10)
    KNN_CASE(11)
    KNN_CASE(12)
    KNN_CASE(13)
    KNN_CASE(14)
    KNN_CASE(15)
    KNN_CASE(16)
  }
#undef KNN_CASE
  CHECK_LAUNCH("k_knn");
  return NAVGPU_OK;
}

extern "C" {

int navgpu_knn_dev(navgpu_ctx *ctx, const double *tgt, size_t nt,
                   const double *queries, size_t nq, int k, int32_t *idx,
                   double *dist) {
  return knn_run(ctx, tgt, nt, queries, nq, k, idx, dist);
}

int navgpu_knn_host(navgpu_ctx *ctx, const double *tgt, size_t nt,
                    const double *queries, size_t nq, int k, int32_t *idx,
                    double *dist) {
  ARG_CHECK(ctx && k >= 1 && k <= 16);
  if (!nq) return NAVGPU_OK;
  ARG_CHECK(queries && idx && dist && (tgt || nt == 0));
  double *dt = nullptr, *dq, *dd;
  int32_t *di;
  if (nt) RC(ws(ctx, kH0, 3 * nt, &dt));
  RC(ws(ctx, kH1, 3 * nq, &dq));
  RC(ws(ctx, kH2, nq * k, &di));
  RC(ws(ctx, kH3, nq * k, &dd));
  if (nt)
    HIP_TRY(hipMemcpyAsync(dt, tgt, 24 * nt, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dq, queries, 24 * nq, hipMemcpyHostToDevice, ctx->stream));
  RC(navgpu_knn_dev(ctx, dt, nt, dq, nq, k, di, dd));
  HIP_TRY(hipMemcpyAsync(idx, di, 4 * nq * k, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dist, dd, 8 * nq * k, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return NAVGPU_OK;
}

int navgpu_pair_knn_dev(navgpu_ctx *ctx, const double *src, const double *tgt,
                        int R, int C, int k, int32_t *src_mask,
                        int32_t *tgt_mask, int32_t *idx, double *dist) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  const size_t N = (size_t)R * C;
  if (!N) return NAVGPU_OK;
  ARG_CHECK(src && tgt);
  if (!src_mask && !tgt_mask) return navgpu_knn_dev(ctx, tgt, N, src, N, k, idx, dist);
  // One curvature launch over both clouds, on a side stream forked from and
  // joined back into the context's stream: it is f64-bound and independent
  // of the (latency-bound) index build and query, so the two overlap.
  if (!ctx->aux) {
    HIP_TRY(hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
  }
  CurvJob J = {{src, tgt}, {src_mask, tgt_mask}, {nullptr, nullptr}};
  if (!src_mask) {  // only the target: it becomes cloud 0
    J.pts[0] = tgt;
    J.mask[0] = tgt_mask;
  }
  HIP_TRY(hipEventRecord(ctx->ev_fork, ctx->stream));
  HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
  {
    TimedRegion tr(ctx, "curvature", ctx->aux);
    dim3 grid((C + kCurvTile - 1) / kCurvTile, R, (src_mask && tgt_mask) ? 2 : 1);
    hipLaunchKernelGGL(k_curvature, grid, dim3(kCurvTile), 0, ctx->aux, J, R, C);
    CHECK_LAUNCH("k_curvature");
  }
  HIP_TRY(hipEventRecord(ctx->ev_join, ctx->aux));
  const int rc = knn_run(ctx, tgt, N, src, N, k, idx, dist);
  HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));  // join before returning
  return rc;
}

}  // extern "C"

// ---- measured HBM ceiling (a STREAM-copy figure beside the 8 TB/s
// peak). 16-B loads and stores, kStreamU vectors per lane with all loads
// issued before any store; blocks dealt round-robin over the XCDs like every
// other launch, each taking a contiguous span so a wave streams whole lines.
namespace {
#ifndef NAVGPU_COPY_U
#define NAVGPU_COPY_U 1  // 1 / 2 / 4 / 8 vectors per thread: 6.2 / 5.7 / 5.4 / 3.6 TB/s (r2)
#endif
constexpr int kStreamU = NAVGPU_COPY_U;
__global__ __launch_bounds__(256) void k_stream_copy(const int4 *__restrict__ src,
                                                     int4 *__restrict__ dst, size_t n) {
  // one contiguous span of kStreamU x 256 vectors per block, no grid-stride
  // loop: every block streams its span once
  const size_t b = (size_t)blockIdx.x * kStreamU * blockDim.x + threadIdx.x;
  int4 v[kStreamU];
#pragma unroll
  for (int u = 0; u < kStreamU; ++u) {
    const size_t i = b + (size_t)u * blockDim.x;
    if (i < n) v[u] = src[i];
  }
#pragma unroll
  for (int u = 0; u < kStreamU; ++u) {
    const size_t i = b + (size_t)u * blockDim.x;
#ifdef NAVGPU_COPY_NT
    if (i < n) __builtin_nontemporal_store(v[u], dst + i);
#else
    if (i < n) dst[i] = v[u];
#endif
  }
}
}  // namespace

extern "C" {

int navgpu_stream_copy_dev(navgpu_ctx *ctx, void *dst, const void *src, size_t bytes) {
  ARG_CHECK(ctx);
  if (!bytes) return NAVGPU_OK;
  ARG_CHECK(dst && src && bytes % 16 == 0 && (uintptr_t)dst % 16 == 0 &&
            (uintptr_t)src % 16 == 0);
  const size_t n = bytes / 16;
  const size_t per = (size_t)kStreamU * 256;
  ARG_CHECK((n + per - 1) / per < (size_t)INT32_MAX);
  const unsigned nb = (unsigned)std::max<size_t>(1, (n + per - 1) / per);
  TimedRegion tr(ctx, "stream_copy");
  hipLaunchKernelGGL(k_stream_copy, dim3(nb), dim3(256), 0, ctx->stream, (const int4 *)src,
                     (int4 *)dst, n);
  CHECK_LAUNCH("k_stream_copy");
  return NAVGPU_OK;
}

}  // extern "C"
