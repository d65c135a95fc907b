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
//   (global mode: the grid index and exact k-NN live in knn.hip)
#include "navgpu_common.h"

#define NAVGPU_VERSION "navgpu 0.2 (gfx950)"

namespace nv {
char g_err[1024] = "";

void set_err(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace nv

using namespace nv;

namespace {


constexpr int kRowsBlock = 512;     // 8 waves per row workgroup
#ifndef NAVGPU_ROWS_MATCH_BLOCK
#define NAVGPU_ROWS_MATCH_BLOCK 1024  // (r6: K2i 0.716 -> 0.696 ms against 512, three interleaved rounds)
#endif
// k_rows_match's threads (the tie pass): the build by all of them, the walk
// by the first kRowsBlock (their stacks are what rows_lds sizes)
constexpr int kRowsMatchBlock = NAVGPU_ROWS_MATCH_BLOCK;
static_assert(kRowsMatchBlock >= kRowsBlock && kRowsMatchBlock <= 1024, "rows match block");
#ifndef NAVGPU_ROWS_BUILD_BLOCK
#define NAVGPU_ROWS_BUILD_BLOCK 512
#endif
constexpr int kRowsBuildBlock = NAVGPU_ROWS_BUILD_BLOCK;  // k_rows_build (trees only)
constexpr int kStackDepth = 14;     // implicit-tree height bound, n < 8192
constexpr int kMaxRowCols = 8191;   // 13-bit stack-entry fields
constexpr int kCurvTile = 256;

// Diagnostic phase stamps (build with -DNAVGPU_STAMPS; never in the product
// ============================================================ device helpers


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
  // (p - s + k) / k exactly, with no integer divide: the f32 quotient
  // a * rcp(k) has a relative error below 2^-22 (rcp 1 ulp, two roundings),
  // so it is within one of a / k while a / k < 2^22, which holds for every
  // caller (positions are 16-bit: rows and LDS windows below 2^16, a < 2^17);
  // then one correction
  const int a = p - s + k;
  int q = (int)((float)a * __builtin_amdgcn_rcpf((float)k));
  const int r = a - q * k;
  q += r >= k ? 1 : (r < 0 ? -1 : 0);
  return p - k * q;
}

// The same nth_element for a window of at most 64 positions, held in the
// wave's registers (lane l = position first + l) from its first pass to its
// last (r4): a pass is two ballots, the tape chains resolved by shuffles, two
// forward permutes (ds_permute) and one key read; P is written once at the
// end. The window shrinks in lane space ([a, b]); lanes outside keep their
// final elements.
#ifndef NAVGPU_WAVE_REGS
#define NAVGPU_WAVE_REGS 1
#endif
constexpr bool kWaveRegs = NAVGPU_WAVE_REGS;
template <class IdxT>
__device__ void wave_nth_element_regs(const double *key, IdxT *P, int first, int last,
                                      int nth, int lane) {
  const int len = last - first + 1;  // <= 64
  int e = lane < len ? (int)P[first + lane] : 0;
  double k = key[e];
  const unsigned long long below = (1ull << lane) - 1ull;
  const int nl = nth - first;
  int a = 0, b = len - 1;
  while (a < b) {
    const int pe = __shfl(e, b, kWave);
    const double pk = __shfl(k, b, kWave);
    const bool inw = lane >= a && lane < b;
    const bool small = inw && ((k - pk) <= 0.0);  // kdtree.c:31-43
    const unsigned long long bal = __ballot(small);
    const unsigned long long lbal = __ballot(inw && !small);
    const int sp = a + __popcll(bal & below);  // a small's destination lane
    const int ps = a + __popcll(bal);          // the pivot's lane
    // tape word: bit 31 = resolved element, else the lane it equals
    unsigned w = 0x80000000u | (unsigned)e;
    if (small && sp != lane) w = (unsigned)tape_jump(lane, sp, lbal & below, 0);
    while (__ballot(!(w >> 31))) {
      const unsigned o = __shfl(w, (w >> 31) ? lane : (int)(w & (kWave - 1)), kWave);
      if (!(w >> 31)) w = o;
    }
    const int tv = (int)(w & 0x7fffffffu);
    // smalls to a .. ps-1; tape[ps] to b, tape[ps+1 .. b-1] stay; pivot at ps
    // (lanes with nothing to send write the pivot's lane, which takes pe)
    const int v1 = __builtin_amdgcn_ds_permute((small ? sp : ps) * 4, e);
    const bool tl = lane >= ps && lane < b;
    const int v2 = __builtin_amdgcn_ds_permute((tl ? (lane == ps ? b : lane) : ps) * 4, tv);
    if (lane >= a && lane < ps)
      e = v1;
    else if (lane == ps)
      e = pe;
    else if (lane > ps && lane <= b)
      e = v2;
    k = key[e];
    if (ps == nl) break;
    if (ps < nl)
      a = ps + 1;
    else
      b = ps - 1;
  }
  if (lane < len) P[first + lane] = (IdxT)e;
  wave_sync_mem();  // the writes before the next pass reads P
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
    if (!GMEM && kWaveRegs && last - first < kWave) {
      wave_nth_element_regs(key, P, first, last, nth, lane);
      return;
    }
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
// block pass form: 1 = r3 (a barrier per chunk for the counts, then
// barrier rounds for chains that cross waves), 2 = r4 (one barrier per chunk)
#ifndef NAVGPU_BLOCK_NTH_V
#define NAVGPU_BLOCK_NTH_V 2
#endif
template <class IdxT, bool GMEM = false>
__device__ void block_nth_element_r3(const double *key, IdxT *P, IdxT *T, int first,
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

template <class IdxT, bool GMEM = false>
__device__ void block_nth_element(const double *key, IdxT *P, IdxT *T, int first,
                                  int last, int nth) {
#if NAVGPU_BLOCK_NTH_V == 1
  block_nth_element_r3<IdxT, GMEM>(key, P, T, first, last, nth);
#else
  // r4: ONE barrier per chunk. Before it every wave publishes its small and
  // large ballots, its small count and the chunk's elements (E); after it a
  // lane follows its tape chain by itself: a run of smalls is one tape_jump,
  // a position of an earlier chunk reads its final T, a large position or a
  // fixed point (sp == p) reads E, and a small position of another wave of
  // this chunk takes that wave's ballots from LDS and jumps again (on scan
  // rows 59 % of the waves need no hop and the mean of a wave's longest
  // chain is 1.5 hops). The buffers alternate between chunks, so a wave one
  // chunk ahead never overwrites what a slower wave still reads.
  constexpr int NWM = kBlockNthMax / kWave;
  __shared__ unsigned long long bsb[2][NWM], blb[2][NWM];
  __shared__ int bcn[2][NWM];
  __shared__ uint32_t bel[2][kBlockNthMax];
  __shared__ int bpre[NWM][NWM + 1];  // per wave: its copy of the chunk's wave prefix
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const int bd = blockDim.x, nw = bd / kWave, wbase = wid * kWave;
  const unsigned long long below = (1ull << lane) - 1ull;
  int chunk = 0;
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
    int e_n = tid < m ? (int)P[first + tid] : 0;
    double k_n = key[e_n];
    for (int cs = 0; cs < m; cs += bd, ++chunk) {
      const int b = chunk & 1;
      const int p = cs + tid;
      const bool act = p < m;
      const int e = e_n;
      const bool small = act && ((k_n - pk) <= 0.0);  // kdtree.c:31-43
      if (cs + bd < m) {  // the next chunk's reads (this chunk writes below it)
        const int pn = p + bd;
        e_n = pn < m ? (int)P[first + pn] : 0;
        k_n = key[e_n];
      }
      const unsigned long long bal = __ballot(small);
      const unsigned long long lbal = __ballot(act && !small);
      bel[b][tid] = (uint32_t)e;
      if (lane == 0) {
        bsb[b][wid] = bal;
        blb[b][wid] = lbal;
        bcn[b][wid] = __popcll(bal);
      }
      __syncthreads();
      // the chunk's wave prefix (lane x of every wave: smalls in waves < x;
      // lane nw: the chunk's total), by DPP; this wave's own entries by
      // readlane, the others' (for hops) through bpre
      const int c = lane < nw ? bcn[b][lane] : 0;
      const int excl = wave_scan_add(c) - c;
      if (lane <= nw) bpre[wid][lane] = excl;
      const int before = __builtin_amdgcn_readlane(excl, wid);
      const int tot = __builtin_amdgcn_readlane(excl, nw);
      const int sp = S + before + lanes_below(bal);
      uint32_t w = (uint32_t)e;
      const bool hop = small && sp != p;
      if (__any(hop)) wave_sync_mem();  // bpre before the hops read it
      if (hop) {
        int y = tape_jump(p, sp, lbal & below, cs + wbase);
        for (;;) {
          if (y < cs) {
            w = (uint32_t)T[first + y];
            break;
          }
          const int wy = (y - cs) >> 6, ly = (y - cs) & (kWave - 1);
          const unsigned long long yb = (1ull << ly) - 1ull;
          const unsigned long long ysb = bsb[b][wy], ylb = blb[b][wy];
          const int spy = S + bpre[wid][wy] + __popcll(ysb & yb);
          if (((ylb >> ly) & 1ull) || spy == y) {
            w = bel[b][y - cs];
            break;
          }
          y = tape_jump(y, spy, ylb & yb, cs + (wy << 6));
        }
      }
      if (act) T[first + p] = (IdxT)w;
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
#endif
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

#ifndef NAVGPU_LANE_SUBTREE
#define NAVGPU_LANE_SUBTREE 16  // (r4: 32 -> 16, rows_probe --integer: build 593 -> 577 us)
#endif
constexpr int kLaneSubtree = NAVGPU_LANE_SUBTREE;  // subarrays this short: one lane per subtree
#ifndef NAVGPU_BLOCK_NTH_MIN
#define NAVGPU_BLOCK_NTH_MIN 256
#endif
constexpr int kBlockNthMin = NAVGPU_BLOCK_NTH_MIN;  // root partition by the block from here
#ifndef NAVGPU_BLOCK_LEVEL_MIN
#define NAVGPU_BLOCK_LEVEL_MIN 1024  // (r5: 512 -> 1024, K2i 0.728 -> 0.715 ms, K4i flat)
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
//
// stop: the query's minimum distance when the caller knows it (the screen's
// exact minimum, for a query whose answer the tree decides only by visit
// order), else -1. The first visited point at that distance is the answer
// (no later point is strictly closer, kdtree.c:117), so the walk ends there.
__device__ __forceinline__ void kd_query(const double *TX, const double *TY,
                                         const double *TZ, int n, double qx,
                                         double qy, double qz, uint32_t *stk,
                                         int stride, int *best_pos,
                                         double *best_dist, double stop = -1.0) {
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
        if (d == stop) {
          sp = 0;
          break;
        }
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
                                   int32_t *mask_out, bool build = true) {
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
  if (build) {
    block_build_kdtree<uint16_t>(FC, NS, n, P, (uint16_t *)(smem + L.t), 0);
  } else {  // the compacted features in column order (flattenPoints) only
    for (int i = threadIdx.x; i < n; i += blockDim.x) P[i] = (uint16_t)i;
    __syncthreads();
  }
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
// i+2's m2 (|a - b| squares to the same bits as |b - a|): two sqrt per point
// instead of four.
// One wave per 60 consecutive columns of a row: lane l holds column
// c0 - 2 + l (a 2-column halo on each side), the neighbours' points and the
// shared distances move between lanes by shuffles; no LDS, no barrier
// (r3: 24.4 -> 18.2 us for both 1M-point clouds of a K3 pair, against a
// 256-point LDS tile with two barriers).
// (r5) Each wave takes kCurvU consecutive segments of its row and issues all
// their loads, from clamped addresses, before any is used (one point per
// lane in flight left the kernel latency-bound).
constexpr int kCurvSeg = kWave - 4;  // output columns per segment
#ifndef NAVGPU_CURV_U
#define NAVGPU_CURV_U 4
#endif
constexpr int kCurvU = NAVGPU_CURV_U;  // segments per wave
__global__ __launch_bounds__(kCurvTile) void k_curvature(CurvJob J, int R, int C) {
  const int z = blockIdx.z;
  const double *pts = J.pts[z];
  const int r = blockIdx.y;
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = (int)blockIdx.x * (kCurvTile / kWave) + (int)threadIdx.x / kWave;
  if (wv * kCurvU * kCurvSeg >= C) return;  // wave-uniform
  const size_t rowoff = (size_t)r * C;
  double x[kCurvU], y[kCurvU], w[kCurvU];
#pragma unroll
  for (int u = 0; u < kCurvU; ++u) {
    const int j = (wv * kCurvU + u) * kCurvSeg - 2 + lane;  // this lane's column
    const double *p = pts + 3 * (rowoff + min(max(j, 0), C - 1));
    x[u] = p[0];
    y[u] = p[1];
    w[u] = p[2];
  }
#pragma unroll
  for (int u = 0; u < kCurvU; ++u) {
    const int c0 = (wv * kCurvU + u) * kCurvSeg;
    if (c0 >= C) break;  // wave-uniform
    const int j = c0 - 2 + lane;
    const bool in = j >= 0 && j < C;
    const double xx = in ? x[u] : 0.0, yy = in ? y[u] : 0.0, ww = in ? w[u] : 0.0;
    const double x1 = __shfl_down(xx, 1), y1 = __shfl_down(yy, 1), w1 = __shfl_down(ww, 1);
    const double x2 = __shfl_down(xx, 2), y2 = __shfl_down(yy, 2), w2 = __shfl_down(ww, 2);
    const double dA = ref_dist(xx, yy, ww, x1, y1, w1);  // d(j, j+1)
    const double dB = ref_dist(xx, yy, ww, x2, y2, w2);  // d(j, j+2)
    const double dAm = __shfl_up(dA, 1);                 // d(j-1, j)
    const double dBm = __shfl_up(dB, 2);                 // d(j-2, j)
    if (lane < 2 || lane >= kWave - 2 || j >= C) continue;
    double cv = 0.0;
    if (j >= 2 && j < C - 2) cv = curvature_of(dBm, dAm, dA, dB);  // src/slam.c:16-58
    J.mask[z][rowoff + j] = cv > 0.1 ? 1 : 0;
    if (J.curv[z]) J.curv[z][rowoff + j] = cv;
  }
}
constexpr int curv_grid_x(int C) {
  return ((C + kCurvSeg * kCurvU - 1) / (kCurvSeg * kCurvU) + kCurvTile / kWave - 1) /
         (kCurvTile / kWave);
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

__global__ __launch_bounds__(kRowsMatchBlock) void k_rows_match(
    const double *__restrict__ src, const double *__restrict__ tgt, int R,
    int C, int32_t *__restrict__ src_mask, int32_t *__restrict__ tgt_mask,
    int32_t *__restrict__ nn_idx, double *__restrict__ nn_dist,
    const int32_t *__restrict__ tie, int S) {
  const RowsLds L = rows_lds(C, kRowsBlock, true);
  const int r = blockIdx.x;
  if (tie && !row_has_tie(tie, r, S)) return;  // uniform
  const size_t rowoff = (size_t)r * C;
  const int pair_row0 = (r % R) * C;  // this row's offset within its pair
  NV_STAMP(rm0);
  const int n = row_stage_and_build(tgt, tgt, r, C, L, tgt_mask);
  NV_STAMP(rm1);
  NV_STAMP_ADD0(4, rm0, rm1);  // stage + build (slots 8-12 split it)
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
  for (int i = threadIdx.x; (int)threadIdx.x < kRowsBlock && i < nq; i += kRowsBlock) {
    const int c = QL[i];
    int bpos;
    double bd;
    // a tied query's exact minimum came from the screen (-1: walk it all)
    kd_query(TX, TY, TZ, n, sraw[3 * c], sraw[3 * c + 1], sraw[3 * c + 2],
             stk + threadIdx.x, kRowsBlock, &bpos, &bd, tie ? nn_dist[rowoff + c] : -1.0);
    nn_idx[rowoff + c] = bpos >= 0 ? pair_row0 + canon_col(TX, TY, TZ, T, n, bpos) : -1;
    nn_dist[rowoff + c] = bd;
  }
#ifdef NAVGPU_STAMPS
  NV_STAMP_ADD0(6, 0ull, (unsigned long long)nq);  // queries walked
  NV_COUNT0(7);                                    // rows that built
  __syncthreads();
  NV_STAMP(rm2);
  NV_STAMP_ADD0(5, rm1, rm2);  // source staging, masks and the walk (slowest lane)
#endif
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
// (r3) the SoA features are sized for F <= C of them: a tie pass runs first
// at F = kLeanF (three rows per CU instead of two), then again at F = C for
// the rows whose feature count exceeded it (flagged in `over` by the first
// launch; the others return at once); tree walks, only the tied queries'
// there, take one wave
constexpr int kLeanF = 1536;

__host__ __device__ inline int rows_lean_walkers(bool tie, int nt) { return tie ? kWave : nt; }

__host__ __device__ inline int rows_lean_lds(int C, int F, int walkers) {
  return align16(24 * F) + 3 * align16(2 * C) + align16(4 * walkers * kStackDepth) +
         align16(4 * 40);
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
    const int32_t *__restrict__ tie, int S, int F, int32_t *__restrict__ over, int second) {
  constexpr int kHold = kLeanMaxC / NT;
  const int r = blockIdx.x;
  if (tie && !row_has_tie(tie, r, S)) return;  // uniform
  if (second && !over[r]) return;              // the first launch did this row
  const size_t rowoff = (size_t)r * C;
  const int pair_row0 = (r % R) * C;
  const int walkers = rows_lean_walkers(tie != nullptr, NT);
  double *FC = (double *)smem;  // SoA, stride F
  uint16_t *FCOL = (uint16_t *)(smem + align16(24 * F));
  uint16_t *P = (uint16_t *)(smem + align16(24 * F) + align16(2 * C));
  uint16_t *T = (uint16_t *)(smem + align16(24 * F) + 2 * align16(2 * C));
  uint32_t *stk = (uint32_t *)(smem + align16(24 * F) + 3 * align16(2 * C));
  int *scan = (int *)(smem + align16(24 * F) + 3 * align16(2 * C) +
                      align16(4 * walkers * kStackDepth));
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
        if (pos < F) {
          FC[pos] = tg[3 * j];
          FC[F + pos] = tg[3 * j + 1];
          FC[2 * F + pos] = tg[3 * j + 2];
          FCOL[pos] = (uint16_t)j;
        }
      });
  // more features than this launch holds: the F = C launch takes the row
  if (!second) {
    if (threadIdx.x == 0) over[r] = n > F;
    if (n > F) return;  // uniform
  }
  block_build_kdtree<uint16_t, false, false>(FC, F, n, P, T, 0);
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
        hy[u] = FC[F + e];
        hz[u] = FC[2 * F + e];
        hc[u] = FCOL[e];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kHold; ++u) {
      const int pos = (int)threadIdx.x + u * NT;
      if (pos < n) {
        FC[pos] = hx[u];
        FC[F + pos] = hy[u];
        FC[2 * F + pos] = hz[u];
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
  const double *TX = FC, *TY = FC + F, *TZ = FC + 2 * F;
  for (int i = threadIdx.x; i < nq && (int)threadIdx.x < walkers; i += walkers) {
    const int c = QL[i];
    int bpos;
    double bd;
    kd_query(TX, TY, TZ, n, sg[3 * c], sg[3 * c + 1], sg[3 * c + 2], stk + threadIdx.x, walkers,
             &bpos, &bd, tie ? nn_dist[rowoff + c] : -1.0);
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
template <int NT, class Flag, class Load, class Put>
__device__ int compact_cols_f(int c0, int c1, Flag flag, Load load, Put put, uint16_t *rank_at,
                              int *cnt);
template <int NT, class Load, class Put>
__device__ int compact_cols(int c0, int c1, const int32_t *__restrict__ mask, Load load,
                            Put put, uint16_t *rank_at, int *cnt) {
  return compact_cols_f<NT>(
      c0, c1, [&](int j) { return mask[j] != 0; }, load, put, rank_at, cnt);
}
// the same with the keep test a functor (called once per column in [c0, c1))
template <int NT, class Flag, class Load, class Put>
__device__ int compact_cols_f(int c0, int c1, Flag flag, Load load, Put put, uint16_t *rank_at,
                              int *cnt) {
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
      // (evaluated at a clamped column, unconditionally: a condition around
      // a load makes hipcc branch and wait per element; a flag with side
      // effects must tolerate a repeated column)
      f[u] = (j < c1) & (bool)flag(min(j, c1 - 1));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // the kept columns' loads, all in flight
      const int j = j0 + u * NT + (int)threadIdx.x;
      v[u] = load(min(j, c1 - 1));  // (unconditional, as the flags)
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
  __device__ double3 at(int e) const { return double3{TX[e], TY[e], TZ[e]}; }
};
// The same set read from the caller's row (r4, k_rows_screen32 keeps only
// f32 offsets in LDS): compacted position e -> column FCOL[e] of the row
// tg[3 * C]; positions from n on (the last chunk's tail) are +inf.
struct ScreenSetG {
  const double *tg;
  const uint16_t *FCOL;
  const double *BOX;
  int nch, n;
  __device__ double3 at(int e) const {
    // (clamped, and column 0 for an empty row: never a load outside the row)
    const double *p = tg + 3 * (n > 0 ? (int)FCOL[min(max(e, 0), n - 1)] : 0);
    const double x = p[0], y = p[1], z = p[2];
    return e < n ? double3{x, y, z} : double3{INFINITY, INFINITY, INFINITY};
  }
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
template <int NT, class Set>
__device__ void screen_boxes(const Set &T, double *BOX, int n, int nch) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  constexpr int NW = NT / kWave, CPW = kWave / kScreenChunk;
  static_assert(kWave % kScreenChunk == 0, "chunks tile a wave");
  for (int b0 = CPW * wid; b0 < nch; b0 += CPW * NW) {
    const int b = b0 + lane / kScreenChunk, e = b * kScreenChunk + lane % kScreenChunk;
    const bool in = b < nch && e < n;
    double lo[3], hi[3];
    const double3 p = T.at(in ? e : 0);
    const double v[3] = {in ? p.x : NAN, in ? p.y : NAN, in ? p.z : NAN};
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
template <class Set>
__device__ void screen_query(const Set &T, bool act, double qx, double qy, double qz,
                             int s0, int s1, double &d1, double &d2, int &j1,
                             double bound2 = INFINITY) {
  const int lane = threadIdx.x & (kWave - 1);
  auto scan_chunk = [&](int k) {
    NV_STAMP_ADD(13, 0ull, 1ull);
    const int e0 = k * kScreenChunk;
#pragma unroll 8
    for (int u = 0; u < kScreenChunk; ++u) {
      const int e = e0 + u;
      const double3 p = T.at(e);
      const double dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
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
template <class Set>
__device__ void screen_verify(const Set &T, bool act, double qx, double qy, double qz,
                              double d1, double d2, int j1, bool &genuine, int &emin) {
  const double dist = __builtin_sqrt(d1);
  const bool suspect = act && d1 < INFINITY && __builtin_sqrt(d2) == dist;
  genuine = false;
  emin = j1;
  if (!__any(suspect)) return;
  const int jr = j1 >= 0 ? j1 : 0;
  const double3 pr = T.at(jr);
  const long long rx = __double_as_longlong(pr.x), ry = __double_as_longlong(pr.y),
                  rz = __double_as_longlong(pr.z);
  for (int k = 0; k < T.nch; ++k) {
    const double lb = screen_box_lb(T.BOX + 6 * k, qx, qx, qy, qy, qz, qz);
    if (!__any(suspect && __builtin_sqrt(lb) <= dist)) continue;
    for (int u = 0; u < kScreenChunk; ++u) {
      const int e = k * kScreenChunk + u;
      const double3 p = T.at(e);
      const double dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
      const double d = dx * dx + dy * dy + dz * dz;
      if (suspect && __builtin_sqrt(d) == dist) {
        const bool same = __double_as_longlong(p.x) == rx &&
                          __double_as_longlong(p.y) == ry &&
                          __double_as_longlong(p.z) == rz;
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
  screen_boxes<NT>(ScreenSet{TX, TY, TZ, BOX, nch}, BOX, n, nch);
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
      const bool under = d1 < INFINITY && dist > 0.0 && dist < 1e-150;
      if (genuine || under) {
        nn_idx[rowoff + c] = kTiePending;
        nn_dist[rowoff + c] = under ? -1.0 : dist;  // the tie pass's stop distance
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

// ---- k_rows_screen32 (r4): the screen's candidate scan in packed f32 -------
// k_rows_screen's f64 scan issues ~12 VALU per candidate and the K4 batch is
// VALU-bound. This kernel returns the same nn_idx / nn_dist /
// tie flags from a packed-f32 scan with an f64 certificate:
//  * LDS holds the row's target features as f32 offsets from the row's first
//    feature o (12 B each instead of 24); the f64 points stay in the caller's
//    row and are read through FCOL where an exact value is needed;
//  * one query per lane keeps the two smallest keys, key = f32 dsq bits with
//    the low kb bits replaced by the position (v_and_or + v_med3 + v_min per
//    candidate; the distances two candidates per packed op);
//  * certificate: the winner's reference dsq d1 is computed in f64. Every
//    other candidate's f32 dsq is >= the runner-up key's truncated value, so
//    when f32_bound(d1 (1 + 2^-40)) is below it, no other point is within
//    sqrt-equality of d1: the answer is the unique argmin, which is what the
//    f64 screen returns (no tie, no verify pass);
//  * chunks are pruned by their exact f64 box bound against f32_upper of the
//    runner-up key (>= the exact dsq of both key holders, so >= the final
//    runner-up: a pruned point can neither win nor tie);
//  * lanes without a certificate (near-ties within the key's 2^-(23-kb)
//    resolution, duplicates, NaN / inf, coordinates beyond f32 range) run
//    k_rows_screen's f64 screen + verify over the caller's row, pruned by that
//    same runner-up bound.
__host__ __device__ inline int rows_screen32_lds(int C, int w) {
  const int cp = (C + kScreenChunk - 1) / kScreenChunk * kScreenChunk;
  return 3 * align16(4 * cp) + 2 * align16(2 * C) + align16(48 * (cp / kScreenChunk)) +
         align16(2 * w) + align16(4 * 160) + 16;
}

template <int NT>
__global__ __launch_bounds__(NT) void k_rows_screen32(
    const double *__restrict__ src, const double *__restrict__ tgt, int R, int C,
    int32_t *__restrict__ src_mask, int32_t *__restrict__ tgt_mask,
    int32_t *__restrict__ nn_idx, double *__restrict__ nn_dist, int32_t *__restrict__ tie,
    int fuse) {
  const int r = blockIdx.x, S = gridDim.y, sp = blockIdx.y;
  const int w = (C + S - 1) / S;
  const int c0 = sp * w, c1 = min(C, c0 + w);
  const size_t rowoff = (size_t)r * C;
  const int pair_row0 = (r % R) * C;
  const int cp = (C + kScreenChunk - 1) / kScreenChunk * kScreenChunk;
  float *XF = (float *)smem;
  float *YF = (float *)(smem + align16(4 * cp));
  float *ZF = (float *)(smem + 2 * align16(4 * cp));
  uint16_t *FCOL = (uint16_t *)(smem + 3 * align16(4 * cp));
  uint16_t *RANK = (uint16_t *)((unsigned char *)FCOL + align16(2 * C));
  double *BOX = (double *)((unsigned char *)RANK + align16(2 * C));
  uint16_t *QL = (uint16_t *)((unsigned char *)BOX + align16(48 * (cp / kScreenChunk)));
  int *scan = (int *)((unsigned char *)QL + align16(2 * w));
  unsigned *DT = (unsigned *)((unsigned char *)scan + align16(4 * 160));
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  NV_STAMP(z0);
  const double *tg = tgt + 3 * rowoff;
  if (threadIdx.x == 0) *DT = 0u;
  // the offsets' origin: the row's column 0, feature or not (known before the
  // compaction, so the row is read from HBM once)
  const double3 o = double3{tg[0], tg[1], tg[2]};
  // target row features in column order (flattenPoints) as f32 offsets, and
  // Dt >= every |t - o| (inf when some offset is not a finite f32: no lane of
  // the row is certified)
  float dtl = 0.0f;
  // features: from the masks k_curvature wrote, or (fuse) the curvature
  // itself from the rows (src/slam.c:16-58; split 0 writes the target mask
  // when the caller wants it)
  const int n = compact_cols_f<NT>(
      0, C,
      [&](int j) -> int {
        if (!fuse) return tgt_mask[rowoff + j] != 0;
        const int f = row_feature_global(tg, C, j);
        if (tgt_mask && sp == 0) tgt_mask[rowoff + j] = f;
        return f;
      },
      [&](int j) { return double3{tg[3 * j], tg[3 * j + 1], tg[3 * j + 2]}; },
      [&](int j, int pos, const double3 &p) {
        const double ex = p.x - o.x, ey = p.y - o.y, ez = p.z - o.z;
        XF[pos] = (float)ex;
        YF[pos] = (float)ey;
        ZF[pos] = (float)ez;
        FCOL[pos] = (uint16_t)j;
        const double m = fmax(fabs(ex), fmax(fabs(ey), fabs(ez)));
        dtl = m <= 1e37 ? fmaxf(dtl, (float)(m * (1.0 + 0x1p-20))) : INFINITY;
        if (!(ex == ex && ey == ey && ez == ez)) dtl = INFINITY;
      },
      RANK, scan);
  const int nch = (n + kScreenChunk - 1) / kScreenChunk;
  const ScreenSetG G = {tg, FCOL, BOX, nch, n};
  for (int e = n + (int)threadIdx.x; e < nch * kScreenChunk; e += NT)
    XF[e] = YF[e] = ZF[e] = INFINITY;  // the last chunk's tail: never taken
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) dtl = fmaxf(dtl, __shfl_xor(dtl, off, kWave));
  if (lane == 0) atomicMax(DT, __float_as_uint(dtl));  // >= 0: the bits order as the values
  __syncthreads();  // offsets, tail and Dt
  // chunk boxes from the f32 offsets, widened by their rounding (each offset
  // is within 2^-24 Dt of the exact one): lower bounds on the exact f64 box
  {
    const double Dt0 = (double)__uint_as_float(*DT);
    const double w = Dt0 * 0x1p-22;
    constexpr int CPW = kWave / kScreenChunk;
    for (int b0 = CPW * wid; b0 < nch; b0 += CPW * (NT / kWave)) {
      const int b = b0 + lane / kScreenChunk, e = b * kScreenChunk + lane % kScreenChunk;
      const bool in = b < nch && e < n;
      const float v[3] = {in ? XF[e] : NAN, in ? YF[e] : NAN, in ? ZF[e] : NAN};
      float lo[3], hi[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const bool ok = v[a] == v[a];
        lo[a] = ok ? v[a] : INFINITY;
        hi[a] = ok ? v[a] : -INFINITY;
      }
#pragma unroll
      for (int off = kScreenChunk / 2; off > 0; off >>= 1)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          lo[a] = fminf(lo[a], __shfl_xor(lo[a], off, kWave));
          hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off, kWave));
        }
      if (b < nch && lane % kScreenChunk == 0) {
        const double oo[3] = {o.x, o.y, o.z};
        double *bx = BOX + 6 * b;
#pragma unroll
        for (int a = 0; a < 3; ++a) {  // (an all-NaN chunk keeps an empty box)
          bx[2 * a] = (oo[a] + (double)lo[a]) - w - fabs(oo[a]) * 0x1p-50;
          bx[2 * a + 1] = (oo[a] + (double)hi[a]) + w + fabs(oo[a]) * 0x1p-50;
        }
      }
    }
  }
  // this split's source features (compact_cols synchronises: offsets, boxes
  // and Dt are visible after it)
  const double *sg = src + 3 * rowoff;
  const int nq = compact_cols_f<NT>(
      c0, c1,
      [&](int j) -> int {
        int f;
        if (fuse) {
          f = row_feature_global(sg, C, j);
          if (src_mask) src_mask[rowoff + j] = f;
        } else {
          f = src_mask[rowoff + j] != 0;
        }
        if (!f) {  // no feature, no correspondence
          nn_idx[rowoff + j] = -1;
          nn_dist[rowoff + j] = INFINITY;
        }
        return f;
      },
      [&](int) { return 0; }, [&](int j, int pos, int) { QL[pos] = (uint16_t)j; }, nullptr,
      scan);
  NV_STAMP(z1);
  NV_STAMP_ADD(4, z0, z1);  // setup: compaction, offsets, boxes, query list
  const double Dt = (double)__uint_as_float(*DT);
  // key: f32 dsq bits, the low kb bits the position (nch * 32 <= 2^kb)
  const int kb = 32 - __builtin_clz((unsigned)max(nch * kScreenChunk - 1, 1));
  const uint32_t idm = (1u << kb) - 1u, vmask = ~idm;
  int mytie = 0;
  for (int i0 = wid * kWave; i0 < nq; i0 += NT) {  // wave-uniform trip count
    const int i = i0 + lane;
    const bool act = i < nq;
    const int c = QL[act ? i : i0];
    const double *qp = src + 3 * (rowoff + c);
    const double qx = qp[0], qy = qp[1], qz = qp[2];
    // the chunks where the wave's columns start first (as k_rows_screen)
    const int s0 = __builtin_amdgcn_readfirstlane(
        min((int)RANK[QL[i0]] / kScreenChunk, max(nch - 1, 0)));
    const int s1 = min(s0 + 1, max(nch - 1, 0));
    const double rx = qx - o.x, ry = qy - o.y, rz = qz - o.z;
    const double Dq = fmax(Dt, fmax(fabs(rx), fmax(fabs(ry), fabs(rz))));
    // each f32 difference is within dl of the exact one: the target offset
    // and the query offset are rounded once each (<= u D), the subtraction
    // once (<= 2 u D), u = 2^-24
    const double dl = Dq * 0x1p-21;
    const f2 qx2 = {(float)rx, (float)rx}, qy2 = {(float)ry, (float)ry},
             qz2 = {(float)rz, (float)rz};
    uint32_t k1 = kNoKey32, k2 = kNoKey32;
    auto scan32 = [&](int k) {
      const int e0 = k * kScreenChunk;
#pragma unroll
      for (int u = 0; u < kScreenChunk; u += 2) {
        const float2 xx = *(const float2 *)(XF + e0 + u);
        const float2 yy = *(const float2 *)(YF + e0 + u);
        const float2 zz = *(const float2 *)(ZF + e0 + u);
        const f2 dx = f2{xx.x, xx.y} - qx2, dy = f2{yy.x, yy.y} - qy2, dz = f2{zz.x, zz.y} - qz2;
        const f2 d = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
        const uint32_t a = knn_key(d[0], vmask, (uint32_t)(e0 + u));
        const uint32_t b = knn_key(d[1], vmask, (uint32_t)(e0 + u + 1));
        k2 = umed3(k1, k2, a);
        k1 = min(k1, a);
        k2 = umed3(k1, k2, b);
        k1 = min(k1, b);
      }
    };
    // upper bound of the exact dsq of both key holders (inf: no bound)
    auto ub2 = [&]() {
      const float V = __uint_as_float(k2 | idm);
      return (V < INFINITY && dl < INFINITY) ? f32_upper((double)V, dl) : (double)INFINITY;
    };
    NV_STAMP(z2);
    if (nch > 0) {
      scan32(s0);
      if (s1 != s0) scan32(s1);
    }
    NV_STAMP(z3);
    NV_STAMP_ADD(5, z2, z3);  // the two start chunks
    // the winner so far is usually the final one: its f64 point is loaded now
    // and arrives during the box loop (gathered again below if it changed)
    const uint32_t k1s = k1;
    const double3 p1s = G.at((int)(k1s & idm));
    double UB2 = ub2();  // refreshed after each further chunk scan
    const bool qok = act && qx == qx && qy == qy && qz == qz;
    double wl[3] = {qok ? qx : INFINITY, qok ? qy : INFINITY, qok ? qz : INFINITY};
    double wh[3] = {qok ? qx : -INFINITY, qok ? qy : -INFINITY, qok ? qz : -INFINITY};
    double wd2 = qok ? UB2 : -INFINITY;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        wl[a] = fmin(wl[a], __shfl_xor(wl[a], off, kWave));
        wh[a] = fmax(wh[a], __shfl_xor(wh[a], off, kWave));
      }
      wd2 = fmax(wd2, __shfl_xor(wd2, off, kWave));
    }
    for (int k0 = 0; k0 < nch; k0 += kWave) {
      const int kl = k0 + lane;
      bool pass = false;
      if (kl < nch && kl != s0 && kl != s1)
        pass = screen_box_lb(BOX + 6 * kl, wl[0], wh[0], wl[1], wh[1], wl[2], wh[2]) <= wd2;
      unsigned long long m = __ballot(pass);
      while (m) {
        const int k = k0 + __builtin_ctzll(m);
        m &= m - 1;
        const double lb = screen_box_lb(BOX + 6 * k, qx, qx, qy, qy, qz, qz);
        if (__any(act && lb <= UB2)) {
          NV_STAMP_ADD(3, 0ull, 1ull);  // chunks scanned past the first two
          scan32(k);
          UB2 = ub2();
        }
      }
    }
    NV_STAMP(z4);
    NV_STAMP_ADD(6, z3, z4);  // the box loop and its scans
    // the certificate (nch = 0: no candidate, nothing to certify)
    int j1 = -1;
    double d1 = INFINITY;
    bool cert = nch == 0;
    if (act && nch > 0) {
      j1 = (int)(k1 & idm);
      const double3 p = k1 == k1s ? p1s : G.at(j1);
      const double dx = p.x - qx, dy = p.y - qy, dz = p.z - qz;
      d1 = dx * dx + dy * dy + dz * dz;  // utils/kdtree.c:16
      const float lb2 = k2 == kNoKey32 ? INFINITY : __uint_as_float(k2 & vmask);
      cert = d1 < INFINITY && Dq < 1e17 && f32_bound(d1 * (1.0 + 0x1p-40), dl) < lb2;
    }
    bool genuine = false;
    int emin = j1;
    const bool need = act && !cert;
#ifdef NAVGPU_STAMPS
    NV_STAMP_ADD(0, 0ull, 1ull);                                       // waves
    NV_STAMP_ADD(1, 0ull, __any(need) ? 1ull : 0ull);                   // ... with a fallback
    NV_STAMP_ADD(2, 0ull, (unsigned long long)__popcll(__ballot(need)));  // fallback lanes
#endif
    if (__any(need)) {
      // Uncertified lanes. With a finite winner and finite errors the answer
      // is decided inside the band of points whose f32 dsq could be within
      // sqrt-equality of the minimum: f32 dsq <= f32_bound(d1 (1 + 2^-40)),
      // d1 the winner's exact dsq (>= the true minimum). Band points (a few)
      // get their exact dsq from the caller's row; pass 1 takes the exact
      // minimum and runner-up over them, pass 2 (only if the runner-up has
      // the minimum's sqrt) separates duplicates from genuine ties, as
      // screen_verify does. The rest (non-finite data, offsets past f32
      // range) runs k_rows_screen's f64 screen over the caller's row.
      const bool band = need && d1 < INFINITY && Dq < 1e17 && dl < INFINITY;
      const bool hard = need && !band;
      if (__any(band)) {
        const double Tb = d1 * (1.0 + 0x1p-40);
        const float Bf = band ? f32_bound(Tb, dl) : -1.0f;
        double e1 = INFINITY, e2 = INFINITY;
        int ej = -1;
        // visit(f) runs f(e, exact dsq, point) for every band point of this lane
        auto visit = [&](auto f) {
          for (int k = 0; k < nch; ++k) {
            const double lb = screen_box_lb(BOX + 6 * k, qx, qx, qy, qy, qz, qz);
            const bool in = band && lb <= Tb;
            if (!__any(in)) continue;
            const int e0 = k * kScreenChunk;
            for (int u = 0; u < kScreenChunk; u += 2) {
              const float2 xx = *(const float2 *)(XF + e0 + u);
              const float2 yy = *(const float2 *)(YF + e0 + u);
              const float2 zz = *(const float2 *)(ZF + e0 + u);
              const f2 dx = f2{xx.x, xx.y} - qx2, dy = f2{yy.x, yy.y} - qy2,
                       dz = f2{zz.x, zz.y} - qz2;
              const f2 dd =
                  __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const bool ib = in && dd[h] <= Bf;
                if (__any(ib) && ib) {
                  const int e = e0 + u + h;
                  const double3 pp = G.at(e);
                  const double ddx = pp.x - qx, ddy = pp.y - qy, ddz = pp.z - qz;
                  f(e, ddx * ddx + ddy * ddy + ddz * ddz, pp);  // utils/kdtree.c:16
                }
              }
            }
          }
        };
        visit([&](int e, double d, const double3 &) {
          ej = d < e1 ? e : ej;
          e2 = fmin(e2, fmax(e1, d));
          e1 = fmin(e1, d);
        });
        const double edist = __builtin_sqrt(e1);
        const bool suspect = band && ej >= 0 && __builtin_sqrt(e2) == edist;
        bool gen = false;
        int em = ej;
        if (__any(suspect)) {
          const double3 pr = G.at(ej);
          const long long rx = __double_as_longlong(pr.x), ry = __double_as_longlong(pr.y),
                          rz = __double_as_longlong(pr.z);
          visit([&](int e, double d, const double3 &pp) {
            if (suspect && __builtin_sqrt(d) == edist) {
              const bool same = __double_as_longlong(pp.x) == rx &&
                                __double_as_longlong(pp.y) == ry &&
                                __double_as_longlong(pp.z) == rz;
              gen |= !same;
              em = same ? min(em, e) : em;
            }
          });
        }
        if (band) {
          d1 = e1;
          j1 = ej;
          genuine = gen;
          emin = em;
        }
      }
      if (__any(hard)) {  // k_rows_screen's f64 path over the caller's row
        double f1 = INFINITY, f2v = INFINITY;
        int fj = -1;
        screen_query(G, hard, qx, qy, qz, nch > 0 ? s0 : -1, nch > 0 ? s1 : -1, f1, f2v, fj,
                     UB2);
        bool gen;
        int em;
        screen_verify(G, hard, qx, qy, qz, f1, f2v, fj, gen, em);
        if (hard) {
          d1 = f1;
          j1 = fj;
          genuine = gen;
          emin = em;
        }
      }
    }
    NV_STAMP(z5);
    NV_STAMP_ADD(7, z4, z5);  // certificate + fallback
    if (act) {
      const double dist = __builtin_sqrt(d1);
      const bool under = d1 < INFINITY && dist > 0.0 && dist < 1e-150;
      if (genuine || under) {
        nn_idx[rowoff + c] = kTiePending;
        nn_dist[rowoff + c] = under ? -1.0 : dist;  // the tie pass's stop distance
        mytie = 1;
      } else {
        nn_idx[rowoff + c] = j1 >= 0 ? pair_row0 + (int)FCOL[emin] : -1;
        nn_dist[rowoff + c] = j1 >= 0 ? dist : INFINITY;
      }
    }
  }
  const int any = __syncthreads_or(mytie);
  if (threadIdx.x == 0) tie[(size_t)r * S + sp] = any;
}

// ------------------------------------------- split per-row build / query
__global__ __launch_bounds__(kRowsBuildBlock) void k_rows_build(
    const double *__restrict__ feat_src, const double *__restrict__ coords,
    int R, int C, double *__restrict__ tree_pts, int32_t *__restrict__ tree_col,
    int32_t *__restrict__ tree_n, int32_t *__restrict__ mask_out, int build,
    int32_t *__restrict__ built) {
  const RowsLds L = rows_lds(C, kRowsBlock, false);
  const int r = blockIdx.x;
  if (built && threadIdx.x == 0) built[r] = 0;  // the row is back in column order (r5: no memset)
  const size_t rowoff = (size_t)r * C;
  const int n = row_stage_and_build(feat_src, coords, r, C, L, mask_out, build != 0);
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
    int32_t *__restrict__ nn_pos, double *__restrict__ nn_dist, int32_t *__restrict__ mask_out,
    int32_t *__restrict__ tie, const int32_t *__restrict__ tree_col,
    const int32_t *__restrict__ built) {
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
  // lazy rows (column order, no tree): the walk stack's region holds the
  // rows' feature columns instead (no query walks here). A lazy row an
  // earlier call already rebuilt (built[r]) holds the reference tree: it is
  // screened and walked as a built one.
  uint16_t *TCOL = (uint16_t *)stk;
  const bool rowbuilt = built && built[r];
  const bool lazy = tree_col != nullptr && !rowbuilt;
  const int n = tree_n[r];
  const int nch = (n + kScreenChunk - 1) / kScreenChunk;
  for (int pos = threadIdx.x; pos < nch * kScreenChunk; pos += NT) {
    if (pos < n) {
      const double *t = tree_pts + 3 * (rowoff + pos);
      TX[pos] = t[0];
      TY[pos] = t[1];
      TZ[pos] = t[2];
      if (lazy) TCOL[pos] = (uint16_t)tree_col[rowoff + pos];
    } else {
      TX[pos] = TY[pos] = TZ[pos] = INFINITY;  // dsq = inf: never taken
    }
  }
  const int lo = max(c0 - 2, 0), hi = min(c1 + 2, C);  // slice + curvature halo
  block_copy(rs, feat_src + 3 * (rowoff + lo), 3 * (hi - lo));
  __syncthreads();
  screen_boxes<NT>(ScreenSet{TX, TY, TZ, BOX, nch}, BOX, n, nch);
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
    // lazy rows: the scan starts at the chunks holding the first feature at or
    // after the wave's first query column (a scan row is an azimuth sweep)
    int s0 = -1, s1 = -1;
    if (lazy && nch > 0) {
      const int q0 = QL[i0];
      int lo = 0, hi = n;  // lower bound of q0 in the row's sorted columns
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int)TCOL[mid] < q0)
          lo = mid + 1;
        else
          hi = mid;
      }
      s0 = __builtin_amdgcn_readfirstlane(min(lo / kScreenChunk, nch - 1));
      s1 = min(s0 + 1, nch - 1);
    }
    if (!lazy) {
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
    screen_query(T, act, qx, qy, qz, s0, s1, d1, d2, j1, e2);
    const double dist = __builtin_sqrt(d1);
    bool genuine;
    int emin;
    screen_verify(T, act, qx, qy, qz, d1, d2, j1, genuine, emin);
    if (act) {
      int bpos = j1 >= 0 ? emin : -1;
      double bd = j1 >= 0 ? dist : INFINITY;
      const bool under = d1 < INFINITY && dist > 0.0 && dist < 1e-150;
      if (genuine || under) {
        if (lazy) {  // the row holds no tree yet: k_rows_retree walks all its queries
          tie[r] = 1;
          bd = under ? -1.0 : bd;  // its walk's stop distance (-1: the whole walk)
        } else {
          kd_query(TX, TY, TZ, n, qx, qy, qz, stk + threadIdx.x, NT, &bpos, &bd,
                   under ? -1.0 : dist);
        }
      }
      nn_pos[rowoff + c] = bpos;
      nn_dist[rowoff + c] = bd;
    }
  }
}

// K5 with the row trees left unbuilt (navgpu_kd_query_rows_lazy_dev): a row
// whose screen found a genuine tie gets the reference's tree now, from the
// compacted features that k_rows_build (build = 0) left in tree_pts in
// column order (the array buildKDTree permutes, utils/kdtree.c:65-82), and
// ALL its queries are answered by the walk (utils/kdtree.c:110-152), since
// their positions now index the permuted row. Rows without a tie return.
__device__ void rows_corr_body(int row, unsigned char *corr_lds, const double *tree_pts,
                               const int32_t *tree_n, const int32_t *nn_pos,
                               const double *nn_dist, const double *ori, int C, int HS,
                               int32_t *keep, double *sums, double *ent, int32_t *ent_n);

// The lazy rows' tie pass: a row whose screen met a tie gets the reference
// tree and all its queries walked. With `ori` (r5, the fast mode) every row's
// workgroup then runs the row's correspondences and sums (rows_corr_body,
// the k_rows_corr launch saved).
__global__ __launch_bounds__(kRowsBlock) void k_rows_retree(
    double *__restrict__ tree_pts, int32_t *__restrict__ tree_col,
    const int32_t *__restrict__ tree_n, const double *__restrict__ feat_src,
    const double *__restrict__ queries, int C, int32_t *__restrict__ nn_pos,
    double *__restrict__ nn_dist, int32_t *__restrict__ tie, int32_t *__restrict__ built,
    const double *__restrict__ ori, int HS, double *__restrict__ sums) {
  const int r = blockIdx.x;
  const int tied = tie[r];
  __syncthreads();  // every thread has read the flag before it is cleared
  if (tied) {  // uniform (a built row's ties were walked by the screen)
  if (threadIdx.x == 0) tie[r] = 0;  // zero again for the next call (no memset, r5)
  const RowsLds L = rows_lds(C, kRowsBlock, true);
  const size_t rowoff = (size_t)r * C;
  const int n = tree_n[r];
  double *raw = (double *)(smem + L.raw);
  double *FC = (double *)(smem + L.fc);
  uint16_t *FCOL = (uint16_t *)(smem + L.fcol);
  uint16_t *P = (uint16_t *)(smem + L.p);
  uint16_t *T = (uint16_t *)(smem + L.t);
  uint32_t *stk = (uint32_t *)(smem + L.stk);
  int *scan = (int *)(smem + L.scan);
  for (int pos = threadIdx.x; pos < n; pos += blockDim.x) {
    const double *t = tree_pts + 3 * (rowoff + pos);
    FC[pos] = t[0];
    FC[C + pos] = t[1];
    FC[2 * C + pos] = t[2];
    FCOL[pos] = (uint16_t)tree_col[rowoff + pos];
  }
  __syncthreads();
  block_build_kdtree<uint16_t>(FC, C, n, P, T, 0);
  // the tree in position order: back to tree_pts / tree_col, and SoA in raw
  double *TX = raw, *TY = raw + C, *TZ = raw + 2 * C;
  for (int pos = threadIdx.x; pos < n; pos += blockDim.x) {
    const int e = P[pos];
    TX[pos] = FC[e];
    TY[pos] = FC[C + e];
    TZ[pos] = FC[2 * C + e];
    T[pos] = FCOL[e];
  }
  __syncthreads();
  for (int pos = threadIdx.x; pos < n; pos += blockDim.x) {
    double *o = tree_pts + 3 * (rowoff + pos);
    o[0] = TX[pos];
    o[1] = TY[pos];
    o[2] = TZ[pos];
    tree_col[rowoff + pos] = T[pos];
  }
  if (built && threadIdx.x == 0) built[r] = 1;  // a later lazy query walks this tree
  // the query row's features (its curvature, src/slam.c:11-61) -> the walk
  double *sraw = FC;
  uint16_t *SM = P;
  block_copy(sraw, feat_src + 3 * rowoff, 3 * C);
  __syncthreads();
  for (int j = threadIdx.x; j < C; j += blockDim.x) {
    const int f = row_curv_lds(sraw, C, j) > 0.1 ? 1 : 0;
    SM[j] = (uint16_t)f;
    if (!f) {
      nn_pos[rowoff + j] = -1;
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
    const double *q = queries + 3 * (rowoff + c);
    int bpos;
    double bd;
    // the screen left each query's exact minimum (-1 where it must not stop)
    kd_query(TX, TY, TZ, n, q[0], q[1], q[2], stk + threadIdx.x, blockDim.x, &bpos, &bd,
             nn_dist[rowoff + c]);
    if (bpos >= 0) {  // the lowest position holding bit-identical coordinates
      const long long rx = __double_as_longlong(TX[bpos]), ry = __double_as_longlong(TY[bpos]),
                      rz = __double_as_longlong(TZ[bpos]);
      for (int p = 0; p < bpos; ++p)
        if (__double_as_longlong(TX[p]) == rx && __double_as_longlong(TY[p]) == ry &&
            __double_as_longlong(TZ[p]) == rz) {
          bpos = p;
          break;
        }
    }
    nn_pos[rowoff + c] = bpos;
    nn_dist[rowoff + c] = bd;
  }
  }
  if (ori) {
    __syncthreads();  // the walk's results and the LDS are free for the row's pairs
    rows_corr_body(r, smem, tree_pts, tree_n, nn_pos, nn_dist, ori, C, HS, nullptr, sums,
                   nullptr, nullptr);
  }
}

// ---------------------------------------- R5 for one arbitrary array
// kdtree.h buildKDTree: n points, in place, root axis depth0 % 3.
// Diagnostic (r6): one reference nth_element (utils/kdtree.c:20-52) as the
// per-row builds run it, by one wave (wave_nth_element: ordinary and register
// passes) or by the block (block_nth_element), on keys and a
// permutation of n <= kMaxRowCols positions (navgpu_debug_nth_element)
__global__ __launch_bounds__(1024) void k_debug_nth(const double *__restrict__ key,
                                                    int32_t *__restrict__ perm, int n, int first,
                                                    int last, int nth, int block) {
  double *K = (double *)smem;
  uint16_t *P = (uint16_t *)(smem + align16(8 * n));
  uint16_t *T = P + align16(2 * n) / 2;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    K[i] = key[i];
    P[i] = (uint16_t)perm[i];
  }
  __syncthreads();
  if (block)
    block_nth_element<uint16_t>(K, P, T, first, last, nth);
  else if (threadIdx.x < kWave)
    wave_nth_element<uint16_t>(K, P, T, first, last, nth, (int)threadIdx.x);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) perm[i] = P[i];
}

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

// one row's correspondences (the k_rows_corr workgroup's work; r5: also the
// tail of k_rows_retree for the fast lazy path), LDS from `corr_lds`
__device__ void rows_corr_body(
    int row, unsigned char *corr_lds, const double *__restrict__ tree_pts,
    const int32_t *__restrict__ tree_n, const int32_t *__restrict__ nn_pos,
    const double *__restrict__ nn_dist, const double *__restrict__ ori, int C, int HS,
    int32_t *__restrict__ keep, double *__restrict__ sums, double *__restrict__ ent,
    int32_t *__restrict__ ent_n) {
  unsigned long long *bdist = (unsigned long long *)corr_lds;  // [HS]
  int *owner = (int *)(bdist + HS);                            // [HS]
  int *bcol = owner + HS;                                      // [HS]
  int *fcol = bcol + HS;                                       // [HS] (ent only)
  int *canon = fcol + HS;                                      // [C]
  __shared__ double red[kCorrBlock / kWave][6];
  __shared__ int cscan[kCorrBlock / kWave + 1];
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

__global__ __launch_bounds__(kCorrBlock) void k_rows_corr(
    const double *__restrict__ tree_pts, const int32_t *__restrict__ tree_n,
    const int32_t *__restrict__ nn_pos, const double *__restrict__ nn_dist,
    const double *__restrict__ ori, int C, int HS, int32_t *__restrict__ keep,
    double *__restrict__ sums, double *__restrict__ ent, int32_t *__restrict__ ent_n) {
  extern __shared__ __attribute__((aligned(8))) unsigned char corr_lds[];
  rows_corr_body(blockIdx.x, corr_lds, tree_pts, tree_n, nn_pos, nn_dist, ori, C, HS, keep,
                 sums, ent, ent_n);
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

}  // namespace

// =================================================================== host
namespace nv {

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

int ensure_aux(navgpu_ctx *ctx) {
  if (!ctx->aux) {
    HIP_TRY(hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
  }
  return NAVGPU_OK;
}

int launch_curvature(const double *pts0, int32_t *mask0, double *curv0,
                     const double *pts1, int32_t *mask1, double *curv1, int R, int C,
                     hipStream_t stream) {
  CurvJob J = {{pts0, pts1}, {mask0, mask1}, {curv0, curv1}};
  dim3 grid(curv_grid_x(C), R, pts1 ? 2 : 1);
  hipLaunchKernelGGL(k_curvature, grid, dim3(kCurvTile), 0, stream, J, R, C);
  CHECK_LAUNCH("k_curvature");
  return NAVGPU_OK;
}

}  // namespace nv

namespace {

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
  if (const char *o = getenv("NAVGPU_PAIR_SIDE")) c->pair_side = atoi(o) != 0;
  if (const char *o = getenv("NAVGPU_KNN_MODE")) {  // 1 or 2; anything else keeps the default
    const int m = atoi(o);
    if (m == 1 || m == 2) c->knn_mode = m;
  }
  if (const char *o = getenv("NAVGPU_KNN_SX")) {
    const int v = atoi(o);
    if (v >= 1 && v <= kKnnMaxSx) c->knn_sx = v;
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

void navgpu_timing_select(navgpu_ctx *ctx, const char *name) {
  if (ctx) ctx->timing_only = name ? name : "";
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
  unsigned long long z[16] = {0}, k[16];
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, 16 * 8));
  RC(knn_stamps_take(k));
  for (int i = 0; i < 16; ++i) out16[i] += k[i];
  return NAVGPU_OK;
#else
  (void)out16;
  return NAVGPU_EINVAL;
#endif
}

int navgpu_debug_nth_element(navgpu_ctx *ctx, const double *key, int32_t *perm, int n,
                             int first, int last, int nth, int block) {
  ARG_CHECK(ctx && key && perm);
  ARG_CHECK(n >= 1 && n <= kMaxRowCols && 0 <= first && first <= nth && nth <= last && last < n);
  const int lds = align16(8 * n) + 2 * align16(2 * n);
  RC(set_lds(k_debug_nth, lds));
  hipLaunchKernelGGL(k_debug_nth, dim3(1), dim3(block ? 1024 : kWave), lds, ctx->stream, key,
                     perm, n, first, last, nth, block ? 1 : 0);
  CHECK_LAUNCH("k_debug_nth");
  return NAVGPU_OK;
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
  dim3 grid(curv_grid_x(C), R, 1);
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
static int rows_build_launch(navgpu_ctx *ctx, const double *feat_src,
                             const double *coords, int R, int C,
                             double *tree_pts, int32_t *tree_col,
                             int32_t *tree_n, int32_t *mask_out, int build,
                             int32_t *built = nullptr) {
  ARG_CHECK(ctx);
  RC(check_rows_shape(R, C, false));
  if (R == 0) return NAVGPU_OK;
  ARG_CHECK(tree_n);
  if (C == 0) {
    HIP_TRY(hipMemsetAsync(tree_n, 0, 4 * (size_t)R, ctx->stream));
    if (built) HIP_TRY(hipMemsetAsync(built, 0, 4 * (size_t)R, ctx->stream));
    return NAVGPU_OK;
  }
  ARG_CHECK(feat_src && coords && tree_pts && tree_col);
  const RowsLds L = rows_lds(C, kRowsBlock, false);
  RC(set_lds(k_rows_build, L.total));
  TimedRegion tr(ctx, "rows_build");
  hipLaunchKernelGGL(k_rows_build, dim3(R), dim3(kRowsBuildBlock), L.total,
                     ctx->stream, feat_src, coords, R, C, tree_pts, tree_col,
                     tree_n, mask_out, build, built);
  CHECK_LAUNCH("k_rows_build");
  return NAVGPU_OK;
}

int navgpu_kd_build_rows_dev(navgpu_ctx *ctx, const double *feat_src,
                             const double *coords, int R, int C,
                             double *tree_pts, int32_t *tree_col,
                             int32_t *tree_n, int32_t *mask_out) {
  return rows_build_launch(ctx, feat_src, coords, R, C, tree_pts, tree_col, tree_n, mask_out, 1);
}

int navgpu_kd_compact_rows_dev(navgpu_ctx *ctx, const double *feat_src,
                               const double *coords, int R, int C,
                               double *tree_pts, int32_t *tree_col,
                               int32_t *tree_n, int32_t *mask_out, int32_t *tree_built) {
  ARG_CHECK(ctx && R >= 0);
  // every row back in column order: k_rows_build zeroes tree_built[r]
  return rows_build_launch(ctx, feat_src, coords, R, C, tree_pts, tree_col, tree_n, mask_out, 0,
                           tree_built);
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

int navgpu_host_register(navgpu_ctx *ctx, void *hptr, size_t bytes) {
  ARG_CHECK(ctx && hptr && bytes);
  const hipError_t e = hipHostRegister(hptr, bytes, hipHostRegisterDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // not sticky: the range simply stays pageable
    set_err("hipHostRegister(%zu): %s", bytes, hipGetErrorString(e));
    return NAVGPU_ERANGE;
  }
  return NAVGPU_OK;
}

void navgpu_host_unregister(navgpu_ctx *ctx, void *hptr) {
  if (!ctx || !hptr) return;
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->aux) (void)hipStreamSynchronize(ctx->aux);
  if (hipHostUnregister(hptr) != hipSuccess) (void)hipGetLastError();
}

// The per-row query over built trees (tie == nullptr), or over the
// compacted, unbuilt rows of navgpu_kd_compact_rows_dev (tie: per-row flags,
// then k_rows_retree on the flagged rows).
static int rows_query_launch(navgpu_ctx *ctx, const double *tree_pts,
                             const int32_t *tree_n, const double *feat_src,
                             const double *queries, int R, int C,
                             int32_t *nn_pos, double *nn_dist,
                             int32_t *mask_out, int32_t *tie,
                             const int32_t *tree_col = nullptr,
                             const int32_t *built = nullptr) {
  ARG_CHECK(ctx);
  RC(check_rows_shape(R, C, true));
  if ((size_t)R * C == 0) return NAVGPU_OK;
  ARG_CHECK(tree_pts && tree_n && feat_src && queries && nn_pos && nn_dist);
  const char *qt = getenv("NAVGPU_ROWS_QUERY_TREE");
  if (tie || !(qt && *qt && *qt != '0')) {
    // the screen (default): >= 512 workgroups, >= 128 columns each (two
    // ~74 KB workgroups per CU at C = 2048; r5: 128 x 2048 frames 107 -> 103
    // us against >= 1024)
    int S = 1;
    while (S < 16 && (long long)R * S < 512 && C / (2 * S) >= 128) S <<= 1;
    if (const char *e = getenv("NAVGPU_ROWSQ_S"); e && *e)  // A/B: column splits per row
      S = std::max(1, std::min(64, atoi(e)));
    const int w = (C + S - 1) / S;
    const int cp = (C + kScreenChunk - 1) / kScreenChunk * kScreenChunk;
    // (the last region: the walk stacks, or the lazy rows' feature columns)
    const int lds = 3 * align16(8 * cp) + align16(48 * (cp / kScreenChunk)) +
                    align16(24 * (w + 4)) + 2 * align16(2 * w) + align16(4 * 40) +
                    std::max(4 * kRowsQBlock * kStackDepth, align16(2 * C));
    if (lds > lds_limit()) {
      set_err("rows_query: C=%d needs %d B of LDS (device limit %d)", C, lds, lds_limit());
      return NAVGPU_ERANGE;
    }
    RC(set_lds(k_rows_query_screen<kRowsQBlock>, lds));
    TimedRegion tr(ctx, "rows_query");
    hipLaunchKernelGGL(k_rows_query_screen<kRowsQBlock>, dim3(R, S), dim3(kRowsQBlock), lds,
                       ctx->stream, tree_pts, tree_n, feat_src, queries, R, C, nn_pos, nn_dist,
                       mask_out, tie, tie ? tree_col : nullptr, tie ? built : nullptr);
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

int navgpu_kd_query_rows_dev(navgpu_ctx *ctx, const double *tree_pts,
                             const int32_t *tree_n, const double *feat_src,
                             const double *queries, int R, int C,
                             int32_t *nn_pos, double *nn_dist,
                             int32_t *mask_out) {
  return rows_query_launch(ctx, tree_pts, tree_n, feat_src, queries, R, C, nn_pos, nn_dist,
                           mask_out, nullptr);
}

static int rows_query_lazy(navgpu_ctx *ctx, double *tree_pts, int32_t *tree_col,
                           const int32_t *tree_n, const double *feat_src,
                           const double *queries, int R, int C, int32_t *nn_pos,
                           double *nn_dist, int32_t *mask_out, int32_t *tree_built,
                           const double *ori, double *sums) {
  ARG_CHECK(ctx);
  RC(check_rows_shape(R, C, true));
  if ((size_t)R * C == 0) return NAVGPU_OK;
  ARG_CHECK(tree_col);
  ARG_CHECK(!ori || (sums && C <= kMaxRowCols));
  int32_t *tie;
  RC(ws(ctx, kRowTieLazy, (size_t)R, &tie));
  if (tie != ctx->lazy_tie || R > ctx->lazy_tie_rows) {  // a new buffer: zero it once
    HIP_TRY(hipMemsetAsync(tie, 0, 4 * (size_t)R, ctx->stream));
    ctx->lazy_tie = tie;
    ctx->lazy_tie_rows = R;
  }
  // Everything that can refuse the call is checked BEFORE the screen runs:
  // the screen sets tie flags that only k_rows_retree clears, so a refusal
  // between the two would leave them set for the next call on this context,
  // which would then rebuild already-built rows from tree order.
  const RowsLds L = rows_lds(C, kRowsBlock, true);
  // (with ori: the rows' correspondences in the same launch, from the same LDS)
  int HS = 64;
  while (HS < 2 * C) HS <<= 1;
  const int lds = ori ? std::max(L.total, HS * (8 + 4 + 4 + 4) + 4 * C) : L.total;
  if (lds > lds_limit()) {
    set_err("rows_query_lazy: C=%d needs %d B of LDS (device limit %d)", C, lds, lds_limit());
    return NAVGPU_ERANGE;
  }
  RC(set_lds(k_rows_retree, lds));
  RC(rows_query_launch(ctx, tree_pts, tree_n, feat_src, queries, R, C, nn_pos, nn_dist,
                       mask_out, tie, tree_col, tree_built));
  TimedRegion tr(ctx, "rows_retree");
  hipLaunchKernelGGL(k_rows_retree, dim3(R), dim3(kRowsBlock), lds, ctx->stream, tree_pts,
                     tree_col, tree_n, feat_src, queries, C, nn_pos, nn_dist,
                     tie, tree_built, ori, HS, sums);
  CHECK_LAUNCH("k_rows_retree");
  return NAVGPU_OK;
}

int navgpu_kd_query_rows_lazy_dev(navgpu_ctx *ctx, double *tree_pts, int32_t *tree_col,
                                  const int32_t *tree_n, const double *feat_src,
                                  const double *queries, int R, int C, int32_t *nn_pos,
                                  double *nn_dist, int32_t *mask_out, int32_t *tree_built) {
  return rows_query_lazy(ctx, tree_pts, tree_col, tree_n, feat_src, queries, R, C, nn_pos,
                         nn_dist, mask_out, tree_built, nullptr, nullptr);
}

int navgpu_kd_query_rows_lazy_corr_dev(navgpu_ctx *ctx, double *tree_pts, int32_t *tree_col,
                                       const int32_t *tree_n, const double *feat_src,
                                       const double *queries, int R, int C, int32_t *nn_pos,
                                       double *nn_dist, int32_t *mask_out, int32_t *tree_built,
                                       const double *ori, double *sums) {
  ARG_CHECK(ori && sums);
  return rows_query_lazy(ctx, tree_pts, tree_col, tree_n, feat_src, queries, R, C, nn_pos,
                         nn_dist, mask_out, tree_built, ori, sums);
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
  if (lds > lds_limit()) {
    set_err("rows_corr: C=%d needs %d B of LDS (device limit %d; C <= 2048 fits)", C, lds,
            lds_limit());
    return NAVGPU_ERANGE;
  }
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
  if (lds > lds_limit()) {
    set_err("rows_corr: C=%d needs %d B of LDS (device limit %d; C <= 2048 fits)", C, lds,
            lds_limit());
    return NAVGPU_ERANGE;
  }
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
    const char *f32e = getenv("NAVGPU_SCREEN_F32");
    const bool f32 = !(f32e && *f32e == '0');
    // the f32 screen computes the features itself (no k_curvature pass, no
    // mask round trip through HBM); the masks are written only if asked for
    // column splits: >= 512 workgroups in all (two per CU: ~64 KB of LDS
    // each), >= 128 columns each; 512 threads once a split holds >= 512
    // columns (measured: K2 83 us at S = 4 x 512 threads, 102 us at S = 8 x
    // 256; a K4 batch is fastest unsplit at 512 threads)
    while (S < 8 && (long long)rows * S < 512 && C / (2 * S) >= 128) S <<= 1;
    if (const char *e = getenv("NAVGPU_SCREEN_S")) S = std::max(1, std::min(64, atoi(e)));
    // unsplit rows (batches): the f32 screen computes the features itself
    // (r4: K4 5.43 -> 5.04 ms; split rows would each redo the target row's:
    // K2 79 -> 84 us, so they keep k_curvature)
    const char *fue = getenv("NAVGPU_SCREEN_FUSE");
    const bool fuse = f32 && (fue ? *fue != '0' : S == 1);
    if (!fuse) {
      if (!src_mask) RC(ws(ctx, kRowMaskS, N, &src_mask));
      if (!tgt_mask) RC(ws(ctx, kRowMaskT, N, &tgt_mask));
    }
    const int w = (C + S - 1) / S;
    int32_t *tf;
    RC(ws(ctx, kRowTie, (size_t)rows * S, &tf));
    tie = tf;
    ctx->screen_rows = rows;
    ctx->screen_S = S;
    // R1 on both clouds, <= 65535 rows per launch (grid y)
    for (int r0 = 0; r0 < rows && !fuse; r0 += 65535) {
      const int nr = std::min(rows - r0, 65535);
      const size_t o = (size_t)r0 * C;
      CurvJob J = {{src + 3 * o, tgt + 3 * o}, {src_mask + o, tgt_mask + o}, {nullptr, nullptr}};
      hipLaunchKernelGGL(k_curvature, dim3(curv_grid_x(C), nr, 2),
                         dim3(kCurvTile), 0, ctx->stream, J, nr, C);
      CHECK_LAUNCH("k_curvature");
    }
    const int lds = f32 ? rows_screen32_lds(C, w) : rows_screen_lds(C, w);
    if (lds > lds_limit()) {
      set_err("rows_screen: C=%d needs %d B of LDS (device limit %d)", C, lds, lds_limit());
      return NAVGPU_ERANGE;
    }
    const char *nte = getenv("NAVGPU_SCREEN_NT");
    // f32 screen: 256-thread workgroups for unsplit rows (r4: K4 5.04 ->
    // 4.12 ms: twice the resident rows per CU at the same waves)
    if (f32 && (nte ? atoi(nte) == 512 : (w >= 512 && S > 1))) {
      RC(set_lds(k_rows_screen32<512>, lds));
      hipLaunchKernelGGL(k_rows_screen32<512>, dim3(rows, S), dim3(512), lds, ctx->stream, src,
                         tgt, R, C, src_mask, tgt_mask, nn_idx, nn_dist, tf, (int)fuse);
    } else if (f32) {
      RC(set_lds(k_rows_screen32<256>, lds));
      hipLaunchKernelGGL(k_rows_screen32<256>, dim3(rows, S), dim3(256), lds, ctx->stream, src,
                         tgt, R, C, src_mask, tgt_mask, nn_idx, nn_dist, tf, (int)fuse);
    } else if (nte ? atoi(nte) == 512 : w >= 512) {
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
    // threads per row (NAVGPU_LEAN_NT = 256 | 512 | 1024; r6: K4 integer-mm
    // 30.80 / 26.87 / 36.35 ms, profiles/r6/k4i_lean_threads_ab.txt)
    static const int ntl = getenv("NAVGPU_LEAN_NT") ? atoi(getenv("NAVGPU_LEAN_NT")) : 512;
    const int NTl = ntl == 1024 ? 1024 : (ntl == 256 ? 256 : 512);
    const int walkers = rows_lean_walkers(tie != nullptr, NTl);
    const int F1 = std::min(C, kLeanF);
    int32_t *over;
    RC(ws(ctx, kOvf, rows, &over));
    auto launch = [&](auto kern, int F, int pass, int lds) -> int {
      hipLaunchKernelGGL(kern, dim3(rows), dim3(NTl), lds, ctx->stream, src, tgt, R, C, src_mask,
                         tgt_mask, nn_idx, nn_dist, tie, S, F, over, pass);
      CHECK_LAUNCH("k_rows_match_lean");
      return NAVGPU_OK;
    };
    auto run = [&](auto kern) -> int {
      int lds = rows_lean_lds(C, F1, walkers);
      RC(set_lds(kern, std::max(lds, rows_lean_lds(C, C, walkers))));
      RC(launch(kern, F1, 0, lds));
      if (F1 < C)  // the rows with more than F1 features
        RC(launch(kern, C, 1, rows_lean_lds(C, C, walkers)));
      return NAVGPU_OK;
    };
    if (NTl == 1024) return run(k_rows_match_lean<1024>);
    if (NTl == 512) return run(k_rows_match_lean<512>);
    return run(k_rows_match_lean<256>);
  }
  const RowsLds L = rows_lds(C, kRowsBlock, true);
  RC(set_lds(k_rows_match, L.total));
  hipLaunchKernelGGL(k_rows_match, dim3(rows), dim3(kRowsMatchBlock), L.total, ctx->stream, src,
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
  if (n >= ((size_t)1 << 30)) {
    set_err("kd_build: %zu points (at most 2^30 - 1)", n);
    return NAVGPU_ERANGE;
  }
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
  // levels above the leaves: until every subarray (<= ceil(n / 2^L)) fits
  // the LDS build of k_kd_leaves
  int L = 0;
  while (L < 30 && !(((n + ((size_t)1 << L) - 1) >> L) <= 65535 &&
                     kd_build_lds_bytes((int)((n + ((size_t)1 << L) - 1) >> L)) <= lds_limit()))
    ++L;
  const int nWmax = 1 << std::max(0, L - 1);
  // the selection kernels put a level's windows on grid.y (checked before
  // any workspace is sized for n)
  if (nWmax > 65535) {
    set_err("kd_build: %zu points need %d windows per level (grid.y limit 65535)", n, nWmax);
    return NAVGPU_ERANGE;
  }
  double *fc;
  uint32_t *P, *T;
  RC(ws(ctx, kKdFc, 3 * n, &fc));
  RC(ws(ctx, kKdP, n, &P));
  RC(ws(ctx, kKdT, n, &T));
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
  // per-level chunk counters: nW windows x chunks of one window, at most
  // about n / kSelChunk + nW at any level (not nWmax x all chunks of n)
  size_t ncnt = 0;
  for (int d = 0; d < L; ++d)
    ncnt = std::max(ncnt, ((size_t)1 << d) * (((n >> d) + kSelChunk - 1) / kSelChunk));
  RC(ws(ctx, kKdSel, (size_t)7 * nWmax + ncnt + kRounds + 1, &stbuf));
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
      // every iteration places its pivot, so a window of at most maxlen + 1
      // positions is done within maxlen + 1 iterations: a level still active
      // past that is stuck (a logic error), and fails at once instead of
      // spinning through 4 n iterations
      if ((long long)it > (long long)maxlen + 64) {
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
