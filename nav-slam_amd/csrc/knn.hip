// knn.hip — global-mode exact k-NN on MI355X (gfx950): the K3 configuration
// (BASELINE.json configs[2]) and the batched global queries of the API.
//
// The reference has one nearest-neighbour search, per scan row over a KD tree
// (utils/kdtree.c:110-152, driven from src/slam.c:236-252). Global mode is its
// generalisation to one index over a whole target cloud and k neighbours per
// query, ordered by (distance, index); for k = 1 it returns the reference KD
// answer whenever the nearest distance is unique. Distances are
// the reference formula, sqrt((dx*dx + dy*dy) + dz*dz) in f64, bit for bit.
//
// Pipeline of one call (DESIGN.md §3-§4 has the HBM layout and the roofline
// of each kernel):
//   k_bbox_partial                  target bbox partials
//   k_bin_hist, k_bin_colscan, k_bin_scatter, k_bin_fine
//                                   both clouds counting-sorted by cell of a
//                                   uniform grid (cells h/sx x h x h, ~occ
//                                   targets per h^3; every k_bin_hist block
//                                   derives the grid from the partials) with
//                                   LDS atomics only: the targets as
//                                   cell-sorted 32-B PRec records (f64 point,
//                                   index, x column) and 16-B SRec staging
//                                   records (f32 offsets), the queries as
//                                   cell-sorted 32-B records (point, index,
//                                   cell)
//   k_nb_fill                       (mode 2) the row neighbourhood lists
//   k_knnw<K>                       (mode 1) one wave per chunk of 64
//                                   cell-sorted queries: the chunk's row
//                                   pieces staged in LDS column-major, one
//                                   query per lane: packed-f32 keys into a
//                                   sorted top-(K+1) (v_med3 insertion), f64
//                                   exact stage, a certificate that the
//                                   answer is exact
//   k_knng<K>                       (mode 2) the same pass, each chunk's
//                                   image staged as slices of the row lists
//   k_knn_slow<K>                   the uncertified rest, one wave per query
#include "navgpu_common.h"

using namespace nv;

namespace {

// ============================================================ the grid
// Cells are numbered x-fastest, so the cells x-sx..x+sx of one (y,z) row are
// contiguous in the cell-sorted arrays.
struct GridParams {
  double o[3];            // origin = target bbox min
  double e[3], inv_e[3];  // cell edge per axis: x h / sx, y and z h
  double h;               // the coarse edge
  double delta;           // slack on cell boxes (cell assignment is f64 arithmetic)
  double emax;            // largest bbox extent
  int g[3];
  int ncells;
  int sx;                 // x cells per h: a query's block is cells x-sx .. x+sx,
                          // y-1 .. y+1, z-1 .. z+1 (the reach is >= h on every axis)
  int clamped;            // some axis hit the 2048-cell cap: its boundary cells
                          // hold points beyond their nominal box
  double c[3];            // (r5) the grid's centre: the one f32 frame of k_knng
  double Dt;              // bound on |t - c| per axis for every target (slack included)
};

// one point of a cell-sorted cloud: the caller's f64 coordinates, its index
// in the caller's array and the x index of its grid cell (the f64 binning's)
struct __align__(16) PRec {
  double x, y, z;
  int idx, cx;
};
// the same point as k_knnw stages it (r4): the f32 offset from the f64
// centre of its cell, o + (c + 0.5) e per axis, and the cell's x index
struct __align__(16) SRec {
  float x, y, z;
  int cx;
};

constexpr int kKeyBits = 8;        // local id in the low bits of a packed key
constexpr uint32_t kKeyMask = (1u << kKeyBits) - 1;
constexpr uint32_t kNoKey = 0xffffffffu;

constexpr int kBBoxBlocks = 256;  // bbox partials (every k_bin_hist block reduces them)

#ifndef NAVGPU_BBOX_U
#define NAVGPU_BBOX_U 4
#endif
#ifndef NAVGPU_BBOX_THREADS
#define NAVGPU_BBOX_THREADS 512  // (r6, 200-step bench A/B: 6 of 7 interleaved rounds faster than 256, ~1 %)
#endif
constexpr int kBBoxThreads = NAVGPU_BBOX_THREADS;  // threads per k_bbox_partial block
static_assert(kBBoxThreads % kWave == 0 && kBBoxThreads <= 1024, "bbox block");
// per-block min/max of the finite coordinates -> part[block][6]
__global__ __launch_bounds__(kBBoxThreads) void k_bbox_partial(const double *__restrict__ p,
                                                               size_t n, double *__restrict__ part) {
  __shared__ double s[kBBoxThreads / kWave][6];
  double v6[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  // batches of U points per thread, all loads of a batch in flight together,
  // issued unconditionally from clamped indices (r5: a conditional load per
  // element makes hipcc branch and wait around each)
  constexpr int U = NAVGPU_BBOX_U;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t ib = (size_t)blockIdx.x * blockDim.x + threadIdx.x; ib < n; ib += U * stride) {
    double v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = ib + u * stride;
      const double *q = p + 3 * (i < n ? i : n - 1);
#pragma unroll
      for (int a = 0; a < 3; ++a) v[u][a] = q[a];
      if (i >= n) v[u][0] = v[u][1] = v[u][2] = INFINITY;
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
    for (int w = 1; w < kBBoxThreads / kWave; ++w) r = a < 3 ? fmin(r, s[w][a]) : fmax(r, s[w][a]);
    part[blockIdx.x * 6 + a] = r;
  }
}

// what the grid is derived from: the bbox partials and the sizing knobs
struct GridArgs {
  const double *part;
  int nparts, cap, sx;
  double occ;
  size_t n, nq;
};

// bbox from the partials, then the grid: h for ~occ points per h^3, capped
// at `cap` cells; the tile width of k_knn. Run by a whole 256-thread block
// (every k_bin_hist block derives its own copy: one launch fewer than a
// separate grid kernel); thread 0 writes *out.
// this thread's share of the bbox partials (loaded first, so that a caller
// can issue other loads behind them and still wait for these alone)
struct Part6 {
  double v[6];
};
// One partial per thread at most (nparts <= kBBoxBlocks <= the block size):
// loaded unconditionally from a clamped slot, masked only when used.
__device__ __forceinline__ Part6 grid_partials(const GridArgs A) {
  Part6 P;
  const double *q = A.part + 6 * min((int)threadIdx.x, max(A.nparts - 1, 0));
#pragma unroll
  for (int a = 0; a < 6; ++a) P.v[a] = q[a];
  return P;
}
__device__ void grid_params_block(const GridArgs A, GridParams *out, const Part6 &P) {
  const int cap = A.cap, sx = A.sx;
  const double occ = A.occ;
  const size_t n = A.n;
  __shared__ double s[16][6];  // one row per wave (<= 1024 threads)
  double v6[6];
  const bool has = (int)threadIdx.x < A.nparts;  // (a select, not a branch: the
  for (int a = 0; a < 6; ++a)                     // wait stays behind the points)
    v6[a] = has ? P.v[a] : (a < 3 ? INFINITY : -INFINITY);
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
    G.clamped = 0;
    for (int a = 0; a < 3; ++a) G.c[a] = 0.5;
    G.Dt = 1.0;
    *out = G;
    return;
  }
  const double emax = fmax(ext[0], fmax(ext[1], ext[2]));
  const double floor_e = fmax(emax * 1e-3, 1e-9);
  double vol = 1.0;
  for (int a = 0; a < 3; ++a) vol *= fmax(ext[a], floor_e);
  double h = cbrt(vol * occ / (double)n);
  if (!(h > 0) || !(h < INFINITY)) h = fmax(emax, 1.0);
  int g[3], clamped = 0;
  for (int it = 0; it < 200; ++it) {
    long long tot = 1;
    clamped = 0;
    for (int a = 0; a < 3; ++a) {
      const double ea = a == 0 ? h / sx : h;
      double ga = floor(ext[a] / ea) + 1.0;  // covers [lo, lo + ext] inclusive
      if (ga > 2048) {
        ga = 2048;
        clamped = 1;
      }
      g[a] = (int)ga;
      tot *= g[a];
    }
    if (tot <= cap) break;
    h *= 1.1;
  }
  G.clamped = clamped;
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
  // the grid's centre, and a bound on |t - c| for every target: the bbox
  // [lo, lo + ext] lies in [o, o + g e] unless an axis was clamped, and in
  // [o, o + emax] always
  double half = 0.0;
  for (int a = 0; a < 3; ++a) {
    G.c[a] = G.o[a] + 0.5 * (g[a] * G.e[a]);
    half = fmax(half, 0.5 * (g[a] * G.e[a]));
  }
  G.Dt = (clamped ? fmax(half, emax) : half) + 4.0 * G.delta;
  *out = G;
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

constexpr int kBinMaxBuckets = 4096;  // coarse buckets per side (k_bin_*)

// (r5) Lean build kernels: 256-thread blocks of at most 64 VGPRs and a few KB
// of LDS, so that with two pairs in flight each of them fits on a CU beside
// the other pair's query pass (k_knng: 3 waves per SIMD of 147 VGPRs, 115 KB
// of LDS per CU) instead of waiting for it to drain.
#ifndef NAVGPU_BUILD_LEAN
#define NAVGPU_BUILD_LEAN 0
#endif
constexpr bool kLean = NAVGPU_BUILD_LEAN;
constexpr int kBuildMinW = kLean ? 8 : 1;  // launch-bounds waves per SIMD (8: <= 64 VGPRs)

// ---- (bucket, block) offsets of the binning (k_bin_*) ---------------------
// The count table is block-major per side, T[tab + blk * nb + b], so that
// k_bin_hist writes and k_bin_scatter reads one contiguous row per block.
// k_bin_colscan turns each bucket's column into an exclusive prefix over the
// blocks, in place, and its total into btot[side * nb + b]; the bucket bases
// (the exclusive scan of btot) are recomputed in LDS by every k_bin_scatter
// block (cheaper than a one-block launch); block 0 of each side publishes them
// to bbase[side * (nb + 1) + 0 .. nb] for k_bin_fine.
constexpr int kColB = kLean ? 16 : 64;  // buckets per k_bin_colscan block
constexpr int kColY = 16;              // block-row chunks per bucket column
constexpr int kColU = kLean ? 8 : 16;  // loads in flight per thread
__global__ __launch_bounds__(kColB * kColY, kBuildMinW) void k_bin_colscan(int *__restrict__ T, int nb,
                                                               int tab0, int nblk0, int tab1,
                                                               int nblk1, int *__restrict__ btot) {
  __shared__ int part[kColY][kColB];
  const int per_side = (nb + kColB - 1) / kColB;
  const int side = (int)blockIdx.x >= per_side ? 1 : 0;
  const int b = ((int)blockIdx.x - side * per_side) * kColB + (int)threadIdx.x % kColB;
  const int y = (int)threadIdx.x / kColB;
  const int tab = side ? tab1 : tab0, nblk = side ? nblk1 : nblk0;
  const int ch = (nblk + kColY - 1) / kColY;
  const int k0 = min(nblk, y * ch), k1 = min(nblk, k0 + ch);
  // a chunk's counts: every load in flight before any is used
  constexpr int U = kColU;
  int v[U], sum = 0;
  for (int k = k0; k < k1; k += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (b < nb && k + u < k1) ? T[tab + (k + u) * nb + b] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) sum += v[u];
  }
  part[y][threadIdx.x % kColB] = sum;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kColY; ++w) {
    const int c = part[w][threadIdx.x % kColB];
    pre += w < y ? c : 0;
    tot += c;
  }
  if (b >= nb) return;
  for (int k = k0; k < k1; k += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = k + u < k1 ? T[tab + (k + u) * nb + b] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k + u < k1) {
        T[tab + (k + u) * nb + b] = pre;
        pre += v[u];
      }
  }
  if (y == 0) btot[side * nb + b] = tot;
}

// ---- cell binning: counting sort of both clouds by grid cell --------------
// Scattered global atomics run at the memory side on this part (~24 G/s
// whatever their scope), so the sort uses none: LDS histograms and LDS ranks.
//  k_bin_hist    each block takes a contiguous chunk of points and counts
//                their coarse bucket (cell >> shift) in LDS; the counts land
//                in a block-major table[block * nb + b] (one contiguous row
//                per block); k_bin_colscan turns it into every (bucket,
//                block)'s offset within its bucket and the buckets' totals.
//  k_bin_scatter same chunks: each point gets an LDS rank within its
//                (bucket, block) and moves to the coarse-bucketed array
//                (BinPt, 32 B).
//  k_bin_fine    one block per bucket: LDS counting sort over the bucket's
//                2^shift cells, writes start[] for them (targets); every
//                point at its final cell-sorted position: targets as a PRec
//                (the exact stage's f64 record) and an SRec (the f32 record
//                the query passes stage), queries as their BinPt (the query
//                passes read 64 consecutive ones per chunk).
//                Order inside a cell is unspecified: the k-NN result does not
//                depend on it (ties are resolved by (distance, index)).
// Side 0 = targets, side 1 = queries; both go through the same launches
// (block ranges) and their tables are concatenated so one scan covers both.
struct BinPt {
  double x, y, z;
  int idx, cell;
};
// k_knng's staged target record (r5): the f32 offset from the grid centre, 12 B
// (the record's position comes from the row list)
struct F3 {
  float x, y, z;
};
#ifndef NAVGPU_KNNG_PACK
#define NAVGPU_KNNG_PACK 1  // 0: k_knng stages from the 16-B SRec (r5 A/B knob)
#endif
constexpr bool kKnngPack = NAVGPU_KNNG_PACK;
// a query's coarse-bucketed key (k_bin_scatter -> k_bin_fine)
struct QKey {
  int cell, idx;
};
struct BinSide {
  const double *p;
  int n, P, nblk;
  int tab;  // offset of this side's table in the concatenated table
  int *start;
  BinPt *bin;    // targets: coarse-bucketed points
  QKey *key;     // queries: coarse-bucketed (cell, index) keys
  PRec *sorted;  // targets: cell-sorted records
  SRec *srec;    // targets: the same, as k_knnw stages them
  F3 *frec;      // targets: the same, as k_knng stages them (instead of srec)
  int *perm;     // queries: cell-sorted position -> the caller's index
  int *qcell;    // queries: cell-sorted position -> cell
  int *rawcell;  // queries: the cell of each point in the caller's order
};
// the queries as the query passes read them: the caller's cloud, through the
// cell-sorted permutation
struct QSide {
  const double *pts;
  const int *idx, *cell;
};
__device__ __forceinline__ BinPt qload(const QSide &QS, int pos) {
  BinPt Q;
  Q.idx = QS.idx[pos];
  Q.cell = QS.cell[pos];
  const double *p = QS.pts + 3 * (size_t)Q.idx;
  Q.x = p[0];
  Q.y = p[1];
  Q.z = p[2];
  return Q;
}
struct BinJob {
  BinSide s[2];
  int shift, nb;  // buckets per side
  int sglobal;    // SRec form: 1 = k_knng's (grid-centre frame + position), 0 = k_knnw's
};

// the SRec of the target at cell-sorted position pos: k_knng reads f32
// offsets from the grid centre and the record's position (its image needs no
// per-record shift: DESIGN.md §4 r5); k_knnw the offset from the record's own
// cell centre and its x column
__device__ __forceinline__ SRec make_srec(const GridParams &G, bool sglobal, double x, double y,
                                          double z, int cell, int pos) {
  SRec r;
  if (sglobal) {
    r.x = (float)(x - G.c[0]);
    r.y = (float)(y - G.c[1]);
    r.z = (float)(z - G.c[2]);
    r.cx = pos;
    return r;
  }
  const int g0 = G.g[0], g1 = G.g[1];
  const int row = cell / g0, cx = cell - row * g0;
  const int cy = row % g1, cz = row / g1;
  r.x = (float)(x - (G.o[0] + (cx + 0.5) * G.e[0]));
  r.y = (float)(y - (G.o[1] + (cy + 0.5) * G.e[1]));
  r.z = (float)(z - (G.o[2] + (cz + 0.5) * G.e[2]));
  r.cx = cx;
  return r;
}
// k_knng's staged record: the f32 offsets from the grid centre
__device__ __forceinline__ F3 make_f3(const GridParams &G, double x, double y, double z) {
  return F3{(float)(x - G.c[0]), (float)(y - G.c[1]), (float)(z - G.c[2])};
}
constexpr int kBinMaxShift = 15;
#ifndef NAVGPU_BIN_UNROLL
#define NAVGPU_BIN_UNROLL (NAVGPU_BUILD_LEAN ? 4 : 8)
#endif
constexpr int kBinUnroll = NAVGPU_BIN_UNROLL;  // points per thread with loads in flight
// (compile-time knobs for A/B variant builds, scripts/build_variants.sh)
#ifndef NAVGPU_BIN_P
#define NAVGPU_BIN_P 4096
#endif
#ifndef NAVGPU_BIN_MIN_SHIFT
#define NAVGPU_BIN_MIN_SHIFT 10
#endif
#ifndef NAVGPU_BIN_FINE_THREADS
#define NAVGPU_BIN_FINE_THREADS (NAVGPU_BUILD_LEAN ? 256 : 512)
#endif
constexpr int kBinP = NAVGPU_BIN_P;  // minimum points per k_bin_hist / k_bin_scatter block
constexpr int kBinMinShift = NAVGPU_BIN_MIN_SHIFT;  // coarse buckets of 2^10 cells (r2 A/B)
constexpr int kBinFineThreads = NAVGPU_BIN_FINE_THREADS;
constexpr int kBinFineHold = kLean ? 2 : 4096 / kBinFineThreads;  // points per thread held in registers

__device__ __forceinline__ int bin_side(const BinJob &J, int &blk) {
  const int side = blk >= J.s[0].nblk ? 1 : 0;
  if (side) blk -= J.s[0].nblk;
  return side;
}

struct P3 {
  double x, y, z;
};
#ifndef NAVGPU_BIN_PRELOAD
#define NAVGPU_BIN_PRELOAD 1  // (r6) the first batch's point loads before the block's setup
#endif
constexpr bool kBinPreload = NAVGPU_BIN_PRELOAD;

// the block's chunk in batches of kBinUnroll points per thread: every load of
// a batch is issued before any of its cells is used. `prep` runs once, after
// the first batch's loads are issued and before any is used, and returns the
// grid (r6: the block's setup -- deriving the grid, scanning the bucket
// bases -- then overlaps the first round trip to HBM instead of preceding it)
// (`fallback`: any 24 readable device bytes, the source of an empty chunk's
// first loads, which are issued unconditionally so that no branch makes the
// compiler's wait counts conservative)
template <class Prep, class F>
__device__ __forceinline__ void bin_chunk(const BinSide &S, int blk, const void *fallback,
                                          Prep prep, F f) {
  const int i0 = blk * S.P, i1 = min(S.n, (blk + 1) * S.P);
  const int bd = (int)blockDim.x;
  const double *src = i1 > i0 ? S.p : (const double *)fallback;
  P3 v[kBinUnroll];
  auto load = [&](int ib) {
    // every load issued unconditionally from a clamped index (r5, as in
    // k_bbox_partial); the lanes past the chunk drop theirs below
#pragma unroll
    for (int u = 0; u < kBinUnroll; ++u) {
      const int i = ib + u * bd + (int)threadIdx.x;
      v[u] = *(const P3 *)(src + 3 * (size_t)max(min(i, i1 - 1), 0));
    }
  };
  if (kBinPreload) load(i0);
  const GridParams G = prep();
  for (int ib = i0; ib < i1; ib += kBinUnroll * bd) {
    if (!kBinPreload || ib != i0) load(ib);
#pragma unroll
    for (int u = 0; u < kBinUnroll; ++u) {
      const int i = ib + u * bd + (int)threadIdx.x;
      if (i < i1) f(i, v[u], cell_of(&v[u].x, G));
    }
  }
}

// Also derives the grid (grid_params_block; block 0 publishes it to *gp and
// resets the call's k-NN counters) and keeps each query's cell for
// k_bin_scatter (4 B instead of re-reading its 24-B point).
#ifndef NAVGPU_BIN_THREADS
#define NAVGPU_BIN_THREADS 512  // (r6 A/B: k_bin_scatter 25.9 -> 23.9 us against 256; 1024: k_bin_hist 14.8 -> 22)
#endif
constexpr int kBinThreads = NAVGPU_BIN_THREADS;  // threads per k_bin_hist / k_bin_scatter block
static_assert(kBBoxBlocks <= kBinThreads, "grid_partials: one bbox partial per thread");
__global__ __launch_bounds__(kBinThreads, kBuildMinW) void k_bin_hist(BinJob J, const GridArgs A,
                                                  GridParams *__restrict__ gp,
                                                  int *__restrict__ counters,
                                                  int *__restrict__ table) {
  extern __shared__ int hist[];  // J.nb counters
  __shared__ GridParams sG;
  int blk = blockIdx.x;
  const BinSide S = J.s[bin_side(J, blk)];
  for (int b = threadIdx.x; b < J.nb; b += blockDim.x) hist[b] = 0;
  const Part6 P = grid_partials(A);  // (issued before the points: waited for alone)
  bin_chunk(
      S, blk, A.part,
      [&]() {
        grid_params_block(A, &sG, P);
        if (blockIdx.x == 0 && threadIdx.x < 16) counters[threadIdx.x] = 0;  // [4, 12): tickets
        __syncthreads();
        const GridParams G = sG;  // (by value: registers, not an LDS read per point)
        if (blockIdx.x == 0 && threadIdx.x == 0) *gp = G;
        return G;
      },
      [&](int i, const P3 &, int c) {
        atomicAdd(&hist[c >> J.shift], 1);
        if (S.rawcell) S.rawcell[i] = c;
      });
  __syncthreads();
  for (int b = threadIdx.x; b < J.nb; b += blockDim.x) table[S.tab + blk * J.nb + b] = hist[b];
}

__global__ __launch_bounds__(kBinThreads, kBuildMinW) void k_bin_scatter(BinJob J, const GridParams *__restrict__ gp,
                                                     const int *__restrict__ offs,
                                                     const int *__restrict__ btot,
                                                     int *__restrict__ bbase) {
  extern __shared__ int cur[];  // J.nb cursors
  __shared__ int scratch[40];
  int blk = blockIdx.x;
  const int side = bin_side(J, blk);
  const BinSide S = J.s[side];
  // the side's bucket bases: exclusive scan of btot, each thread a run (run
  // once the block's first batch of points or cells is in flight)
  auto bases = [&]() {
    const int *bt = btot + side * J.nb;
    const int per = (J.nb + blockDim.x - 1) / blockDim.x;
    const int j0 = min(J.nb, (int)threadIdx.x * per), j1 = min(J.nb, j0 + per);
    int sum = 0;
    for (int j = j0; j < j1; ++j) sum += bt[j];
    int total;
    int acc = block_excl_scan(sum, scratch, &total);
    // the side's first block also publishes the bases for k_bin_fine
    int *bo = blk == 0 ? bbase + side * (J.nb + 1) : nullptr;
    for (int j = j0; j < j1; ++j) {
      const int v = bt[j];
      cur[j] = acc + offs[S.tab + blk * J.nb + j];
      if (bo) bo[j] = acc;
      acc += v;
    }
    if (bo && threadIdx.x == 0) bo[J.nb] = total;
    __syncthreads();
  };
  if (side) {  // queries: their cells as k_bin_hist kept them
    const int i0 = blk * S.P, i1 = min(S.n, (blk + 1) * S.P);
    const int bd = (int)blockDim.x;
    int c[kBinUnroll];
    auto load = [&](int ib) {
#pragma unroll
      for (int u = 0; u < kBinUnroll; ++u) {
        const int i = ib + u * bd + (int)threadIdx.x;
        c[u] = S.rawcell[max(min(i, i1 - 1), 0)];  // (clamped, unconditional; dropped below)
      }
    };
    if (kBinPreload) load(i0);  // (an empty chunk reads its clamped slot 0: nq > 0 here)
    bases();
    for (int ib = i0; ib < i1; ib += kBinUnroll * bd) {
      if (!kBinPreload || ib != i0) load(ib);
#pragma unroll
      for (int u = 0; u < kBinUnroll; ++u) {
        const int i = ib + u * bd + (int)threadIdx.x;
        if (i < i1) S.key[atomicAdd(&cur[c[u] >> J.shift], 1)] = QKey{c[u], i};
      }
    }
    return;
  }
  bin_chunk(
      S, blk, gp,
      [&]() {
        bases();
        return *gp;
      },
      [&](int i, const P3 &v, int c) {
        const int pos = atomicAdd(&cur[c >> J.shift], 1);
        BinPt t;
        t.x = v.x;
        t.y = v.y;
        t.z = v.z;
        t.idx = i;
        t.cell = c;
        S.bin[pos] = t;
      });
}

// One bucket: count its points per cell (LDS), scan, write the cell starts,
// then place every target (its PRec and SRec) or every query (its index in the
// caller's cloud and its cell: qperm, qcell).
// Queries of a bucket of at most kFineStage points (the usual case) are
// staged: each output position gets its input slot in LDS (lslot) and the
// positions are written in order, coalesced, instead of one scattered 4-B
// store each (r3 A/B: build 107 -> 106 us; staging the targets' 32-B records
// the same way measured 113 us: their LDS halves the resident blocks, and a
// scattered 32-B record store is already a whole sector). Otherwise the
// first kBinFineHold * blockDim points stay in registers between the count
// and the placement and the rest are re-read.
constexpr int kFineStage = 2048;
#ifndef NAVGPU_FINE_TSTAGE
#define NAVGPU_FINE_TSTAGE 1
#endif
constexpr bool kFineTStage = NAVGPU_FINE_TSTAGE;
constexpr int kFineStageHold = kFineStage / kBinFineThreads;
// dynamic LDS: cnt[2^shift], then lslot[kFineStage] when queries are staged
constexpr size_t fine_lds_bytes(int shift, bool stage_q) {
  return ((size_t)4 << shift) + (stage_q ? (size_t)kFineStage * sizeof(uint16_t) : 0);
}
__global__ __launch_bounds__(kBinFineThreads, kBuildMinW) void k_bin_fine(BinJob J,
                                                              const GridParams *__restrict__ gp,
                                                              const int *__restrict__ bbase,
                                                              int nscan, int qstage) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fine_lds[];
  int *cnt = (int *)fine_lds;                                        // 2^shift
  uint16_t *lslot = (uint16_t *)(fine_lds + ((size_t)4 << J.shift));  // qstage
  __shared__ int scratch[40];
  const int side = blockIdx.x >= J.nb ? 1 : 0;
  const int b = blockIdx.x - (side ? J.nb : 0);
  const BinSide S = J.s[side];
  const int ncell = 1 << J.shift, base = b << J.shift;
  const int lo = bbase[side * (J.nb + 1) + b], hi = bbase[side * (J.nb + 1) + b + 1];
  const int n = hi - lo;
  // staged placement: the queries' (qstage > 0) and, since r4, the targets'
  // (NAVGPU_FINE_TSTAGE): output positions are written in order, coalesced;
  // the scattered 32-B PRec / 16-B SRec stores cost partial-line writes
  const bool staged = n <= qstage && (side || kFineTStage);
  const BinPt *src = S.bin;
  const QKey *qk = S.key;
  const int bd = (int)blockDim.x, tid = (int)threadIdx.x;
  if (n == 0) {
    // an empty bucket (about half of them: the buckets span the cell cap,
    // twice the grid's cells): its cells all start at lo, no count or scan
    if (S.start)
      for (int j = tid; j < ncell; j += bd)
        if (base + j < nscan) S.start[base + j] = lo;
    return;
  }
  for (int j = tid; j < ncell; j += bd) cnt[j] = 0;
  __syncthreads();
  // unstaged: queries hold only their cell (the placement writes the position)
  BinPt hold[kBinFineHold];
  int scell[kFineStageHold];
  const int held_end = min(hi, lo + kBinFineHold * bd);
  if (staged) {
    // (loads issued unconditionally from clamped slots when the bucket is
    // not empty, as in bin_chunk; the slots past n are never used)
    if (n > 0) {
#pragma unroll
      for (int u = 0; u < kFineStageHold; ++u) {
        const int sl = lo + min(u * bd + tid, n - 1);
        scell[u] = side ? qk[sl].cell : src[sl].cell;
      }
    }
#pragma unroll
    for (int u = 0; u < kFineStageHold; ++u)
      if (u * bd + tid < n) atomicAdd(&cnt[scell[u] - base], 1);
  } else {
#pragma unroll
    for (int u = 0; u < kBinFineHold; ++u) {
      const int i = lo + u * bd + tid;
      if (i < held_end) {
        if (side) {
          const QKey e = qk[i];
          hold[u].cell = e.cell;
          hold[u].idx = e.idx;
        } else {
          hold[u] = src[i];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kBinFineHold; ++u) {
      const int i = lo + u * bd + tid;
      if (i < held_end) atomicAdd(&cnt[hold[u].cell - base], 1);
    }
    for (int i = held_end + tid; i < hi; i += bd)
      atomicAdd(&cnt[(side ? qk[i].cell : src[i].cell) - base], 1);
  }
  __syncthreads();
  // exclusive scan over the bucket's cells: each thread owns a contiguous run
  const int per = ncell / bd;  // ncell is a multiple of the block size
  const int j0 = tid * per;
  int sum = 0;
  for (int u = 0; u < per; ++u) sum += cnt[j0 + u];
  int total;
  int acc = lo + block_excl_scan(sum, scratch, &total);
  for (int u = 0; u < per; ++u) {
    const int v = cnt[j0 + u];
    cnt[j0 + u] = acc;
    if (S.start && base + j0 + u < nscan) S.start[base + j0 + u] = acc;
    acc += v;
  }
  __syncthreads();
  const GridParams &G = *gp;
  const int g0 = G.g[0];
  if (staged) {
#pragma unroll
    for (int u = 0; u < kFineStageHold; ++u) {
      const int sl = u * bd + tid;
      if (sl < n) lslot[atomicAdd(&cnt[scell[u] - base], 1) - lo] = (uint16_t)sl;
    }
    __syncthreads();
    if (side) {
      for (int j = tid; j < n; j += bd) {
        const QKey e = qk[lo + lslot[j]];
        S.perm[lo + j] = e.idx;
        S.qcell[lo + j] = e.cell;
      }
    } else {
      for (int j = tid; j < n; j += bd) {
        const BinPt e = src[lo + lslot[j]];  // (the bucket's records are in L2)
        PRec t;
        t.x = e.x;
        t.y = e.y;
        t.z = e.z;
        t.idx = e.idx;
        const int row = e.cell / g0;
        t.cx = e.cell - row * g0;
        S.sorted[lo + j] = t;
        if (S.frec)
          S.frec[lo + j] = make_f3(G, e.x, e.y, e.z);
        else
          S.srec[lo + j] = make_srec(G, J.sglobal, e.x, e.y, e.z, e.cell, lo + j);
      }
    }
    return;
  }
  auto place = [&](const BinPt &e, int i) {
    const int pos = atomicAdd(&cnt[e.cell - base], 1);
    if (side) {
      S.perm[pos] = e.idx;
      S.qcell[pos] = e.cell;
    } else {
      PRec t;
      t.x = e.x;
      t.y = e.y;
      t.z = e.z;
      t.idx = e.idx;
      const int row = e.cell / g0;
      t.cx = e.cell - row * g0;
      S.sorted[pos] = t;
      if (S.frec)
        S.frec[pos] = make_f3(G, e.x, e.y, e.z);
      else
        S.srec[pos] = make_srec(G, J.sglobal, e.x, e.y, e.z, e.cell, pos);
    }
  };
#pragma unroll
  for (int u = 0; u < kBinFineHold; ++u) {
    const int i = lo + u * bd + tid;
    if (i < held_end) place(hold[u], i);
  }
  for (int i = held_end + tid; i < hi; i += bd) {
    if (side) {
      BinPt e;
      e.cell = qk[i].cell;
      e.idx = qk[i].idx;
      place(e, i);
    } else {
      place(src[i], i);
    }
  }
}

// ---- (r5) the row neighbourhood lists k_knng stages from -------------------
// For grid row R = (y, z), its list GL_R holds, column by column (x = 0 ..
// g0-1), the cell-sorted positions of the targets of the 9 cells (x, y+dy,
// z+dz), dy, dz in {-1, 0, 1} in the order s = 3 (dz+1) + (dy+1), each cell's
// run in order. A query in cell (x, R) then finds its whole block (cells
// x-sx .. x+sx of the 9 rows) as ONE contiguous range of GL_R, and a run of
// query cells of one row stages ONE contiguous slice.
//
// Where GL_R starts needs no scan. Pad the (y, z) plane with one empty row of
// cells on every side and number the padded rows P in the grid's order; every
// padded row gets the list of its 9 neighbours, and the lists lie in P order.
// Row P's 9 neighbours are P + sigma_s (sigma_s = dz (g1+2) + dy, no wrap can
// reach a non-empty row), so the targets in the lists before P's number
// sum_s C(P + sigma_s), C(Q) = the targets in real rows before padded row Q,
// which is tstart at that row's first cell (0 below the grid, nt above it, a
// z slab's start or end beside it). Within the row, column x starts after
// tstart[(R_s) g0 + x] - tstart[(R_s) g0] more of each neighbour R_s, so
//   npg(R, x) = sum_s T_s(x),  T_s(x) = tstart[(y+dy, z+dz) g0 + x] for an
//   in-grid neighbour, C(P + sigma_s) otherwise,
// and the lists take exactly 9 nt positions. npg is stored per row with g0+1
// entries (x = g0: the row's end; rows are not adjacent in the padded order).
// One thread per (row, x): 18 tstart loads (L2), the npg entry and the
// column's ~9 occ positions written in order.
__device__ __forceinline__ int nb_pos(int yy, int zz, int x, int g0, int g1, int g2, int &real) {
  real = 0;
  if (zz < 0) return 0;                              // tstart[0] = 0
  if (zz >= g2) return g0 * g1 * g2;                 // = nt
  if (yy < 0) return zz * g1 * g0;                   // the slab's start
  if (yy >= g1) return (zz + 1) * g1 * g0;           // its end
  real = 1;
  return (zz * g1 + yy) * g0 + x;
}

// One WAVE per task = 64 consecutive columns of one row: lane = column for the
// loads and npg, then lane = (column, s) cell run for the list writes, so one
// store instruction covers 64 consecutive runs (a few cache lines) instead of
// 64 columns ~15 positions apart. (r5: writing each task's positions 64 at a
// time, coalesced, through LDS run marks and a running max measured 33 against
// 25 us: the marks' 32 KB per workgroup cost residency.)
#ifndef NAVGPU_NB_WAVES
#define NAVGPU_NB_WAVES 4
#endif
constexpr int kNbWaves = NAVGPU_NB_WAVES;  // waves per k_nb_fill workgroup
__global__ __launch_bounds__(kWave * kNbWaves) void k_nb_fill(const GridParams *__restrict__ gp,
                                                              const int *__restrict__ tstart,
                                                              int *__restrict__ npg,
                                                              int *__restrict__ gl) {
  __shared__ int tab[kNbWaves][2][kWave * 9 + 1];  // per (column, s): start, list offset
  const int g0 = gp->g[0], g1 = gp->g[1], g2 = gp->g[2];
  const int w = g0 + 1;
  const int tpr = (w + kWave - 1) / kWave;  // tasks per row
  const int ntask = g1 * g2 * tpr;
  const int wid = (int)threadIdx.x / kWave, lane = (int)threadIdx.x & (kWave - 1);
  int *ta = tab[wid][0], *to = tab[wid][1];  // run r's count: to[r + 1] - to[r]
  for (int t = blockIdx.x * kNbWaves + wid; t < ntask; t += gridDim.x * kNbWaves) {
    const int R = t / tpr, x0 = (t - R * tpr) * kWave;
    const int y = R % g1, z = R / g1;
    const int x = x0 + lane;
    const int xc = min(x, g0);
    int a[9], c[9], base = 0;
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      int real;
      const int p = nb_pos(y + s % 3 - 1, z + s / 3 - 1, xc, g0, g1, g2, real);
      // both loads unconditional (a branch per load would wait for each)
      const int va = tstart[p];
      const int vb = tstart[real && xc < g0 ? p + 1 : p];
      a[s] = va;
      c[s] = x < g0 ? vb - va : 0;
      base += va;
    }
    if (x <= g0) npg[R * w + x] = base;
    int off = base;
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      ta[lane * 9 + s] = a[s];
      to[lane * 9 + s] = off;
      off += c[s];
    }
    if (lane == kWave - 1) to[kWave * 9] = off;
    wave_sync_mem();
#pragma unroll
    for (int it = 0; it < 9; ++it) {
      const int r = it * kWave + lane;
      const int va = ta[r], o = to[r], n = to[r + 1] - o;
      for (int k = 0; k < n; ++k) gl[o + k] = va + k;
    }
    wave_sync_mem();  // the tables are rewritten by the wave's next task
  }
}

// ============================================================ k-NN helpers
// (d, i) < (kd, ki): distance first, then index. Never true for d = inf/NaN.
__device__ __forceinline__ bool knn_less(double d, int i, double kd, int ki) {
  return d < kd || (d == kd && i < ki);
}

// the same without short-circuit evaluation (selects, no branches)
__device__ __forceinline__ bool knn_less_bf(double d, int i, double kd, int ki) {
  return (d < kd) | ((d == kd) & (i < ki));
}

// compare-exchange: (ad, ai) <= (bd, bi) by (distance, index) afterwards
__device__ __forceinline__ void knn_cx(double &ad, int &ai, double &bd, int &bi) {
  const bool sw = knn_less_bf(bd, bi, ad, ai);
  const double td = sw ? bd : ad, ud = sw ? ad : bd;
  const int ti = sw ? bi : ai, ui = sw ? ai : bi;
  ad = td;
  ai = ti;
  bd = ud;
  bi = ui;
}

// squared distance from q to the box of cells [x0..x1] x [y0..y1] x [z0..z1]
// grown by delta: a lower bound on the reference dsq of any point binned there
__device__ __forceinline__ double box_d2(const GridParams &G, const double *qv, int x0, int x1,
                                         int y0, int y1, int z0, int z1) {
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


struct KnnLists {
  int *slow_q, *n_slow;  // queries (cell-sorted positions) the fast path could not certify
  double *slow_thr;      // their starting bound (K-th dsq upper bound), or inf
  int *n_unstaged;       // of them: queries whose block exceeded the LDS budget
  int *err;              // set when a kernel had to clamp an index (navgpu_knn_check)
  int vec_out;           // outputs 16-B aligned: results may be stored as vectors
};

__device__ __forceinline__ void push_slow(const KnnLists &L_, int qi, double thr) {
  const int e = atomicAdd(L_.n_slow, 1);
  L_.slow_q[e] = qi;
  L_.slow_thr[e] = thr;
}

// ============================================================ k_knnw
// The query pass in wave chunks (r4): one WAVE per chunk of 64 consecutive
// cell-sorted queries, no block barriers. k_knn's tiles were W query cells of
// one grid row on a 3-wave block: ~146 queries on 192 lanes (0.77 of the
// lanes), every tile paying stage -> barrier -> scan -> barrier. Here a chunk
// is exactly 64 queries wherever the grid rows break; its queries fall into a
// few SEGMENTS (one per grid row they touch, 1-2 on uniform data) and the
// wave stages every segment's 9 neighbouring row pieces into its own LDS
// region, column-major as in k_knn: segment s owns virtual columns
// [vc0_s, vc0_s + ncol_s), its cells xf_s - S .. xl_s + S, each column the
// records of its 9 (y, z) rows in turn, so a query's block is still ONE
// contiguous slot range. Each segment has its own f32 frame (the tile centre
// of k_knn for the segment's query cells). A chunk whose segments need more
// than kWCols columns or kWRec records is done in rounds over a prefix of its
// lanes; a lane whose block alone exceeds kWRec goes to k_knn_slow.
// The per-query scan, exact stage and certificate are k_knn's.
#ifndef NAVGPU_KNNW_REC
#define NAVGPU_KNNW_REC 800
#endif
#ifndef NAVGPU_KNNW_MINW
#define NAVGPU_KNNW_MINW 4  // (r4 A/B: query 165 -> 161 us against 3)
#endif
constexpr int kWRec = NAVGPU_KNNW_REC;   // staged records per wave (16 B each)
constexpr int kWPairs = kWRec / 2 + 2;   // two spare pairs: read-ahead
constexpr int kWZg = 4 * kWPairs;        // floats from the XY plane to the ZG plane
constexpr int kWCols = 2 * kWave;        // staged columns per round: two per lane
#ifndef NAVGPU_KNNW_SEGS
#define NAVGPU_KNNW_SEGS 8
#endif
constexpr int kWSegs = NAVGPU_KNNW_SEGS;  // segments (grid rows) per round
// waves per workgroup, each with its own chunk and LDS region
#ifndef NAVGPU_KNNW_WPB
#define NAVGPU_KNNW_WPB 1
#endif
constexpr int kWPB = NAVGPU_KNNW_WPB;
#ifndef NAVGPU_KNNW_U
#define NAVGPU_KNNW_U 1
#endif

// inclusive wave64 prefix sum by DPP (row_shr 1/2/4/8, row_bcast 15/31):
// every lane must be active
__device__ __forceinline__ int rdlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// the f32 frame of a segment whose query cells are xf .. xl of row (y, z):
// k_knn's tile centre; Dt bounds every staged offset (cell slack included)
struct WFrame {
  double o[3], Dt;
};
__device__ __forceinline__ WFrame wframe(const GridParams &G, int xf, int xl, int y, int z) {
  WFrame F;
  F.o[0] = G.o[0] + (xf + 0.5 * (xl - xf + 1)) * G.e[0];
  F.o[1] = G.o[1] + (y + 0.5) * G.h;
  F.o[2] = G.o[2] + (z + 0.5) * G.h;
  F.Dt = G.clamped ? G.emax + 2.0 * G.h
                   : fmax((0.5 * (xl - xf + 1) + G.sx + 1) * G.e[0], 2.0 * G.h) + 4.0 * G.delta;
  return F;
}

#ifdef NAVGPU_STAMPS
// k_knnw's phase stamps: one record per chunk, written by lane 0 (atomics on
// shared slots from every wave would serialise at the memory side and
// distort what they time); knn_stamps_take sums them
constexpr int kWStampChunks = 1 << 15;
__device__ unsigned long long g_wstamps[kWStampChunks][8];
#define NV_WFLUSH(chunk)                                             \
  if ((threadIdx.x & 63) == 0 && (chunk) < kWStampChunks) {          \
    _Pragma("unroll") for (int s_ = 1; s_ < 9; ++s_)                 \
      g_wstamps[chunk][s_ - 1] = nv_acc[s_];                         \
  }
#else
#define NV_WFLUSH(chunk)
#endif

// k_knnw asks for 4 waves per SIMD; its LDS allows 3, so the backend reports
// the occupancy target as missed ("pass failed"); the request still measured
// faster (r4), and only this kernel's warning is silenced
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
template <int K>
__global__ __launch_bounds__(kWave * kWPB, NAVGPU_KNNW_MINW) void k_knnw(const GridParams *__restrict__ gp,
                                                   const int *__restrict__ tstart,
                                                   const PRec *__restrict__ tsort,
                                                   const SRec *__restrict__ srec,
                                                   const QSide QS, int nq, int ntg,
                                                   int32_t *__restrict__ oidx,
                                                   double *__restrict__ odist, KnnLists L_) {
  // one region per wave of the workgroup (the waves never synchronise)
  __shared__ __attribute__((aligned(16))) float spair_w[kWPB][2 * kWZg];
  __shared__ int colst_w[kWPB][kWCols + 1];  // first slot of virtual column v; [kWCols] = total
  // each segment's 9 row pieces: [sbnd[s][r][0], sbnd[s][r][1])
  __shared__ int sbnd_w[kWPB][kWSegs][9][2];
  const int wid = kWPB > 1 ? (int)threadIdx.x / kWave : 0;
  float *spair = spair_w[wid];
  int *colst = colst_w[wid];
  int(*sbnd)[9][2] = sbnd_w[wid];
  constexpr int KL = K + 1;
  static_assert(K >= 1 && K <= 16, "K");
  const GridParams G = *gp;
  const int S = G.sx;
  const int g0 = G.g[0], g1 = G.g[1], g2 = G.g[2];
  // chunks dealt to the 8 XCDs in contiguous ranges (block b -> XCD b % 8),
  // kWPB consecutive chunks per workgroup
  const int nchunk = (nq + kWave - 1) / kWave;
  const int per = (nchunk + 7) / 8;
  const int cx = (int)(blockIdx.x >> 3) * kWPB + wid;
  const int chunk = (int)(blockIdx.x & 7) * per + cx;
  if (cx >= per || chunk >= nchunk) return;  // (no workgroup barrier follows)
  const int lane = (int)threadIdx.x & (kWave - 1);
  NV_ACC_DECL;
  NV_STAMP(w0);
  const int nlive = min(kWave, nq - chunk * kWave);
  const int qi = chunk * kWave + lane;
  const bool live = lane < nlive;
  BinPt Q;
  Q = qload(QS, min(qi, nq - 1));  // (unconditional: see the table loads)
  // the query's cell: x, row = (z g1 + y); rows ascend over the lanes
  const int qrow = live ? Q.cell / g0 : 0x7fffffff;
  const int qx = live ? Q.cell - qrow * g0 : 0;
  const int qy = live ? qrow % g1 : 0, qz = live ? qrow / g1 : 0;
  const uint32_t vmask = ~kKeyMask;
  int bad = 0;  // an index that had to be clamped (a logic error)
  // rows ascend over the live lanes: a lane starts (ends) a grid row when the
  // lane before (after) it holds another one (the shuffles run on every lane:
  // a lane masked off by a short-circuit would hand its neighbour garbage)
  const int prow = __shfl_up(qrow, 1, kWave), nrow = __shfl_down(qrow, 1, kWave);
  const unsigned long long rowfirst = __ballot(live && (lane == 0 || prow != qrow));
  const unsigned long long rowlast = __ballot(live && (lane == nlive - 1 || nrow != qrow));
  NV_STAMP(w1);
  NV_ACC(1, w0, w1);
  for (int la = 0; la < nlive;) {
    NV_STAMP(r0);
    NV_ACC(7, 0ull, 1ull);
    // ---- segments of lanes [la, nlive): a grid row each (the first one may
    // start mid-row after a cut round)
    const bool in = lane >= la && live;
    const unsigned long long fall = (rowfirst & (~0ull << la)) | (1ull << la);
    const unsigned long long below = (2ull << lane) - 1;  // lanes <= lane (lane 63: all)
    const int sf = 63 - __builtin_clzll((fall & below) | 1ull);  // the lane's segment: first lane
    const int sl = (int)__builtin_ctzll((rowlast & ~(below >> 1)) | (1ull << 63));  // ... last
    const bool first = in && sf == lane, last = in && sl == lane;
    const int xf = __shfl(qx, sf, kWave);  // the segment's first query cell
    const int colq = qx - xf + S;          // the lane's cell: column in its segment
    const int val = last ? colq + S + 1 : 0;  // columns of a segment, at its last lane
    const int incv = wave_scan_add(val);
    const int pre = in ? incv - val : 0;   // columns of earlier segments
    const int vcq = pre + colq;            // the lane's cell: virtual column
    const int cum = vcq + S + 1;           // columns if the round ended here
    // the round: the lane prefix whose columns fit (cum ascends over the
    // lanes) in at most kWSegs segments
    const int segi = __popcll(fall & below) - 1;
    int lb = la + __popcll(__ballot(in && cum <= kWCols && segi < kWSegs));
    const int lbc = lb;  // the frames use the column-fit round (a budget cut keeps them)
    int NC = rdlane(cum, lb - 1);
    unsigned long long fb = __ballot(first && lane < lb);  // segment starts
    // ---- column tables: virtual column v = lane + 64 p -> cell (vx, vy, vz);
    // cs = its records (the 9 rows'), cbr[p][r] + g = the slot of the record
    // at cell-sorted position g of row r; dxc = the column's cell centre in
    // its segment's frame (x)
    int cbr[2][9], st[2][9], en[2][9];
    float dxc[2];
    int total;
    {
      int cs[2], vx[2], vy[2], vz[2];
      double fox[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        vx[p] = vy[p] = vz[p] = 0;
        cs[p] = 0;
        fox[p] = 0.0;
      }
      for (unsigned long long b = fb; b; b &= b - 1) {
        const int f = (int)__builtin_ctzll(b);
        const int f_vc0 = rdlane(pre, f), f_xf = rdlane(qx, f), f_x0 = f_xf - S;
        const int f_y = rdlane(qy, f), f_z = rdlane(qz, f);
        const int f_xl = rdlane(qx, min(rdlane(sl, f), lbc - 1));
        const double f_ox = wframe(G, f_xf, f_xl, f_y, f_z).o[0];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int v = lane + kWave * p;
          if (v >= f_vc0) {
            vx[p] = f_x0 + (v - f_vc0);
            vy[p] = f_y;
            vz[p] = f_z;
            fox[p] = f_ox;
          }
        }
      }
      const int np = NC > kWave ? 2 : 1;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int v = lane + kWave * p;
        // the f64 cell centre k_bin_fine measured the SRec offsets from
        dxc[p] = (float)((G.o[0] + (vx[p] + 0.5) * G.e[0]) - fox[p]);
        if (p < np) {  // wave-uniform
          // every load issued unconditionally (cells off the grid read
          // tstart[0] and are zeroed after): a per-element condition makes
          // hipcc branch around each load and wait for it
          bool ok[9];
#pragma unroll
          for (int r = 0; r < 9; ++r) {
            const int yy = vy[p] + (r % 3) - 1, zz = vz[p] + (r / 3) - 1;
            ok[r] = v < NC && yy >= 0 && yy < g1 && zz >= 0 && zz < g2;
            const int base = ok[r] ? (zz * g1 + yy) * g0 : 0;
            st[p][r] = tstart[ok[r] ? base + min(max(vx[p], 0), g0) : 0];
            en[p][r] = tstart[ok[r] ? base + min(max(vx[p] + 1, 0), g0) : 0];
          }
#pragma unroll
          for (int r = 0; r < 9; ++r) {
            st[p][r] = ok[r] ? st[p][r] : 0;
            en[p][r] = ok[r] ? en[p][r] : 0;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 9; ++r) st[p][r] = en[p][r] = 0;
        }
#pragma unroll
        for (int r = 0; r < 9; ++r) cs[p] += en[p][r] - st[p][r];
      }
      const int inc0 = wave_scan_add(cs[0]);
      const int tot0 = rdlane(inc0, kWave - 1);
      const int inc1 = np > 1 ? wave_scan_add(cs[1]) + tot0 : tot0;
      total = rdlane(inc1, kWave - 1);
      const int ex[2] = {inc0 - cs[0], inc1 - cs[1]};
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        int a = ex[p];
#pragma unroll
        for (int r = 0; r < 9; ++r) {
          cbr[p][r] = a - st[p][r];
          a += en[p][r] - st[p][r];
        }
        colst[lane + kWave * p] = ex[p];
      }
      if (lane == 0) colst[kWCols] = total;
    }
    wave_sync_mem();
    NV_STAMP(r1);
    NV_ACC(2, r0, r1);
    if (total > kWRec) {
      // the lane prefix whose blocks end within the budget (slot ends ascend)
      const bool inr = in && lane < lb;
      const int endslot = inr ? colst[vcq + S + 1] : 0x7fffffff;
      const int lb2 = la + __popcll(__ballot(inr && endslot <= kWRec));
      if (lb2 == la) {
        // the first lane's block alone exceeds the budget: it and every lane
        // of its cell go to k_knn_slow from an infinite bound
        const int vq0 = rdlane(vcq, la);
        const bool same = inr && vcq == vq0;
        if (same) {
          push_slow(L_, qi, INFINITY);
          atomicAdd(L_.n_unstaged, 1);
        }
        la += __popcll(__ballot(same));
        wave_sync_mem();  // colst is rewritten by the next round
        continue;
      }
      lb = lb2;
      NC = rdlane(cum, lb - 1);
      fb &= lb >= kWave ? ~0ull : ((1ull << lb) - 1);
    }
    // ---- each segment's row pieces: the starts at its first column, the
    // ends at its last (the round's cut included), from the tables
    {
      int si = 0;
      for (unsigned long long b = fb; b; b &= b - 1, ++si) {
        const int f = (int)__builtin_ctzll(b);
        const int lsl = min(rdlane(sl, f), lb - 1);
        const int vc0 = rdlane(pre, f), vlast = rdlane(cum, lsl) - 1;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int v = lane + kWave * p;
#pragma unroll
          for (int r = 0; r < 9; ++r) {
            if (v == vc0) sbnd[si][r][0] = st[p][r];
            if (v == vlast) sbnd[si][r][1] = en[p][r];
          }
        }
      }
    }
    wave_sync_mem();
    // ---- staging: per segment, its 9 row pieces as SRec (16 B: f32 offset
    // from the record's cell centre + x cell); every load of a segment in
    // flight before any is used; slot from cbr, x shift from dxc (the
    // record's column's lane), y and z shifts per row. TWO: the round has
    // columns past 64 (the second table of each lane), a separate copy so
    // the usual one-table round shuffles only once per value.
    auto stage = [&](auto TWO) {
      int si = 0;
      for (unsigned long long b = fb; b; b &= b - 1, ++si) {
        const int f = (int)__builtin_ctzll(b);
        const int lsl = min(rdlane(sl, f), lb - 1);
        const int vc0 = rdlane(pre, f), vlast = rdlane(cum, lsl) - 1;
        const int sxf = rdlane(qx, f), sy = rdlane(qy, f), sz = rdlane(qz, f);
        const WFrame F = wframe(G, sxf, rdlane(qx, min(rdlane(sl, f), lbc - 1)), sy, sz);
        const int x0 = sxf - S;
        const int tlast = max(ntg - 1, 0);  // (srec holds at least one record)
        constexpr int U = NAVGPU_KNNW_U;
        int glo[9], nr[9];
#pragma unroll
        for (int r = 0; r < 9; ++r) {  // wave-uniform: scalar registers
          glo[r] = __builtin_amdgcn_readfirstlane(sbnd[si][r][0]);
          nr[r] = __builtin_amdgcn_readfirstlane(sbnd[si][r][1]) - glo[r];
        }
        for (int k0 = 0;; k0 += U * kWave) {
          SRec v[9][U];
          bool more = false;
          // every load is issued, unconditionally, from a position clamped
          // into the cloud (a per-element condition makes hipcc branch around
          // each load and wait for it: nine serial round trips); lanes past a
          // row piece discard theirs below. A clamp inside a piece would be a
          // logic error: it sets the call's error flag (navgpu_knn_check).
#pragma unroll
          for (int r = 0; r < 9; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int k = k0 + u * kWave + lane;
              // (a wave-uniform row base and a 32-bit lane offset)
              bad |= (k < nr[r]) & ((unsigned)(glo[r] + k) >= (unsigned)ntg);
              v[r][u] = (srec + glo[r])[min(k, tlast - glo[r])];
            }
#pragma unroll
          for (int r = 0; r < 9; ++r) {
            more |= k0 + U * kWave < nr[r];
            const int yy = sy + (r % 3) - 1, zz = sz + (r / 3) - 1;
            const float dy = (float)((G.o[1] + (yy + 0.5) * G.e[1]) - F.o[1]);
            const float dz = (float)((G.o[2] + (zz + 0.5) * G.e[2]) - F.o[2]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int k = k0 + u * kWave + lane;
              const int vcol = vc0 + v[r][u].cx - x0;
              const int il = vcol & (kWave - 1);
              int cb = __shfl(cbr[0][r], il, kWave);
              float dx = __shfl(dxc[0], il, kWave);
              if constexpr (decltype(TWO)::value) {
                const int c1 = __shfl(cbr[1][r], il, kWave);
                const float d1 = __shfl(dxc[1], il, kWave);
                cb = vcol >= kWave ? c1 : cb;
                dx = vcol >= kWave ? d1 : dx;
              }
              if (k < nr[r] && vcol <= vlast) {
                const int slot = cb + glo[r] + k;
                float *d = spair + (slot >> 1) * 4 + (slot & 1);
                d[0] = v[r][u].x + dx;
                d[2] = v[r][u].y + dy;
                d[kWZg] = v[r][u].z + dz;
                d[kWZg + 2] = __int_as_float(glo[r] + k);
              }
            }
          }
          if (!more) break;  // wave-uniform: nr and k0 are
        }
      }
    };
    if (NC > kWave)
      stage(std::true_type{});
    else
      stage(std::false_type{});
    wave_sync_mem();
    NV_STAMP(r2);
    NV_ACC(3, r1, r2);
    // the last query cell of the lane's segment in the column-fit round (its frame)
    const int xl = __shfl(qx, min(sl, lbc - 1), kWave);
    // ---- the round's queries, one per lane (k_knn's scan, exact stage and
    // certificate on the lane's block [t0, t1))
    if (in && lane < lb) {
      const double qv[3] = {Q.x, Q.y, Q.z};
      const int c[3] = {qx, qy, qz};
      const int t0 = colst[vcq - S], t1 = colst[vcq + S + 1];
      const WFrame F = wframe(G, xf, xl, qy, qz);
      const double qr[3] = {qv[0] - F.o[0], qv[1] - F.o[1], qv[2] - F.o[2]};
      const double Dq = fmax(F.Dt, fmax(fabs(qr[0]), fmax(fabs(qr[1]), fabs(qr[2]))));
      // each f32 difference is within dl of the exact one: the staged target
      // offset s + d carries <= 4 u Dq (s from the cell centre, the centre's
      // shift d, their sum), the query's u Dq, the subtraction 2 u Dq, with
      // u = 2^-24 (SRec)
      const double dl = Dq * 0x1p-21;
      const f2 qx2 = {(float)qr[0], (float)qr[0]}, qy2 = {(float)qr[1], (float)qr[1]},
               qz2 = {(float)qr[2], (float)qr[2]};
      const double Lr = block_reach(G, qv, c, 1);
      uint32_t key[KL];
#pragma unroll
      for (int s = 0; s < KL; ++s) key[s] = kNoKey;
      auto ins = [&](uint32_t kk) {  // keep the K+1 smallest keys sorted
#pragma unroll
        for (int s = K; s > 0; --s) key[s] = umed3(key[s - 1], key[s], kk);
        key[0] = min(key[0], kk);
      };
      auto dist2 = [&](const float *p) {  // packed f32 squared distances of a pair
        const float4 xy = *(const float4 *)p;
        const float2 zz = *(const float2 *)(p + kWZg);
        const f2 fx2 = f2{xy.x, xy.y} - qx2, fy2 = f2{xy.z, xy.w} - qy2,
                 fz2 = f2{zz.x, zz.y} - qz2;
        return __builtin_elementwise_fma(fz2, fz2, __builtin_elementwise_fma(fy2, fy2, fx2 * fx2));
      };
      const int ta = t0 & ~1;
      const int npr = (t1 - ta + 1) >> 1;  // pairs the block touches
      const bool overflow = (t1 - ta) > (1 << kKeyBits);
      const float *cur = spair + (ta >> 1) * 4;
      if (npr > 0) {  // first pair: may start before the block (odd t0) or end past it
        const f2 d = dist2(cur);
        const uint32_t k0 = knn_key(d[0], vmask, 0u), k1 = knn_key(d[1], vmask, 1u);
        if (ta >= t0) ins(k0);
        if (ta + 1 < t1) ins(k1);
        cur += 4;
      }
      if (npr > 2) {  // interior pairs: the key's local id is the wave-uniform pair counter
        const float *lastp = spair + ((ta >> 1) + npr - 1) * 4;
        uint32_t v2 = 2;
        float4 xy = *(const float4 *)cur;
        float2 zz = *(const float2 *)(cur + kWZg);
        do {
          const float4 nxy = *(const float4 *)(cur + 4);
          const float2 nzz = *(const float2 *)(cur + 4 + kWZg);
          const f2 fx2 = f2{xy.x, xy.y} - qx2, fy2 = f2{xy.z, xy.w} - qy2,
                   fz2 = f2{zz.x, zz.y} - qz2;
          const f2 d =
              __builtin_elementwise_fma(fz2, fz2, __builtin_elementwise_fma(fy2, fy2, fx2 * fx2));
          ins(knn_key(d[0], vmask, v2));
          ins(knn_key(d[1], vmask, v2 + 1));
          cur += 4;
          v2 += 2;
          xy = nxy;
          zz = nzz;
        } while (cur < lastp);
      }
      if (npr > 1) {  // last pair: may end past the block
        const f2 d = dist2(cur);
        const uint32_t lid = (uint32_t)(2 * (npr - 1)) & kKeyMask;
        const uint32_t k0 = (__float_as_uint(d[0]) & vmask) | lid;
        const uint32_t k1 = (__float_as_uint(d[1]) & vmask) | (lid + 1);
        ins(k0);
        if (ta + 2 * (npr - 1) + 1 < t1) ins(k1);
      }
      NV_STAMP(r3);
      NV_ACC(4, r2, r3);
      bool ok = !overflow && Dq < 1e17;
      // exact f64 stage on the K best keys (as in k_knn)
      double ed[K];
      int ei[K];
      if (key[0] != kNoKey) {
        int gpos[K];
#pragma unroll
        for (int s = 0; s < K; ++s) {
          const uint32_t kk = key[s] != kNoKey ? key[s] : key[0];
          const int p = min(max(ta + (int)(kk & kKeyMask), t0), max(t1 - 1, t0));
          gpos[s] = __float_as_int(spair[kWZg + (p >> 1) * 4 + 2 + (p & 1)]);
        }
        // all 2 K gathers in flight before any is used (the scheduler would
        // otherwise sink each pair to its use: a chain of round trips)
        double2 gxy[K], gzi[K];
#pragma unroll
        for (int s = 0; s < K; ++s) {
          bad |= (unsigned)gpos[s] >= (unsigned)ntg;  // (flagged, as the staging clamp above)
          gpos[s] = min(max(gpos[s], 0), max(ntg - 1, 0));
          const PRec *tp = tsort + gpos[s];
          gxy[s] = *(const double2 *)&tp->x;
          gzi[s] = *(const double2 *)&tp->z;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < K; ++s) {
          const bool val = key[s] != kNoKey;
          const double2 xy = gxy[s], zi = gzi[s];
          const double pz = zi.x;
          const int pid = __double2loint(zi.y);
          const double ddx = xy.x - qv[0], ddy = xy.y - qv[1], ddz = pz - qv[2];
          const double dsq = ddx * ddx + ddy * ddy + ddz * ddz;  // utils/kdtree.c:16
          ei[s] = val ? pid : -1;
          ed[s] = val ? __builtin_sqrt(dsq) : INFINITY;
          if (val && !(ed[s] < INFINITY)) {  // an inf/NaN distance is never a neighbour (kdtree.c:117)
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
      // certificate bound on every candidate left out
      double B = INFINITY;
      if (Lr < INFINITY) {
        const double Lg = Lr - 2.0 * G.delta;
        B = Lg > 0.0 ? Lg * Lg : 0.0;
      }
      if (key[K] != kNoKey) {
        const double V = (double)__uint_as_float(key[K] & vmask);
        B = fmin(B, V - f32_err(V, dl));
      }
      bool sorted = true;
#pragma unroll
      for (int s = 1; s < K; ++s) sorted &= !knn_less_bf(ed[s], ei[s], ed[s - 1], ei[s - 1]);
      for (int pass = 0; pass < K - 1 && __any(!sorted); ++pass) {
#pragma unroll
        for (int u = 1; u < K; ++u) knn_cx(ed[u - 1], ei[u - 1], ed[u], ei[u]);
        sorted = true;
#pragma unroll
        for (int s = 1; s < K; ++s) sorted &= !knn_less_bf(ed[s], ei[s], ed[s - 1], ei[s - 1]);
      }
      const double dk = ed[K - 1];
      const double dk2 = dk * dk;
      if (dk < INFINITY)
        ok = ok && B > dk2 * (1.0 + 0x1p-46);
      else
        ok = ok && B == INFINITY;
      if (ok) {
        const size_t q = (size_t)Q.idx;
        if (K % 4 == 0 && L_.vec_out) {
#pragma unroll
          for (int s = 0; s < K; s += 4)
            *(int4 *)(oidx + q * K + s) = make_int4(ei[s], ei[s + 1], ei[s + 2], ei[s + 3]);
#pragma unroll
          for (int s = 0; s < K; s += 2)
            *(double2 *)(odist + q * K + s) = make_double2(ed[s], ed[s + 1]);
        } else {
#pragma unroll
          for (int s = 0; s < K; ++s) {
            oidx[q * K + s] = ei[s];
            odist[q * K + s] = ed[s];
          }
        }
      } else {
        push_slow(L_, qi, (dk < INFINITY && !overflow) ? dk2 * (1.0 + 0x1p-46) : INFINITY);
      }
      NV_STAMP(r4);
      NV_ACC(5, r3, r4);
    }
    NV_STAMP(r5);
    NV_ACC(6, r2, r5);
    la = lb;
    wave_sync_mem();  // LDS is restaged by the next round
  }
  if (__any(bad) && lane == 0) atomicOr(L_.err, 1);
  NV_STAMP(w9);
  NV_ACC(8, w0, w9);
  NV_WFLUSH(chunk);
}
#pragma clang diagnostic pop

// ============================================================ k_knng
// The query pass on the row neighbourhood lists (r5, default): one WAVE per
// chunk of 64 consecutive cell-sorted queries, as k_knnw, but with no column
// tables, no per-segment frames and no per-record shift or shuffle:
//  * a lane's block is [npg(R, x - sx), npg(R, x + sx + 1)) of its row's list
//    GL_R (k_nb_fill): two loads;
//  * the chunk's queries fall in a few grid rows (segments); a segment's
//    image is ONE slice of its row's list, so the round's LDS image is the
//    concatenation of the segments' slices: slot j holds gl[j + delta], delta
//    per segment; every position and record load of the round is in flight
//    at once (kGU batches), then each record is written to its slot with its
//    cell-sorted position (the exact stage reads the K best positions there);
//  * every record is an f32 offset from ONE frame, the grid centre c (SRec,
//    k_bin_fine), so staging copies it as it is; each coordinate difference
//    is still within dl = Dq 2^-21 of the exact one with Dq >= |t - c|,
//    |q - c| (G.Dt), only Dq is larger than a segment frame's.
// The scan, exact stage and certificate are k_knnw's.
// Indices are checked where they are clamped: a position outside the list or
// the cloud sets the call's error flag (navgpu_knn_check returns
// NAVGPU_EINTERNAL).
#ifndef NAVGPU_KNNG_REC
#define NAVGPU_KNNG_REC 800
#endif
#ifndef NAVGPU_KNNG_MINW
#define NAVGPU_KNNG_MINW 3
#endif
// 3 waves per SIMD: 4 (<= 128 VGPRs) spills, and more waves only lengthen
// every wave's memory round trips (r5 timeline)
constexpr int kGRec = NAVGPU_KNNG_REC;          // staged records per round (16 B each)
constexpr int kGPairs = kGRec / 2 + 2;          // two spare pairs: read-ahead
constexpr int kGZg = 4 * kGPairs;               // floats from the XY plane to the ZG plane
constexpr int kGU = (kGRec + kWave - 1) / kWave;  // staging batches of a full round

#ifdef NAVGPU_STAMPS
// k_knng's per-chunk timeline (stamps builds only): [0] start, [1] end
// (s_memrealtime, 100 MHz, one clock for the chip), [2] HW_ID, [3] XCC_ID,
// [4] staging, [5] scan, [6] exact stage (s_memtime cycles), [7] rounds
constexpr int kGStampChunks = 1 << 15;
__device__ unsigned long long g_gstamps[kGStampChunks][8];
#define NV_GT(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define NV_GADD(i, a, b) gst[i] += (b) - (a)
#else
#define NV_GT(v)
#define NV_GADD(i, a, b)
#endif

// Timing-only ablations (-DNAVGPU_ABL=bits, scripts/build_variants.sh; never
// the product build, the results are wrong): 1 the exact stage's record
// gathers, 8 the staged records read from a 1024-record window (L2-resident,
// same request count); 4 no result stores.
#ifndef NAVGPU_ABL
#define NAVGPU_ABL 0
#endif
constexpr int kAbl = NAVGPU_ABL;
// non-temporal hints on the accesses nobody re-reads (r5 A/B knobs): the
// random query-point lines and the result stores, so that they do not evict
// the neighbourhood's records from the XCD's L2
#ifndef NAVGPU_KNNG_NT_Q
#define NAVGPU_KNNG_NT_Q 0
#endif
#ifndef NAVGPU_KNNG_NT_OUT
#define NAVGPU_KNNG_NT_OUT 1  // (r5 bench A/B: 0.2544 against 0.2589 ms; NT_Q lost)
#endif
constexpr bool kNtQ = NAVGPU_KNNG_NT_Q, kNtOut = NAVGPU_KNNG_NT_OUT;
typedef double d2v __attribute__((ext_vector_type(2)));
typedef int i4v __attribute__((ext_vector_type(4)));

// The tail of one lane's query in k_knng: the exact f64 stage on
// the K best keys (their cell-sorted positions from posf(slot)), the
// certificate that no candidate left out (outside the block, or past the
// (K+1)-th key) can rank among the K, and the result: into the LDS rows of a
// chunk done in one round (tstore), else straight to the outputs; an
// uncertified query goes to k_knn_slow with its K-th dsq bound.
template <int K, class PosF>
__device__ __forceinline__ void knng_finish(
    const uint32_t *key, int ta, int t0, int t1, bool overflow, double Dq, double dl, double Lr,
    uint32_t vmask, const GridParams &G, const double *qv, int qidx, int qi,
    const PRec *__restrict__ tsort, int ntg, bool tstore, double *rd, int *ri, int *rq, int lane,
    int32_t *__restrict__ oidx, double *__restrict__ odist, const KnnLists &L_, int &bad,
    PosF posf) {
  bool ok = !overflow && Dq < 1e17;
  double ed[K];
  int ei[K];
  // exact f64 stage on the K best keys
  if (key[0] != kNoKey) {
    int gq[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
      const uint32_t kk = key[s] != kNoKey ? key[s] : key[0];
      const int p = min(max(ta + (int)(kk & kKeyMask), t0), max(t1 - 1, t0));
      gq[s] = posf(p);
    }
    // all 2 K gathers in flight before any is used
    double2 gxy[K], gzi[K];
#pragma unroll
    for (int s = 0; s < K; ++s) {
      bad |= (unsigned)gq[s] >= (unsigned)ntg;
      const PRec *tp = tsort + min(max((kAbl & 1) ? (gq[s] & 1023) : gq[s], 0), max(ntg - 1, 0));
      gxy[s] = *(const double2 *)&tp->x;
      gzi[s] = *(const double2 *)&tp->z;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < K; ++s) {
      const bool val = key[s] != kNoKey;
      const double2 xy = gxy[s], zi = gzi[s];
      const double pz = zi.x;
      const int pid = __double2loint(zi.y);
      const double ddx = xy.x - qv[0], ddy = xy.y - qv[1], ddz = pz - qv[2];
      const double dsq = ddx * ddx + ddy * ddy + ddz * ddz;  // utils/kdtree.c:16
      ei[s] = val ? pid : -1;
      ed[s] = val ? __builtin_sqrt(dsq) : INFINITY;
      if (val && !(ed[s] < INFINITY)) {  // an inf/NaN distance is never a neighbour (kdtree.c:117)
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
  // certificate bound on every candidate left out
  double B = INFINITY;
  if (Lr < INFINITY) {
    const double Lg = Lr - 2.0 * G.delta;
    B = Lg > 0.0 ? Lg * Lg : 0.0;
  }
  if (key[K] != kNoKey) {
    const double V = (double)__uint_as_float(key[K] & vmask);
    B = fmin(B, V - f32_err(V, dl));
  }
  bool sorted = true;
#pragma unroll
  for (int s = 1; s < K; ++s) sorted &= !knn_less_bf(ed[s], ei[s], ed[s - 1], ei[s - 1]);
  for (int pass = 0; pass < K - 1 && __any(!sorted); ++pass) {
#pragma unroll
    for (int u = 1; u < K; ++u) knn_cx(ed[u - 1], ei[u - 1], ed[u], ei[u]);
    sorted = true;
#pragma unroll
    for (int s = 1; s < K; ++s) sorted &= !knn_less_bf(ed[s], ei[s], ed[s - 1], ei[s - 1]);
  }
  const double dk = ed[K - 1];
  const double dk2 = dk * dk;
  if (dk < INFINITY)
    ok = ok && B > dk2 * (1.0 + 0x1p-46);
  else
    ok = ok && B == INFINITY;
  if (tstore) rq[lane] = ok ? qidx : -1;
  if (ok && tstore) {
#pragma unroll
    for (int s = 0; s < K; s += 2)
      *(double2 *)(rd + lane * 8 + s) = make_double2(ed[s], ed[s + 1]);
#pragma unroll
    for (int s = 0; s < K; s += 4)
      *(int4 *)(ri + lane * 8 + s) = make_int4(ei[s], ei[s + 1], ei[s + 2], ei[s + 3]);
  } else if (ok && (!(kAbl & 4) || ed[0] == -1.0)) {
    const size_t q = (size_t)qidx;
    if (K % 4 == 0 && L_.vec_out) {
#pragma unroll
      for (int s = 0; s < K; s += 4)
        *(int4 *)(oidx + q * K + s) = make_int4(ei[s], ei[s + 1], ei[s + 2], ei[s + 3]);
#pragma unroll
      for (int s = 0; s < K; s += 2)
        *(double2 *)(odist + q * K + s) = make_double2(ed[s], ed[s + 1]);
    } else {
#pragma unroll
      for (int s = 0; s < K; ++s) {
        oidx[q * K + s] = ei[s];
        odist[q * K + s] = ed[s];
      }
    }
  } else if (!ok) {
    push_slow(L_, qi, (dk < INFINITY && !overflow) ? dk2 * (1.0 + 0x1p-46) : INFINITY);
  }
}

// A chunk done in one round writes its results as whole rows (k = 8): lane l
// left its 8 distances at rd + 8 l, its indices at ri + 8 l and its query in
// rq[l] (-1: no row; lanes outside the round are marked here, after every
// lane's reads of the image, which the rows overlap). Instruction i then
// writes 16-B piece l & 3 of query 16 i + l / 4's distance row and piece
// l & 1 of query 32 i + l / 2's index row.
__device__ __forceinline__ void knng_store_rows(const double *rd, const int *ri, int *rq,
                                                bool active, int lane, int32_t *__restrict__ oidx,
                                                double *__restrict__ odist) {
  if (!active) rq[lane] = -1;
  wave_sync_mem();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qa = 16 * i + (lane >> 2), pc = lane & 3;
    const int q = rq[qa];
    const double2 v = *(const double2 *)(rd + qa * 8 + 2 * pc);
    if (q >= 0) {
      double2 *o = (double2 *)(odist + (size_t)q * 8 + 2 * pc);
      if (kNtOut)
        __builtin_nontemporal_store(d2v{v.x, v.y}, (d2v *)o);
      else
        *o = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int qa = 32 * i + (lane >> 1), pc = lane & 1;
    const int q = rq[qa];
    const int4 v = *(const int4 *)(ri + qa * 8 + 4 * pc);
    if (q >= 0) {
      int4 *o = (int4 *)(oidx + (size_t)q * 8 + 4 * pc);
      if (kNtOut)
        __builtin_nontemporal_store(i4v{v.x, v.y, v.z, v.w}, (i4v *)o);
      else
        *o = v;
    }
  }
}

template <int K>
__global__ __launch_bounds__(kWave, NAVGPU_KNNG_MINW) void k_knng(
    const GridParams *__restrict__ gp, const int *__restrict__ npg, const int *__restrict__ gl,
    int ngl, const PRec *__restrict__ tsort, const F3 *__restrict__ frec, int fstride,
    const QSide QS,
    int nq, int ntg, int32_t *__restrict__ oidx, double *__restrict__ odist, KnnLists L_) {
  // the round's image: an XY plane (x0 x1 y0 y1 per pair of slots) and a ZG
  // plane (z0 z1 g0 g1, g = the cell-sorted position)
  __shared__ __attribute__((aligned(16))) float spair[2 * kGZg];
  constexpr int KL = K + 1;
  static_assert(K >= 1 && K <= 16, "K");
  const GridParams G = *gp;
  const int S = G.sx, g0 = G.g[0], g1 = G.g[1];
  // chunks dealt to the 8 XCDs in contiguous pools (block b -> XCD b % 8):
  // one chunk per wave, the pool's chunk b / 8. (Persistent waves were
  // measured in r5 and lost, with the next chunk's cells and block bounds
  // loaded during this one's scan: drawing chunks from per-pool ticket
  // counters 269 us, since each atomic serialises at the memory side and its
  // return stays in the wave's vmcnt, so every later wait also waits for it;
  // a static round robin 188 us, its uneven per-wave totals leaving a 76 us
  // tail; against 144 us for one chunk per wave.)
  const int nchunk = (nq + kWave - 1) / kWave;
  const int per = (nchunk + 7) / 8;
  const int pool = (int)(blockIdx.x & 7);
  const int pend = min(nchunk, (pool + 1) * per);  // the pool's end
  const int chunk = pool * per + (int)(blockIdx.x >> 3);
  if (chunk >= pend) return;
  const int lane = (int)threadIdx.x;
  const uint32_t vmask = ~kKeyMask;
  int bad = 0;  // an index that had to be clamped (a logic error)
  // a chunk's per-lane inputs: the query's cell and index (cell-sorted),
  // its block bounds in the row's list (k_nb_fill), its f64 point from the
  // caller's cloud (issued after the bounds: only the scan needs it).
  // (Carrying the points through the build instead, so that a chunk reads 64
  // consecutive records, was measured in r5: the pass's raw FETCH 165 ->
  // 105 MB and its time -3 us, the build +16-20 us. So were 2 or 3
  // consecutive chunks per wave, the next chunk's cells and bounds loaded
  // during this one: 140 -> 155 and 161 us, the extra registers spilling.)
  const int qc = min(chunk * kWave + lane, nq - 1);
  const int qcell = QS.cell[qc], qidx = QS.idx[qc];
  int ga, gb;
  {
    const bool lv = chunk * kWave + lane < nq;
    const int row = lv ? qcell / g0 : 0;
    const int x = lv ? qcell - row * g0 : 0;
    ga = npg[row * (g0 + 1) + max(x - S, 0)];
    gb = npg[row * (g0 + 1) + min(x + S + 1, g0)];
  }
  const double *qp = QS.pts + 3 * (size_t)qidx;
  const double qv[3] = {kNtQ ? __builtin_nontemporal_load(qp) : qp[0],
                        kNtQ ? __builtin_nontemporal_load(qp + 1) : qp[1],
                        kNtQ ? __builtin_nontemporal_load(qp + 2) : qp[2]};
#ifdef NAVGPU_STAMPS
  unsigned long long gst[8] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0, 0, 0};
#endif
  const int nlive = min(kWave, nq - chunk * kWave);
  const int qi = chunk * kWave + lane;
  const bool live = lane < nlive;
  // the query's cell: x, row = (z g1 + y); rows ascend over the lanes.
  // (Cell-sorted query records written by k_bin_fine were measured in r5:
  // the query pass 142 -> 138 us, the build's gather of the points 115 ->
  // 147 us.)
  const int qrow = live ? qcell / g0 : 0x7fffffff;
  const int qx = live ? qcell - qrow * g0 : 0;
  const int prow = __shfl_up(qrow, 1, kWave), nrow = __shfl_down(qrow, 1, kWave);
  const unsigned long long rowfirst = __ballot(live && (lane == 0 || prow != qrow));
  const unsigned long long rowlast = __ballot(live && (lane == nlive - 1 || nrow != qrow));
  for (int la = 0; la < nlive;) {
    // ---- segments of lanes [la, nlive): a grid row each (the first one may
    // start mid-row after a cut round)
    const bool in = lane >= la && live;
    const unsigned long long fall = (rowfirst & (~0ull << la)) | (1ull << la);
    const unsigned long long below = (2ull << lane) - 1;  // lanes <= lane (lane 63: all)
    const int sf = 63 - __builtin_clzll((fall & below) | 1ull);  // the lane's segment: first lane
    const int sl = (int)__builtin_ctzll((rowlast & ~(below >> 1)) | (1ull << 63));  // ... last
    const bool first = in && sf == lane, last = in && sl == lane;
    const int A = __shfl(ga, sf, kWave);       // the segment's first list position
    const int val = last ? gb - A : 0;         // a segment's slots, at its last lane
    const int incv = wave_scan_add(val);
    const int pre = in ? incv - val : 0;       // slots of the earlier segments
    const int cum = pre + (gb - A);            // slots if the round ended at this lane
    // the round: the lane prefix whose image fits (cum ascends over the lanes)
    const int lb = la + __popcll(__ballot(in && cum <= kGRec));
    if (lb == la) {
      // lane la's block alone exceeds the budget: it and every lane of its
      // cell (the same block) go to k_knn_slow from an infinite bound
      const bool same = in && qcell == rdlane(qcell, la);
      if (same) {
        push_slow(L_, qi, INFINITY);
        atomicAdd(L_.n_unstaged, 1);
      }
      la += __popcll(__ballot(same));
      continue;
    }
    const int total = rdlane(cum, lb - 1);
    NV_GT(ts0);
    if (total > 0) {
      // ---- staging: slot j of the round holds gl[j + delta(segment of j)]
      const unsigned long long fb = __ballot(first && lane < lb);
      int dl_[kGU];
      {
        const int f0 = (int)__builtin_ctzll(fb);
        const int d0 = rdlane(A - pre, f0);
#pragma unroll
        for (int u = 0; u < kGU; ++u) dl_[u] = d0;
        for (unsigned long long b = fb & (fb - 1); b; b &= b - 1) {
          const int f = (int)__builtin_ctzll(b);
          const int pf = rdlane(pre, f), df = rdlane(A - pre, f);
#pragma unroll
          for (int u = 0; u < kGU; ++u) dl_[u] = u * kWave + lane >= pf ? df : dl_[u];
        }
      }
      // every load of the round issued unconditionally from a clamped index
      // (a per-element condition makes hipcc branch around each load and wait
      // for it); slots past the image discard theirs, a clamp inside it is
      // an error (flagged)
      int gpos[kGU];
#pragma unroll
      for (int u = 0; u < kGU; ++u) {
        const int j = u * kWave + lane;
        const int gi = min(j, total - 1) + dl_[u];
        bad |= (unsigned)gi >= (unsigned)ngl;
        gpos[u] = gl[min(max(gi, 0), ngl - 1)];
      }
      F3 rec[kGU];  // (12 of the record's 16 B: one dwordx3 each)
#pragma unroll
      for (int u = 0; u < kGU; ++u) {
        bad |= (unsigned)gpos[u] >= (unsigned)ntg;
        rec[u] = *(const F3 *)((const float *)frec +
                               (size_t)fstride *
                                   min(max((kAbl & 8) ? (gpos[u] & 1023) : gpos[u], 0), ntg - 1));
      }
#pragma unroll
      for (int u = 0; u < kGU; ++u) {
        const int j = u * kWave + lane;
        if (j < total) {
          float *d = spair + (j >> 1) * 4 + (j & 1);
          d[0] = rec[u].x;
          d[2] = rec[u].y;
          d[kGZg] = rec[u].z;
          d[kGZg + 2] = __int_as_float(gpos[u]);
        }
      }
    }
    wave_sync_mem();
    NV_GT(ts1);
    NV_GADD(4, ts0, ts1);
#ifdef NAVGPU_STAMPS
    gst[7] += 1;
#endif
    // ---- the round's queries, one per lane (k_knnw's scan, exact stage and
    // certificate on the lane's block [t0, t1))
    // a chunk done in one round, k = 8: its results leave through LDS, so
    // that every store instruction writes whole 64-B (distances) and 32-B
    // (indices) rows of 16 and 32 queries instead of 64 scattered 16-B
    // pieces (r5 ablation: the direct stores cost ~18 us of the pass)
    const bool tstore = K == 8 && L_.vec_out && la == 0 && lb == nlive && !(kAbl & 4);
    // its LDS rows (over the dead image, each lane after its own reads of it):
    // lane l's distances at 8 l doubles, indices after them, then its query
    double *rd = (double *)spair;
    int *ri = (int *)(rd + kWave * 8);
    int *rq = ri + kWave * 8;
    if (in && lane < lb) {
      const int c[3] = {qx, qrow % g1, qrow / g1};
      const int t0 = pre + (ga - A), t1 = pre + (gb - A);
      const double qr[3] = {qv[0] - G.c[0], qv[1] - G.c[1], qv[2] - G.c[2]};
      const double Dq = fmax(G.Dt, fmax(fabs(qr[0]), fmax(fabs(qr[1]), fabs(qr[2]))));
      // each f32 difference is within dl of the exact one: the staged target
      // offset and the query's carry <= u Dq each (u = 2^-24, plus the f64
      // subtraction's 2^-53), the f32 subtraction <= 2 u Dq
      const double dl = Dq * 0x1p-21;
      const f2 qx2 = {(float)qr[0], (float)qr[0]}, qy2 = {(float)qr[1], (float)qr[1]},
               qz2 = {(float)qr[2], (float)qr[2]};
      const double Lr = block_reach(G, qv, c, 1);
      uint32_t key[KL];
#pragma unroll
      for (int s = 0; s < KL; ++s) key[s] = kNoKey;
      auto ins = [&](uint32_t kk) {  // keep the K+1 smallest keys sorted
#pragma unroll
        for (int s = K; s > 0; --s) key[s] = umed3(key[s - 1], key[s], kk);
        key[0] = min(key[0], kk);
      };
      auto dist2 = [&](const float *p) {  // packed f32 squared distances of a pair
        const float4 xy = *(const float4 *)p;
        const float2 zz = *(const float2 *)(p + kGZg);
        const f2 fx2 = f2{xy.x, xy.y} - qx2, fy2 = f2{xy.z, xy.w} - qy2,
                 fz2 = f2{zz.x, zz.y} - qz2;
        return __builtin_elementwise_fma(fz2, fz2, __builtin_elementwise_fma(fy2, fy2, fx2 * fx2));
      };
      const int ta = t0 & ~1;
      const int npr = (t1 - ta + 1) >> 1;  // pairs the block touches
      const bool overflow = (t1 - ta) > (1 << kKeyBits);
      const float *cur = spair + (ta >> 1) * 4;
      if (npr > 0) {  // first pair: may start before the block (odd t0) or end past it
        const f2 d = dist2(cur);
        const uint32_t k0 = knn_key(d[0], vmask, 0u), k1 = knn_key(d[1], vmask, 1u);
        if (ta >= t0) ins(k0);
        if (ta + 1 < t1) ins(k1);
        cur += 4;
      }
      if (npr > 2) {  // interior pairs: the key's local id is the wave-uniform pair counter
        const float *lastp = spair + ((ta >> 1) + npr - 1) * 4;
        uint32_t v2 = 2;
        float4 xy = *(const float4 *)cur;
        float2 zz = *(const float2 *)(cur + kGZg);
        do {
          const float4 nxy = *(const float4 *)(cur + 4);
          const float2 nzz = *(const float2 *)(cur + 4 + kGZg);
          const f2 fx2 = f2{xy.x, xy.y} - qx2, fy2 = f2{xy.z, xy.w} - qy2,
                   fz2 = f2{zz.x, zz.y} - qz2;
          const f2 d =
              __builtin_elementwise_fma(fz2, fz2, __builtin_elementwise_fma(fy2, fy2, fx2 * fx2));
          ins(knn_key(d[0], vmask, v2));
          ins(knn_key(d[1], vmask, v2 + 1));
          cur += 4;
          v2 += 2;
          xy = nxy;
          zz = nzz;
        } while (cur < lastp);
      }
      if (npr > 1) {  // last pair: may end past the block
        const f2 d = dist2(cur);
        const uint32_t lid = (uint32_t)(2 * (npr - 1)) & kKeyMask;
        const uint32_t k0 = (__float_as_uint(d[0]) & vmask) | lid;
        const uint32_t k1 = (__float_as_uint(d[1]) & vmask) | (lid + 1);
        ins(k0);
        if (ta + 2 * (npr - 1) + 1 < t1) ins(k1);
      }
      NV_GT(ts2);
      NV_GADD(5, ts1, ts2);
      knng_finish<K>(key, ta, t0, t1, overflow, Dq, dl, Lr, vmask, G, qv, qidx, qi, tsort, ntg,
                     tstore, rd, ri, rq, lane, oidx, odist, L_, bad, [&](int p) {
                       return __float_as_int(spair[kGZg + (p >> 1) * 4 + 2 + (p & 1)]);
                     });
      NV_GT(ts3);
      NV_GADD(6, ts2, ts3);
    }
    if (tstore) knng_store_rows(rd, ri, rq, in && lane < lb, lane, oidx, odist);
    la = lb;
    wave_sync_mem();  // LDS is restaged by the next round
  }
#ifdef NAVGPU_STAMPS
  gst[1] = __builtin_amdgcn_s_memrealtime();
  gst[2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
  gst[3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
  // the scan and exact-stage times: the wave's (the max over its lanes)
#pragma unroll
  for (int i = 5; i < 7; ++i) {
    unsigned long long v = gst[i];
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long w = (unsigned long long)__shfl_xor((long long)v, o, kWave);
      v = v > w ? v : w;
    }
    gst[i] = v;
  }
  if (lane == 0 && chunk < kGStampChunks)
#pragma unroll
    for (int i = 0; i < 8; ++i) g_gstamps[chunk][i] = gst[i];
#endif
  if (__any(bad) && lane == 0) atomicOr(L_.err, 1);
}

// ============================================================ k_knn_slow
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
      const bool take = knn_less(od, oi, bd, bi) || (!knn_less(bd, bi, od, oi) && ol < bl);
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

// the reference f64 distance of record t; inserted into the lane's sorted
// list when its dsq is within thr
template <int K>
__device__ __forceinline__ void knn_visit(const PRec &tp, const double qv[3], double thr,
                                          double *kd, int *ki) {
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
// 64 lanes. Each lane keeps a sorted list (reference f64 distance); one wave
// merge gives the answer. An infinite bound, or a cube beyond kSlowMaxR,
// takes the ring search: rings of cells split over the lanes, merged after
// every ring, the merged K-th bounding the next ring.
template <int K>
__global__ __launch_bounds__(256) void k_knn_slow(const GridParams *__restrict__ gp,
                                                  const int *__restrict__ start,
                                                  const PRec *__restrict__ tsort,
                                                  const QSide QS,
                                                  int32_t *__restrict__ oidx,
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
    const BinPt Q = qload(QS, L_.slow_q[e]);
    const size_t q = (size_t)Q.idx;
    double thr = L_.slow_thr[e];
    const double qv[3] = {Q.x, Q.y, Q.z};
    const int c[3] = {cell_axis(qv[0], G, 0), cell_axis(qv[1], G, 1), cell_axis(qv[2], G, 2)};
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
        if (j < total) knn_visit<K>(tsort[pb + (j - pp)], qv, thr, kd, ki);
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
        }
        if (lane >= tot && lane < K) {  // fewer than K survivors: empty slots
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
        for (int t = b; t < en; ++t) knn_visit<K>(tsort[t], qv, thr, kd, ki);
      }
      knn_wave_merge<K>(kd, ki, md, mi, lane);
      // lane 0 carries the merged list into the next ring
#pragma unroll
      for (int s = 0; s < K; ++s) {
        kd[s] = lane == 0 ? md[s] : INFINITY;
        ki[s] = lane == 0 ? mi[s] : -1;
      }
      if (md[K - 1] < INFINITY) thr = fmin(thr, md[K - 1] * md[K - 1] * (1.0 + 0x1p-46));
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

// counters of the last call: [n_unstaged, n_slow, err, pad]
long long read_counter(navgpu_ctx *ctx, int which) {
  if (!ctx) return -1;
  auto it = ctx->bufs.find(kStats);
  if (it == ctx->bufs.end() || !it->second.first) return -1;
  int v[4] = {0, 0, 0, 0};
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return -1;
  if (hipMemcpy(v, it->second.first, 16, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (long long)v[which];
}

}  // namespace

// ============================================================ host
namespace nv {
int knn_stamps_take(unsigned long long *out16) {
#ifdef NAVGPU_STAMPS
  HIP_TRY(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_stamps), 16 * 8));
  unsigned long long z[16] = {0};
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, 16 * 8));
  // k_knnw's per-chunk records, summed into slots 1..8 (zeroed after)
  std::vector<unsigned long long> w((size_t)kWStampChunks * 8);
  HIP_TRY(hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(g_wstamps), w.size() * 8));
  for (size_t i = 0; i < w.size(); ++i) out16[1 + i % 8] += w[i];
  std::fill(w.begin(), w.end(), 0ull);
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_wstamps), w.data(), w.size() * 8));
  return NAVGPU_OK;
#else
  (void)out16;
  return NAVGPU_EINVAL;
#endif
}
}  // namespace nv

// The k-NN call (navgpu_knn_dev): index build, query pass, slow pass; all on
// the context's stream, nothing allocated once the workspace is warm.
static int knn_run(navgpu_ctx *ctx, const double *tgt, size_t nt, const double *queries,
                   size_t nq, int k, int32_t *idx, double *dist) {
  ARG_CHECK(ctx && k >= 1 && k <= 16);
  ARG_CHECK(nt < (size_t)INT32_MAX / 2 && nq < (size_t)INT32_MAX / 2);
  if (!nq) {
    // an empty call is clean: its counters (navgpu_knn_check reads the
    // error flag of the LAST call) are zeroed, not left from the previous one
    int *counters;
    RC(ws(ctx, kStats, 16, &counters));
    HIP_TRY(hipMemsetAsync(counters, 0, 16 * sizeof(int), ctx->stream));
    return NAVGPU_OK;
  }
  ARG_CHECK(queries && idx && dist && (tgt || nt == 0));
  const double occ = ctx->knn_occ;
  const int sx = ctx->knn_sx;
  const long long capl = (long long)((double)nt / occ) * 2 * sx + 1024;
  ARG_CHECK(capl < INT32_MAX / 2);
  const int cap = (int)capl;
  const int nscan = cap + 1;  // start[] has one entry past the last cell
  // binning geometry (k_bin_*): coarse buckets of 2^shift cells, at most
  // kBinMaxBuckets of them, at least one cell per fine-pass thread
  int shift = kBinMinShift;
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
    S.P = (int)std::max<size_t>(kBinP, (ns[side] / 2000 + 256) / 256 * 256);
    S.nblk = (int)std::max<size_t>(1, (ns[side] + S.P - 1) / S.P);
    S.tab = (int)ntab;
    ntab += (long long)J.nb * S.nblk;
  }
  if (ntab >= INT32_MAX) {
    set_err("knn: binning table of %lld entries exceeds the int range", ntab);
    return NAVGPU_ERANGE;
  }
  const int nparts = (int)std::min<size_t>(kBBoxBlocks, std::max<size_t>(1, grid1d(nt, 256)));
  double *part;
  GridParams *gp;
  int *tab, *tstart, *bbase, *counters;
  BinPt *tbin = nullptr;
  QKey *qkey;
  int *qcell;
  PRec *tsort = nullptr;
  SRec *srec = nullptr;
  int *qperm;
  RC(ws(ctx, kBBox, (size_t)kBBoxBlocks * 6, &part));
  RC(ws(ctx, kParams, 1, &gp));
  RC(ws(ctx, kCnt, (size_t)ntab, &tab));
  RC(ws(ctx, kStart, nscan, &tstart));
  int *btot;
  RC(ws(ctx, kBSum, 2 * (size_t)J.nb, &btot));
  RC(ws(ctx, kCellId, 2 * ((size_t)J.nb + 1), &bbase));
  RC(ws(ctx, kStats, 16, &counters));  // zeroed by k_bin_hist
  if (nt) RC(ws(ctx, kSlotBuf, nt, &tbin));
  // at least one record each: k_knnw loads from clamped positions unconditionally
  RC(ws(ctx, kTSort, std::max<size_t>(nt, 1), &tsort));
  RC(ws(ctx, kSRec, std::max<size_t>(nt, 1), &srec));
  RC(ws(ctx, kQCell, nq, &qkey));
  RC(ws(ctx, kQPerm, nq, &qperm));
  RC(ws(ctx, kQSort, nq, &qcell));
  int *qraw;
  RC(ws(ctx, kQSlot, nq, &qraw));
  // k_knng's row neighbourhood lists: 9 positions per target, and g0 + 1
  // column starts per grid row (rows * (g0 + 1) <= 2 ncells <= 2 cap). A
  // target cloud whose lists would pass the int32 range (> ~238M points)
  // takes k_knnw (mode 1), which has no lists.
  int *npg = nullptr, *gl = nullptr;
  const long long ngl = std::max<long long>(9LL * (long long)nt, 1);
  const int mode = (ctx->knn_mode == 2 && ngl >= INT32_MAX) ? 1 : ctx->knn_mode;
  const bool lists = mode == 2;  // k_knng stages from the row lists
  if (lists) {
    RC(ws(ctx, kNpg, 2 * (size_t)cap + 2, &npg));
    RC(ws(ctx, kGl, (size_t)ngl, &gl));
  }
  J.sglobal = lists;
  J.s[0].p = tgt;
  J.s[1].p = queries;
  J.s[0].start = tstart;
  J.s[1].start = nullptr;  // the query passes read no query cell starts
  J.s[0].bin = tbin;
  J.s[1].bin = nullptr;
  J.s[0].key = nullptr;
  J.s[1].key = qkey;
  J.s[0].qcell = nullptr;
  J.s[1].qcell = qcell;
  J.s[0].rawcell = nullptr;
  J.s[1].rawcell = qraw;
  J.s[0].sorted = tsort;
  // k_knng reads 12-B F3 records (kKnngPack) in the same buffer, k_knnw the SRec
  const bool pack = mode == 2 && kKnngPack;
  J.s[0].srec = pack ? nullptr : srec;
  J.s[0].frec = pack ? (F3 *)srec : nullptr;
  J.s[1].srec = nullptr;
  J.s[1].frec = nullptr;
  J.s[1].sorted = nullptr;
  J.s[0].perm = nullptr;
  J.s[1].perm = qperm;
  hipStream_t s = ctx->stream;
  {
    TimedRegion tb(ctx, "knn_build");
    if (nt) {
      hipLaunchKernelGGL(k_bbox_partial, dim3(nparts), dim3(kBBoxThreads), 0, s, tgt, nt, part);
      CHECK_LAUNCH("k_bbox_partial");
    }
    GridArgs A;
    A.part = part;
    A.nparts = nt ? nparts : 0;
    A.cap = cap;
    A.sx = sx;
    A.occ = occ;
    A.n = nt;
    A.nq = nq;
    const dim3 gb(J.s[0].nblk + J.s[1].nblk);
    hipLaunchKernelGGL(k_bin_hist, gb, dim3(kBinThreads), 4 * (size_t)J.nb, s, J, A, gp, counters, tab);
    CHECK_LAUNCH("k_bin_hist");
    const dim3 gc(2 * ((J.nb + kColB - 1) / kColB));
    hipLaunchKernelGGL(k_bin_colscan, gc, dim3(kColB * kColY), 0, s, tab, J.nb, J.s[0].tab,
                       J.s[0].nblk, J.s[1].tab, J.s[1].nblk, btot);
    CHECK_LAUNCH("k_bin_colscan");
    hipLaunchKernelGGL(k_bin_scatter, gb, dim3(kBinThreads), 4 * (size_t)J.nb, s, J, gp, (const int *)tab,
                       (const int *)btot, bbase);
    CHECK_LAUNCH("k_bin_scatter");
    // staged query placement when its LDS fits beside a 2^shift count table
    const bool st_q = fine_lds_bytes(shift, true) <= 144 * 1024;
    const size_t lds = fine_lds_bytes(shift, st_q);
    if (lds > 48 * 1024)
      HIP_TRY(hipFuncSetAttribute((const void *)k_bin_fine,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_bin_fine, dim3(2 * J.nb), dim3(kBinFineThreads), lds, s, J, gp,
                       (const int *)bbase, nscan, st_q ? kFineStage : 0);
    CHECK_LAUNCH("k_bin_fine");
    if (lists) {
      // tasks (64 columns of a row) <= 2 cap / 64 + rows; a few per wave
      // (4096 workgroups, one task per wave: build -2 us, bench flat in r5)
      const unsigned nbl = std::min<unsigned>(1024, std::max<unsigned>(1, grid1d(2 * (size_t)cap, 64 * kNbWaves * 2)));
      hipLaunchKernelGGL(k_nb_fill, dim3(nbl), dim3(kWave * kNbWaves), 0, s, gp,
                         (const int *)tstart, npg, gl);
      CHECK_LAUNCH("k_nb_fill");
    }
  }
  KnnLists klists;
  RC(ws(ctx, kSlowQ, nq, &klists.slow_q));
  RC(ws(ctx, kSlowThr, nq, &klists.slow_thr));
  klists.n_unstaged = counters;
  klists.n_slow = counters + 1;
  klists.err = counters + 2;
  klists.vec_out = ((uintptr_t)idx % 16 == 0 && (uintptr_t)dist % 16 == 0) ? 1 : 0;
  TimedRegion tr(ctx, "knn_query");
  const dim3 gs(std::max<unsigned>(1, std::min<unsigned>(2048, grid1d(nq, 256))));
  // one 64-lane block per chunk of 64 cell-sorted queries, chunks dealt to
  // the XCDs in contiguous ranges (block b -> XCD b % 8, the placement
  // HW_REG_XCC_ID reports)
  const int nchunk = (int)((nq + kWave - 1) / kWave);
  const dim3 gw(8 * (((nchunk + 7) / 8 + kWPB - 1) / kWPB)), bw(kWave * kWPB);
  const QSide QS{queries, qperm, qcell};
  const dim3 gg(8 * (unsigned)((nchunk + 7) / 8));
#define KNN_CASE(KK)                                                                        \
  case KK:                                                                                  \
    if (mode == 2)                                                                          \
      hipLaunchKernelGGL((k_knng<KK>), gg, dim3(kWave), 0, s, gp, (const int *)npg,         \
                         (const int *)gl, (int)ngl, tsort, (const F3 *)srec,                \
                         pack ? 3 : 4, QS, (int)nq, (int)nt, idx,                           \
                         dist, klists);                                                     \
    else                                                                                    \
      hipLaunchKernelGGL((k_knnw<KK>), gw, bw, 0, s, gp, tstart, tsort, srec, QS, (int)nq,      \
                         (int)nt, idx, dist, klists);                                       \
    hipLaunchKernelGGL((k_knn_slow<KK>), gs, dim3(256), 0, s, gp, tstart, tsort, QS,       \
                       idx, dist, klists);                                                  \
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

int navgpu_knn_dev(navgpu_ctx *ctx, const double *tgt, size_t nt, const double *queries,
                   size_t nq, int k, int32_t *idx, double *dist) {
  return knn_run(ctx, tgt, nt, queries, nq, k, idx, dist);
}

int navgpu_knn_host(navgpu_ctx *ctx, const double *tgt, size_t nt, const double *queries,
                    size_t nq, int k, int32_t *idx, double *dist) {
  ARG_CHECK(ctx && k >= 1 && k <= 16);
  if (!nq) return NAVGPU_OK;
  ARG_CHECK(queries && idx && dist && (tgt || nt == 0));
  double *dt = nullptr, *dq, *dd;
  int32_t *di;
  if (nt) RC(ws(ctx, kH0, 3 * nt, &dt));
  RC(ws(ctx, kH1, 3 * nq, &dq));
  RC(ws(ctx, kH2, nq * k, &di));
  RC(ws(ctx, kH3, nq * k, &dd));
  if (nt) HIP_TRY(hipMemcpyAsync(dt, tgt, 24 * nt, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dq, queries, 24 * nq, hipMemcpyHostToDevice, ctx->stream));
  RC(navgpu_knn_dev(ctx, dt, nt, dq, nq, k, di, dd));
  HIP_TRY(hipMemcpyAsync(idx, di, 4 * nq * k, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dist, dd, 8 * nq * k, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return navgpu_knn_check(ctx);
}

int navgpu_pair_knn_dev(navgpu_ctx *ctx, const double *src, const double *tgt, int R, int C,
                        int k, int32_t *src_mask, int32_t *tgt_mask, int32_t *idx,
                        double *dist) {
  ARG_CHECK(ctx && R >= 0 && C >= 0);
  const size_t N = (size_t)R * C;
  if (!N) return NAVGPU_OK;
  ARG_CHECK(src && tgt);
  if (!src_mask && !tgt_mask) return navgpu_knn_dev(ctx, tgt, N, src, N, k, idx, dist);
  // One curvature launch over both clouds, on a side stream forked from and
  // joined back into the context's stream: it is f64-bound and independent
  // of the (latency-bound) index build and query, so the two overlap.
  // (NAVGPU_PAIR_SIDE=0: on the context's stream, one stream per context.)
  const bool side = ctx->pair_side;
  if (side) {
    RC(ensure_aux(ctx));
    HIP_TRY(hipEventRecord(ctx->ev_fork, ctx->stream));
    HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
  }
  hipStream_t cs = side ? ctx->aux : ctx->stream;
  {
    TimedRegion tr(ctx, "curvature", cs);
    if (src_mask && tgt_mask)
      RC(launch_curvature(src, src_mask, nullptr, tgt, tgt_mask, nullptr, R, C, cs));
    else if (src_mask)
      RC(launch_curvature(src, src_mask, nullptr, nullptr, nullptr, nullptr, R, C, cs));
    else
      RC(launch_curvature(tgt, tgt_mask, nullptr, nullptr, nullptr, nullptr, R, C, cs));
  }
  if (side) HIP_TRY(hipEventRecord(ctx->ev_join, ctx->aux));
  const int rc = knn_run(ctx, tgt, N, src, N, k, idx, dist);
  if (side) HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));  // join before returning
  return rc;
}

long long navgpu_knn_fallbacks(navgpu_ctx *ctx) { return read_counter(ctx, 1); }

long long navgpu_knn_overflows(navgpu_ctx *ctx) { return read_counter(ctx, 0); }

#ifdef NAVGPU_STAMPS
// stamps builds only (not in navgpu.h): k_knng's per-chunk timeline of the
// last call, 8 words per chunk, up to n chunks; returns the chunks copied
int navgpu_debug_knng_timeline(unsigned long long *out, int n) {
  n = std::min(n, kGStampChunks);
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gstamps), (size_t)n * 64) != hipSuccess) return -1;
  return n;
}
#endif

int navgpu_knn_check(navgpu_ctx *ctx) {
  ARG_CHECK(ctx);
  const long long e = read_counter(ctx, 2);
  if (e < 0) {
    nv::set_err("knn_check: could not read the call's counters");
    return NAVGPU_EHIP;
  }
  if (e) {
    nv::set_err("knn: a kernel clamped an out-of-range index (internal error)");
    return NAVGPU_EINTERNAL;
  }
  return NAVGPU_OK;
}

}  // extern "C"
