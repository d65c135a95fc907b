/*
 * oracle_grid.c — full-size checkers and all-cores CPU-baseline drivers.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): tests/ use orc_knn_grid to check
 * every one of the 1,048,576 K3 queries, not a sample; bench.py's
 * cpu_baseline leg uses the *_mt drivers for its all-cores figure. Nothing in
 * the product links this file.
 *
 * orc_knn_grid computes exactly what orc_knn_brute computes -- per query the
 * k targets with the smallest reference distance sqrt((dx*dx+dy*dy)+dz*dz)
 * (utils/kdtree.c:14-17, dx = target - query), ordered by (distance, index),
 * +INFINITY/NaN never a neighbour (utils/kdtree.c:117) -- but visits only
 * the cells of a uniform grid in growing cubic shells around the query and
 * stops once every unvisited cell lies provably farther than the k-th
 * distance found. tests/test_oracle.py pins it against orc_knn_brute.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

static int orc_finite3(const double *p)
{
    return isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]);
}

/* (d, i) before (kd, ki): distance first, then index */
static int orc_knn_less(double d, int i, double kd, int ki)
{
    return d < kd || (d == kd && i < ki);
}

typedef struct {
    double o[3], h, inv_h, eps;
    long g[3];
    long *start; /* ncells + 1 */
    int *ids;    /* finite target indices, cell-sorted */
} orc_grid;

static long orc_cell_axis(const orc_grid *G, double v, int a)
{
    double t = (v - G->o[a]) * G->inv_h;
    if (!(t >= 0.0))
        return 0;
    if (t >= (double)G->g[a])
        return G->g[a] - 1;
    return (long)t;
}

static void orc_grid_build(orc_grid *G, const double *tgt, size_t nt)
{
    double lo[3] = {INFINITY, INFINITY, INFINITY};
    double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    size_t nf = 0;
    for (size_t t = 0; t < nt; t++) {
        const double *p = tgt + 3 * t;
        if (!orc_finite3(p))
            continue;
        nf++;
        for (int a = 0; a < 3; a++) {
            lo[a] = fmin(lo[a], p[a]);
            hi[a] = fmax(hi[a], p[a]);
        }
    }
    double emax = 0.0, vol = 1.0;
    for (int a = 0; a < 3; a++)
        emax = fmax(emax, nf ? hi[a] - lo[a] : 0.0);
    double fl = fmax(emax * 1e-3, 1e-9);
    for (int a = 0; a < 3; a++)
        vol *= fmax(nf ? hi[a] - lo[a] : 0.0, fl);
    /* about 2 targets per cell, at most 4 nt + 64 cells */
    double h = cbrt(vol * 2.0 / (double)(nf ? nf : 1));
    if (!(h > 0) || !isfinite(h))
        h = fmax(emax, 1.0);
    for (;;) {
        double tot = 1.0;
        for (int a = 0; a < 3; a++) {
            G->g[a] = nf ? (long)floor((hi[a] - lo[a]) / h) + 1 : 1;
            tot *= (double)G->g[a];
        }
        if (tot <= 4.0 * (double)nf + 64.0)
            break;
        h *= 1.1;
    }
    for (int a = 0; a < 3; a++)
        G->o[a] = nf ? lo[a] : 0.0;
    G->h = h;
    G->inv_h = 1.0 / h;
    G->eps = 1e-9 * (emax + h); /* slack on cell faces (f64 cell assignment) */
    long nc = G->g[0] * G->g[1] * G->g[2];
    G->start = calloc((size_t)nc + 1, sizeof(long));
    G->ids = malloc((nf ? nf : 1) * sizeof(int));
    long *cell = malloc((nt ? nt : 1) * sizeof(long));
    for (size_t t = 0; t < nt; t++) {
        const double *p = tgt + 3 * t;
        if (!orc_finite3(p)) {
            cell[t] = -1;
            continue;
        }
        cell[t] = (orc_cell_axis(G, p[2], 2) * G->g[1] + orc_cell_axis(G, p[1], 1)) * G->g[0] +
                  orc_cell_axis(G, p[0], 0);
        G->start[cell[t] + 1]++;
    }
    for (long c = 0; c < nc; c++)
        G->start[c + 1] += G->start[c];
    long *fill = malloc((size_t)nc * sizeof(long));
    memcpy(fill, G->start, (size_t)nc * sizeof(long));
    for (size_t t = 0; t < nt; t++)
        if (cell[t] >= 0)
            G->ids[fill[cell[t]]++] = (int)t;
    free(fill);
    free(cell);
}

static void orc_grid_query(const orc_grid *G, const double *tgt, const double *qp, int k,
                           int *bi, double *bd)
{
    for (int s = 0; s < k; s++) {
        bi[s] = -1;
        bd[s] = INFINITY;
    }
    if (!orc_finite3(qp) || G->start[G->g[0] * G->g[1] * G->g[2]] == 0)
        return; /* every distance is inf/NaN, or no finite target */
    long c[3];
    for (int a = 0; a < 3; a++)
        c[a] = orc_cell_axis(G, qp[a], a);
    int have = 0;
    for (long s = 0;; s++) {
        long lo[3], hi[3];
        for (int a = 0; a < 3; a++) {
            lo[a] = c[a] - s < 0 ? 0 : c[a] - s;
            hi[a] = c[a] + s > G->g[a] - 1 ? G->g[a] - 1 : c[a] + s;
        }
        /* the shell: cells of the cube at Chebyshev distance exactly s */
        for (long z = lo[2]; z <= hi[2]; z++)
            for (long y = lo[1]; y <= hi[1]; y++) {
                int ring = labs(z - c[2]) == s || labs(y - c[1]) == s;
                for (long x = lo[0]; x <= hi[0]; x++) {
                    if (!ring && labs(x - c[0]) != s) {
                        x = c[0] + s - 1; /* jump to the far face of this row */
                        continue;
                    }
                    long cell = (z * G->g[1] + y) * G->g[0] + x;
                    for (long e = G->start[cell]; e < G->start[cell + 1]; e++) {
                        int t = G->ids[e];
                        const double *tp = tgt + 3 * (size_t)t;
                        double dx = tp[0] - qp[0], dy = tp[1] - qp[1], dz = tp[2] - qp[2];
                        double d = sqrt(dx * dx + dy * dy + dz * dz); /* kdtree.c:16 */
                        if (!(d < INFINITY))
                            continue;
                        if (have == k && !orc_knn_less(d, t, bd[k - 1], bi[k - 1]))
                            continue;
                        int p = have < k ? have : k - 1;
                        while (p > 0 && orc_knn_less(d, t, bd[p - 1], bi[p - 1])) {
                            bd[p] = bd[p - 1];
                            bi[p] = bi[p - 1];
                            p--;
                        }
                        bd[p] = d;
                        bi[p] = t;
                        if (have < k)
                            have++;
                    }
                }
            }
        /* every point outside the cube is at least L away */
        double L = INFINITY;
        for (int a = 0; a < 3; a++) {
            if (c[a] - s > 0)
                L = fmin(L, qp[a] - (G->o[a] + (double)(c[a] - s) * G->h));
            if (c[a] + s < G->g[a] - 1)
                L = fmin(L, (G->o[a] + (double)(c[a] + s + 1) * G->h) - qp[a]);
        }
        if (L == INFINITY)
            return; /* the cube covers the whole grid */
        if (have == k && bd[k - 1] < (L - G->eps) * (1.0 - 1e-12))
            return;
    }
}

void orc_knn_grid(const double *tgt, size_t nt, const double *qs, size_t nq, int k,
                  int *oi, double *od)
{
    orc_grid G;
    orc_grid_build(&G, tgt, nt);
#pragma omp parallel for schedule(dynamic, 1024)
    for (long q = 0; q < (long)nq; q++)
        orc_grid_query(&G, tgt, qs + 3 * (size_t)q, k, oi + (size_t)q * k, od + (size_t)q * k);
    free(G.start);
    free(G.ids);
}

/* ---- all-cores CPU baseline (SURVEY 8d "(2) all cores") ----------------- */
typedef void (*orc_ref_nn_fn_mt)(void *root, const double *target, double *result,
                                 double *bestDist, int depth);

/* nearestNeighborSearch of a reference-ABI tree for every query, OpenMP over
 * the queries (the search only reads the tree: utils/kdtree.c:110-152). */
void orc_ref_nn_batch_mt(void *fn, void *root, const double *qs, size_t nq, double *out_pts,
                         double *out_dist)
{
    orc_ref_nn_fn_mt f = (orc_ref_nn_fn_mt)fn;
#pragma omp parallel for schedule(dynamic, 4096)
    for (long i = 0; i < (long)nq; i++) {
        double best = INFINITY;
        f(root, qs + 3 * i, out_pts + 3 * i, &best, 0);
        out_dist[i] = best;
    }
}

typedef void *(*orc_ref_build_fn)(void *pts, size_t n, int depth);
typedef void (*orc_ref_free_fn)(void *root);

/* The per-row frame step of src/slam.c:162-172 + 236-244 through the
 * reference's own buildKDTree / nearestNeighborSearch / freeKDTree, given
 * the feature masks: rows in parallel (OpenMP) when threads > 1, one after
 * another otherwise. Returns the number of source features queried. */
long orc_ref_rows_match_mt(void *build, void *nn, void *freef, const double *src,
                           const double *tgt, const int *smask, const int *tmask, int R, int C,
                           int threads, double *out_pts, double *out_dist)
{
    orc_ref_build_fn fb = (orc_ref_build_fn)build;
    orc_ref_nn_fn_mt fq = (orc_ref_nn_fn_mt)nn;
    orc_ref_free_fn ff = (orc_ref_free_fn)freef;
    long total = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total) num_threads(threads)
    for (int r = 0; r < R; r++) {
        double *flat = malloc(sizeof(double) * 3 * (size_t)(C ? C : 1));
        size_t n = 0;
        for (int c = 0; c < C; c++) /* flattenPoints, src/slam.c:64-81 */
            if (tmask[(size_t)r * C + c]) {
                memcpy(flat + 3 * n, tgt + 3 * ((size_t)r * C + c), 24);
                n++;
            }
        void *root = fb(flat, n, 0);
        for (int c = 0; c < C; c++) {
            size_t g = (size_t)r * C + c;
            if (!smask[g])
                continue;
            total++;
            double best = INFINITY;
            if (root)
                fq(root, src + 3 * g, out_pts + 3 * g, &best, 0);
            out_dist[g] = best;
        }
        ff(root);
        free(flat);
    }
    return total;
}

/* extract_feature (orc_extract_feature, src/slam.c:11-61) split over row
 * blocks: the curvature of a point depends only on its own row. */
void orc_extract_feature_mt(const double *pts, int R, int C, int *feature, int threads)
{
#pragma omp parallel for schedule(static) num_threads(threads)
    for (int r = 0; r < R; r++)
        orc_extract_feature(pts + 3 * (size_t)r * C, 1, C, feature + (size_t)r * C, NULL);
}

int orc_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
