/*
 * oracle.h — CPU restatement of the NAV-SLAM scan-matching hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (nav-slam_amd/, include/)
 * links, loads or calls this code. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * Every function restates one reference function statement by statement, in
 * the same floating-point operation order, and is compiled with
 * `-O2 -std=gnu11 -ffp-contract=off` (no FMA contraction, no fast-math), the
 * same arithmetic the reference x86-64 build performs. Parity of this
 * restatement with the reference itself is pinned by tests/test_oracle.py
 * against fixtures generated from the reference sources compiled as-is
 * (oracle/Makefile target `ref`, tests/golden/make_golden.py).
 *
 * Layouts: a cloud is `double[R*C*3]` row-major (x,y,z interleaved), i.e. the
 * reference `Point ToF_position[MAX_ROWS][MAX_COLS]` (utils/pointcloud.h:32-44)
 * with runtime R, C instead of compile-time MAX_ROWS/MAX_COLS.
 */
#ifndef NAVSLAM_ORACLE_H
#define NAVSLAM_ORACLE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* utils/pointcloud.c:8-48 — depth grid (mm) -> xyz (mm). */
void orc_convert_to_pointcloud(const int *dist, int R, int C, double *pts);

/* src/slam.c:11-61 — edge-feature mask (0/1 for every cell; the reference
 * only writes 1s into a caller-zeroed array). `curv` (optional) gets the
 * curvature value, 0 where the reference computes none. */
void orc_extract_feature(const double *pts, int R, int C, int *feature,
                         double *curv);

/* src/slam.c:8,95-115 — R from (roll, pitch, yaw) in degrees, row-major. */
void orc_rotation_matrix_deg(double roll, double pitch, double yaw,
                             double Rm[9]);

/* src/slam.c:145-160 / 193-207 / 402-416 — out = t + R*p per point. */
void orc_transform_cloud(const double *pts, size_t n, const double Rm[9],
                         const double t[3], double *out);

/* src/slam.c:118-131 — out = g - tr per point. */
void orc_map_to_last(const double *g, size_t n, const double tr[3],
                     double *out);

/* src/slam.c:64-81 — stable compaction of a row's feature points; the
 * column of each kept point goes to flat_col. Returns the count. */
size_t orc_flatten_row(const double *row_pts, const int *row_feat, int C,
                       double *flat, int *flat_col);

/* utils/kdtree.c:20-62 — Lomuto quickselect (pivot = last, `cmp <= 0` goes
 * left). idx (optional) is permuted alongside the points. */
void orc_nth_element(double *pts, int *idx, size_t first, size_t last,
                     size_t nth, int axis);

/* utils/kdtree.c:65-82 — median-split build. Permutes pts/idx in place; the
 * result IS the tree: node of range [lo,hi) sits at lo+(hi-lo)/2, its left
 * child is [lo,mid), its right child [mid+1,hi), split axis = depth % 3. */
void orc_kd_build(double *pts, int *idx, size_t n);

/* utils/kdtree.c:14-17,110-152 — exact 1-NN over a tree built by
 * orc_kd_build; first-visited point wins ties. out_pos = tree position of the
 * winner (or -1 for an empty tree, where the reference leaves `result`
 * untouched); out_dist = +INFINITY when empty. */
void orc_kd_nn(const double *tree, size_t n, const double q[3],
               long *out_pos, double *out_dist);

/* The scan-pair composition of SURVEY.md S4 in per-row mode (the slam.c
 * semantics, src/slam.c:162-172 + 236-244): features of src and tgt, one tree
 * per target row over the row's feature points, every src feature point
 * queried against its own row's tree. Outputs per src grid cell:
 *   nn_idx  = linear index r*C+c of the nearest target point, or -1 when the
 *             cell is not a feature or its row tree is empty;
 *   nn_dist = the reference distance, +INFINITY when nn_idx == -1.
 * src_mask/tgt_mask (optional) receive the two feature masks. */
void orc_rows_match(const double *src, const double *tgt, int R, int C,
                    int *src_mask, int *tgt_mask, int *nn_idx,
                    double *nn_dist);

/* k-NN definition for the global mode (the reference implements k = 1 only,
 * utils/kdtree.c:110-152; k > 1 is a restatement): per query, the k target
 * points with the smallest reference distance (utils/kdtree.c:14-17,
 * dx = target_point - query), ordered by (distance, index) ascending, so
 * equal distances resolve to the lowest index. Missing slots get index -1
 * and distance +INFINITY; an infinite/NaN distance is never a neighbour
 * (kdtree.c:117 takes a point only if dist < best, best = INFINITY).
 * Brute force, O(nq * nt). */
void orc_knn_brute(const double *tgt, size_t nt, const double *qs, size_t nq,
                   int k, int *out_idx, double *out_dist);

/* CPU-baseline drivers: orc_kd_nn over nq queries; and a loop calling a
 * reference-ABI nearestNeighborSearch through `fn` (bestDist = INFINITY per
 * query, as src/slam.c:243). */
void orc_kd_nn_batch(const double *tree, size_t n, const double *qs, size_t nq,
                     long *out_pos, double *out_dist);
void orc_ref_nn_batch(void *fn, void *root, const double *qs, size_t nq,
                      double *out_pts, double *out_dist);

/* oracle_grid.c: the same k-NN as orc_knn_brute (identical results, pinned
 * by tests/test_oracle.py) over a uniform grid searched in growing shells,
 * OpenMP over the queries: checks all 1M K3 queries in seconds. */
void orc_knn_grid(const double *tgt, size_t nt, const double *qs, size_t nq,
                  int k, int *out_idx, double *out_dist);

/* oracle_grid.c: all-cores CPU-baseline drivers (OpenMP). The reference's
 * own buildKDTree / nearestNeighborSearch / freeKDTree are passed in as
 * function pointers (oracle/_ref build). */
void orc_ref_nn_batch_mt(void *fn, void *root, const double *qs, size_t nq,
                         double *out_pts, double *out_dist);
long orc_ref_rows_match_mt(void *build, void *nn, void *freef,
                           const double *src, const double *tgt,
                           const int *smask, const int *tmask, int R, int C,
                           int threads, double *out_pts, double *out_dist);
void orc_extract_feature_mt(const double *pts, int R, int C, int *feature,
                            int threads);
int orc_max_threads(void);

/* src/slam.c:236-284: a frame's correspondence list from per-feature 1-NN
 * results over per-row trees (trees: row r's tree at offset r*C; pos[g]: tree
 * position, -1 = no query/empty tree; dist[g]; ori[g]: the query's
 * transformed point). Writes the list in the reference's order: ori, nearest
 * point, distance and the grid index g of each entry's query. Returns the
 * entry count (CPcount). The same code orc_slam_localization runs. */
int orc_rows_dedup(const double *trees, int R, int C, const long *pos,
                   const double *dist, const double *ori, double *out_ori,
                   double *out_near, double *out_dist, long *out_grid);

/* ---- src/slam.c:134-431 frame loop, runtime dims, buffers sized R*C ---- */
typedef struct orc_slam orc_slam;
orc_slam *orc_slam_create(int R, int C);
void orc_slam_destroy(orc_slam *s);
/* src/slam.c:134-175. pos = {x,y,z,roll,pitch,yaw}. */
void orc_slam_init(orc_slam *s, const double pos[6], const double *lidar);
/* src/slam.c:178-390. Returns the number of Adam iterations run in *iters,
 * the correspondence count in *ncorr. */
void orc_slam_localization(orc_slam *s, const double *lidar,
                           const double pred[6], const double last[6],
                           double out[6], int *iters, int *ncorr);
/* src/slam.c:393-431. */
void orc_slam_mapping(orc_slam *s, const double pos[6], const double *lidar);
double orc_slam_error(const orc_slam *s);
int orc_slam_frame_count(const orc_slam *s);
/* Row tree r (permuted points, count) and the last global frame. */
size_t orc_slam_tree(const orc_slam *s, int r, const double **pts,
                     const int **cols);
const double *orc_slam_last_global(const orc_slam *s);

/* ---- src/ekf.c:9-127 (caller-side filter, restated for stream tests) ---- */
typedef struct {
    double pos[6];
    double P[6][6], Q[6][6], Rn[6][6];
} orc_ekf;
void orc_ekf_init(orc_ekf *e, const double pos[6]);
void orc_ekf_predict(orc_ekf *e, const double last[6], const double cur[6]);
void orc_ekf_modify(orc_ekf *e, const double meas[6]);
void orc_ekf_update_R(orc_ekf *e, double error);

#ifdef __cplusplus
}
#endif
#endif
