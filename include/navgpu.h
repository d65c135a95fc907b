/*
 * navgpu.h — C ABI of the MI355X scan-matching core (libnavgpu.so).
 *
 * Plain pointers and sizes, no C++/torch types. Two families of entry points:
 *
 *  *_dev : inputs and outputs are DEVICE pointers (hipMalloc'd or any HIP
 *          allocation, e.g. a torch tensor's data_ptr()), enqueued on the
 *          context's stream, asynchronous, no host synchronisation and no
 *          allocation once the workspace has grown to the shape (so a warm
 *          call can be captured into a hipGraph).
 *  *_host: the same computation on HOST pointers: copy in, run, copy out,
 *          synchronise. These back the drop-in C shim (slam.h / kdtree.h /
 *          pointcloud.h, see include/slam.h).
 *
 * Clouds are `double[R*C*3]`, row-major, x,y,z interleaved: the reference
 * `Point ToF_position[MAX_ROWS][MAX_COLS]` (utils/pointcloud.h:32-44) with
 * runtime R, C. Every function returns NAVGPU_OK or a negative status; the
 * message of the last failure is navgpu_last_error(). There is NO CPU
 * fallback: without a usable gfx950 device every compute call fails.
 *
 * Reference functions each entry point replaces (file:line in
 * wuHakureReimu/NAV-SLAM):
 *   navgpu_curvature_*     extract_feature            src/slam.c:11-61
 *   navgpu_project_*       convertToPointCloud        utils/pointcloud.c:8-48
 *   navgpu_kd_build_rows_* flattenPoints+buildKDTree  src/slam.c:64-81,
 *                                                     utils/kdtree.c:8-82
 *   navgpu_kd_query_rows_* nearestNeighborSearch loop src/slam.c:236-244,
 *                                                     utils/kdtree.c:110-152
 *   navgpu_rows_match_*    the per-row scan-pair composition:
 *                          extract_feature x2 + per-row build + 1-NN
 *                          (the tree is built only for rows whose queries
 *                          have a distance tie)
 *   navgpu_knn_*           global-mode k-NN (the reference has k = 1 only;
 *                          ordering = (distance, index))
 */
#ifndef NAVGPU_H
#define NAVGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NAVGPU_OK 0
#define NAVGPU_EINVAL (-1)  /* bad argument / shape                      */
#define NAVGPU_EHIP (-2)    /* HIP runtime error (no device, fault, ...) */
#define NAVGPU_ENOMEM (-3)  /* device allocation failed                   */
#define NAVGPU_ERANGE (-4)  /* shape beyond what a kernel supports        */
#define NAVGPU_EINTERNAL (-5) /* a kernel met an out-of-range index (bug)  */

typedef struct navgpu_ctx navgpu_ctx;

/* Context = device + stream + grow-only workspace. stream may be NULL (a
 * private non-blocking stream is created) or a hipStream_t to enqueue on. */
int navgpu_create(int device, void *stream, navgpu_ctx **out);
void navgpu_destroy(navgpu_ctx *ctx);
int navgpu_set_stream(navgpu_ctx *ctx, void *stream);
void *navgpu_stream(navgpu_ctx *ctx);
int navgpu_sync(navgpu_ctx *ctx);
const char *navgpu_last_error(void);
const char *navgpu_version(void);
/* Largest row width the in-LDS row kernels accept (depends on the device's
 * LDS size); larger rows return NAVGPU_ERANGE. */
int navgpu_rows_max_cols(void);

/* ---- R1: curvature / edge features (src/slam.c:11-61) -------------------
 * mask[r*C+c] = 1 iff the reference marks (r,c) a feature, else 0 (the
 * reference writes only 1s into a caller-zeroed array). curv (nullable)
 * receives the curvature value (0 where none is computed). */
int navgpu_curvature_dev(navgpu_ctx *ctx, const double *pts, int R, int C,
                         int32_t *mask, double *curv);
int navgpu_curvature_host(navgpu_ctx *ctx, const double *pts, int R, int C,
                          int32_t *mask, double *curv);

/* ---- R2: depth grid -> points (utils/pointcloud.c:8-48) ----------------- */
int navgpu_project_dev(navgpu_ctx *ctx, const int32_t *depth, int R, int C,
                       double *pts);
int navgpu_project_host(navgpu_ctx *ctx, const int32_t *depth, int R, int C,
                        double *pts);

/* ---- R3: rigid transform (src/slam.c:95-131,145-160,193-210) ------------
 * out = t + Rm*p (Rm row-major 3x3, the reference's left-to-right sums);
 * when out_last != NULL also out_last = out - tr (mapCoordinatesToLastFrame).
 * Rm is passed from the host so no device transcendental is involved. */
int navgpu_transform_dev(navgpu_ctx *ctx, const double *pts, size_t n,
                         const double Rm[9], const double t[3],
                         const double tr[3], double *out, double *out_last);

/* ---- R4+R5: per-row feature trees ---------------------------------------
 * For each row r: the feature points of `coords` row r (feature = mask of
 * `feat_src`, computed here with R1; coords and feat_src may be the same
 * cloud) compacted in column order (flattenPoints) and arranged by the
 * reference's exact buildKDTree permutation (Lomuto nth_element, median
 * n/2, axis depth%3). Outputs, per row r at offset r*C:
 *   tree_pts[3*(r*C+i)] : i-th point of the permuted array (== implicit
 *                         tree: node of [lo,hi) at lo+(hi-lo)/2)
 *   tree_col[r*C+i]     : its column; tree_n[r]: count.
 * mask_out (nullable) receives the feature mask. */
int navgpu_kd_build_rows_dev(navgpu_ctx *ctx, const double *feat_src,
                             const double *coords, int R, int C,
                             double *tree_pts, int32_t *tree_col,
                             int32_t *tree_n, int32_t *mask_out);

/* ---- R5 host trees: KDNode images of the trees of navgpu_kd_build_rows ---
 * Replaces the per-node malloc + linking of buildKDTree (utils/kdtree.c:
 * 65-82) for the per-row trees of updateKDTree (src/slam.c:161-170).
 * row_off (R+1 int32, device): row_off[r] = tree_n[0]+...+tree_n[r-1],
 * row_off[R] = total. nodes (device, 40*total bytes): for row r and tree
 * position i < tree_n[r], a kdtree.h KDNode {Point point; KDNode *left,
 * *right} at nodes + 40*(row_off[r]+i) whose left/right are the host
 * addresses host_base + 40*(row_off[r]+child) of its children in the
 * implicit layout (NULL for none). Downloaded to host_base, row r's tree is
 * rooted at host_base + 40*(row_off[r] + tree_n[r]/2). R <= 65535. */
int navgpu_kd_rows_nodes_dev(navgpu_ctx *ctx, const double *tree_pts,
                             const int32_t *tree_n, int R, int C,
                             uint64_t host_base, void *nodes, int32_t *row_off);

/* ---- R6: per-row 1-NN over the trees of navgpu_kd_build_rows ------------
 * Queries = feature points of `feat_src` (mask via R1), coordinates from
 * `queries`; query (r,c) searches tree r exactly like
 * nearestNeighborSearch (first-visited point wins ties). Per grid cell:
 *   nn_pos[r*C+c]  = tree position (index into row r of tree_pts) holding
 *                    the reference's answer Point (for bit-identical
 *                    duplicates, the lowest position with those coordinates),
 *                    -1 if (r,c) is not a feature or tree r is empty;
 *   nn_dist[r*C+c] = reference distance, +INFINITY when nn_pos == -1.
 * mask_out (nullable) receives the query feature mask. */
int navgpu_kd_query_rows_dev(navgpu_ctx *ctx, const double *tree_pts,
                             const int32_t *tree_n, const double *feat_src,
                             const double *queries, int R, int C,
                             int32_t *nn_pos, double *nn_dist,
                             int32_t *mask_out);

/* ---- R4 without R5, and R6 over such rows: trees only where ties need them
 * navgpu_kd_compact_rows_dev: navgpu_kd_build_rows_dev without the
 * permutation: tree_pts/tree_col row r = the feature points in column order
 * (flattenPoints, src/slam.c:64-81), tree_n as there. navgpu_kd_query_rows_
 * lazy_dev: navgpu_kd_query_rows_dev over such rows: a query's minimum is
 * unique, or its duplicates bit-identical, except on a genuine distance tie
 * (DESIGN.md §2), and only those rows then get the reference's tree, built
 * in place (tree_pts/tree_col row r permuted as navgpu_kd_build_rows_dev
 * would), with all their queries walked. nn_pos indexes the row as it is on
 * return (column order for untied rows). For a caller that needs no host
 * KDNode trees (the shim with NAVSLAM_HOST_TREES=0): the per-row Lomuto
 * chain (utils/kdtree.c:20-82) runs only for tied rows. tree_built (device,
 * R ints, nullable; zeroed by the compaction): 1 for a row the lazy query has
 * already turned into the reference tree, so that a second lazy query over
 * the same rows (two localisations between mappings) walks that tree instead
 * of rebuilding it from an order that is no longer the column order. NULL:
 * the caller re-compacts before every lazy query. */
int navgpu_kd_compact_rows_dev(navgpu_ctx *ctx, const double *feat_src,
                               const double *coords, int R, int C,
                               double *tree_pts, int32_t *tree_col,
                               int32_t *tree_n, int32_t *mask_out,
                               int32_t *tree_built);
int navgpu_kd_query_rows_lazy_dev(navgpu_ctx *ctx, double *tree_pts, int32_t *tree_col,
                                  const int32_t *tree_n, const double *feat_src,
                                  const double *queries, int R, int C, int32_t *nn_pos,
                                  double *nn_dist, int32_t *mask_out,
                                  int32_t *tree_built);
/* The same, then each row's correspondence sums of the fast mode
 * (navgpu_rows_corr_dev with keep = NULL: `ori` the queries' global
 * coordinates, `sums` 6 doubles per row) in the same launch as the tie
 * pass (r5: one launch and its gap fewer per K5 frame). Not part of the
 * reference interface. */
int navgpu_kd_query_rows_lazy_corr_dev(navgpu_ctx *ctx, double *tree_pts, int32_t *tree_col,
                                       const int32_t *tree_n, const double *feat_src,
                                       const double *queries, int R, int C, int32_t *nn_pos,
                                       double *nn_dist, int32_t *mask_out,
                                       int32_t *tree_built, const double *ori, double *sums);

/* ---- R7: correspondence dedup per row (src/slam.c:247-284) -------------
 * Over the output of navgpu_kd_query_rows: of the queries of row r whose
 * nearest points have equal coordinates, keep the first column at the
 * smallest distance (the reference list's final entry). keep[r*C+c] = 1 for
 * a kept correspondence (nullable); sums[r*6 .. r*6+4] over the row's kept
 * pairs of d = ori - nearest: sum d.x, d.y, d.z; sum |d - mean|^2 (centred,
 * mean = the row's own mean of d); count; sums[r*6+5] =
 * the row's queries that found a nearest point. Order-free: used
 * by the shim's closed-form Adam (NAVSLAM_ADAM=fast); the bit-exact mode
 * keeps the reference's sequential list on the host. */
int navgpu_rows_corr_dev(navgpu_ctx *ctx, const double *tree_pts,
                         const int32_t *tree_n, const int32_t *nn_pos,
                         const double *nn_dist, const double *ori, int R, int C,
                         int32_t *keep, double *sums);

/* The bit-exact counterpart: the reference's correspondence list itself
 * (src/slam.c:235-284), rows in order, each row's entries in first-insertion
 * order (the column of the first query that found that nearest point), each
 * entry holding the query kept for it (smallest distance, then first
 * column). list[7*i .. 7*i+6] = oriPoint (ori at the kept query), nearestPoint,
 * distance: the NeighborResult layout of utils/kdtree.h. list holds up to
 * R*C entries; count[0] = entries, count[1] = queries that found a point.
 * Queries with nn_pos == -1 (no feature, empty row tree) make no entry. */
int navgpu_rows_corr_list_dev(navgpu_ctx *ctx, const double *tree_pts,
                              const int32_t *tree_n, const int32_t *nn_pos,
                              const double *nn_dist, const double *ori, int R, int C,
                              double *list, int32_t *count);

/* ---- The K2 scan-pair step, per-row mode (fused, one kernel) ------------
 * masks of src and tgt (R1), per-row target trees (R4+R5), every src
 * feature queried against its row's tree (R6). nn_idx = linear target index
 * r*C+c of the nearest point (-1: not a feature / empty row tree),
 * nn_dist as above. src_mask / tgt_mask nullable. */
int navgpu_rows_match_dev(navgpu_ctx *ctx, const double *src,
                          const double *tgt, int R, int C, int32_t *src_mask,
                          int32_t *tgt_mask, int32_t *nn_idx, double *nn_dist);
int navgpu_rows_match_host(navgpu_ctx *ctx, const double *src,
                           const double *tgt, int R, int C, int32_t *src_mask,
                           int32_t *tgt_mask, int32_t *nn_idx,
                           double *nn_dist);

/* The same over a batch of independent pairs (K4), one launch: src, tgt are
 * [npairs][R][C] clouds, masks / nn_idx / nn_dist [npairs][R][C]; nn_idx is
 * the target index r*C+c within the query's own pair. */
int navgpu_rows_match_batch_dev(navgpu_ctx *ctx, const double *src,
                                const double *tgt, int npairs, int R, int C,
                                int32_t *src_mask, int32_t *tgt_mask,
                                int32_t *nn_idx, double *nn_dist);

/* ---- Global-mode k-NN (K3) ----------------------------------------------
 * For each of nq queries the k (1..16) target points with the smallest
 * reference distance sqrt((dx*dx+dy*dy)+dz*dz), dx = target - query,
 * ordered by (distance, index) ascending. idx[q*k+s] / dist[q*k+s]; slots
 * left unfilled get -1 / +INFINITY. As in the reference 1-NN (a candidate
 * is taken only if dist < best, best starting at +INFINITY), a target whose
 * distance is +INFINITY or NaN is never a neighbour. Index: a radix-binned uniform grid over the
 * target cloud, rebuilt every call. */
int navgpu_knn_dev(navgpu_ctx *ctx, const double *tgt, size_t nt,
                   const double *queries, size_t nq, int k, int32_t *idx,
                   double *dist);
int navgpu_knn_host(navgpu_ctx *ctx, const double *tgt, size_t nt,
                    const double *queries, size_t nq, int k, int32_t *idx,
                    double *dist);

/* The K3 scan-pair step: curvature masks of both R x C clouds + global k-NN
 * of every src point against tgt. Masks nullable. */
int navgpu_pair_knn_dev(navgpu_ctx *ctx, const double *src, const double *tgt,
                        int R, int C, int k, int32_t *src_mask,
                        int32_t *tgt_mask, int32_t *idx, double *dist);

/* ---- R5 for one arbitrary point array (kdtree.h buildKDTree) ------------
 * pts: n points (AoS), permuted in place into the reference's buildKDTree
 * order for a root at depth `depth0` (axis = (depth0 + level) % 3).
 * n < 2^30 and at most 2^15 windows per level (about 383M points; larger n
 * returns NAVGPU_ERANGE). Up to ~5.7k points the build runs in one
 * workgroup's LDS.
 * Larger arrays run the reference's Lomuto passes grid-wide, level by level
 * (DESIGN.md §4). The number of quickselect rounds depends on the data, so
 * that path reads a device flag back every 4 rounds: unlike the other
 * *_dev calls it synchronises the host with the context's stream. */
int navgpu_kd_build_dev(navgpu_ctx *ctx, double *pts, size_t n, int depth0);
int navgpu_kd_build_host(navgpu_ctx *ctx, double *pts, size_t n, int depth0);

/* ---- device memory helpers (for C callers without HIP headers) --------- */
int navgpu_malloc(navgpu_ctx *ctx, size_t bytes, void **dptr);
void navgpu_free(navgpu_ctx *ctx, void *dptr);
/* page-locked host memory (copies to and from it skip the staging buffer);
 * navgpu_host_free waits for the context's streams first */
int navgpu_host_alloc(navgpu_ctx *ctx, size_t bytes, void **hptr);
void navgpu_host_free(navgpu_ctx *ctx, void *hptr);
/* page-lock a caller's host range in place (copies to and from it then run by
 * DMA, no staging). The range must stay allocated until
 * navgpu_host_unregister: memory freed while registered keeps the old pages
 * behind its addresses, so a later allocation there would copy the wrong
 * data (which is why the drop-in shim, which cannot see when its caller
 * frees a SLAM_attr, does not use it). NAVGPU_ERANGE when the runtime
 * refuses (the range stays pageable and every copy still works) */
int navgpu_host_register(navgpu_ctx *ctx, void *hptr, size_t bytes);
void navgpu_host_unregister(navgpu_ctx *ctx, void *hptr);
/* stream-ordered copies on the context's stream (host memory pageable) */
int navgpu_upload(navgpu_ctx *ctx, void *dst_dev, const void *src_host,
                  size_t bytes);
int navgpu_download(navgpu_ctx *ctx, void *dst_host, const void *src_dev,
                    size_t bytes);
/* Measured HBM ceiling for the roofline: a device-to-device copy
 * of `bytes` (a multiple of 16, both pointers 16-B aligned) by a plain
 * streaming kernel on the context's stream, timed as "stream_copy". Not part
 * of the reference interface. */
int navgpu_stream_copy_dev(navgpu_ctx *ctx, void *dst_dev, const void *src_dev,
                           size_t bytes);

/* Copies that overlap later work: navgpu_side_mark records the current
 * point of the context's stream; navgpu_side_download copies device->host on
 * a side stream once that point is reached, while work enqueued after the
 * mark keeps running on the main stream. navgpu_sync waits for both. */
int navgpu_side_mark(navgpu_ctx *ctx);
int navgpu_side_download(navgpu_ctx *ctx, void *dst_host, const void *src_dev,
                         size_t bytes);

/* Kernel-level timing hook for bench.py: HIP events recorded around the
 * dominant kernel of the last *_dev call on the context's stream. Returns
 * the summed milliseconds of the named kernel since the last reset
 * (name: "knn_query", "rows_match", "curvature"), or -1. */
void navgpu_timing_enable(navgpu_ctx *ctx, int on);
/* Record only the region `name` while timing is on (NULL or "" = every
 * region): fewer event packets in a measured run (r5: events around every
 * region of every K3 step cost the step ~2 %). */
void navgpu_timing_select(navgpu_ctx *ctx, const char *name);
double navgpu_timing_read(navgpu_ctx *ctx, const char *name, int reset);
int navgpu_timing_count(navgpu_ctx *ctx, const char *name);
/* Diagnostic: queries of the last navgpu_knn_* call that left the fast path
 * for the exact ring search (synchronises). Recorded only when the context
 * was created with NAVGPU_KNN_STATS=1 in the environment; -1 otherwise. */
long long navgpu_knn_fallbacks(navgpu_ctx *ctx);
/* Diagnostic: k_knn tiles of the last navgpu_knn_* call whose neighbourhood
 * exceeded the LDS tile budget and ran from global memory (synchronises). */
long long navgpu_knn_overflows(navgpu_ctx *ctx);
/* Integrity check of the last navgpu_knn_* / navgpu_pair_knn_dev call
 * (synchronises): NAVGPU_EINTERNAL when a k-NN kernel met a list, cloud or
 * record index out of range (it clamps the address so the device cannot
 * fault, and flags the call); NAVGPU_OK otherwise. navgpu_knn_host checks
 * it itself. */
int navgpu_knn_check(navgpu_ctx *ctx);
/* Diagnostic: rows of the last navgpu_rows_match_* call that had a query
 * with a distance tie and so ran the reference tree (synchronises); -1 when
 * the last call did not screen (NAVGPU_ROWS_SCREEN=0) or none was made. */
long long navgpu_rows_tie_rows(navgpu_ctx *ctx);
/* Diagnostic: one reference nth_element (utils/kdtree.c:20-52: Lomuto,
 * pivot = last, `<= 0` goes left) over keys[perm[first..last]] as the
 * per-row builds run it (block = 0: one wave, its ordinary and register
 * passes; 1: the 1024-thread block pass), permuting the device
 * array perm (values < n, n <= 8191) in place; asynchronous on the stream. */
int navgpu_debug_nth_element(navgpu_ctx *ctx, const double *key, int32_t *perm, int n,
                             int first, int last, int nth, int block);

#ifdef __cplusplus
}
#endif
#endif
