/*
 * navslam_shim.c — the drop-in C ABI of NAV-SLAM's scan-matching path:
 * slam.h (init_slam / slam_localization / slam_mapping), kdtree.h
 * (buildKDTree / freeKDTree / nearestNeighborSearch / printKDTree),
 * pointcloud.h (convertToPointCloud / printPointCloud) and slam.c's
 * extract_feature, implemented over libnavgpu (include/navgpu.h).
 *
 * Built once per grid size (libnavslam_<R>x<C>.so, -DMAX_ROWS/-DMAX_COLS),
 * because the reference's structs embed the dims. src/main.c and src/ekf.c
 * link against it unchanged.
 *
 * What runs where, per frame:
 *   GPU : rigid transform (src/slam.c:145-160,193-210,402-416), curvature
 *         (src/slam.c:11-61), per-row feature compaction + the reference's
 *         exact KD permutation (src/slam.c:64-81, utils/kdtree.c:20-82), and
 *         the per-feature 1-NN batch (src/slam.c:236-244, utils/kdtree.c:
 *         110-152).
 *         The correspondence list (src/slam.c:247-284) is built on the GPU
 *         in the reference's first-insertion order; only the list comes back.
 *   host: the 3-DOF Adam loop (src/slam.c:300-389), a sequential
 *         floating-point sum whose rounding order is part of the result,
 *         kept bit-identical here. NAVSLAM_ADAM=fast: GPU sums + closed form.
 * There is no CPU fallback for the GPU part: a device failure prints the
 * error and aborts (the reference API has no status codes).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stddef.h>
#include <time.h>

#include "navgpu.h"
#include "slam.h"

#define ROWS MAX_ROWS
#define COLS MAX_COLS
#define NPTS ((size_t)MAX_ROWS * MAX_COLS)
#define DEG2RAD(x) ((x) * M_PI / 180.0) /* src/slam.c:8 */

/* ----------------------------------------------------------- context */
static navgpu_ctx *g_ctx;

static void die(const char *what, int rc)
{
    fprintf(stderr, "navslam: %s failed (%d): %s\n", what, rc,
            navgpu_last_error());
    abort();
}

#define CK(x)                        \
    do {                             \
        int rc_ = (x);               \
        if (rc_ != NAVGPU_OK)        \
            die(#x, rc_);            \
    } while (0)

static navgpu_ctx *ctx(void)
{
    if (!g_ctx) {
        const char *d = getenv("NAVSLAM_DEVICE");
        CK(navgpu_create(d ? atoi(d) : 0, NULL, &g_ctx));
    }
    return g_ctx;
}

/* NAVSLAM_PROFILE=1: host-side phase times, printed at exit (diagnostic) */
static double g_prof[8];
static long g_prof_n[8];
static int g_prof_on = -1;
static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}
static void prof_dump(void)
{
    static const char *names[8] = {"map: gpu+copies", "map: link trees", "loc: gpu+copies",
                                   "loc: adam", "", "", "", ""};
    for (int i = 0; i < 8; i++)
        if (g_prof_n[i])
            fprintf(stderr, "navslam profile %-18s %8.3f ms avg over %ld\n", names[i],
                    1e3 * g_prof[i] / g_prof_n[i], g_prof_n[i]);
}
static int prof_on(void)
{
    if (g_prof_on < 0) {
        const char *e = getenv("NAVSLAM_PROFILE");
        g_prof_on = e && *e == '1';
        if (g_prof_on)
            atexit(prof_dump);
    }
    return g_prof_on;
}
#define PROF_ADD(i, t0)                     \
    do {                                    \
        if (prof_on()) {                    \
            g_prof[i] += now_s() - (t0);    \
            g_prof_n[i]++;                  \
        }                                   \
    } while (0)

static int quiet(void)
{
    const char *q = getenv("NAVSLAM_QUIET");
    return q && *q && *q != '0';
}

/* NAVSLAM_ADAM=fast: correspondence dedup on the GPU and the Adam loop on
 * closed-form residual sums (order-free, so not bit-identical to the
 * reference's sequential sums; the pose difference is reported by
 * bench.py --workload k5 --k5-mode fast). Default: bit-exact host path. */
static int adam_fast(void)
{
    const char *q = getenv("NAVSLAM_ADAM");
    return q && strcmp(q, "fast") == 0;
}

/* Where the map slot downloads (NAVSLAM_D2H=1 side stream, =0 main stream;
 * r5 A/B knob). Default: on the side stream while the host trees build
 * (k_rows_build, ~0.5 ms to overlap), on the main stream after the lazy
 * rows' ~14 us compaction (the side stream's blit path started ~370 us
 * late in r5's trace). Either is a pageable copy: the runtime locks the
 * caller's pages per call, at a cost that varied from ~0.1 to ~0.45 ms per
 * 6.3 MB slot across r5's boxes; page-locked bounce buffers and piecewise
 * copies did not beat it. */
static int host_trees(void);
static int side_d2h(void)
{
    const char *q = getenv("NAVSLAM_D2H");
    if (q && (*q == '0' || *q == '1'))
        return *q == '1';
    return host_trees();
}

static int host_trees(void)
{
    const char *q = getenv("NAVSLAM_HOST_TREES");
    return !(q && *q == '0');
}

/* Fast mode on lazy rows: the row sums in the tie pass's launch (default), or
 * NAVSLAM_LAZY_CORR=0 for the separate k_rows_corr launch (r5 A/B knob) */
static int lazy_corr(void)
{
    const char *q = getenv("NAVSLAM_LAZY_CORR");
    return !(q && *q == '0');
}

/* ------------------------------------- host KDNode blocks + registry */
/* Every tree this library hands out is one malloc'd block of KDNode laid
 * out in the implicit order (node of [lo,hi) at lo+(hi-lo)/2), linked like
 * the reference's per-node mallocs. freeKDTree recognises block roots. */
typedef struct {
    KDNode *root, *base;
    size_t n;
} kd_block;
static kd_block *g_blocks;
static size_t g_nblocks, g_capblocks;

static KDNode *link_range(KDNode *b, const Point *pts, size_t lo, size_t hi)
{
    if (lo >= hi)
        return NULL;
    size_t mid = lo + (hi - lo) / 2;
    KDNode *nd = &b[mid];
    nd->point = pts[mid];
    nd->left = link_range(b, pts, lo, mid);
    nd->right = link_range(b, pts, mid + 1, hi);
    return nd;
}

static KDNode *make_block(const Point *pts, size_t n)
{
    if (n == 0)
        return NULL;
    KDNode *b = malloc(sizeof(KDNode) * n);
    if (!b) {
        fprintf(stderr, "navslam: out of host memory\n");
        abort();
    }
    KDNode *root = link_range(b, pts, 0, n);
    if (g_nblocks == g_capblocks) {
        g_capblocks = g_capblocks ? 2 * g_capblocks : 64;
        g_blocks = realloc(g_blocks, sizeof(kd_block) * g_capblocks);
    }
    g_blocks[g_nblocks].root = root;
    g_blocks[g_nblocks].base = b;
    g_blocks[g_nblocks].n = n;
    g_nblocks++;
    return root;
}

/* A slab of row trees owned by a SLAM_attr's state (map_frame): freeKDTree
 * on any node inside it is a no-op, the slab lives as long as the state. */
_Static_assert(sizeof(KDNode) == 40 && offsetof(KDNode, left) == 24 &&
                   offsetof(KDNode, right) == 32,
               "KDNode layout of utils/kdtree.h:7-11 (navgpu_kd_rows_nodes_dev)");
static void register_slab(KDNode *base, size_t n)
{
    if (g_nblocks == g_capblocks) {
        g_capblocks = g_capblocks ? 2 * g_capblocks : 64;
        g_blocks = realloc(g_blocks, sizeof(kd_block) * g_capblocks);
    }
    if (!g_blocks) {
        fprintf(stderr, "navslam: out of host memory\n");
        abort();
    }
    g_blocks[g_nblocks].root = NULL;
    g_blocks[g_nblocks].base = base;
    g_blocks[g_nblocks].n = n;
    g_nblocks++;
}

static int release_block(KDNode *root)
{
    for (size_t i = g_nblocks; i-- > 0;) {
        if (g_blocks[i].root == root) {
            free(g_blocks[i].base);
            g_blocks[i] = g_blocks[--g_nblocks];
            return 1;
        }
    }
    return 0;
}

/* utils/kdtree.c:84-91 */
void freeKDTree(KDNode *root)
{
    if (!root)
        return;
    if (release_block(root))
        return;
    /* a subtree of one of our blocks: freed with its block's root */
    for (size_t i = 0; i < g_nblocks; i++)
        if (root >= g_blocks[i].base && root < g_blocks[i].base + g_blocks[i].n)
            return;
    /* a tree the caller built node by node with malloc */
    freeKDTree(root->left);
    freeKDTree(root->right);
    free(root);
}

/* utils/kdtree.c:65-82 — the permutation is computed on the GPU. */
KDNode *buildKDTree(Point *points, size_t numPoints, int depth)
{
    if (numPoints == 0)
        return NULL;
    CK(navgpu_kd_build_host(ctx(), (double *)points, numPoints, depth));
    return make_block(points, numPoints);
}

/* utils/kdtree.c:94-107 */
void printKDTree(KDNode *node, int depth)
{
    if (node == NULL)
        return;
    printf("\xe6\xb7\xb1\xe5\xba\xa6 %d: Point(x=%.2f, y=%.2f, z=%.2f)\n", depth,
           node->point.x, node->point.y, node->point.z);
    printKDTree(node->left, depth + 1);
    printKDTree(node->right, depth + 1);
}

/* utils/kdtree.c:110-152 — one query against a linked host tree. */
void nearestNeighborSearch(KDNode *root, Point *target, Point *result,
                           double *bestDist, int depth)
{
    if (root == NULL)
        return;
    double dx = root->point.x - target->x;
    double dy = root->point.y - target->y;
    double dz = root->point.z - target->z;
    double dist = sqrt(dx * dx + dy * dy + dz * dz);
    if (dist < *bestDist) {
        *bestDist = dist;
        *result = root->point;
    }
    int axis = depth % 3;
    double t = axis == 0 ? target->x : axis == 1 ? target->y : target->z;
    double n = axis == 0 ? root->point.x : axis == 1 ? root->point.y
                                                     : root->point.z;
    KDNode *near = t < n ? root->left : root->right;
    KDNode *far = t < n ? root->right : root->left;
    nearestNeighborSearch(near, target, result, bestDist, depth + 1);
    if (fabs(t - n) < *bestDist)
        nearestNeighborSearch(far, target, result, bestDist, depth + 1);
}

/* --------------------------------------------------------- pointcloud.h */
void convertToPointCloud(int distances[MAX_ROWS][MAX_COLS],
                         Point pointCloud[MAX_ROWS][MAX_COLS])
{
    CK(navgpu_project_host(ctx(), (const int32_t *)&distances[0][0], ROWS,
                           COLS, &pointCloud[0][0].x));
}

void printPointCloud(PointCloud pointcloud) /* utils/pointcloud.c:50-58 */
{
    for (int i = 0; i < MAX_ROWS; i++)
        for (int j = 0; j < MAX_COLS; j++) {
            Point p = pointcloud.ToF_position[i][j];
            printf("point %d: (%f, %f, %f) \n", i * MAX_ROWS + j, p.x, p.y, p.z);
        }
}

/* src/slam.c:11-61 — writes 1 where the reference does, leaves the rest. */
void extract_feature(PointCloud *lidarPointCloud,
                     int feature[MAX_ROWS][MAX_COLS])
{
    static int32_t mask[MAX_ROWS][MAX_COLS];
    CK(navgpu_curvature_host(ctx(), &lidarPointCloud->ToF_position[0][0].x,
                             ROWS, COLS, &mask[0][0], NULL));
    for (int i = 0; i < ROWS; i++)
        for (int j = 0; j < COLS; j++)
            if (mask[i][j])
                feature[i][j] = 1;
}

/* ------------------------------------------ extras (not in the reference) */
static int g_last_queries, g_last_cp, g_last_iters;

/* The navgpu context the shim runs on, so a host harness can switch its
 * kernel timing on (navgpu_timing / navgpu_timing_read). */
void *navslam_context(void)
{
    return ctx();
}

/* Counts of the last slam_localization call: feature queries searched,
 * correspondences after the dedup (CPcount, src/slam.c:284) and Adam
 * iterations run (src/slam.c:300-379). Returns 0. */
int navslam_last_frame_stats(int *queries, int *correspondences, int *iterations)
{
    if (queries)
        *queries = g_last_queries;
    if (correspondences)
        *correspondences = g_last_cp;
    if (iterations)
        *iterations = g_last_iters;
    return 0;
}

/* ------------------------------------------------ SLAM_attr side table */

typedef struct {
    SLAM_attr *key;
    double *d_lidar, *d_global, *d_last, *d_tree, *d_dist, *d_sums, *d_list;
    double h_sums[6 * ROWS];
    double *h_sums_pin; /* page-locked, written by k_rows_corr itself (r5), or NULL */
    int32_t *d_tcol, *d_tn, *d_pos, *d_count;
    int32_t *d_built; /* lazy rows already turned into the reference tree */
    int have_trees;
    int lazy; /* the rows hold compacted features, trees only where ties need them */
    double prof_t0; /* NAVSLAM_PROFILE */
    int32_t *d_off;         /* row offsets of the node image (ROWS+1) */
    void *d_nodes;          /* KDNode image of the row trees, device */
    KDNode *h_nodes;        /* its host copy: the trees handed out */
    int h_nodes_pinned;
    int32_t h_off[ROWS + 1];
    NeighborResult *result; /* correspondence list (src/slam.c:214) */
} slam_state;

static slam_state **g_states;
static int g_nstates;

static slam_state *state_for(SLAM_attr *a)
{
    for (int i = 0; i < g_nstates; i++)
        if (g_states[i]->key == a)
            return g_states[i];
    slam_state *s = calloc(1, sizeof(*s));
    if (!s) {
        fprintf(stderr, "navslam: out of host memory\n");
        abort();
    }
    s->key = a;
    navgpu_ctx *c = ctx();
    CK(navgpu_malloc(c, 24 * NPTS, (void **)&s->d_lidar));
    CK(navgpu_malloc(c, 24 * NPTS, (void **)&s->d_global));
    CK(navgpu_malloc(c, 24 * NPTS, (void **)&s->d_last));
    CK(navgpu_malloc(c, 24 * NPTS, (void **)&s->d_tree));
    CK(navgpu_malloc(c, 8 * NPTS, (void **)&s->d_dist));
    CK(navgpu_malloc(c, 4 * NPTS, (void **)&s->d_tcol));
    CK(navgpu_malloc(c, 4 * ROWS, (void **)&s->d_tn));
    CK(navgpu_malloc(c, 4 * ROWS, (void **)&s->d_built));
    CK(navgpu_malloc(c, 4 * NPTS, (void **)&s->d_pos));
    CK(navgpu_malloc(c, 8 * 6 * ROWS, (void **)&s->d_sums));
    CK(navgpu_malloc(c, 56 * (size_t)NPTS, (void **)&s->d_list));
    CK(navgpu_malloc(c, 8, (void **)&s->d_count));
    CK(navgpu_malloc(c, 4 * (ROWS + 1), (void **)&s->d_off));
    CK(navgpu_malloc(c, sizeof(KDNode) * (size_t)NPTS, &s->d_nodes));
    /* page-locked when the runtime allows it: the image then downloads by
     * DMA straight into the trees */
    s->h_nodes_pinned =
        navgpu_host_alloc(c, sizeof(KDNode) * (size_t)NPTS, (void **)&s->h_nodes) == 0;
    if (!s->h_nodes_pinned)
        s->h_nodes = malloc(sizeof(KDNode) * (NPTS ? (size_t)NPTS : 1));
    if (!s->h_nodes) {
        fprintf(stderr, "navslam: out of host memory\n");
        abort();
    }
    register_slab(s->h_nodes, NPTS);
    /* the fast mode's per-row sums land here straight from the kernel: no
     * copy launch per frame (NULL when page-locked memory is refused) */
    if (navgpu_host_alloc(c, sizeof(s->h_sums), (void **)&s->h_sums_pin) != 0)
        s->h_sums_pin = NULL;
    g_states = realloc(g_states, sizeof(*g_states) * (g_nstates + 1));
    g_states[g_nstates++] = s;
    return s;
}

/* src/slam.c:95-115 with the DEG2RAD of the callers */
static void rotation(double roll, double pitch, double yaw, double R[9])
{
    double cr = cos(DEG2RAD(roll)), sr = sin(DEG2RAD(roll));
    double cp = cos(DEG2RAD(pitch)), sp = sin(DEG2RAD(pitch));
    double cy = cos(DEG2RAD(yaw)), sy = sin(DEG2RAD(yaw));
    R[0] = cy * cp;
    R[1] = cy * sp * sr - sy * cr;
    R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp;
    R[4] = sy * sp * sr + cy * cr;
    R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;
    R[7] = cp * sr;
    R[8] = cp * cr;
}

/* src/slam.c:143-172 / 395-427: global frame into the map slot, trees of
 * the lidar-frame features over the global coordinates. */
static void map_frame(SLAM_attr *attr, slam_state *s, Pos pos,
                      PointCloud *lidar, int slot)
{
    navgpu_ctx *c = ctx();
    const double pt0 = prof_on() ? now_s() : 0.0;
    double R[9], t[3] = {pos.x, pos.y, pos.z};
    rotation(pos.roll, pos.pitch, pos.yaw, R);
    attr->globalPointCloud[slot].ToF_timestamps = lidar->ToF_timestamps;
    CK(navgpu_upload(c, s->d_lidar, &lidar->ToF_position[0][0], 24 * NPTS));
    CK(navgpu_transform_dev(c, s->d_lidar, NPTS, R, t, NULL, s->d_global, NULL));
    const int side = side_d2h();
    if (side)
        CK(navgpu_side_mark(c)); /* the map slot is final here */
    /* without host trees nobody walks a tree the next localisation does not
     * need: the rows keep their features in column order and only rows with
     * a distance tie get the reference's tree (navgpu_kd_query_rows_lazy_dev) */
    s->lazy = !host_trees();
    if (s->lazy)
        CK(navgpu_kd_compact_rows_dev(c, s->d_lidar, s->d_global, ROWS, COLS,
                                      s->d_tree, s->d_tcol, s->d_tn, NULL, s->d_built));
    else
        CK(navgpu_kd_build_rows_dev(c, s->d_lidar, s->d_global, ROWS, COLS,
                                    s->d_tree, s->d_tcol, s->d_tn, NULL));
    if (side) /* the map slot comes back while the trees build */
        CK(navgpu_side_download(c, &attr->globalPointCloud[slot].ToF_position[0][0],
                                s->d_global, 24 * NPTS));
    else
        CK(navgpu_download(c, &attr->globalPointCloud[slot].ToF_position[0][0],
                           s->d_global, 24 * NPTS));
    s->have_trees = 1;
    if (!host_trees()) {
        CK(navgpu_sync(c));
        for (int r = 0; r < ROWS; r++)
            attr->kdtree_lastframe[r] = NULL;
        PROF_ADD(0, pt0);
        return;
    }
    /* the host trees: their linked KDNode image is written on the GPU with
     * the slab's host addresses and lands in place (no per-node malloc or
     * linking on the host). The slab is this state's: the previous frame's
     * trees (which the reference leaks) are overwritten, not freed. */
    CK(navgpu_kd_rows_nodes_dev(c, s->d_tree, s->d_tn, ROWS, COLS,
                                (uint64_t)(uintptr_t)s->h_nodes, s->d_nodes, s->d_off));
    CK(navgpu_download(c, s->h_off, s->d_off, sizeof(s->h_off)));
    CK(navgpu_sync(c));
    PROF_ADD(0, pt0);
    const double pt1 = prof_on() ? now_s() : 0.0;
    const int32_t total = s->h_off[ROWS];
    if (total < 0 || total > NPTS) {
        fprintf(stderr, "navslam: bad tree sizes from the device (%d)\n", (int)total);
        abort();
    }
    CK(navgpu_download(c, s->h_nodes, s->d_nodes, sizeof(KDNode) * (size_t)total));
    CK(navgpu_sync(c));
    for (int r = 0; r < ROWS; r++) {
        const int32_t n = s->h_off[r + 1] - s->h_off[r];
        attr->kdtree_lastframe[r] = n > 0 ? s->h_nodes + s->h_off[r] + n / 2 : NULL;
    }
    PROF_ADD(1, pt1);
}

void init_slam(SLAM_attr *attr, Pos pos, PointCloud *lidarPointCloud)
{
    slam_state *s = state_for(attr);
    attr->frameCount = 0;
    attr->error = 0.0;
    map_frame(attr, s, pos, lidarPointCloud, 0);
    attr->frameCount++;
}

void slam_mapping(SLAM_attr *attr, Pos pos, PointCloud *lidarPointCloud)
{
    slam_state *s = state_for(attr);
    /* the reference writes globalPointCloud[frameCount] with no bound
     * (src/slam.c:395); past SLAM_MAP_FRAMES the map is a ring here */
    map_frame(attr, s, pos, lidarPointCloud, attr->frameCount % SLAM_MAP_FRAMES);
    attr->frameCount++;
}


/* The NAVSLAM_ADAM=fast tail of slam_localization: dedup + residual sums on
 * the GPU (navgpu_rows_corr_dev), then src/slam.c:300-389's Adam loop with
 * every per-iteration sum in closed form. With d_i = ori_i - near_i, its
 * mean m and dx_i = (ori_i - t) - near_i = d_i - t:
 *   sum dx = n (m - t),   totalError = sum |d_i - t|^2 = M2 + n |m - t|^2
 * where M2 = sum |d_i - m|^2 comes centred from the GPU (per row, merged
 * here), so no cancellation and never negative (exact in real arithmetic;
 * rounding differs from the reference's sequential sums). */
static Pos localization_fast(SLAM_attr *attr, slam_state *s, double transform[6],
                             Pos pos_last, int corr_done)
{
    navgpu_ctx *c = ctx();
    if (!corr_done) /* (the lazy rows' query launched it with their tie pass) */
        CK(navgpu_rows_corr_dev(c, s->d_tree, s->d_tn, s->d_pos, s->d_dist, s->d_global,
                                ROWS, COLS, NULL, s->h_sums_pin ? s->h_sums_pin : s->d_sums));
    if (!s->h_sums_pin)
        CK(navgpu_download(c, s->h_sums, s->d_sums, sizeof(s->h_sums)));
    CK(navgpu_sync(c));
    const double *sums = s->h_sums_pin ? s->h_sums_pin : s->h_sums;
    PROF_ADD(2, s->prof_t0);
    /* merge the rows' (count, mean, centred M2) with Chan et al.'s pairwise
     * update: M2 = M2a + M2b + |mb - ma|^2 na nb / (na + nb) */
    double mean[3] = {0.0, 0.0, 0.0}, M2 = 0.0, n = 0.0, nq = 0.0;
    for (int r = 0; r < ROWS; r++) {
        const double *h = sums + 6 * r;
        nq += h[5];
        const double nb = h[4];
        if (!(nb > 0))
            continue;
        const double tot = n + nb;
        double dm[3], dd = 0.0;
        for (int j = 0; j < 3; j++) {
            dm[j] = h[j] / nb - mean[j];
            dd += dm[j] * dm[j];
            mean[j] += dm[j] * (nb / tot);
        }
        M2 += h[3] + dd * (n * nb / tot);
        n = tot;
    }
    double learningRate = 0.1, tolerance = 1e-6;
    double previousTotalError = 0, totalError = 0;
    double m[3] = {0.0, 0.0, 0.0}, v[3] = {0.0, 0.0, 0.0};
    double beta1 = 0.9, beta2 = 0.999, epsilon = 1e-8;
    int q = quiet();
    int iter;
    for (iter = 0; iter < 200; ++iter) {
        const double *t = transform;
        double gradient[3];
        /* sum dx_i = n (mean - t); sum |dx_i|^2 = M2 + n |mean - t|^2 >= 0 */
        double off2 = 0.0;
        for (int j = 0; j < 3; j++) {
            const double e = mean[j] - t[j];
            gradient[j] = -(n * e);
            off2 += e * e;
        }
        totalError = M2 + n * off2;
        if (fabs(totalError - previousTotalError) < tolerance) {
            if (!q)
                printf("\xe6\x94\xb6\xe6\x95\x9b\xef\xbc\x8c\xe5\x81\x9c\xe6\xad\xa2"
                       "\xe8\xbf\xad\xe4\xbb\xa3\xef\xbc\x81\n");
            break;
        }
        previousTotalError = totalError;
        if (n > 0) {
            gradient[0] /= n;
            gradient[1] /= n;
            gradient[2] /= n;
        }
        int tt = iter + 1;
        for (int j = 0; j < 3; j++) {
            m[j] = beta1 * m[j] + (1 - beta1) * gradient[j];
            v[j] = beta2 * v[j] + (1 - beta2) * gradient[j] * gradient[j];
            double m_hat = m[j] / (1 - pow(beta1, tt));
            double v_hat = v[j] / (1 - pow(beta2, tt));
            transform[j] -= learningRate * m_hat / (sqrt(v_hat) + epsilon);
        }
        if (!q)
            printf("Iteration %d, Total Error: %.6f\n", iter, totalError);
    }
    g_last_queries = (int)nq;
    g_last_cp = (int)n;
    g_last_iters = iter;
    attr->error = n > 0 ? sqrt(totalError / n) : 0.0;
    Pos out;
    out.x = pos_last.x + transform[0];
    out.y = pos_last.y + transform[1];
    out.z = pos_last.z + transform[2];
    out.roll = pos_last.roll + transform[3];
    out.pitch = pos_last.pitch + transform[4];
    out.yaw = pos_last.yaw + transform[5];
    return out;
}

Pos slam_localization(SLAM_attr *attr, PointCloud *lidarPointCloud,
                      Pos pos_predict, Pos pos_last)
{
    navgpu_ctx *c = ctx();
    slam_state *s = state_for(attr);
    double R[9];
    rotation(pos_predict.roll, pos_predict.pitch, pos_predict.yaw, R);
    double transform[6]; /* compute_posdiff, src/slam.c:84-92 */
    transform[0] = pos_predict.x - pos_last.x;
    transform[1] = pos_predict.y - pos_last.y;
    transform[2] = pos_predict.z - pos_last.z;
    transform[3] = pos_predict.roll - pos_last.roll;
    transform[4] = pos_predict.pitch - pos_last.pitch;
    transform[5] = pos_predict.yaw - pos_last.yaw;
    double t[3] = {pos_predict.x, pos_predict.y, pos_predict.z};

    s->prof_t0 = prof_on() ? now_s() : 0.0;
    /* GPU: transform, features, per-row 1-NN (src/slam.c:185-244) */
    CK(navgpu_upload(c, s->d_lidar, &lidarPointCloud->ToF_position[0][0],
                     24 * NPTS));
    CK(navgpu_transform_dev(c, s->d_lidar, NPTS, R, t, transform, s->d_global,
                            s->d_last));
    if (!s->have_trees) { /* localisation before any init/mapping: no map */
        CK(navgpu_upload(c, s->d_tn, (int32_t[ROWS]){0}, 4 * ROWS));
        s->have_trees = 1;
    }
    const int fast = adam_fast();
    int corr_done = 0;
    if (s->lazy && fast && lazy_corr()) { /* the fast mode's row sums in the tie pass's launch */
        CK(navgpu_kd_query_rows_lazy_corr_dev(c, s->d_tree, s->d_tcol, s->d_tn, s->d_lidar,
                                              s->d_last, ROWS, COLS, s->d_pos, s->d_dist, NULL,
                                              s->d_built, s->d_global,
                                              s->h_sums_pin ? s->h_sums_pin : s->d_sums));
        corr_done = 1;
    } else if (s->lazy)
        CK(navgpu_kd_query_rows_lazy_dev(c, s->d_tree, s->d_tcol, s->d_tn, s->d_lidar,
                                         s->d_last, ROWS, COLS, s->d_pos, s->d_dist, NULL,
                                         s->d_built));
    else
        CK(navgpu_kd_query_rows_dev(c, s->d_tree, s->d_tn, s->d_lidar, s->d_last,
                                    ROWS, COLS, s->d_pos, s->d_dist, NULL));
    if (fast)
        return localization_fast(attr, s, transform, pos_last, corr_done);
    /* GPU: the reference's correspondence list (src/slam.c:235-284), built
     * and compacted in its first-insertion order on the device; only the
     * list itself comes back */
    if (!s->result) {
        s->result = malloc(sizeof(NeighborResult) * (NPTS ? NPTS : 1));
        if (!s->result) {
            fprintf(stderr, "navslam: out of host memory\n");
            abort();
        }
    }
    _Static_assert(sizeof(NeighborResult) == 7 * sizeof(double),
                   "NeighborResult is 7 doubles (utils/kdtree.h:14-18)");
    CK(navgpu_rows_corr_list_dev(c, s->d_tree, s->d_tn, s->d_pos, s->d_dist, s->d_global,
                                 ROWS, COLS, s->d_list, s->d_count));
    int32_t cnt[2];
    CK(navgpu_download(c, cnt, s->d_count, sizeof(cnt)));
    CK(navgpu_sync(c));
    int CPcount = cnt[0], nqueries = cnt[1];
    NeighborResult *result = s->result;
    if (CPcount > 0)
        CK(navgpu_download(c, result, s->d_list, sizeof(NeighborResult) * (size_t)CPcount));
    CK(navgpu_sync(c));
    PROF_ADD(2, s->prof_t0);
    const double pt1 = prof_on() ? now_s() : 0.0;

    /* host: Adam on the translation (src/slam.c:218-379) */
    double learningRate = 0.1, tolerance = 1e-6;
    double previousTotalError = 0, totalError = 0;
    int validGradientCount = 0;
    double m[3] = {0.0, 0.0, 0.0}, v[3] = {0.0, 0.0, 0.0};
    double beta1 = 0.9, beta2 = 0.999, epsilon = 1e-8;
    int q = quiet();
    int iter;
    for (iter = 0; iter < 200; ++iter) {
        double gradient[3] = {0.0, 0.0, 0.0};
        totalError = 0;
        validGradientCount = 0;
        for (int i = 0; i < CPcount; i++) {
            double dx = (result[i].oriPoint.x - transform[0]) - result[i].nearestPoint.x;
            double dy = (result[i].oriPoint.y - transform[1]) - result[i].nearestPoint.y;
            double dz = (result[i].oriPoint.z - transform[2]) - result[i].nearestPoint.z;
            double dist_sq = dx * dx + dy * dy + dz * dz;
            totalError += dist_sq;
            gradient[0] -= dx;
            gradient[1] -= dy;
            gradient[2] -= dz;
            validGradientCount++;
        }
        if (fabs(totalError - previousTotalError) < tolerance) {
            if (!q)
                printf("\xe6\x94\xb6\xe6\x95\x9b\xef\xbc\x8c\xe5\x81\x9c\xe6\xad\xa2"
                       "\xe8\xbf\xad\xe4\xbb\xa3\xef\xbc\x81\n");
            break;
        }
        previousTotalError = totalError;
        if (validGradientCount > 0) {
            gradient[0] /= validGradientCount;
            gradient[1] /= validGradientCount;
            gradient[2] /= validGradientCount;
        }
        int tt = iter + 1;
        for (int j = 0; j < 3; j++) {
            m[j] = beta1 * m[j] + (1 - beta1) * gradient[j];
            v[j] = beta2 * v[j] + (1 - beta2) * gradient[j] * gradient[j];
            double m_hat = m[j] / (1 - pow(beta1, tt));
            double v_hat = v[j] / (1 - pow(beta2, tt));
            transform[j] -= learningRate * m_hat / (sqrt(v_hat) + epsilon);
        }
        if (!q)
            printf("Iteration %d, Total Error: %.6f\n", iter, totalError);
    }
    g_last_queries = nqueries;
    g_last_cp = CPcount;
    g_last_iters = iter; /* the iteration that converged, or 200 */
    PROF_ADD(3, pt1);
    if (validGradientCount > 0)
        attr->error = sqrt(totalError / validGradientCount);
    else
        attr->error = 0.0;
    Pos out;
    out.x = pos_last.x + transform[0];
    out.y = pos_last.y + transform[1];
    out.z = pos_last.z + transform[2];
    out.roll = pos_last.roll + transform[3];
    out.pitch = pos_last.pitch + transform[4];
    out.yaw = pos_last.yaw + transform[5];
    return out;
}
