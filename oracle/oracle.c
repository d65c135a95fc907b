/*
 * oracle.c — CPU restatement of the NAV-SLAM hot path (see oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY: the checker and the CPU baseline, never the
 * product. Build: oracle/Makefile (-O2 -std=gnu11 -ffp-contract=off).
 * Each function cites the reference statement range it follows; the
 * floating-point expressions keep the reference's association order.
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_PI 3.14159265358979323846 /* == M_PI, glibc math.h */

/* utils/pointcloud.c:8-48 */
void orc_convert_to_pointcloud(const int *dist, int R, int C, double *pts)
{
    const double fov_h = 45.0;
    const double fov_v = 45.0;
    const double theta_step_deg = fov_h / (C - 1);
    const double phi_step_deg = fov_v / (R - 1);
    for (int j = 0; j < R; ++j) {
        for (int i = 0; i < C; ++i) {
            double distance = dist[(size_t)j * C + i];
            double *p = pts + 3 * ((size_t)j * C + i);
            if (distance <= 0) {
                p[0] = p[1] = p[2] = 0.0;
                continue;
            }
            double theta = -fov_h / 2.0 + i * theta_step_deg;
            double phi = -fov_v / 2.0 + j * phi_step_deg;
            theta = theta * ORC_PI / 180.0;
            phi = phi * ORC_PI / 180.0;
            p[0] = distance;
            p[1] = -(distance)*tan(theta);
            p[2] = -(distance)*tan(phi);
        }
    }
}

/* src/slam.c:11-61 */
void orc_extract_feature(const double *P, int R, int C, int *feature,
                         double *curv)
{
    const int w = 2; /* smooth_window, src/slam.c:12 */
    memset(feature, 0, sizeof(int) * (size_t)R * C);
    if (curv)
        memset(curv, 0, sizeof(double) * (size_t)R * C);
    for (int i = 0; i < R; i++) {
        for (int j = w; j < C - w; j++) {
            const double *cp = P + 3 * ((size_t)i * C + j);
            double sum_dist = 0.0;
            int count = 0;
            for (int k = -w; k <= w; k++) {
                if (k == 0)
                    continue;
                const double *np = P + 3 * ((size_t)i * C + j + k);
                double dx = cp[0] - np[0];
                double dy = cp[1] - np[1];
                double dz = cp[2] - np[2];
                double dist_sq = dx * dx + dy * dy + dz * dz;
                sum_dist += sqrt(dist_sq);
                count++;
            }
            double avg_dist = (count > 0) ? sum_dist / count : 0;
            double curvature = 0.0;
            if (count > 0 && avg_dist > 0) {
                double sum_var = 0.0;
                for (int k = -w; k <= w; k++) {
                    if (k == 0)
                        continue;
                    const double *np = P + 3 * ((size_t)i * C + j + k);
                    double dx = cp[0] - np[0];
                    double dy = cp[1] - np[1];
                    double dz = cp[2] - np[2];
                    double dist = sqrt(dx * dx + dy * dy + dz * dz);
                    sum_var += (dist - avg_dist) * (dist - avg_dist);
                }
                curvature = sum_var / count / (avg_dist * avg_dist + 1e-6f);
            }
            if (curvature > 0.1)
                feature[(size_t)i * C + j] = 1;
            if (curv)
                curv[(size_t)i * C + j] = curvature;
        }
    }
}

/* src/slam.c:8 (DEG2RAD) + src/slam.c:95-115 */
void orc_rotation_matrix_deg(double roll_d, double pitch_d, double yaw_d,
                             double R[9])
{
    double roll = roll_d * ORC_PI / 180.0;
    double pitch = pitch_d * ORC_PI / 180.0;
    double yaw = yaw_d * ORC_PI / 180.0;
    double cr = cos(roll);
    double sr = sin(roll);
    double cp = cos(pitch);
    double sp = sin(pitch);
    double cy = cos(yaw);
    double sy = sin(yaw);
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

/* src/slam.c:145-160 (same statements at :193-207 and :402-416) */
void orc_transform_cloud(const double *pts, size_t n, const double R[9],
                         const double t[3], double *out)
{
    for (size_t i = 0; i < n; i++) {
        double lx = pts[3 * i], ly = pts[3 * i + 1], lz = pts[3 * i + 2];
        double rx = R[0] * lx + R[1] * ly + R[2] * lz;
        double ry = R[3] * lx + R[4] * ly + R[5] * lz;
        double rz = R[6] * lx + R[7] * ly + R[8] * lz;
        out[3 * i] = t[0] + rx;
        out[3 * i + 1] = t[1] + ry;
        out[3 * i + 2] = t[2] + rz;
    }
}

/* src/slam.c:118-131 */
void orc_map_to_last(const double *g, size_t n, const double tr[3],
                     double *out)
{
    for (size_t i = 0; i < n; i++) {
        out[3 * i] = g[3 * i] - tr[0];
        out[3 * i + 1] = g[3 * i + 1] - tr[1];
        out[3 * i + 2] = g[3 * i + 2] - tr[2];
    }
}

/* src/slam.c:64-81 */
size_t orc_flatten_row(const double *row, const int *feat, int C, double *flat,
                       int *flat_col)
{
    size_t n = 0;
    for (int i = 0; i < C; ++i) {
        if (feat[i] == 1) {
            flat[3 * n] = row[3 * i];
            flat[3 * n + 1] = row[3 * i + 1];
            flat[3 * n + 2] = row[3 * i + 2];
            if (flat_col)
                flat_col[n] = i;
            n++;
        }
    }
    return n;
}

static inline void swap_pt(double *p, int *ix, size_t a, size_t b)
{
    double t0 = p[3 * a], t1 = p[3 * a + 1], t2 = p[3 * a + 2];
    p[3 * a] = p[3 * b];
    p[3 * a + 1] = p[3 * b + 1];
    p[3 * a + 2] = p[3 * b + 2];
    p[3 * b] = t0;
    p[3 * b + 1] = t1;
    p[3 * b + 2] = t2;
    if (ix) {
        int t = ix[a];
        ix[a] = ix[b];
        ix[b] = t;
    }
}

/* utils/kdtree.c:20-62. The tail recursion is a loop; same visit order. */
void orc_nth_element(double *p, int *ix, size_t first, size_t last,
                     size_t nth, int axis)
{
    while (first < last) {
        size_t i = first;
        double pivot = p[3 * last + axis];
        for (size_t j = first; j < last; j++) {
            double cmp = p[3 * j + axis] - pivot; /* kdtree.c:31-42 */
            if (cmp <= 0) {
                swap_pt(p, ix, i, j);
                i++;
            }
        }
        swap_pt(p, ix, i, last);
        if (i == nth)
            return;
        else if (i < nth)
            first = i + 1;
        else
            last = i - 1;
    }
}

/* utils/kdtree.c:65-82 */
static void kd_build_rec(double *p, int *ix, size_t n, int depth)
{
    if (n == 0)
        return;
    int axis = depth % 3; /* getAxis, kdtree.c:8-11 */
    size_t median = n / 2;
    orc_nth_element(p, ix, 0, n - 1, median, axis);
    kd_build_rec(p, ix, median, depth + 1);
    kd_build_rec(p + 3 * (median + 1), ix ? ix + median + 1 : NULL,
                 n - median - 1, depth + 1);
}

void orc_kd_build(double *p, int *ix, size_t n) { kd_build_rec(p, ix, n, 0); }

/* utils/kdtree.c:110-152 over the implicit tree of orc_kd_build */
static void kd_nn_rec(const double *p, size_t lo, size_t hi, const double *q,
                      int depth, long *best_i, double *best)
{
    if (lo >= hi)
        return;
    size_t mid = lo + (hi - lo) / 2;
    const double *np = p + 3 * mid;
    /* euclideanDistance(root->point, *target), kdtree.c:14-17; gcc folds
     * pow(v, 2) to v*v. */
    double dx = np[0] - q[0], dy = np[1] - q[1], dz = np[2] - q[2];
    double dist = sqrt(dx * dx + dy * dy + dz * dz);
    if (dist < *best) {
        *best = dist;
        *best_i = (long)mid;
    }
    int axis = depth % 3;
    int go_left = (axis == 0 && q[0] < np[0]) || (axis == 1 && q[1] < np[1]) ||
                  (axis == 2 && q[2] < np[2]);
    size_t nlo, nhi, flo, fhi;
    if (go_left) {
        nlo = lo; nhi = mid; flo = mid + 1; fhi = hi;
    } else {
        nlo = mid + 1; nhi = hi; flo = lo; fhi = mid;
    }
    kd_nn_rec(p, nlo, nhi, q, depth + 1, best_i, best);
    double diff = axis == 0 ? q[0] - np[0] : axis == 1 ? q[1] - np[1]
                                                       : q[2] - np[2];
    if (fabs(diff) < *best)
        kd_nn_rec(p, flo, fhi, q, depth + 1, best_i, best);
}

void orc_kd_nn(const double *tree, size_t n, const double q[3], long *out_pos,
               double *out_dist)
{
    long bi = -1;
    double bd = INFINITY;
    kd_nn_rec(tree, 0, n, q, 0, &bi, &bd);
    *out_pos = bi;
    *out_dist = bd;
}

void orc_rows_match(const double *src, const double *tgt, int R, int C,
                    int *src_mask, int *tgt_mask, int *nn_idx, double *nn_dist)
{
    size_t N = (size_t)R * C;
    int *sm = malloc(sizeof(int) * N), *tm = malloc(sizeof(int) * N);
    double *flat = malloc(sizeof(double) * 3 * (size_t)C);
    int *fcol = malloc(sizeof(int) * (size_t)C);
    orc_extract_feature(src, R, C, sm, NULL);
    orc_extract_feature(tgt, R, C, tm, NULL);
    for (int r = 0; r < R; r++) {
        size_t n = orc_flatten_row(tgt + 3 * (size_t)r * C, tm + (size_t)r * C,
                                   C, flat, fcol);
        orc_kd_build(flat, fcol, n);
        for (int c = 0; c < C; c++) {
            size_t g = (size_t)r * C + c;
            nn_idx[g] = -1;
            nn_dist[g] = INFINITY;
            if (sm[g] != 1)
                continue;
            long pos;
            double d;
            orc_kd_nn(flat, n, src + 3 * g, &pos, &d);
            if (pos >= 0) {
                /* the reference returns the Point (kdtree.c:121); its index
                 * is the lowest column among the row's features holding
                 * exactly those coordinates (bitwise), so duplicated points
                 * name one canonical index whichever the tree visits first */
                int col = fcol[pos];
                for (size_t p = 0; p < n; p++)
                    if (memcmp(flat + 3 * p, flat + 3 * pos, 3 * sizeof(double)) == 0 &&
                        fcol[p] < col)
                        col = fcol[p];
                nn_idx[g] = r * C + col;
                nn_dist[g] = d;
            }
        }
    }
    if (src_mask)
        memcpy(src_mask, sm, sizeof(int) * N);
    if (tgt_mask)
        memcpy(tgt_mask, tm, sizeof(int) * N);
    free(sm);
    free(tm);
    free(flat);
    free(fcol);
}

void orc_knn_brute(const double *tgt, size_t nt, const double *qs, size_t nq,
                   int k, int *oi, double *od)
{
    for (size_t q = 0; q < nq; q++) {
        int *bi = oi + q * (size_t)k;
        double *bd = od + q * (size_t)k;
        for (int s = 0; s < k; s++) {
            bi[s] = -1;
            bd[s] = INFINITY;
        }
        const double *qp = qs + 3 * q;
        int have = 0;
        for (size_t t = 0; t < nt; t++) {
            const double *tp = tgt + 3 * t;
            double dx = tp[0] - qp[0], dy = tp[1] - qp[1], dz = tp[2] - qp[2];
            double d = sqrt(dx * dx + dy * dy + dz * dz);
            /* as the reference 1-NN (kdtree.c:117, best starts at INFINITY):
             * an infinite or NaN distance is never a neighbour */
            if (!(d < INFINITY))
                continue;
            /* indices ascend, so an equal distance never displaces */
            if (have == k && !(d < bd[k - 1]))
                continue;
            int s = have < k ? have : k - 1;
            while (s > 0 && d < bd[s - 1]) {
                bd[s] = bd[s - 1];
                bi[s] = bi[s - 1];
                s--;
            }
            bd[s] = d;
            bi[s] = (int)t;
            if (have < k)
                have++;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* src/slam.c:134-431 with runtime dims. Correspondence buffers are sized
 * R*C (the reference's fixed result[100] overflows past 100, slam.c:214). */
struct orc_slam {
    int R, C;
    double *tree;   /* R*C*3: row r's tree at offset r*C */
    int *tcol;      /* R*C   */
    size_t *tn;     /* R     */
    double *global; /* R*C*3 last global frame */
    int frameCount;
    double error;
};

orc_slam *orc_slam_create(int R, int C)
{
    orc_slam *s = calloc(1, sizeof(*s));
    size_t N = (size_t)R * C;
    s->R = R;
    s->C = C;
    s->tree = calloc(3 * N, sizeof(double));
    s->tcol = calloc(N, sizeof(int));
    s->tn = calloc((size_t)R, sizeof(size_t));
    s->global = calloc(3 * N, sizeof(double));
    return s;
}

void orc_slam_destroy(orc_slam *s)
{
    if (!s)
        return;
    free(s->tree);
    free(s->tcol);
    free(s->tn);
    free(s->global);
    free(s);
}

/* src/slam.c:162-172 / 418-427: features of the lidar-frame cloud, trees over
 * the global-frame coordinates. */
static void rebuild_trees(orc_slam *s, const double *lidar)
{
    int R = s->R, C = s->C;
    int *feat = malloc(sizeof(int) * (size_t)R * C);
    orc_extract_feature(lidar, R, C, feat, NULL);
    for (int r = 0; r < R; r++) {
        double *t = s->tree + 3 * (size_t)r * C;
        int *tc = s->tcol + (size_t)r * C;
        s->tn[r] = orc_flatten_row(s->global + 3 * (size_t)r * C,
                                   feat + (size_t)r * C, C, t, tc);
        orc_kd_build(t, tc, s->tn[r]);
    }
    free(feat);
}

void orc_slam_init(orc_slam *s, const double pos[6], const double *lidar)
{
    s->frameCount = 0;
    s->error = 0.0;
    double Rm[9];
    orc_rotation_matrix_deg(pos[3], pos[4], pos[5], Rm);
    orc_transform_cloud(lidar, (size_t)s->R * s->C, Rm, pos, s->global);
    rebuild_trees(s, lidar);
    s->frameCount++;
}

void orc_slam_mapping(orc_slam *s, const double pos[6], const double *lidar)
{
    double Rm[9];
    orc_rotation_matrix_deg(pos[3], pos[4], pos[5], Rm);
    orc_transform_cloud(lidar, (size_t)s->R * s->C, Rm, pos, s->global);
    rebuild_trees(s, lidar);
    s->frameCount++;
}

typedef struct {
    double ori[3], near[3], dist;
} orc_corr;

/* src/slam.c:236-284: the correspondence list of one frame, built row by row
 * from the per-feature 1-NN results (pos[g] = tree position in row g / C, -1
 * for a non-feature or an empty row tree; dist[g] its distance). Within a
 * row, a nearest point equal in x, y and z (==) to an entry already listed
 * for that row replaces the entry only when strictly closer; otherwise it is
 * appended. `col` (nullable) receives the grid index of each entry's
 * current query. Returns CPcount. */
static int orc_dedup_list(const double *trees, int R, int C, const long *pos,
                          const double *dist, const double *tp, orc_corr *res, long *col)
{
    int CPcount = 0, flag = 0;
    for (int row = 0; row < R; ++row) {
        const double *tree = trees + 3 * (size_t)row * C;
        for (int col_ = 0; col_ < C; ++col_) {
            size_t g = (size_t)row * C + col_;
            /* Empty row tree: the reference reads an uninitialised Point
             * (slam.c:242-252, undefined behaviour); here the query makes no
             * correspondence. */
            if (pos[g] < 0)
                continue;
            const double *np = tree + 3 * pos[g];
            double bestDist = dist[g];
            if (flag == CPcount) {
                memcpy(res[CPcount].ori, tp + 3 * g, 24);
                memcpy(res[CPcount].near, np, 24);
                res[CPcount].dist = bestDist;
                if (col)
                    col[CPcount] = (long)g;
                CPcount++;
                continue;
            }
            int found = 0;
            for (int i = flag; i < CPcount; i++) {
                if (res[i].near[0] == np[0] && res[i].near[1] == np[1] &&
                    res[i].near[2] == np[2]) {
                    if (res[i].dist > bestDist) {
                        memcpy(res[i].ori, tp + 3 * g, 24);
                        memcpy(res[i].near, np, 24);
                        res[i].dist = bestDist;
                        if (col)
                            col[i] = (long)g;
                    }
                    found = 1;
                    break;
                }
            }
            if (!found) {
                memcpy(res[CPcount].ori, tp + 3 * g, 24);
                memcpy(res[CPcount].near, np, 24);
                res[CPcount].dist = bestDist;
                if (col)
                    col[CPcount] = (long)g;
                CPcount++;
            }
        }
        flag = CPcount;
    }
    return CPcount;
}

int orc_rows_dedup(const double *trees, int R, int C, const long *pos, const double *dist,
                   const double *ori, double *out_ori, double *out_near, double *out_dist,
                   long *out_grid)
{
    size_t N = (size_t)R * C;
    orc_corr *res = malloc(sizeof(orc_corr) * (N ? N : 1));
    int n = orc_dedup_list(trees, R, C, pos, dist, ori, res, out_grid);
    for (int i = 0; i < n; i++) {
        memcpy(out_ori + 3 * (size_t)i, res[i].ori, 24);
        memcpy(out_near + 3 * (size_t)i, res[i].near, 24);
        out_dist[i] = res[i].dist;
    }
    free(res);
    return n;
}

void orc_slam_localization(orc_slam *s, const double *lidar,
                           const double pred[6], const double last[6],
                           double out[6], int *iters_out, int *ncorr_out)
{
    int R = s->R, C = s->C;
    size_t N = (size_t)R * C;
    double Rm[9];
    orc_rotation_matrix_deg(pred[3], pred[4], pred[5], Rm);
    int *feature = malloc(sizeof(int) * N);
    orc_extract_feature(lidar, R, C, feature, NULL);
    double transform[6]; /* compute_posdiff, slam.c:84-92 */
    for (int i = 0; i < 6; i++)
        transform[i] = pred[i] - last[i];
    double *tp = malloc(sizeof(double) * 3 * N);
    double *ql = malloc(sizeof(double) * 3 * N);
    orc_transform_cloud(lidar, N, Rm, pred, tp);
    orc_map_to_last(tp, N, transform, ql);

    orc_corr *res = malloc(sizeof(orc_corr) * (N ? N : 1));
    long *pos = malloc(sizeof(long) * (N ? N : 1));
    double *bd = malloc(sizeof(double) * (N ? N : 1));
    int CPcount = 0;
    double learningRate = 0.1, tolerance = 1e-6;
    double previousTotalError = 0, totalError = 0;
    int validGradientCount = 0;
    double m[3] = {0, 0, 0}, v[3] = {0, 0, 0};
    double beta1 = 0.9, beta2 = 0.999, epsilon = 1e-8;
    int iter;
    for (iter = 0; iter < 200; ++iter) {
        if (iter % 200 == 0) { /* slam.c:233-284 */
            for (int row = 0; row < R; ++row)
                for (int col = 0; col < C; ++col) {
                    size_t g = (size_t)row * C + col;
                    pos[g] = -1;
                    if (feature[g] == 1)
                        orc_kd_nn(s->tree + 3 * (size_t)row * C, s->tn[row], ql + 3 * g,
                                  &pos[g], &bd[g]);
                }
            CPcount = orc_dedup_list(s->tree, R, C, pos, bd, tp, res, NULL);
        }
        /* slam.c:318-373 (ErrDistance, slam.c:301-308, has no effect) */
        double gradient[3] = {0.0, 0.0, 0.0};
        totalError = 0;
        validGradientCount = 0;
        for (int i = 0; i < CPcount; i++) {
            double dx = (res[i].ori[0] - transform[0]) - res[i].near[0];
            double dy = (res[i].ori[1] - transform[1]) - res[i].near[1];
            double dz = (res[i].ori[2] - transform[2]) - res[i].near[2];
            double dist_sq = dx * dx + dy * dy + dz * dz;
            totalError += dist_sq;
            gradient[0] -= dx;
            gradient[1] -= dy;
            gradient[2] -= dz;
            validGradientCount++;
        }
        if (fabs(totalError - previousTotalError) < tolerance)
            break;
        previousTotalError = totalError;
        if (validGradientCount > 0) {
            gradient[0] /= validGradientCount;
            gradient[1] /= validGradientCount;
            gradient[2] /= validGradientCount;
        }
        int t = iter + 1;
        for (int j = 0; j < 3; j++) {
            m[j] = beta1 * m[j] + (1 - beta1) * gradient[j];
            v[j] = beta2 * v[j] + (1 - beta2) * gradient[j] * gradient[j];
            double m_hat = m[j] / (1 - pow(beta1, t));
            double v_hat = v[j] / (1 - pow(beta2, t));
            transform[j] -= learningRate * m_hat / (sqrt(v_hat) + epsilon);
        }
    }
    if (validGradientCount > 0)
        s->error = sqrt(totalError / validGradientCount);
    else
        s->error = 0.0;
    for (int i = 0; i < 6; i++)
        out[i] = last[i] + transform[i]; /* slam.c:381-387 */
    if (iters_out)
        *iters_out = iter;
    if (ncorr_out)
        *ncorr_out = CPcount;
    free(feature);
    free(tp);
    free(ql);
    free(res);
    free(pos);
    free(bd);
}

double orc_slam_error(const orc_slam *s) { return s->error; }
int orc_slam_frame_count(const orc_slam *s) { return s->frameCount; }
size_t orc_slam_tree(const orc_slam *s, int r, const double **pts,
                     const int **cols)
{
    if (pts)
        *pts = s->tree + 3 * (size_t)r * s->C;
    if (cols)
        *cols = s->tcol + (size_t)r * s->C;
    return s->tn[r];
}
const double *orc_slam_last_global(const orc_slam *s) { return s->global; }

/* ---------------------------- src/ekf.c -------------------------------- */
void orc_ekf_init(orc_ekf *e, const double pos[6]) /* ekf.c:9-50 */
{
    memcpy(e->pos, pos, sizeof(e->pos));
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) {
            e->P[i][j] = (i == j) ? 1.0 : 0.0;
            e->Q[i][j] = 0.0;
            e->Rn[i][j] = 0.0;
        }
    for (int i = 0; i < 6; i++)
        e->Q[i][i] = 0.05;
    e->Rn[0][0] = e->Rn[1][1] = e->Rn[2][2] = 0.05;
    e->Rn[3][3] = e->Rn[4][4] = e->Rn[5][5] = 0.1;
}

void orc_ekf_predict(orc_ekf *e, const double last[6], const double cur[6])
{ /* ekf.c:53-77 */
    for (int i = 0; i < 6; i++)
        e->pos[i] += cur[i] - last[i];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++)
            e->P[i][j] += e->Q[i][j];
}

void orc_ekf_modify(orc_ekf *e, const double z[6]) /* ekf.c:80-112 */
{
    double K[6];
    for (int i = 0; i < 6; i++)
        K[i] = e->P[i][i] / (e->P[i][i] + e->Rn[i][i]);
    double y[6];
    for (int i = 0; i < 6; i++)
        y[i] = z[i] - e->pos[i];
    for (int i = 0; i < 6; i++)
        e->pos[i] += K[i] * y[i];
    for (int i = 0; i < 6; i++)
        e->P[i][i] = (1 - K[i]) * e->P[i][i];
}

void orc_ekf_update_R(orc_ekf *e, double error) /* ekf.c:114-127 */
{
    const double base_R[6] = {0.05, 0.05, 0.05, 0.1, 0.1, 0.1};
    double gain = 10.0;
    double scale = 1 + gain * error / (1 + error);
    for (int i = 0; i < 6; i++) {
        for (int j = 0; j < 6; j++)
            e->Rn[i][j] = 0.0;
        e->Rn[i][i] = base_R[i] * scale;
    }
}

/* Batch drivers for the CPU baseline: the query loop stays in C so the
 * timing measures the search, not a Python call per query. */
void orc_kd_nn_batch(const double *tree, size_t n, const double *qs, size_t nq,
                     long *out_pos, double *out_dist)
{
    for (size_t i = 0; i < nq; i++)
        orc_kd_nn(tree, n, qs + 3 * i, out_pos + i, out_dist + i);
}

/* Calls a reference-ABI nearestNeighborSearch (utils/kdtree.c:110) through a
 * function pointer for each query, with bestDist reset to INFINITY as
 * src/slam.c:243 does. */
typedef void (*orc_ref_nn_fn)(void *root, const double *target, double *result,
                              double *bestDist, int depth);
void orc_ref_nn_batch(void *fn, void *root, const double *qs, size_t nq,
                      double *out_pts, double *out_dist)
{
    orc_ref_nn_fn f = (orc_ref_nn_fn)fn;
    for (size_t i = 0; i < nq; i++) {
        double best = INFINITY;
        f(root, qs + 3 * i, out_pts + 3 * i, &best, 0);
        out_dist[i] = best;
    }
}
