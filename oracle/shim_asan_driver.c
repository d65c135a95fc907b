/*
 * shim_asan_driver.c — TEST INFRASTRUCTURE ONLY. Drives the drop-in shim
 * (nav-slam_amd/csrc/navslam_shim.c, the reference's slam.h / kdtree.h /
 * pointcloud.h over libnavgpu) on the CPU stub of libnavgpu
 * (navgpu_cpu_stub.c) under -fsanitize=address,undefined: the L5/L9 frame
 * loop of src/main.c (init_slam, then slam_localization + slam_mapping per
 * frame) past the 100-frame map ring, in the bit-exact mode (poses compared
 * with the oracle's frame loop, oracle.c orc_slam_*) and in the fast mode
 * (NAVSLAM_ADAM=fast), with host trees on and off; plus buildKDTree /
 * nearestNeighborSearch / freeKDTree on a point set and a caller-linked
 * tree. Prints "shim_asan ok" when every check passed.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "slam.h"

#define NF 130 /* frames: past SLAM_MAP_FRAMES (headers/slam.h:12) */

static void depth_frame(int f, int d[MAX_ROWS][MAX_COLS])
{
    for (int r = 0; r < MAX_ROWS; r++)
        for (int c = 0; c < MAX_COLS; c++)
            d[r][c] = 900 + (int)(300 * sin(0.7 * r + 0.05 * f) + 200 * cos(0.45 * c - 0.03 * f)) +
                      (r * 7 + c * 13 + f * 3) % 17;
}

static int fail(const char *what, int f)
{
    fprintf(stderr, "shim_asan: %s at frame %d\n", what, f);
    return 1;
}

static int run_loop(int exact)
{
    SLAM_attr *attr = calloc(1, sizeof(SLAM_attr));
    PointCloud *pc = calloc(1, sizeof(PointCloud));
    orc_slam *os = exact ? orc_slam_create(MAX_ROWS, MAX_COLS) : NULL;
    static int depth[MAX_ROWS][MAX_COLS];
    Pos last = {0, 0, 0, 0, 0, 0};
    double olast[6] = {0, 0, 0, 0, 0, 0};
    int bad = 0;
    for (int f = 0; f < NF && !bad; f++) {
        depth_frame(f, depth);
        convertToPointCloud(depth, pc->ToF_position);
        const double *pts = &pc->ToF_position[0][0].x;
        if (f == 0) {
            init_slam(attr, last, pc);
            if (os)
                orc_slam_init(os, olast, pts);
            continue;
        }
        Pos pred = last;
        pred.x += 1.5;
        pred.yaw += 0.2;
        Pos est = slam_localization(attr, pc, pred, last);
        if (os) {
            double opred[6] = {pred.x, pred.y, pred.z, pred.roll, pred.pitch, pred.yaw};
            double oout[6];
            int it, nc;
            orc_slam_localization(os, pts, opred, olast, oout, &it, &nc);
            const double got[6] = {est.x, est.y, est.z, est.roll, est.pitch, est.yaw};
            if (memcmp(got, oout, sizeof(got)) != 0)
                bad |= fail("pose differs from the oracle", f);
            if (attr->error != orc_slam_error(os))
                bad |= fail("error differs from the oracle", f);
            orc_slam_mapping(os, oout, pts);
            memcpy(olast, oout, sizeof(olast));
        }
        slam_mapping(attr, est, pc);
        for (int r = 0; r < MAX_ROWS; r++) {  /* walk the handed-out trees */
            KDNode *stack[64];
            int sp = 0;
            if (attr->kdtree_lastframe[r])
                stack[sp++] = attr->kdtree_lastframe[r];
            while (sp > 0) {
                KDNode *n = stack[--sp];
                if (!isfinite(n->point.x))
                    bad |= fail("non-finite tree point", f);
                if (n->left && sp < 64)
                    stack[sp++] = n->left;
                if (n->right && sp < 64)
                    stack[sp++] = n->right;
            }
        }
        last = est;
    }
    if (os)
        orc_slam_destroy(os);
    free(pc);
    free(attr);
    return bad;
}

static int run_kdtree(void)
{
    enum { N = 777 };
    Point *p = malloc(sizeof(Point) * N);
    for (int i = 0; i < N; i++) {
        p[i].x = (i * 37) % 101 - 50.0;
        p[i].y = (i * 53) % 97 * 0.5;
        p[i].z = (i * 11) % 13;
    }
    KDNode *root = buildKDTree(p, N, 0);
    int bad = 0;
    for (int q = 0; q < 50; q++) {
        Point t = {q * 2.0 - 50.0, q * 0.7, q % 13 * 1.0}, res = {0, 0, 0};
        double best = INFINITY;
        nearestNeighborSearch(root, &t, &res, &best, 0);
        double bf = INFINITY;
        for (int i = 0; i < N; i++) {
            const double dx = p[i].x - t.x, dy = p[i].y - t.y, dz = p[i].z - t.z;
            const double d = sqrt(dx * dx + dy * dy + dz * dz);
            bf = d < bf ? d : bf;
        }
        if (best != bf)
            bad |= fail("nearestNeighborSearch distance differs from brute force", q);
    }
    freeKDTree(root);
    /* a tree the caller linked node by node (freeKDTree frees it) */
    KDNode *a = malloc(sizeof(KDNode)), *b = malloc(sizeof(KDNode));
    a->point = p[0];
    b->point = p[1];
    a->left = b;
    a->right = NULL;
    b->left = b->right = NULL;
    freeKDTree(a);
    free(p);
    return bad;
}

int main(void)
{
    int bad = run_kdtree();
    setenv("NAVSLAM_QUIET", "1", 1);
    bad |= run_loop(1);                /* exact mode, host trees */
    setenv("NAVSLAM_HOST_TREES", "0", 1);
    bad |= run_loop(1);                /* exact mode, no host trees */
    setenv("NAVSLAM_ADAM", "fast", 1);
    bad |= run_loop(0);                /* fast mode */
    unsetenv("NAVSLAM_HOST_TREES");
    bad |= run_loop(0);
    if (bad)
        return 1;
    printf("shim_asan ok\n");
    return 0;
}
