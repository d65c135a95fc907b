/*
 * slam.h — drop-in for NAV-SLAM headers/slam.h (same SLAM_attr layout, same
 * three entry points). src/main.c and src/ekf.c compile and link against
 * this header + libnavslam_<R>x<C>.so unchanged.
 *
 * The frame-level work (curvature, rigid transform, per-row KD build and the
 * per-feature nearest-neighbour batch) runs on the GPU; GPU-resident state
 * (row trees, frame buffers) lives in a side table keyed by the SLAM_attr
 * pointer, so the struct keeps the reference's layout byte for byte.
 * Single-threaded, like the reference.
 */
#ifndef SLAM_H
#define SLAM_H

#include <stddef.h>
#include "pointcloud.h"
#include "kdtree.h"

#ifndef SLAM_MAP_FRAMES
#define SLAM_MAP_FRAMES 100   /* headers/slam.h:12 */
#endif

/* headers/slam.h:10-18 */
typedef struct
{
    PointCloud globalPointCloud[SLAM_MAP_FRAMES]; /* global map, one frame per slot */
    int frameCount;
    KDNode* kdtree_lastframe[MAX_ROWS];           /* one tree per row, last frame */
    double error;                                 /* RMS registration residual */
} SLAM_attr;

/* headers/slam.h:22 / src/slam.c:134-175 */
void init_slam(SLAM_attr *attr, Pos pos, PointCloud *lidarPointCloud);

/* headers/slam.h:25 / src/slam.c:178-390 */
Pos slam_localization(SLAM_attr *attr, PointCloud *lidarPointCloud, Pos pos_predict, Pos pos_last);

/* headers/slam.h:28 / src/slam.c:393-431 */
void slam_mapping(SLAM_attr *attr, Pos pos, PointCloud *lidarPointCloud);

/* Extensions (not in the reference; a harness may ignore them) --------- */

/* The navgpu_ctx* the library runs on (include/navgpu.h), e.g. to switch
 * kernel timing on with navgpu_timing(). */
void *navslam_context(void);

/* Counts of the last slam_localization call: feature queries searched,
 * correspondences kept by the dedup (CPcount, src/slam.c:284), Adam
 * iterations run (src/slam.c:300-379). Returns 0. */
int navslam_last_frame_stats(int *queries, int *correspondences, int *iterations);

#endif
