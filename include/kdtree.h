/*
 * kdtree.h — drop-in for NAV-SLAM utils/kdtree.h (same types and signatures).
 *
 * buildKDTree permutes the caller's array exactly as the reference does
 * (the permutation is computed on the GPU, navgpu_kd_build) and returns a
 * malloc'd linked tree over it. nearestNeighborSearch / printKDTree /
 * freeKDTree act on that host structure, as in the reference: a single
 * point query against a linked host tree has no GPU-shaped work in it. The
 * per-frame batch of queries that slam.c issues goes to the GPU behind the
 * slam.h entry points instead.
 */
#ifndef KDTREE_H
#define KDTREE_H

#include <stddef.h>
#include "pointcloud.h"

/* utils/kdtree.h:7-11 */
typedef struct KDNode {
    Point point;
    struct KDNode* left;
    struct KDNode* right;
} KDNode;

/* utils/kdtree.h:14-18 */
typedef struct {
    Point oriPoint;
    Point nearestPoint;
    double distance;
} NeighborResult;

/* utils/kdtree.c:65-82 */
KDNode* buildKDTree(Point *points, size_t numPoints, int depth);

/* utils/kdtree.c:84-91 */
void freeKDTree(KDNode* root);

/* utils/kdtree.c:110-152 */
void nearestNeighborSearch(KDNode* root, Point* target, Point* result, double* bestDist, int depth);

/* utils/kdtree.c:94-107 */
void printKDTree(KDNode* root, int depth);

#endif
