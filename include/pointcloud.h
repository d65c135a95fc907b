/*
 * pointcloud.h — drop-in for NAV-SLAM utils/pointcloud.h (same types, same
 * function signatures, same struct layout), served by libnavslam_<R>x<C>.so.
 *
 * Difference: the grid dims are overridable. The reference #defines
 * MAX_ROWS/MAX_COLS unconditionally (utils/pointcloud.h:9-10, L5 8x8); here
 * they default to the same values but may be set with -DMAX_ROWS=.. -DMAX_COLS=..
 * The shim library must be built with the same dims as its callers (the
 * structs embed them), exactly as the reference bakes them in at compile time.
 */
#ifndef POINTCLOUD_H
#define POINTCLOUD_H

#define L5_MAX_ROWS 8
#define L5_MAX_COLS 8
#define L9_MAX_ROWS 54
#define L9_MAX_COLS 42
#ifndef MAX_ROWS
#define MAX_ROWS L5_MAX_ROWS
#endif
#ifndef MAX_COLS
#define MAX_COLS L5_MAX_COLS
#endif

/* L5 depth frame: timestamp + depth grid in mm (utils/pointcloud.h:13-17) */
typedef struct
{
    int ToF_timestamps;
    int ToF_distances[MAX_ROWS][MAX_COLS];
} L5_LidarDataFrame;

/* IMU frame: angles in degrees, position in metres (utils/pointcloud.h:20-29) */
typedef struct
{
    int IMU_timestamps;
    double roll;
    double pitch;
    double yaw;
    double x;
    double y;
    double z;
} IMUDataFrame;

/* Pose: mm and degrees (utils/pointcloud.h:32-35) */
typedef struct
{
    double x, y, z, roll, pitch, yaw;
} Pos;

/* 3-D point in mm (utils/pointcloud.h:39-44) */
typedef struct
{
    double x;
    double y;
    double z;
} Point;

/* One frame of points on the sensor grid (utils/pointcloud.h:47-51) */
typedef struct
{
    int ToF_timestamps;
    Point ToF_position[MAX_ROWS][MAX_COLS];
} PointCloud;

/* utils/pointcloud.c:8-48 — runs on the GPU (navgpu_project) */
void convertToPointCloud(int distances[MAX_ROWS][MAX_COLS], Point pointCloud[MAX_ROWS][MAX_COLS]);

/* utils/pointcloud.c:50-58 — host printf, same format */
void printPointCloud(PointCloud pointcloud);

#endif
