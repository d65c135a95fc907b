/*
 * asan_driver.c — TEST INFRASTRUCTURE (SURVEY.md §5 "ASan/UBSan on the host
 * restatement"): drives the oracle restatement (oracle.c, oracle_grid.c) and
 * the jansson subset the K1 driver reads its frames through
 * (nav-slam_amd/jansson/jansson_mini.c) under AddressSanitizer +
 * UndefinedBehaviorSanitizer (oracle/Makefile `asan`, tests/test_sanitizers.py).
 *
 * It checks results too (exit 1 on a mismatch), but its purpose is memory and
 * UB safety on edge inputs: empty and single-point trees, duplicates, NaN and
 * infinite coordinates, rows without features, k > n, and hostile JSON
 * (truncated documents, deep nesting, bad escapes, huge numbers).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jansson.h"
#include "oracle.h"

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static double urand(void) {  /* splitmix64 -> [0, 1) */
    uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    return (double)(z >> 11) * 0x1p-53;
}

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "asan_driver: check failed at %d: %s\n", __LINE__, #c); \
            ++fails;                                                    \
        }                                                               \
    } while (0)

static void cloud(double *p, size_t n, double scale, int integer) {
    for (size_t i = 0; i < 3 * n; ++i) {
        p[i] = urand() * scale;
        if (integer) p[i] = floor(p[i]);
    }
}

/* R1/R2/R3: projection, features, rigid transform on a small grid, with
 * zero depths (the (0,0,0) points) and a constant row (avg_dist == 0) */
static void test_features(void) {
    enum { R = 6, C = 40 };
    int depth[R * C];
    for (int i = 0; i < R * C; ++i) depth[i] = (int)(urand() * 3000) - 200;
    for (int c = 0; c < C; ++c) depth[2 * C + c] = 1000;
    double pts[R * C * 3], curv[R * C], out[R * C * 3], back[R * C * 3];
    int feat[R * C];
    orc_convert_to_pointcloud(depth, R, C, pts);
    orc_extract_feature(pts, R, C, feat, curv);
    for (int i = 0; i < R * C; ++i) CHECK(feat[i] == 0 || feat[i] == 1);
    double Rm[9], t[3] = {10, -20, 30};
    orc_rotation_matrix_deg(3.0, -7.5, 91.0, Rm);
    orc_transform_cloud(pts, R * C, Rm, t, out);
    orc_map_to_last(out, R * C, t, back);
    double flat[C * 3];
    int col[C];
    for (int r = 0; r < R; ++r) {
        size_t n = orc_flatten_row(pts + 3 * r * C, feat + r * C, C, flat, col);
        CHECK(n <= C);
    }
}

/* R5/R6: trees of 0, 1, 2, duplicate, NaN/inf and random point sets against
 * the brute force (distances equal; the tree's first-visited tie rule may
 * pick another of several equidistant points) */
static void test_kdtree(void) {
    const size_t sizes[] = {0, 1, 2, 3, 17, 300, 2500};
    for (size_t si = 0; si < sizeof sizes / sizeof *sizes; ++si) {
        for (int kind = 0; kind < 4; ++kind) {
            const size_t n = sizes[si];
            double *p = malloc(3 * n * sizeof(double) + 8);
            int *idx = malloc(n * sizeof(int) + 4);
            cloud(p, n, 100.0, kind == 1);
            if (kind == 2)
                for (size_t i = 0; i < 3 * n; ++i) p[i] = floor(p[i] / 40.0);  /* duplicates */
            if (kind == 3 && n > 4) {
                p[0] = NAN;
                p[4] = INFINITY;
                p[8] = -INFINITY;
            }
            for (size_t i = 0; i < n; ++i) idx[i] = (int)i;
            orc_kd_build(p, idx, n);
            for (int q = 0; q < 20; ++q) {
                double qv[3] = {urand() * 110 - 5, urand() * 110 - 5, urand() * 110 - 5};
                long pos;
                double d;
                orc_kd_nn(p, n, qv, &pos, &d);
                CHECK(n > 0 ? pos >= 0 && pos < (long)n : pos == -1);
                if (kind != 3 && n > 0) {
                    int bi;
                    double bd;
                    orc_knn_brute(p, n, qv, 1, 1, &bi, &bd);
                    CHECK(bd == d);
                }
            }
            free(p);
            free(idx);
        }
    }
}

/* per-row mode and the correspondence list on rows with and without features */
static void test_rows(void) {
    enum { R = 8, C = 64 };
    static double src[R * C * 3], tgt[R * C * 3], nd[R * C];
    static int sm[R * C], tm[R * C], ni[R * C];
    for (int integer = 0; integer < 2; ++integer) {
        cloud(src, R * C, 2000.0, integer);
        cloud(tgt, R * C, 2000.0, integer);
        for (int c = 0; c < C; ++c)  /* a flat row: no features */
            for (int a = 0; a < 3; ++a) tgt[3 * (3 * C + c) + a] = src[3 * (3 * C + c) + a] = 5.0;
        orc_rows_match(src, tgt, R, C, sm, tm, ni, nd);
        for (int g = 0; g < R * C; ++g) CHECK(ni[g] >= -1 && ni[g] < R * C);
    }
}

/* global k-NN: the grid checker against the brute force, k > n included */
static void test_knn(void) {
    const size_t nts[] = {0, 5, 3000};
    for (size_t ti = 0; ti < 3; ++ti) {
        const size_t nt = nts[ti], nq = 400;
        const int k = 8;
        double *t = malloc(3 * nt * sizeof(double) + 8), *q = malloc(3 * nq * sizeof(double));
        cloud(t, nt, 500.0, ti == 2);
        cloud(q, nq, 520.0, 0);
        int *bi = malloc(nq * k * sizeof(int)), *gi = malloc(nq * k * sizeof(int));
        double *bd = malloc(nq * k * sizeof(double)), *gd = malloc(nq * k * sizeof(double));
        orc_knn_brute(t, nt, q, nq, k, bi, bd);
        orc_knn_grid(t, nt, q, nq, k, gi, gd);
        CHECK(memcmp(bi, gi, nq * k * sizeof(int)) == 0);
        CHECK(memcmp(bd, gd, nq * k * sizeof(double)) == 0);
        free(t);
        free(q);
        free(bi);
        free(gi);
        free(bd);
        free(gd);
    }
}

/* src/slam.c:134-431 frame loop over a short synthetic stream */
static void test_slam(void) {
    enum { R = 8, C = 16 };
    orc_slam *s = orc_slam_create(R, C);
    double lidar[R * C * 3], pos[6] = {0, 0, 0, 0, 0, 0}, last[6] = {0}, out[6];
    for (int f = 0; f < 6; ++f) {
        for (int i = 0; i < R * C; ++i) {
            const double az = (i % C) * 0.2, el = (i / C) * 0.05;
            const double r = 1500 + 300 * sin(3 * az + f * 0.1) + urand() * 5;
            lidar[3 * i] = r * cos(az) + 20 * f;
            lidar[3 * i + 1] = r * sin(az);
            lidar[3 * i + 2] = r * el;
        }
        if (f == 0) {
            orc_slam_init(s, pos, lidar);
            continue;
        }
        int iters, ncorr;
        orc_slam_localization(s, lidar, last, last, out, &iters, &ncorr);
        orc_slam_mapping(s, out, lidar);
        memcpy(last, out, sizeof out);
        CHECK(iters >= 0 && ncorr >= 0);
    }
    orc_slam_destroy(s);
    orc_ekf e;
    orc_ekf_init(&e, pos);
    orc_ekf_predict(&e, pos, last);
    orc_ekf_update_R(&e, 3.5);
    orc_ekf_modify(&e, last);
}

/* the jansson subset on well-formed and hostile documents */
static void test_json(void) {
    json_error_t err;
    const char *good = "[{\"time_main\": 1000, \"distance\": [1, -2, 3000000000],"
                       " \"params\": [0.5, -1e-300, 1.7976931348623157e308, 0, 1, 2]},"
                       " {\"s\": \"\\u00e9\\ud83d\\ude00\\\\\\\"\", \"n\": null, \"b\": [true, false]}]";
    json_t *j = json_loads(good, 0, &err);
    CHECK(j != NULL);
    if (j) {
        json_t *f0 = json_array_get(j, 0);
        json_t *d = json_object_get(f0, "distance");
        CHECK(json_array_size(d) == 3);
        CHECK(json_integer_value(json_array_get(d, 2)) == 3000000000LL);
        CHECK(json_array_get(d, 3) == NULL);
        CHECK(json_real_value(json_array_get(json_object_get(f0, "params"), 2)) ==
              1.7976931348623157e308);
        CHECK(json_string_value(json_object_get(json_array_get(j, 1), "s")) != NULL);
        CHECK(json_object_get(f0, "missing") == NULL);
        json_delete(j);
    }
    const char *bad[] = {"", "[", "]", "{", "{\"a\"", "{\"a\":", "{\"a\":1,}", "[1,]", "[01]",
                         "[1e999]", "[-]", "[1.]", "[\"\\x\"]", "[\"\\u12\"]", "[\"\\ud800\"]",
                         "[\"abc", "[tru]", "[nul]", "\"\\u0000\"", "[1] 2", "{1:2}",
                         "[99999999999999999999999]", "\xff\xfe", "[\"\xc3\"]"};
    for (size_t i = 0; i < sizeof bad / sizeof *bad; ++i) {
        json_t *b = json_loads(bad[i], 0, &err);
        if (b) json_delete(b);
    }
    /* deep nesting, both unterminated and balanced */
    const int depth = 5000;
    char *deep = malloc(2 * depth + 1);
    for (int i = 0; i < depth; ++i) deep[i] = '[';
    for (int i = 0; i < depth; ++i) deep[depth + i] = ']';
    deep[2 * depth] = 0;
    json_t *dj = json_loads(deep, 0, &err);
    if (dj) json_delete(dj);
    deep[depth + 10] = 0;
    dj = json_loads(deep, 0, &err);
    CHECK(dj == NULL);
    free(deep);
    /* a long array of reals through json_loadf */
    FILE *fp = tmpfile();
    if (fp) {
        fputc('[', fp);
        for (int i = 0; i < 20000; ++i) fprintf(fp, "%s%.17g", i ? "," : "", urand() * 1e6 - 5e5);
        fputc(']', fp);
        rewind(fp);
        json_t *a = json_loadf(fp, 0, &err);
        CHECK(a != NULL && json_array_size(a) == 20000);
        if (a) json_delete(a);
        fclose(fp);
    }
}

int main(void) {
    test_features();
    test_kdtree();
    test_rows();
    test_knn();
    test_slam();
    test_json();
    if (fails) {
        fprintf(stderr, "asan_driver: %d check(s) failed\n", fails);
        return 1;
    }
    printf("asan_driver ok\n");
    return 0;
}
