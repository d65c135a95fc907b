// Pass statistics of the reference build (utils/kdtree.c:20-82: Lomuto quickselect, pivot = last)
// over rows written by scripts/dump_tie_rows.py; "ident" = passes whose pivot is the window maximum,
// chunksA / chunksB = 64-position chunk steps per call without / with identity runs collapsed.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static long passes_lvl[32], elems_lvl[32], calls_lvl[32], maxp_lvl[32], ident_lvl[32], minp_lvl[32];
static double *K[3];
static long costA_lvl[32], costB_lvl[32];
static long callA, callB;
static int small_(double a, double p) { return (a - p) <= 0.0; }
static int nth_el(int *P, int first, int last, int nth, int ax, int lvl) {
  int np = 0;
  calls_lvl[lvl]++;
  callA = callB = 0;
  int in_run = 0;
  while (first < last) {
    int pe = P[last]; double pk = K[ax][pe];
    int i = first, nsmall = 0;
    for (int j = first; j < last; ++j) if (K[ax][P[j]] - pk <= 0.0) nsmall++;
    int chunks = (last - first + 1 + 63) / 64;
    callA += chunks;
    if (nsmall == last - first) { ident_lvl[lvl]++; if (!in_run) { callB += chunks; in_run = 1; } }
    else { callB += chunks; in_run = 0; }
    if (nsmall == 0) minp_lvl[lvl]++;
    for (int j = first; j < last; ++j) {
      int ej = P[j];
      if (K[ax][ej] - pk <= 0.0) { P[j] = P[i]; P[i] = ej; ++i; }
    }
    P[last] = P[i]; P[i] = pe;
    np++; elems_lvl[lvl] += last - first + 1;
    if (i == nth) break;
    if (i < nth) first = i + 1; else last = i - 1;
  }
  passes_lvl[lvl] += np;
  costA_lvl[lvl] += callA; costB_lvl[lvl] += callB;
  if (np > maxp_lvl[lvl]) maxp_lvl[lvl] = np;
  return np;
}
static void build(int *P, int lo, int hi, int depth) {
  if (hi - lo < 2) return;
  int mid = lo + (hi - lo) / 2;
  nth_el(P, lo, hi - 1, mid, depth % 3, depth);
  build(P, lo, mid, depth + 1);
  build(P, mid + 1, hi, depth + 1);
}
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb");
  int rows; fread(&rows, 4, 1, f);
  for (int r = 0; r < rows; ++r) {
    int n; fread(&n, 4, 1, f);
    double *xyz = malloc(24 * (size_t)n); fread(xyz, 24, n, f);
    for (int a = 0; a < 3; ++a) { K[a] = malloc(8 * (size_t)n); for (int i = 0; i < n; ++i) K[a][i] = xyz[3 * i + a]; }
    int *P = malloc(4 * (size_t)n); for (int i = 0; i < n; ++i) P[i] = i;
    long before = passes_lvl[0];
    long e0 = elems_lvl[0];
    build(P, 0, n, 0);
    if (r < 6) printf("row %d n %d root passes %ld root elems %ld\n", r, n, passes_lvl[0] - before, elems_lvl[0] - e0);
    free(xyz); free(P); for (int a = 0; a < 3; ++a) free(K[a]);
  }
  printf("lvl calls passes/call maxpasses elems/call ident minpiv chunksA/call chunksB/call\n");
  for (int l = 0; l < 14; ++l) if (calls_lvl[l])
    printf("%2d %7ld %8.2f %5ld %10.1f %6ld %6ld %8.1f %8.1f\n", l, calls_lvl[l], (double)passes_lvl[l] / calls_lvl[l], maxp_lvl[l], (double)elems_lvl[l] / calls_lvl[l], ident_lvl[l], minp_lvl[l], (double)costA_lvl[l]/calls_lvl[l], (double)costB_lvl[l]/calls_lvl[l]);
  return 0;
}
