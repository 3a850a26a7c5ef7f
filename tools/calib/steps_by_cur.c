/* Dev analysis: per-Dijkstra step counts of scipy's SAP on one int64 cost
 * matrix (the oracle's algorithm, oracle/oracle.c, with a per-cur counter).
 * Built and loaded by tools/steps_by_cur.py. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void steps_by_cur(int n, const int64_t *C, int32_t *out) {
  int64_t *u = calloc(n, 8), *v = calloc(n, 8), *spc = malloc(n * 8);
  int *path = malloc(n * 4), *c4r = malloc(n * 4), *r4c = malloc(n * 4), *rem = malloc(n * 4);
  char *SR = malloc(n), *SC = malloc(n);
  for (int i = 0; i < n; ++i) { c4r[i] = -1; r4c[i] = -1; path[i] = -1; }
  for (int cur = 0; cur < n; ++cur) {
    int64_t minVal = 0; int nrem = n, steps = 0;
    for (int it = 0; it < n; ++it) rem[it] = n - it - 1;
    memset(SR, 0, n); memset(SC, 0, n);
    for (int j = 0; j < n; ++j) spc[j] = INT64_MAX;
    int i = cur, sink = -1;
    while (sink == -1) {
      int index = -1; int64_t lowest = INT64_MAX; SR[i] = 1; ++steps;
      for (int it = 0; it < nrem; ++it) {
        int j = rem[it]; int64_t r = minVal + C[(int64_t)i * n + j] - u[i] - v[j];
        if (r < spc[j]) { path[j] = i; spc[j] = r; }
        if (spc[j] < lowest || (spc[j] == lowest && r4c[j] == -1)) { lowest = spc[j]; index = it; }
      }
      minVal = lowest; int j = rem[index];
      if (r4c[j] == -1) sink = j; else i = r4c[j];
      SC[j] = 1; rem[index] = rem[--nrem];
    }
    u[cur] += minVal;
    for (int ii = 0; ii < n; ++ii) if (SR[ii] && ii != cur) u[ii] += minVal - spc[c4r[ii]];
    for (int jj = 0; jj < n; ++jj) if (SC[jj]) v[jj] -= minVal - spc[jj];
    int j = sink;
    for (;;) { int ii = path[j]; r4c[j] = ii; int t = c4r[ii]; c4r[ii] = j; j = t; if (ii == cur) break; }
    out[cur] = steps;
  }
  free(u); free(v); free(spc); free(path); free(c4r); free(r4c); free(rem); free(SR); free(SC);
}
