/* Analysis tool (not product code): scipy's SAP (oracle/oracle.c) on Santa
 * singles blocks, reporting how far the "miss count" component m of every
 * value the solve forms strays from 0.  Every value is A * 2^32 + m * E in
 * units of 2^-31 (a wish costs -a * 2^32, a miss E = 10737418); when every
 * value has |m| <= 199, comparing the packed pairs A * K + m (K >= 400)
 * lexicographically makes exactly the decisions of the int64 solve.
 *   mrange_block(n, C, out[4]) -> out = {max|m| over u, v, spc/r, minVal}
 *   mrange_block_a(n, C, out[4], outa[4]) -> also outa = max|A| of the same
 *   values (A = the 2^32 component, a wish of rank r is A = -(100 - r))
 * returns the number of values that do not decompose with |m| < 400. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const int64_t E = 10737418;

static int mof(int64_t x, int *bad) {
  uint32_t lo = (uint32_t)(uint64_t)x;
  if (lo % E == 0 && lo / E < 400) return (int)(lo / E);
  uint64_t hi = (1ull << 32) - lo;
  if (hi % E == 0 && hi / E < 400) return -(int)(hi / E);
  ++*bad;
  return 0;
}
#define UPD(slot, x) do { int64_t xx_ = (x); int mm = mof(xx_, &bad); \
    int64_t aa = (xx_ - (int64_t)mm * E) >> 32; if (aa < 0) aa = -aa; \
    if (mm < 0) mm = -mm; if (mm > out[slot]) out[slot] = mm; \
    if (out8 && aa > out8[slot]) out8[slot] = (int)aa; } while (0)

static int *out8 = 0;  /* optional: max |A| (the 2^32 component) per slot */

int mrange_block_a(int n, const int64_t *C, int *out, int *outa);

int mrange_block(int n, const int64_t *C, int *out) {
  int64_t *u = calloc(n, 8), *v = calloc(n, 8), *spc = malloc(n * 8);
  int *path = malloc(n * 4), *c4r = malloc(n * 4), *r4c = malloc(n * 4), *rem = malloc(n * 4);
  char *SR = malloc(n), *SC = malloc(n);
  int bad = 0;
  out[0] = out[1] = out[2] = out[3] = 0;
  for (int i = 0; i < n; ++i) { c4r[i] = -1; r4c[i] = -1; path[i] = -1; }
  for (int cur = 0; cur < n; ++cur) {
    int64_t minVal = 0;
    int nrem = n;
    for (int it = 0; it < n; ++it) rem[it] = n - it - 1;
    memset(SR, 0, n); memset(SC, 0, n);
    for (int j = 0; j < n; ++j) spc[j] = INT64_MAX;
    int i = cur, sink = -1;
    while (sink == -1) {
      int index = -1;
      int64_t lowest = INT64_MAX;
      SR[i] = 1;
      for (int it = 0; it < nrem; ++it) {
        int j = rem[it];
        int64_t r = minVal + C[(int64_t)i * n + j] - u[i] - v[j];
        UPD(2, r);
        if (r < spc[j]) { path[j] = i; spc[j] = r; }
        if (spc[j] < lowest || (spc[j] == lowest && r4c[j] == -1)) { lowest = spc[j]; index = it; }
      }
      minVal = lowest;
      UPD(3, minVal);
      int j = rem[index];
      if (r4c[j] == -1) sink = j; else i = r4c[j];
      SC[j] = 1;
      rem[index] = rem[--nrem];
    }
    u[cur] += minVal;
    for (int ii = 0; ii < n; ++ii) if (SR[ii] && ii != cur) u[ii] += minVal - spc[c4r[ii]];
    for (int jj = 0; jj < n; ++jj) if (SC[jj]) v[jj] -= minVal - spc[jj];
    for (int ii = 0; ii < n; ++ii) UPD(0, u[ii]);
    for (int jj = 0; jj < n; ++jj) UPD(1, v[jj]);
    int j = sink;
    for (;;) { int ii = path[j]; r4c[j] = ii; int t = c4r[ii]; c4r[ii] = j; j = t; if (ii == cur) break; }
  }
  free(u); free(v); free(spc); free(path); free(c4r); free(r4c); free(rem); free(SR); free(SC);
  return bad;
}

int mrange_block_a(int n, const int64_t *C, int *out, int *outa) {
  outa[0] = outa[1] = outa[2] = outa[3] = 0;
  out8 = outa;
  int b = mrange_block(n, C, out);
  out8 = 0;
  return b;
}
