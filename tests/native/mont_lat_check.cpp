// mont29_lat (latency form, tb_fp.h) == mont29 bit for bit on random and
// top-of-range operands, for N = 1 (product and squaring) and N = 2.
// Host build: tests/test_mont_lat.py.
#include <cstdio>
#include <random>
#include "tb_fp.h"
using namespace tb;
int main() {
  std::mt19937_64 rng(1);
  int bad = 0;
  for (int it = 0; it < 200000; it++) {
    fp a, b;
    for (int i = 0; i < 12; i++) { a.l[i] = (uint32_t)rng(); b.l[i] = (uint32_t)rng(); }
    // inputs anywhere below 2^384 (the contract), incl. top values
    if (it % 7 == 0) for (int i = 0; i < 12; i++) a.l[i] = 0xffffffffu;
    uint32_t x[1][14], y[1][14], z0[1][14], z1[1][14], s0[1][14], s1[1][14];
    to29(x[0], a); to29(y[0], b);
    mont29<1, false>(z0, x, y); mont29_lat<1, false>(z1, x, y);
    mont29<1, true>(s0, x, x); mont29_lat<1, true>(s1, x, x);
    for (int i = 0; i < 14; i++) if (z0[0][i] != z1[0][i] || s0[0][i] != s1[0][i]) { bad++; break; }
    uint32_t X[2][14], Y[2][14], Z0[2][14], Z1[2][14];
    for (int i = 0; i < 14; i++) { X[0][i] = x[0][i]; X[1][i] = y[0][i]; Y[0][i] = y[0][i]; Y[1][i] = x[0][i]; }
    mont29<2, false>(Z0, X, Y); mont29_lat<2, false>(Z1, X, Y);
    for (int j = 0; j < 2; j++) for (int i = 0; i < 14; i++) if (Z0[j][i] != Z1[j][i]) { bad++; j = 2; break; }
  }
  printf("mismatches %d\n", bad);
  return bad != 0;
}
