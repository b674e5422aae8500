// Host fuzz of the device x87 emulation (zhpe-ompi_amd/csrc/mx_x87.hpp)
// against the host's real x87 `long double` arithmetic.  Built and run by
// tests/test_x87_host.py (CPU).  Prints the first mismatches and exits 1.
#define MX_X87_HOST_TEST 1
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <cmath>
#include <cfloat>
#include <random>
#include "mx_x87.hpp"
using namespace mx;

static x87 to_x(long double v) { x87 r; memset(&r, 0, sizeof r); memcpy(&r, &v, 10); return r; }
static bool same(const x87 &a, long double v) {
  x87 b = to_x(v);
  bool an = x87_isnan(a), bn = x87_isnan(b);
  if (an || bn) return an && bn && a.m == b.m && a.se == b.se;
  return a.m == b.m && a.se == b.se;
}
static long double gen(std::mt19937_64 &g) {
  long double v;
  switch (g() % 12) {
    case 10: { x87 r; memset(&r, 0, sizeof r); r.m = g(); r.se = (uint16_t)g(); memcpy(&v, &r, 10); return v; }  // any bits
    case 11: { x87 r; memset(&r, 0, sizeof r); r.m = (g() >> 1) >> (g() % 3 ? 0 : 63);   // unnormal / pseudo-NaN / pseudo-inf
               r.se = (uint16_t)((g() % 2 ? 0x7fff : 1 + g() % 0x7ffe) | ((g() & 1) << 15)); memcpy(&v, &r, 10); return v; }
    case 0: { x87 r; memset(&r, 0, sizeof r); r.m = g() | (1ull << 63); r.se = (uint16_t)(g() % 0x7fff) | ((g() & 1) << 15); memcpy(&v, &r, 10); return v; }
    case 1: { x87 r; memset(&r, 0, sizeof r); r.m = g() >> (g() % 64); r.se = (g() & 1) << 15; memcpy(&v, &r, 10); return v; }  // denormal
    case 2: return (g() & 1) ? LDBL_MAX : -LDBL_MIN * (long double)(g() % 5);
    case 3: { x87 r; memset(&r, 0, sizeof r); r.m = (1ull << 63) | (g() >> 1); r.se = 0x7fff | ((g() & 1) << 15); memcpy(&v, &r, 10); return v; }  // NaN/inf-ish
    case 4: return (long double)((int)(g() % 7) - 3);
    default: { std::uniform_real_distribution<double> u(-4, 4); long double x = u(g); return x * ldexpl(1.0L, (int)(g() % 200) - 100) + (long double)u(g) / 3.0L; }
  }
}
int main(int argc, char **argv) {
  long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 g(12345);
  int bad = 0;
  for (long i = 0; i < n && bad < 10; i++) {
    long double a = gen(g), b = gen(g);
    if (g() % 4 == 0) b = -a * (long double)(1 + (g() % 3));   // cancellation
    if (g() % 8 == 0) b = a * ldexpl(1.0L, -(int)(g() % 70));  // near-equal exponent
    x87 xa = to_x(a), xb = to_x(b);
    volatile long double s = a + b, p = a * b;
    x87 rs = x87_add(xa, xa, xb), rp = x87_mul(xa, xa, xb);
    bool gt = a > b, lt = a < b, eq = a == b;
    {  // complex product: gcc's inline expansion + __mulxc3 (Annex G) vs x87c_mul
      long double c = gen(g), d = gen(g);
      __complex__ long double P, Q;
      __real__ P = a; __imag__ P = b; __real__ Q = c; __imag__ Q = d;
      volatile __complex__ long double R = P * Q;
      x87c xp{to_x(a), to_x(b)}, xq{to_x(c), to_x(d)};
      x87c xr = x87c_mul(xp, xq);
      if (!same(xr.re, __real__ R) || !same(xr.im, __imag__ R)) {
        x87 er = to_x(__real__ R), ei = to_x(__imag__ R), xc = to_x(c), xd = to_x(d);
        printf("CMUL MISMATCH (%04x:%016llx %04x:%016llx)*(%04x:%016llx %04x:%016llx) got %04x:%016llx %04x:%016llx "
               "exp %04x:%016llx %04x:%016llx\n", xp.re.se, (unsigned long long)xp.re.m, xp.im.se,
               (unsigned long long)xp.im.m, xc.se, (unsigned long long)xc.m, xd.se, (unsigned long long)xd.m,
               xr.re.se, (unsigned long long)xr.re.m, xr.im.se, (unsigned long long)xr.im.m, er.se,
               (unsigned long long)er.m, ei.se, (unsigned long long)ei.m);
        bad++;
      }
    }
    if (!same(rs, s) || !same(rp, p) || (xa > xb) != gt || (xa < xb) != lt || (xa == xb) != eq) {
      x87 es = to_x(s), ep = to_x(p);
      printf("MISMATCH a=%04x:%016llx b=%04x:%016llx add got %04x:%016llx exp %04x:%016llx "
             "mul got %04x:%016llx exp %04x:%016llx cmp %d%d%d/%d%d%d\n",
             xa.se, (unsigned long long)xa.m, xb.se, (unsigned long long)xb.m, rs.se, (unsigned long long)rs.m,
             es.se, (unsigned long long)es.m, rp.se, (unsigned long long)rp.m, ep.se, (unsigned long long)ep.m,
             (xa > xb), (xa < xb), (xa == xb), gt, lt, eq);
      bad++;
    }
  }
  printf("%s after %ld cases\n", bad ? "FAIL" : "OK", n);
  return bad ? 1 : 0;
}
