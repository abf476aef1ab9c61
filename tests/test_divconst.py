"""CPU check of the kernel's constant-division trick (swrt_kernels.hpp
div_const): q0 = x*RN(1/d); r = fma(-q0, d, x); q = fma(r, RN(1/d), q0)
must equal the IEEE quotient x/d for d = 3, 5 over the whole exponent range
used by the Lagrange weights (and far beyond)."""
import os
import subprocess

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t nxt(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rnd(void) {  /* random finite double with exponent in [-300, 300] */
  uint64_t m = nxt() & ((1ull << 52) - 1);
  int e = (int)(nxt() % 601) - 300;
  uint64_t bits = ((uint64_t)(e + 1023) << 52) | m | ((nxt() & 1ull) << 63);
  double d; memcpy(&d, &bits, 8); return d;
}
int main(void) {
  const double R3 = 1.0 / 3.0, R5 = 1.0 / 5.0;
  long bad = 0;
  for (long i = 0; i < 20000000; ++i) {
    double x = rnd();
    double q0 = x * R3, r = fma(-q0, 3.0, x), q = fma(r, R3, q0);
    if (q != x / 3.0) ++bad;
    q0 = x * R5; r = fma(-q0, 5.0, x); q = fma(r, R5, q0);
    if (q != x / 5.0) ++bad;
  }
  /* adversarial: mantissas that are multiples of 3/5 (exact quotients) */
  for (long m = 1; m < 3000000; ++m) {
    double x = (double)m * 3.0, y = (double)m * 5.0;
    double q0 = x * R3, r = fma(-q0, 3.0, x), q = fma(r, R3, q0);
    if (q != x / 3.0) ++bad;
    q0 = y * R5; r = fma(-q0, 5.0, y); q = fma(r, R5, q0);
    if (q != y / 5.0) ++bad;
  }
  printf("%ld\n", bad);
  return bad != 0;
}
"""


def test_markstein_division_by_3_and_5_is_correctly_rounded(tmp_path):
    c = tmp_path / "divc.c"
    c.write_text(SRC)
    exe = tmp_path / "divc"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "0", out.stdout


WEIGHTS = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 0x2545F4914F6CDD1Dull;
static uint64_t nxt(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double divc(double x, int d) {  /* the kernel's div_const: exact for |d| in {1,2,4}, Markstein for 3, 5 */
  int a = d < 0 ? -d : d; double q;
  if (a == 1 || a == 2 || a == 4) q = x * (1.0 / a);
  else { double R = 1.0 / a, q0 = x * R, r = fma(-q0, (double)a, x); q = fma(r, R, q0); }
  return d < 0 ? -q : q;
}
static int oddp(int d) { d = d < 0 ? -d : d; while (d % 2 == 0) d /= 2; return d; }
static double scl(int d) { double c = d < 0 ? -1.0 : 1.0; d = d < 0 ? -d : d; while (d % 2 == 0) { d /= 2; c *= 0.5; } return c; }
int main(void) {
  long bad = 0;
  for (long n = 0; n < 4000000; ++n) {
    double a;
    if (n < 64) a = (double)n / 64.0; else { uint64_t m = nxt() >> 12; a = (double)m / 4503599627370496.0; }
    double bump = (n & 1) ? 1e-10 : 1e-13;
    double t[6];
    for (int j = -2; j <= 3; ++j) t[j + 2] = (a - (double)j) + bump;
    for (int i = -2; i <= 3; ++i) {
      double w = 1.0, v = 1.0, c = 1.0;
      for (int j = -2; j <= 3; ++j) {
        if (j == i) continue;
        w = w * t[j + 2] / (double)(j - i);   /* interpolate.m:37 (IEEE division) */
        v = divc(v * t[j + 2], oddp(j - i));  /* odd part in the running product */
        c *= scl(j - i);
      }
      v = v * c;
      if (memcmp(&v, &w, 8) != 0) ++bad;
    }
  }
  printf("%ld\n", bad);
  return bad != 0;
}
"""


def test_lagrange_weights_with_hoisted_powers_of_two_are_bit_exact(tmp_path):
    """swrt_kernels.hpp lagrange_wi: the signs and powers of two of the five
    divisors applied once after the running product of the odd parts give
    interpolate.m's weights bit for bit (4e6 offsets a in [0, 1), both bumps,
    all six weights, including the grid points a = k/64)."""
    c = tmp_path / "w.c"
    c.write_text(WEIGHTS)
    exe = tmp_path / "w"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "0", out.stdout


DRIFT = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 0x2545F4914F6CDD1Dull;
static uint64_t nxt(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rnd(int lo, int hi) {  /* random double, exponent in [lo, hi], random sign */
  uint64_t m = nxt() & ((1ull << 52) - 1);
  int e = lo + (int)(nxt() % (uint64_t)(hi - lo + 1));
  uint64_t bits = ((uint64_t)(e + 1023) << 52) | m | ((nxt() & 1ull) << 63);
  double d; memcpy(&d, &bits, 8); return d;
}
static int same(double a, double b) { return memcmp(&a, &b, 8) == 0; }
/* swrt_kernels.hpp div_rn_z with rb = RN(1/b) */
static double div_rn_z(double a, double b, double rb) {
  double q0 = a * rb, r = fma(q0, b, -a);
  return fma(-r, rb, q0);
}
int main(void) {
  long bad = 0;
  for (long i = 0; i < 20000000; ++i) {
    /* drift_inc operands: gH*k over a wide range, omega >= f */
    const double f2 = fabs(rnd(-60, 60)), gH = fabs(rnd(-30, 30));
    const double k = rnd(-200, 200), l = rnd(-200, 200);
    const double w = sqrt(f2 + gH * (k * k + l * l));
    if (!isfinite(w)) continue;
    const double rw = 1.0 / w, ak = gH * k, al = gH * l;
    if (fabs(ak / w) < 0x1p-1022 || fabs(al / w) < 0x1p-1022) continue;  /* documented range */
    if (!same(div_rn_z(ak, w, rw), ak / w)) ++bad;
    if (!same(div_rn_z(al, w, rw), al / w)) ++bad;
  }
  /* quotients exactly representable, and signed zeros */
  for (long m = 1; m < 2000000; ++m) {
    const double w = (double)(2 * m + 1), a = w * (double)(m % 977 + 1) * ((m & 1) ? -1.0 : 1.0);
    if (!same(div_rn_z(a, w, 1.0 / w), a / w)) ++bad;
  }
  if (!same(div_rn_z(-0.0, 3.0, 1.0 / 3.0), -0.0) || !same(div_rn_z(0.0, 3.0, 1.0 / 3.0), 0.0)) ++bad;
  printf("%ld\n", bad);
  return bad != 0;
}
"""


def test_drift_quotients_from_one_reciprocal_are_ieee(tmp_path):
    """drift_inc's fast path: gH*k/omega and gH*l/omega as div_rn_z from
    RN(1/omega) equal IEEE division bit for bit (zero signs included)."""
    c = tmp_path / "drift.c"
    c.write_text(DRIFT)
    exe = tmp_path / "drift"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "0", out.stdout


CELL = r"""
#include <math.h>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
/* v_cvt_i32_f64: NaN -> 0, saturating */
static int cvt_sat(double v) {
  if (isnan(v)) return 0;
  if (v >= 2147483647.0) return INT_MAX;
  if (v <= -2147483648.0) return INT_MIN;
  return (int)v;
}
static unsigned umin(unsigned a, unsigned b) { return a < b ? a : b; }
static int old_c(double fl, double period, int nx) {
  int c = (fl >= 0.0 && fl <= period) ? (int)fl : 0;
  if (c >= nx) c -= nx;
  if (c >= nx) c %= nx;
  return c;
}
static int new_c(double fl, int iperiod, int nx) {
  int c = cvt_sat(fl);
  c = (unsigned)c > (unsigned)iperiod ? 0 : c;
  c = (int)umin((unsigned)c, (unsigned)(c - nx));
  c = (int)umin((unsigned)c, (unsigned)(c - nx));
  if (iperiod >= 3 * nx) c %= nx;
  return c;
}
int main(void) {
  long bad = 0;
  const int nxs[] = {1, 2, 3, 16, 64, 255, 512, 1024, 4096};
  for (unsigned a = 0; a < sizeof nxs / sizeof nxs[0]; ++a) {
    const int nx = nxs[a];
    const int periods[] = {nx, 2 * nx, 3 * nx, 5 * nx + 1};
    for (int b = 0; b < 4; ++b) {
      const int p = periods[b];
      for (int v = -3 * p - 5; v <= 3 * p + 5; ++v) {
        const double fl = (double)v;
        if (old_c(fl, (double)p, nx) != new_c(fl, p, nx)) ++bad;
      }
      const double spec[] = {NAN, -NAN, INFINITY, -INFINITY, -0.0, 0.0, 1e300, -1e300, 3e9, -3e9};
      for (unsigned q = 0; q < sizeof spec / sizeof spec[0]; ++q)
        if (old_c(spec[q], (double)p, nx) != new_c(spec[q], p, nx)) ++bad;
    }
  }
  printf("%ld\n", bad);
  return bad != 0;
}
"""


def test_cell_index_integer_path_matches_reference_logic(tmp_path):
    """cell_frac's integer tail (saturating cvt, unsigned range test, two
    unsigned-min wraps) equals the (fl >= 0 && fl <= period) ? (int)fl : 0
    then mod-nx logic for every integral fl in [-3p-5, 3p+5] and the special
    values, for periods nx, 2nx, 3nx and 5nx+1."""
    c = tmp_path / "cell.c"
    c.write_text(CELL)
    exe = tmp_path / "cell"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(c), "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "0", out.stdout
