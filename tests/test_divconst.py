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
