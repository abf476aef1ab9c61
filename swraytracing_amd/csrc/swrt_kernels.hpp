// swrt_kernels.hpp — device code of the packet hot path (gfx950 / CDNA4).
//
// One lane per packet.  The six background fields of a snapshot live in HBM
// as a halo-padded, node-interleaved array: node (ix, iy) holds the 48 B
// record {u, v, u_x, u_y, v_x, v_y} and iy is the fast index, so one row of
// the 6x6 Lagrange stencil (fixed ix, six consecutive iy) is one contiguous
// 288 B segment and no tap needs a periodic wrap (2 ghost nodes below, 3
// above in each direction).
//
// Arithmetic is fp64 in exactly the reference's operation order (see
// oracle/swrt_oracle.c for the CPU twin); this translation unit is compiled
// with -ffp-contract=off so no FMA is formed behind our back.  Divisions and
// square roots are IEEE correctly rounded.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swrt_share.hpp"

namespace swrt {

constexpr int kNT = 6;            // taps per direction (Iord = 2, interpolate.m:12)
constexpr int kPadLo = 2;         // ghost nodes below (offset -2)
constexpr int kPadTot = 5;        // npad = nx + 5 (offsets -2..+3 from cells 0..nx-1)
constexpr int kRec = 6;           // doubles per node record

struct FieldView {
  const double* nodes;  // (nx+5) x (nx+5) records, x-major, y contiguous
  int nx;               // grid size (periodic in x and y with nx nodes)
  int npad;             // nx + 5
  double dx;            // L / nx (interpolate.m dx = dy = h)
  double px, py;        // mod periods of x/dx and y/dy (nx, ny_period)
  double inv_px, inv_py;
  int ipx, ipy;          // the periods as ints
  double inv_dx;        // RN(1/dx): locality keys, and x/dx via div_rn (correctly rounded)
};

// a / b correctly rounded (== IEEE a/b) from rb = RN(1/b), in one multiply
// and two FMAs (Markstein; Handbook of Floating-Point Arithmetic, Thm 4.10):
// q0 = RN(a*rb) is within 1 ulp of a/b, r = a - b*q0 is exact in an FMA, and
// RN(q0 + r*rb) is then the correctly rounded quotient.  Outside the normal
// range the result may differ from IEEE division, which does not matter here:
// |a/b| < 2^-54 gives the same cell and offset (1 + xl rounds to 1 either
// way), and an overflowing quotient is NaN instead of Inf, which cell_frac
// turns into NaN anyway (Inf - Inf).  Checked bit-exact against a/b on 1e9
// random pairs (a and b over 120 binades each) on the host.
__device__ __forceinline__ double div_rn(double a, double b, double rb) {
  const double q0 = a * rb;
  const double r = __builtin_fma(-q0, b, a);
  return __builtin_fma(r, rb, q0);
}

// a / b correctly rounded from rb = RN(1/b), as div_rn, with the sign of a
// zero quotient kept: r = a - q0*b is formed as -(q0*b - a) (the same value,
// exact), so a = -0 gives -0 like IEEE division (div_rn gives +0).  The
// negations are FMA source modifiers: still one multiply and two FMAs.
__device__ __forceinline__ double div_rn_z(double a, double b, double rb) {
  const double q0 = a * rb;
  const double r = __builtin_fma(q0, b, -a);
  return __builtin_fma(-r, rb, q0);
}

// sqrt(x), correctly rounded, for 2^-767 <= x < +inf: the instruction
// sequence the compiler emits for sqrt() (v_rsq_f64 + Goldschmidt/Newton
// steps) without its input scaling (an identity on this range) and its
// +-0/+inf class select (not reachable on it) — 10 instructions instead of 17.
// Callers guarantee the range through f^2 >= 2^-767 (dispersion_fast()).
__device__ __forceinline__ double sqrt_rn_normal(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  double d = __builtin_fma(-g, g, x);
  h = __builtin_fma(h, r, h);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}

// RN(1/b) for 2^-766 <= b <= 2^1022: the compiler's IEEE division sequence
// for 1.0/b (v_rcp_f64, two Newton steps, then q = 1*y, r = 1 - b*q and the
// final q + r*y) without v_div_scale (which scales only outside this range)
// and v_div_fixup (special operands only) — 7 instructions instead of 11.
__device__ __forceinline__ double rcp_rn_normal(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-b, y, 1.0);
  y = __builtin_fma(y, e, y);
  const double r = __builtin_fma(-b, y, 1.0);
  return __builtin_fma(r, y, y);
}

// Half-step drift increment of ode_symplectic.m:10-16,
//   (hcx, hcy) = half * (gH*k/omega, gH*l/omega),  omega = sqrt(f^2 + gH*|k|^2),
// in IEEE operations.  fast (f^2 >= 2^-767, uniform): omega by sqrt_rn_normal
// and both quotients from ONE correctly rounded reciprocal (div_rn_z,
// Markstein), 23 instructions instead of 39 — the same bits for every packet
// with |gH*k/omega| >= 2^-1022 and f^2 + gH*|k|^2 finite (|k| < ~1e154):
// outside that the packet's state is already meaningless.
__device__ __forceinline__ void drift_inc(double k, double l, double f2, double gH, double half, bool fast,
                                          double& hcx, double& hcy) {
  const double x = f2 + gH * (k * k + l * l);
  if (fast) {
    const double w = sqrt_rn_normal(x);
    const double rw = rcp_rn_normal(w);
    hcx = half * div_rn_z(gH * k, w, rw);
    hcy = half * div_rn_z(gH * l, w, rw);
  } else {
    const double w = sqrt(x);
    hcx = half * (gH * k / w);
    hcy = half * (gH * l / w);
  }
}

// n1 / sqrt(r) and n2 / sqrt(r) in IEEE operations (odefun's Cg*k/s,
// qgsw_raytrace.m:262-263): fast (r >= f^2 >= 2^-767, uniform) as drift_inc.
__device__ __forceinline__ void quot2_sqrt(double r, double n1, double n2, bool fast, double& q1, double& q2) {
  if (fast) {
    const double w = sqrt_rn_normal(r);
    const double rw = rcp_rn_normal(w);
    q1 = div_rn_z(n1, w, rw);
    q2 = div_rn_z(n2, w, rw);
  } else {
    const double w = sqrt(r);
    q1 = n1 / w;
    q2 = n2 / w;
  }
}

// Host-side: may drift_inc take its fast path for this f^2?
__host__ __device__ inline bool dispersion_fast(double f2) { return f2 >= 0x1p-767 && f2 < 0x1p+1000; }

// Hardware conformance check of the short sequences (swrt_check_arith):
// random operands over their whole documented ranges, compared bit for bit
// with the compiler's IEEE sqrt / division.  mismatches[0..2] = sqrt, 1/w,
// drift quotients.
__global__ void __launch_bounds__(256) check_arith_kernel(int64_t n, uint64_t seed,
                                                          unsigned long long* mismatches) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint64_t s = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(p + 1));
  auto nxt = [&]() {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return s;
  };
  auto rnd = [&](int lo, int hi) {  // random positive double, exponent in [lo, hi]
    const uint64_t m = nxt() & ((1ull << 52) - 1);
    const int e = lo + (int)(nxt() % (uint64_t)(hi - lo + 1));
    return __longlong_as_double((long long)(((uint64_t)(e + 1023) << 52) | m));
  };
  unsigned bad[3] = {0, 0, 0};
  for (int it = 0; it < 16; ++it) {
    const double x = rnd(-767, 1023);
    if (__double_as_longlong(sqrt_rn_normal(x)) != __double_as_longlong(sqrt(x))) ++bad[0];
    const double w = rnd(-383, 511);
    if (__double_as_longlong(rcp_rn_normal(w)) != __double_as_longlong(1.0 / w)) ++bad[1];
    const double f2 = rnd(-60, 60), gH = rnd(-30, 30);
    const double k = (nxt() & 1 ? -1.0 : 1.0) * rnd(-40, 40), l = (nxt() & 1 ? -1.0 : 1.0) * rnd(-40, 40);
    double hx, hy, gx, gy;
    drift_inc(k, l, f2, gH, 0.5, true, hx, hy);
    drift_inc(k, l, f2, gH, 0.5, false, gx, gy);
    if (__double_as_longlong(hx) != __double_as_longlong(gx) || __double_as_longlong(hy) != __double_as_longlong(gy))
      ++bad[2];
  }
  for (int q = 0; q < 3; ++q)
    if (bad[q]) atomicAdd(&mismatches[q], (unsigned long long)bad[q]);
}

// v_cvt_i32_f64 with the hardware's defined behaviour (NaN -> 0, saturation
// outside the int range); C++'s (int) would be undefined there.
__device__ __forceinline__ int cvt_i32_sat(double v) {
  int c;
  asm("v_cvt_i32_f64 %0, %1" : "=v"(c) : "v"(v));
  return c;
}

// interpolate.m:21-31 — xl = mod(x/dx, n); i0 = 1 + floor(xl); a = 1 + xl - i0.
// Returns the 0-based cell reduced mod nx and the fractional offset a.
// inv_dx = RN(1/dx) and inv_period = RN(1/period) from the host, iperiod =
// the period as an int.  q/period is div_rn for every period: for a power of
// two inv_period is exact, q0 = q*inv_period is already the quotient and the
// correction adds r = 0 (a zero of either sign gives the same cell and
// offset), so no per-lane select between a plain multiply and div_rn is needed.
__device__ __forceinline__ int cell_frac(double x, double dx, double inv_dx, double period,
                                         double inv_period, int iperiod, int nx, double& a) {
  const double q = div_rn(x, dx, inv_dx);
  const double r = div_rn(q, period, inv_period);
  const double xl = q - floor(r) * period;   // MATLAB mod (a - floor(a/m)*m)
  const double fl = floor(xl);
  a = (1.0 + xl) - (1.0 + fl);
  // NaN/Inf positions: keep the index in range (the result is NaN anyway).
  // fl outside [0, period] (or NaN: cvt gives 0) -> cell 0, as
  // (fl >= 0 && fl <= period) ? (int)fl : 0 in two integer instructions.
  int c = cvt_i32_sat(fl);
  c = (unsigned)c > (unsigned)iperiod ? 0 : c;
  // c mod nx: i0 may equal the period after round-up of mod, and the 2-layer
  // y-period is 2*nx (interpolate.m:45-46 wrap by nx).  Two unsigned-min
  // subtractions (c - nx wraps above c when c < nx) reduce c <= 3nx - 1;
  // wider generic periods (uniform) take the integer remainder.
  c = (int)min((unsigned)c, (unsigned)(c - nx));
  c = (int)min((unsigned)c, (unsigned)(c - nx));
  if (iperiod >= 3 * nx) c %= nx;
  return c;
}

// x / d for a small integer constant d, correctly rounded (== IEEE x/d).
// |d| in {1,2,4}: exact scaling.  |d| in {3,5}: Markstein's correction,
//   q0 = RN(x*RN(1/d)), r = fma(-q0, d, x) (exact), q = RN(q0 + r*RN(1/d)),
// which is the correctly rounded quotient because x/d is never within
// 1/(2|d|) ulp of a rounding midpoint (its binary expansion is periodic with
// period |d|-1), far more than the 2^-52-relative error of the correction.
template <int D>
__device__ __forceinline__ double div_const(double x) {
  constexpr int A = D < 0 ? -D : D;
  static_assert(A >= 1 && A <= 5, "divisor");
  double q;
  if constexpr (A == 1 || A == 2 || A == 4) {
    q = x * (1.0 / (double)A);
  } else {
    constexpr double R = 1.0 / (double)A;  // RN(1/A), evaluated in double
    const double q0 = x * R;
    const double r = __builtin_fma(-q0, (double)A, x);
    q = __builtin_fma(r, R, q0);
  }
  return D < 0 ? -q : q;
}

// interpolate.m:33-41 — w(i) = prod_{j != i} (a - j + bump)/(j - i), running
// product in the reference order (multiply, then divide by the constant).
// Dividing by d = s * 2^e * m (sign s, odd part m in {1, 3, 5}) is an exact
// scaling by s * 2^-e of the division by m, and a scaling by +-2^n commutes
// with every rounding of the running product (|w| stays far inside the
// normal range: |a - j + bump| <= 4), so the signs and powers of two of all
// five divisors are applied once, as the exact constant factor kScale<I>,
// after the running product of the odd parts: the same bits with 6 fewer
// multiplications per direction.
constexpr int odd_part(int d) { return d < 0 ? odd_part(-d) : (d % 2 == 0 ? odd_part(d / 2) : d); }
constexpr double pow2_sign_inv(int d) {  // s * 2^-e of d = s * 2^e * odd_part(d)
  return d < 0 ? -pow2_sign_inv(-d) : (d % 2 == 0 ? 0.5 * pow2_sign_inv(d / 2) : 1.0);
}
template <int I>
constexpr double kScale() {
  double c = 1.0;
  for (int j = -2; j <= 3; ++j)
    if (j != I) c *= pow2_sign_inv(j - I);
  return c;
}

template <int I, int J>
__device__ __forceinline__ double wstep(double w, const double* t) {
  if constexpr (I == J) {
    return w;
  } else {
    return div_const<odd_part(J - I)>(w * t[J + 2]);
  }
}

template <int I>
__device__ __forceinline__ double lagrange_wi(const double* t) {
  double w = 1.0;
  w = wstep<I, -2>(w, t);
  w = wstep<I, -1>(w, t);
  w = wstep<I, 0>(w, t);
  w = wstep<I, 1>(w, t);
  w = wstep<I, 2>(w, t);
  w = wstep<I, 3>(w, t);
  constexpr double S = kScale<I>();
  return S == 1.0 ? w : w * S;
}

__device__ __forceinline__ void lagrange_w(double a, double bump, double w[kNT]) {
  double t[kNT];
#pragma unroll
  for (int j = -2; j <= 3; ++j) t[j + 2] = (a - (double)j) + bump;
  w[0] = lagrange_wi<-2>(t);
  w[1] = lagrange_wi<-1>(t);
  w[2] = lagrange_wi<0>(t);
  w[3] = lagrange_wi<1>(t);
  w[4] = lagrange_wi<2>(t);
  w[5] = lagrange_wi<3>(t);
}

// Cell index for LOCALITY only (binning keys, in-tile sort keys): floor of
// x*(1/dx) mod nx — a multiply instead of the correctly rounded division of
// cell_frac.  A packet classified one cell off near a cell edge is merely
// sorted or binned next door; every result is computed by cell_frac.
__device__ __forceinline__ int fast_cell(double x, double inv_dx, int nx) {
  const double q = floor(x * inv_dx);
  int c = (q > -1073741824.0 && q < 1073741824.0) ? (int)q : 0;  // NaN/huge -> 0
  c %= nx;
  return c < 0 ? c + nx : c;
}

// Cell and 1-D weights of a point: shared by every field and snapshot of the
// same grid (the reference recomputes them per interpolate call; the values
// are identical).
struct Stencil {
  int ic, jc;
  double wx[kNT], wy[kNT];
};

__device__ __forceinline__ void stencil_at(const FieldView& fv, double x, double y, double bump,
                                           Stencil& s) {
  double ax, ay;
  s.ic = cell_frac(x, fv.dx, fv.inv_dx, fv.px, fv.inv_px, fv.ipx, fv.nx, ax);
  s.jc = cell_frac(y, fv.dx, fv.inv_dx, fv.py, fv.inv_py, fv.ipy, fv.nx, ay);
  lagrange_w(ax, bump, s.wx);
  lagrange_w(ay, bump, s.wy);
}

// Six-field stencil sums of one or two snapshots:
//   out[f] = sum_i sum_j (wx_i * wy_j) * F_f[ig, jg]
// accumulated i-outer / j-inner exactly as interpolate.m:43-49 does per field.
// The sums start from -0.0, the additive identity (-0 + p == p for every p,
// so the first add folds away; +0 + p differs from p only in the sign of an
// all-negative-zero sum, which is numerically equal).
template <bool TWO>
__device__ __forceinline__ void gather6(const double* nodes0, const double* nodes1, int npad,
                                        const Stencil& s, double o0[kRec], double o1[kRec]) {
#pragma unroll
  for (int f = 0; f < kRec; ++f) { o0[f] = -0.0; o1[f] = -0.0; }
  const size_t off = ((size_t)s.ic * npad + s.jc) * kRec;
#pragma unroll
  for (int i = 0; i < kNT; ++i) {
    const size_t ro = off + (size_t)i * npad * kRec;
    const double2* r0 = reinterpret_cast<const double2*>(nodes0 + ro);
    const double2* r1 = reinterpret_cast<const double2*>(nodes1 + ro);
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
      const double wij = s.wx[i] * s.wy[j];
      const double2 a0 = r0[3 * j + 0], a1 = r0[3 * j + 1], a2 = r0[3 * j + 2];
      o0[0] = o0[0] + wij * a0.x; o0[1] = o0[1] + wij * a0.y;
      o0[2] = o0[2] + wij * a1.x; o0[3] = o0[3] + wij * a1.y;
      o0[4] = o0[4] + wij * a2.x; o0[5] = o0[5] + wij * a2.y;
      if constexpr (TWO) {
        const double2 b0 = r1[3 * j + 0], b1 = r1[3 * j + 1], b2 = r1[3 * j + 2];
        o1[0] = o1[0] + wij * b0.x; o1[1] = o1[1] + wij * b0.y;
        o1[2] = o1[2] + wij * b1.x; o1[3] = o1[3] + wij * b1.y;
        o1[4] = o1[4] + wij * b2.x; o1[5] = o1[5] + wij * b2.y;
      }
    }
  }
}

__device__ __forceinline__ void interp6(const FieldView& fv, double x, double y, double bump,
                                        double out[kRec]) {
  Stencil s;
  stencil_at(fv, x, y, bump, s);
  double dummy[kRec];
  gather6<false>(fv.nodes, fv.nodes, fv.npad, s, out, dummy);
}

// The same sums as gather6 (same per-field order: i outer, j inner) with a
// scheduling barrier after every tap, so at most one tap's 6 records are in
// flight: the register-light global fallback of the LDS-tiled kernels, whose
// hot path then needs no spills.  Rare path; its speed is secondary.
// acc + w*v: mul then add (the reference's rounding, bit-exact) or, in the
// opt-in FMA gather mode (swrt_set_gather_mode 1), one fused multiply-add —
// the same sum with one rounding fewer per tap (tolerance parity).
template <bool FMA>
__device__ __forceinline__ double madd(double acc, double w, double v) {
  if constexpr (FMA)
    return __builtin_fma(w, v, acc);
  else
    return acc + w * v;
}

template <bool TWO, bool FMA = false>
__device__ __forceinline__ void gather6_lean(const double* nodes0, const double* nodes1, int npad,
                                             const Stencil& s, double o0[kRec], double o1[kRec]) {
#pragma unroll
  for (int f = 0; f < kRec; ++f) { o0[f] = -0.0; o1[f] = -0.0; }
  const size_t off = ((size_t)s.ic * npad + s.jc) * kRec;
#pragma unroll
  for (int i = 0; i < kNT; ++i) {
    const size_t ro = off + (size_t)i * npad * kRec;
    const double2* r0 = reinterpret_cast<const double2*>(nodes0 + ro);
    const double2* r1 = reinterpret_cast<const double2*>(nodes1 + ro);
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
      const double wij = s.wx[i] * s.wy[j];
      const double2 a0 = r0[3 * j + 0], a1 = r0[3 * j + 1], a2 = r0[3 * j + 2];
      o0[0] = madd<FMA>(o0[0], wij, a0.x); o0[1] = madd<FMA>(o0[1], wij, a0.y);
      o0[2] = madd<FMA>(o0[2], wij, a1.x); o0[3] = madd<FMA>(o0[3], wij, a1.y);
      o0[4] = madd<FMA>(o0[4], wij, a2.x); o0[5] = madd<FMA>(o0[5], wij, a2.y);
      if constexpr (TWO) {
        const double2 b0 = r1[3 * j + 0], b1 = r1[3 * j + 1], b2 = r1[3 * j + 2];
        o1[0] = madd<FMA>(o1[0], wij, b0.x); o1[1] = madd<FMA>(o1[1], wij, b0.y);
        o1[2] = madd<FMA>(o1[2], wij, b1.x); o1[3] = madd<FMA>(o1[3], wij, b1.y);
        o1[4] = madd<FMA>(o1[4], wij, b2.x); o1[5] = madd<FMA>(o1[5], wij, b2.y);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// interpolate_U.m:19-23 — (1 - alpha)*U1 + alpha*U2, per field.  Both
// snapshots live on the same grid (checked on the host).
template <bool TWO>
__device__ __forceinline__ void eval_flow_t(const FieldView& f0, const FieldView& f1, double alpha,
                                            double x, double y, double bump, double I[kRec]) {
  Stencil s;
  stencil_at(f0, x, y, bump, s);
  double J[kRec];
  gather6<TWO>(f0.nodes, f1.nodes, f0.npad, s, I, J);
  if constexpr (TWO) {
    const double oma = 1 - alpha;
#pragma unroll
    for (int q = 0; q < kRec; ++q) I[q] = oma * I[q] + alpha * J[q];
  }
}

__device__ __forceinline__ void eval_flow(const FieldView& f0, const FieldView& f1, int nslots,
                                          double alpha, double x, double y, double bump,
                                          double I[kRec]) {
  if (nslots == 2)
    eval_flow_t<true>(f0, f1, alpha, x, y, bump, I);
  else
    eval_flow_t<false>(f0, f1, alpha, x, y, bump, I);
}

constexpr int kMaxIntervals = 4;  // PDE intervals per multi-interval launch

struct StepArgs {
  FieldView f0, f1;
  int nslots;
  double* x;  // N x 2 column-major
  double* k;
  int64_t n;
  double dt, half, f2, gH;  // f2 = f*f
  int fastdisp;             // dispersion_fast(f2): drift_inc's short sequences
  double alpha0, dalpha;
  int64_t s0;               // global index of the first step of this launch
  int nsteps;
  double bump;
  int64_t save_every;
  double* hist_x;           // frames of N x 2 (NULL: no history)
  double* hist_k;
  int64_t frame0;           // history frame index of global step save_every-1
  const int* perm;          // device order -> original packet index (history)
};


// ode_symplectic.m:13-37 fused: drift(dt/2) -> kick(dt) -> drift(dt/2), nsteps
// times with the packet held in registers.
template <bool TWO>
__global__ void __launch_bounds__(256) leapfrog_kernel(StepArgs a) {
  const int64_t p = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (p >= a.n) return;
  double x0 = a.x[p], y0 = a.x[a.n + p];
  double k0 = a.k[p], l0 = a.k[a.n + p];
  // phi1(x0, k0, dt/2): x + (dt/2) * (gH*k/omega(k))   (ode_symplectic.m:10-16).
  // The drift after a kick and the drift that opens the next step use the
  // same k, so the increment is computed once per step (same bits).
  double hcx, hcy;
  drift_inc(k0, l0, a.f2, a.gH, a.half, a.fastdisp, hcx, hcy);
  for (int s = 0; s < a.nsteps; ++s) {
    const int64_t sg = a.s0 + s;
    const double x1 = x0 + hcx;
    const double y1 = y0 + hcy;
    // phi2(x1, k1, dt): U and (grad U)^T k at x1  (ode_symplectic.m:18-21)
    double I[kRec];
    eval_flow_t<TWO>(a.f0, a.f1, a.alpha0 + (double)sg * a.dalpha, x1, y1, a.bump, I);
    const double x2 = x1 + a.dt * I[0];
    const double y2 = y1 + a.dt * I[1];
    const double k2 = k0 - a.dt * (I[2] * k0 + I[4] * l0);  // RaytracingScheme.m:14
    const double l2 = l0 - a.dt * (I[3] * k0 + I[5] * l0);  // RaytracingScheme.m:15
    // phi1(x2, k2, dt/2)
    drift_inc(k2, l2, a.f2, a.gH, a.half, a.fastdisp, hcx, hcy);
    x0 = x2 + hcx;
    y0 = y2 + hcy;
    k0 = k2;
    l0 = l2;
    if (a.hist_x != nullptr && ((sg + 1) % a.save_every) == 0) {
      const int64_t fr = a.frame0 + (sg + 1) / a.save_every - 1;
      double* hx = a.hist_x + fr * 2 * a.n;
      double* hk = a.hist_k + fr * 2 * a.n;
      const int64_t o = a.perm[p];  // frames are stored in the original packet order
      hx[o] = x0; hx[a.n + o] = y0;
      hk[o] = k0; hk[a.n + o] = l0;
    }
  }
  a.x[p] = x0; a.x[a.n + p] = y0;
  a.k[p] = k0; a.k[a.n + p] = l0;
}

// U, grad U at points: out 6 x n (SpectralScheme.U/grad_U, interpolate_U).
__global__ void __launch_bounds__(256) eval_kernel(FieldView f0, FieldView f1, int nslots,
                                                   double alpha, double bump, const double* x,
                                                   const double* y, int64_t n, double* out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  double I[kRec];
  eval_flow(f0, f1, nslots, alpha, x[p], y[p], bump, I);
#pragma unroll
  for (int q = 0; q < kRec; ++q) out[(int64_t)q * n + p] = I[q];
}

// Generic interpolate(x, y, F, dx, dy) of one nx x nyF column-major grid
// (reads only columns < nx, as F(ig,jg) with jg <= nx does).
__global__ void __launch_bounds__(256) interp1_kernel(const double* F, int nx, double pyF,
                                                      double inv_py, double dx,
                                                      double dy, double bump, const double* x,
                                                      const double* y, int64_t n, double* out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const double px = (double)nx;
  double ax, ay;
  const int ic = cell_frac(x[p], dx, 1.0 / dx, px, 1.0 / px, nx, nx, ax);
  const int jc = cell_frac(y[p], dy, 1.0 / dy, pyF, inv_py, (int)pyF, nx, ay);
  double wx[kNT], wy[kNT];
  lagrange_w(ax, bump, wx);
  lagrange_w(ay, bump, wy);
  double FI = 0.0;
#pragma unroll
  for (int i = 0; i < kNT; ++i) {
    int ig = ic + i - 2;
    ig = ig < 0 ? ig + nx : (ig >= nx ? ig - nx : ig);
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
      int jg = jc + j - 2;
      jg = jg < 0 ? jg + nx : (jg >= nx ? jg - nx : jg);
      FI = FI + wx[i] * wy[j] * F[ig + (size_t)nx * jg];
    }
  }
  out[p] = FI;
}

// Pack 6 column-major planes (F[ig + nx*jg]) into the padded interleaved
// node array with periodic ghosts; u gets `shear` added (grid_U.m:11).
__global__ void pack_nodes_kernel(const double* planes, int nx, int npad, double shear,
                                  double* nodes) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = (int64_t)npad * npad;
  if (idx >= tot) return;
  const int ip = (int)idx / npad, jp = (int)idx % npad;
  int ig = ip - kPadLo, jg = jp - kPadLo;
  ig = ((ig % nx) + nx) % nx;
  jg = ((jg % nx) + nx) % nx;
  const int64_t plane = (int64_t)nx * nx;
  const int64_t src = ig + (int64_t)nx * jg;
  double* dst = nodes + idx * kRec;
#pragma unroll
  for (int f = 0; f < kRec; ++f) dst[f] = planes[f * plane + src] + (f == 0 ? shear : 0.0);
}

// Inverse of pack for downloads: nodes -> 6 column-major planes.
__global__ void unpack_nodes_kernel(const double* nodes, int nx, int npad, double* planes) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t plane = (int64_t)nx * nx;
  if (idx >= plane) return;
  const int ig = (int)idx % nx, jg = (int)idx / nx;
  const double* src = nodes + ((int64_t)(ig + kPadLo) * npad + (jg + kPadLo)) * kRec;
#pragma unroll
  for (int f = 0; f < kRec; ++f) planes[f * plane + idx] = src[f];
}

}  // namespace swrt
