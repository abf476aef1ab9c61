// swrt_qg.hpp — the QG PDE steppers that produce the packets' background
// snapshots, on the device.
//
//   1 layer:  qgsw_raytrace.m:111-137   AB3 (Euler / AB2 start) + filter,
//             update :270-286, inertial_ring :216-220, filter :222-230.
//   2 layers: qg2layersw_raytrace.m:129-181  exponential AB3 (expLdt,
//             expL2dt = LV diag(exp(LD dt)) LV^-1 of factor_L), update
//             :309-323, mmult3 :333-338; adaptive CFL :156-165 (host logic
//             over swrt_qg_max_speed).
//
// State: qk, its two previous tendencies and the previous qk, each
// nlayers x (2kmax+1) x (kmax+1) complex (the g2k half plane), resident in
// HBM in ky-fastest order (h = (kx + kmax)*(kmax+1) + ky) so that the passes
// over the full spectrum (layout [ky + n*kx]) read and write it contiguously;
// the C ABI converts from/to the host's column-major order.  One step is
//   spectra of psi_x + i psi_y and q_x + i q_y per layer (Hermitian
//   completion = fulspec)  ->  inverse 2-D FFT  ->  J = psi_x q_y - psi_y q_x
//   (both layers packed J1 + i J2 into one forward transform)  ->  g2k crop
//   and the AB3 update fused in one pass over the half plane.
// The Fourier transforms are the Stockham passes of swrt_fft.hpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swrt_fft.hpp"

namespace swrt {

struct QGDev {
  int n;          // grid size (power of two)
  int nl;         // layers: 1 or 2
  double kscale;  // 2*pi/L (1 for the 1-layer driver's L = 2*pi)
  double dx;      // L / n
  double K_d2;
  double beta;
  double r_drag;  // 1 layer: the r_drag*K2 term of update (qgsw_raytrace.m:285)
  double force_strength, f, Cg;  // 1 layer: inertial_ring forcing
  int filter;     // 1 layer: apply the exponential filter (qgsw_raytrace.m:137)
  double shear;   // 2 layers: shear_strength (mean-flow terms; grid_U's u offset)
  double nu, hyper, r;  // 2 layers: (nu*K2^alpha + r)*K2 diffusion factor
};

struct cd {
  double x, y;
};
__device__ __forceinline__ cd cmk(double x, double y) { return cd{x, y}; }
__device__ __forceinline__ cd cadd(cd a, cd b) { return cd{a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cd csub(cd a, cd b) { return cd{a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cd cmul(cd a, cd b) { return cd{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ cd crs(double s, cd a) { return cd{s * a.x, s * a.y}; }  // real * complex
__device__ __forceinline__ cd cdivr(cd a, double s) { return cd{a.x / s, a.y / s}; }
__device__ __forceinline__ cd cexp_(cd z) {
  const double e = exp(z.x);
  double sn, cs;
  sincos(z.y, &sn, &cs);
  return cd{e * cs, e * sn};
}
__device__ __forceinline__ cd csqrt_(cd z) {
  const double r = hypot(z.x, z.y);
  if (r == 0.0) return cd{0.0, 0.0};
  if (z.x >= 0.0) {
    const double t = sqrt(0.5 * (r + z.x));
    return cd{t, z.y / (2.0 * t)};
  }
  const double t = sqrt(0.5 * (r - z.x));
  return cd{fabs(z.y) / (2.0 * t), z.y >= 0.0 ? t : -t};
}
__device__ __forceinline__ cd cdiv(cd a, cd b) {
  const double d = b.x * b.x + b.y * b.y;
  return cd{(a.x * b.x + a.y * b.y) / d, (a.y * b.x - a.x * b.y) / d};
}
__device__ __forceinline__ cd ld(const double2* p, int64_t i) { const double2 v = p[i]; return cd{v.x, v.y}; }
__device__ __forceinline__ void st(double2* p, int64_t i, cd v) { p[i] = make_double2(v.x, v.y); }
// (1i*k).*z as MATLAB evaluates it
__device__ __forceinline__ cd ik(double k, cd z) { return cd{-(k * z.y), k * z.x}; }
// pack two real fields' spectra: A + i*B
__device__ __forceinline__ double2 pack2(cd a, cd b) { return make_double2(a.x - b.y, a.y + b.x); }

// 2-layer PV inversion B = [-F-K2, -F; -F, -F-K2] ./ (K2.*(K2+2F)), B = 0 at K2 = 0
// (qg2layersw_raytrace.m:129-136).  Returns B11 (= B22) and B12 (= B21).
__device__ __forceinline__ void qg2_B(double K2, double K_d2, double& b11, double& b12) {
  const double F = K_d2 / 2;
  if (K2 == 0.0) { b11 = 0.0; b12 = 0.0; return; }
  const double det = K2 * (K2 + 2 * F);
  b11 = (-F - K2) / det;
  b12 = -F / det;
}

// Step 1 of update: per full-spectrum index (layout [c + n*r], ky FFT index c
// contiguous) and layer l, Z[2l] = psi_x + i psi_y, Z[2l+1] = q_x + i q_y with
// the Hermitian completion of fulspec.m (kx < 0 on ky = 0 and ky < 0 from
// their conjugate partners; Nyquist row/column zero).
template <int NL, class Sink>
__device__ __forceinline__ void qg_jac_spectra_to(int64_t idx, const double2* qk, QGDev g, Sink out) {
  const int n = g.n;
  const int64_t nn = (int64_t)n * n;
  if (idx >= nn) return;
  const int sh_ = __ffs(n) - 1;  // n is a power of two
  const int c = (int)idx & (n - 1), r = (int)idx >> sh_;
  const int kmax = n / 2 - 1, nkx = 2 * kmax + 1;
  const int64_t nhalf = (int64_t)nkx * (kmax + 1);
  const int kx = signed_k(r, n), ky = signed_k(c, n);
  const bool inband = (kx >= -kmax && kx <= kmax && ky >= -kmax && ky <= kmax);
  int hx = kx, hy = ky;
  bool cj = false;
  if (ky < 0 || (ky == 0 && kx < 0)) { hx = -kx; hy = -ky; cj = true; }
  const int64_t h = inband ? (int64_t)(hx + kmax) * (kmax + 1) + hy : 0;
  const double kxs = (double)hx * g.kscale, kys = (double)hy * g.kscale;
  const double K2 = kxs * kxs + kys * kys;
  cd q[2], ps[2];
#pragma unroll
  for (int l = 0; l < NL; ++l) q[l] = inband ? ld(qk, l * nhalf + h) : cmk(0.0, 0.0);
  if constexpr (NL == 1) {
    // psik = -qk./(K_d2 + K2)   (qgsw_raytrace.m:271)
    const double den = g.K_d2 + K2;
    ps[0] = cmk(-q[0].x / den, -q[0].y / den);
  } else {
    // psik = mmult3(B, qk)      (qg2layersw_raytrace.m:310)
    double b11, b12;
    qg2_B(K2, g.K_d2, b11, b12);
    ps[0] = cadd(crs(b11, q[0]), crs(b12, q[1]));
    ps[1] = cadd(crs(b12, q[0]), crs(b11, q[1]));
  }
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    cd px = ik(kxs, ps[l]), py = ik(kys, ps[l]), qx = ik(kxs, q[l]), qy = ik(kys, q[l]);
    if (cj) { px.y = -px.y; py.y = -py.y; qx.y = -qx.y; qy.y = -qy.y; }
    if (!inband) px = py = qx = qy = cmk(0.0, 0.0);
    out(2 * l, idx, pack2(px, py));
    out(2 * l + 1, idx, pack2(qx, qy));
  }
}
template <int NL>
__device__ __forceinline__ void qg_jac_spectra_at(int64_t idx, const double2* qk, QGDev g, double2* Z) {
  qg_jac_spectra_to<NL>(idx, qk, g, GlobalPlanes{Z, (int64_t)g.n * g.n});
}

template <int NL>
__global__ void __launch_bounds__(256) qg_jac_spectra_kernel(const double2* qk, QGDev g, double2* Z) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  qg_jac_spectra_at<NL>(idx, qk, g, Z);
}

// J = psix.*qy - psiy.*qx per grid point and layer (qgsw_raytrace.m:282);
// both layers packed into one complex field J1 + i J2 for the forward FFT.
__global__ void qg_jacobian_kernel(const double2* T, int nl, int64_t nn, double2* Zj) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  double J[2] = {0.0, 0.0};
  for (int l = 0; l < nl; ++l) {
    const double2 P = T[(2 * l) * nn + i], Q = T[(2 * l + 1) * nn + i];
    J[l] = P.x * Q.y - P.y * Q.x;
  }
  Zj[i] = make_double2(J[0], J[1]);
}

// filter (qgsw_raytrace.m:222-230) at one wavenumber
__device__ __forceinline__ double qg_filter_at(double kx, double ky, double dx) {
  const double ks = sqrt((kx * dx) * (kx * dx) + (ky * dx) * (ky * dx));
  const double kc = 0.75 * 3.14159265358979323846;
  if (!(ks >= kc)) return 1.0;
  const double q = 0.25 * 3.14159265358979323846;
  const double cst = log(1e-15) / (q * q * q * q);
  const double d = ks - kc;
  return exp(cst * (d * d * d * d));
}

// 2-layer factor_L at one wavenumber (qg2layersw_raytrace.m:140-144):
//   B.*((nu*K2.^alpha + r).*K2 - 1i*kx*beta)
//   + 1i*kx*shear .* [-1,0;0,1]*(eye(2) + 2F*B)
__device__ __forceinline__ void qg2_factor_L(const QGDev& g, double kxs, double K2, cd L[4]) {
  double b11, b12;
  qg2_B(K2, g.K_d2, b11, b12);
  const double F = g.K_d2 / 2;
  const cd dfac = cmk((g.nu * pow(K2, g.hyper) + g.r) * K2, -(kxs * g.beta));
  const cd sf = cmk(0.0, kxs * g.shear);
  const double m00 = -(1 + 2 * F * b11), m01 = -(2 * F * b12), m10 = 2 * F * b12, m11 = 1 + 2 * F * b11;
  L[0] = cadd(crs(m00, sf), crs(b11, dfac));
  L[1] = cadd(crs(m01, sf), crs(b12, dfac));
  L[2] = cadd(crs(m10, sf), crs(b12, dfac));
  L[3] = cadd(crs(m11, sf), crs(b11, dfac));
}

// exp(t*M) of a 2x2 complex matrix through its eigenvalues s +- d
// (= LV*diag(exp(t*LD))*LV^-1, qg2layersw_raytrace.m:146-149):
//   exp(tM) = (e1+e2)/2 I + (e1-e2)/(2d) (M - sI),  e1,2 = exp(t(s +- d)),
// with the series of exp(ts) sinh(td)/d near a double eigenvalue.
__device__ __forceinline__ void expm2(const cd M[4], double t, cd E[4]) {
  const cd s = crs(0.5, cadd(M[0], M[3]));
  const cd D = crs(0.5, csub(M[0], M[3]));
  const cd d = csqrt_(cadd(cmul(D, D), cmul(M[1], M[2])));
  const cd td = crs(t, d);
  const cd ets = cexp_(crs(t, s));
  cd A, S;  // A = e^{ts} cosh(td), S = e^{ts} sinh(td)/d
  if (hypot(td.x, td.y) > 1e-3) {
    const cd e1 = cexp_(cadd(crs(t, s), td)), e2 = cexp_(csub(crs(t, s), td));
    A = crs(0.5, cadd(e1, e2));
    S = cdiv(crs(0.5, csub(e1, e2)), d);
  } else {
    const cd z2 = cmul(td, td);
    // cosh = 1 + z2/2 + z2^2/24, sinh(td)/d = t (1 + z2/6 + z2^2/120)
    const cd ch = cadd(cadd(cmk(1.0, 0.0), crs(0.5, z2)), crs(1.0 / 24.0, cmul(z2, z2)));
    const cd sh = crs(t, cadd(cadd(cmk(1.0, 0.0), crs(1.0 / 6.0, z2)), crs(1.0 / 120.0, cmul(z2, z2))));
    A = cmul(ets, ch);
    S = cmul(ets, sh);
  }
  E[0] = cadd(A, cmul(S, D));
  E[1] = cmul(S, M[1]);
  E[2] = cmul(S, M[2]);
  E[3] = csub(A, cmul(S, D));
}

// expLdt and expL2dt for every half-plane wavenumber: E[4*idx + (2i+j)]
// (idx in the ky-fastest state order).
__global__ void qg2_exp_kernel(QGDev g, double dt, double2* E1, double2* E2) {
  const int n = g.n, kmax = n / 2 - 1, nkx = 2 * kmax + 1;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)nkx * (kmax + 1)) return;
  const int shh_ = __ffs(n) - 2;  // kmax + 1 = n/2, a power of two
  const int col = (int)idx & (kmax), row = (int)idx >> shh_;
  const double kxs = (double)(row - kmax) * g.kscale, kys = (double)col * g.kscale;
  const double K2 = kxs * kxs + kys * kys;
  cd L[4], e[4];
  qg2_factor_L(g, kxs, K2, L);
  expm2(L, dt, e);
  for (int q = 0; q < 4; ++q) st(E1, 4 * idx + q, e[q]);
  expm2(L, 2 * dt, e);
  for (int q = 0; q < 4; ++q) st(E2, 4 * idx + q, e[q]);
}

__device__ __forceinline__ void mmul2(const double2* E, int64_t idx, const cd x[2], cd y[2]) {
  const cd a = ld(E, 4 * idx), b = ld(E, 4 * idx + 1), c = ld(E, 4 * idx + 2), d = ld(E, 4 * idx + 3);
  y[0] = cadd(cmul(a, x[0]), cmul(b, x[1]));
  y[1] = cadd(cmul(c, x[0]), cmul(d, x[1]));
}

// g2k crop of the (packed) forward spectrum, the tendency, and the AB3 update
// of qk at one half-plane wavenumber idx = (kx+kmax)*(kmax+1) + ky (both
// layers together for mmult3), from the packed spectrum Z = F1 + i F2 at k
// (Fk) and at -k (Fm):
//   1 layer:  Qn = g2k(J) - beta*psikx + r_drag*K2 + surface_forces
//             qk = Ef.*(qk + dq)                       (qgsw_raytrace.m:121-137)
//   2 layers: Qn = g2k(J);  qk = mmult3(expLdt, qk + dq)   (:168-181)
//   dq = dt*Qn | dt/2*(3Qn - X1) | dt/12*(23Qn - 16X1 + 5X2), X = Qm (1 layer)
//   or mmult3(expL(2)dt, Qm) (2 layers).  Returns the new qk (out), the
// tendency Qn and the previous one m1 (the history shifts Qm2 <- m1,
// Qm1 <- Qn; the callers store what their buffer scheme needs).
template <int NL>
__device__ __forceinline__ void qg_update_at(int64_t idx, int kx, int ky, double2 Fk, double2 Fm, const QGDev& g,
                                             double dt, int abstep, const double2* E1, const double2* E2,
                                             const double2* qk, const double2* Qm1, const double2* Qm2, cd out[NL],
                                             cd Qn[NL], cd m1[NL]) {
  const int n = g.n, kmax = n / 2 - 1, nkx = 2 * kmax + 1;
  const int64_t nhalf = (int64_t)nkx * (kmax + 1);
  const double kxs = (double)kx * g.kscale, kys = (double)ky * g.kscale;
  const double K2 = kxs * kxs + kys * kys;
  const double nn = (double)n * (double)n;
  if constexpr (NL == 1) {
    // g2k(J) = fftshift(fft2(J))/nx^2 of a real J: the packed imaginary part is 0
    (void)Fm;
    Qn[0] = cmk(Fk.x / nn, Fk.y / nn);
  } else {
    const cd F1 = cmk(0.5 * (Fk.x + Fm.x), 0.5 * (Fk.y - Fm.y));
    const cd F2 = cmk(0.5 * (Fk.y + Fm.y), -0.5 * (Fk.x - Fm.x));
    Qn[0] = cdivr(F1, nn);
    Qn[1] = cdivr(F2, nn);
  }
  cd q[NL];
  _Pragma("unroll") for (int l = 0; l < NL; ++l) q[l] = ld(qk, l * nhalf + idx);
  if constexpr (NL == 1) {
    const double den = g.K_d2 + K2;
    const cd psik = cmk(-q[0].x / den, -q[0].y / den);
    const cd psikx = ik(kxs, psik);
    const double omega = sqrt(g.f * g.f + (g.Cg * g.Cg) * K2);
    const double force = (0.9 * g.f < omega && omega < 1.1 * g.f) ? g.force_strength : 0.0;
    Qn[0] = csub(Qn[0], crs(g.beta, psikx));
    Qn[0].x = Qn[0].x + g.r_drag * K2;
    Qn[0].x = Qn[0].x + force;
  }
  cd X1[NL], X2[NL], m2[NL];
  _Pragma("unroll") for (int l = 0; l < NL; ++l) {
    m1[l] = ld(Qm1, l * nhalf + idx);
    m2[l] = ld(Qm2, l * nhalf + idx);
  }
  if constexpr (NL == 1) {
    X1[0] = m1[0];
    X2[0] = m2[0];
  } else {
    mmul2(E1, idx, m1, X1);
    mmul2(E2, idx, m2, X2);
  }
  cd dq[NL];
  _Pragma("unroll") for (int l = 0; l < NL; ++l) {
    if (abstep == 1) {
      dq[l] = crs(dt, Qn[l]);
    } else if (abstep == 2) {
      dq[l] = crs(dt / 2, csub(crs(3.0, Qn[l]), X1[l]));
    } else {
      dq[l] = crs(dt / 12, cadd(csub(crs(23.0, Qn[l]), crs(16.0, X1[l])), crs(5.0, X2[l])));
    }
  }
  if constexpr (NL == 1) {
    const double Ef = g.filter ? qg_filter_at(kxs, kys, g.dx) : 1.0;
    out[0] = crs(Ef, cadd(q[0], dq[0]));
  } else {
    cd s[2] = {cadd(q[0], dq[0]), cadd(q[1], dq[1])};
    mmul2(E1, idx, s, out);
  }
}

// The update over the half plane from the full forward spectrum Fj (layout
// [ky + n*kx], FFT indices).  Qm1/Qm2 are read, and the shifted history
// (Qm2 <- Qm1, Qm1 <- Qn) written to Qm1_out/Qm2_out: the same buffers for a
// committed step, spare ones for a speculative step
// (swrt_qg_step_speculative), which must leave the committed state intact
// until it is accepted.
template <int NL>
__global__ void __launch_bounds__(256) qg_update_kernel(const double2* Fj, QGDev g, double dt, int abstep, const double2* E1,
                                 const double2* E2, const double2* qk, double2* qk_out, const double2* Qm1,
                                 const double2* Qm2, double2* Qm1_out, double2* Qm2_out) {
  const int n = g.n, kmax = n / 2 - 1, nkx = 2 * kmax + 1;
  const int64_t nhalf = (int64_t)nkx * (kmax + 1);
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= nhalf) return;
  const int shh_ = __ffs(n) - 2;  // kmax + 1 = n/2, a power of two
  const int col = (int)idx & (kmax), row = (int)idx >> shh_;
  const int kx = row - kmax, ky = col;
  // packed forward spectrum Z = F1 + i F2 at k and -k (FFT indices)
  const int r = kx < 0 ? kx + n : kx, c = ky;
  const int rm = kx > 0 ? n - kx : -kx, cm = ky > 0 ? n - ky : 0;
  const double2 Fk = Fj[c + (int64_t)n * r], Fm = Fj[cm + (int64_t)n * rm];
  cd out[NL], Qn[NL], m1[NL];
  qg_update_at<NL>(idx, kx, ky, Fk, Fm, g, dt, abstep, E1, E2, qk, Qm1, Qm2, out, Qn, m1);
  _Pragma("unroll") for (int l = 0; l < NL; ++l) {
    st(qk_out, l * nhalf + idx, out[l]);
    st(Qm2_out, l * nhalf + idx, m1[l]);
    st(Qm1_out, l * nhalf + idx, Qn[l]);
  }
}

// The last pass of J's forward transform fused with the update (fused mode,
// n <= 2048): Zr holds J1 + i J2 after its first pass (along x, layout
// [kx + n*y], FFT index kx), workgroup w transforms the two columns kx = r
// and kx = n - r along y — the per-vector FFT of fft_vec_kernel<true,...>'s
// column pass, so the same spectrum bits — and, with both in LDS, updates
// every half-plane wavenumber (+-r, ky), ky = 0..kmax, whose k and -k they
// hold (r = 0 pairs with the Nyquist column, which no wavenumber reads).
// The spectrum never goes to memory (the column pass's write and the update's
// k / -k reads) and the state is read and written along ky, contiguously.
// Only the new tendency is stored, to Qn_out (which may alias Qm2: each
// wavenumber is read and written by one lane); the caller renames the
// history buffers (Qm2 <- Qm1, Qm1 <- Qn_out).  blockDim = n/2 (two vectors
// of n/4 lanes, lane t = ky for the update), dynamic LDS 2*(n+1) double2.
// Block b: XCD b % 8 walks a contiguous range of r, so the columns of each
// 128-B line are read by workgroups of one XCD (one L2).
template <int NL>
__global__ void __launch_bounds__(1024) qg_update_cols_kernel(const double2* Zr, QGDev g, int logn,
                                                               const double2* tw, double dt, int abstep,
                                                               const double2* E1, const double2* E2,
                                                               const double2* qk, double2* qk_out, const double2* Qm1,
                                                               const double2* Qm2, double2* Qn_out) {
  extern __shared__ double2 sbuf[];
  const int n = g.n, kmax = n / 2 - 1, nkx = 2 * kmax + 1;
  const int64_t nhalf = (int64_t)nkx * (kmax + 1);
  const int quarter = n >> 2, t = threadIdx.x, ld = n + 1;
  const int r = (int)(blockIdx.x & 7) * (n >> 4) + (int)(blockIdx.x >> 3);  // 0 .. n/2-1
  const int rb = r == 0 ? n / 2 : n - r;                                     // the partner column
  {
    // lanes 2j, 2j+1 read row j's two columns, every load issued before the first wait
    const int c = t & 1, j0 = t >> 1;
    const double2* src = Zr + (c ? rb : r);
    double2 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = src[(int64_t)(j0 + k * quarter) * n];
#pragma unroll
    for (int k = 0; k < 4; ++k) sbuf[c * ld + j0 + k * quarter] = v[k];
  }
  __syncthreads();
  {
    const int col = t / quarter, b = t - col * quarter;
    fft_stages_one_buffer(sbuf + col * ld, b, n, logn, tw, 0);
  }
  const double2* A = sbuf;       // FFT row r:  kx = r
  const double2* B = sbuf + ld;  // FFT row rb: kx = -r (r > 0)
  const int ky = t, cm = ky > 0 ? n - ky : 0;
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    if (side == 1 && r == 0) break;
    const int kx = side ? -r : r;
    const double2 Fk = side ? B[ky] : A[ky];
    const double2 Fm = r == 0 ? A[cm] : (side ? A[cm] : B[cm]);
    const int64_t idx = (int64_t)(kx + kmax) * (kmax + 1) + ky;
    cd out[NL], Qn[NL], m1[NL];
    qg_update_at<NL>(idx, kx, ky, Fk, Fm, g, dt, abstep, E1, E2, qk, Qm1, Qm2, out, Qn, m1);
    _Pragma("unroll") for (int l = 0; l < NL; ++l) {
      st(qk_out, l * nhalf + idx, out[l]);
      st(Qn_out, l * nhalf + idx, Qn[l]);
    }
  }
}

// u + i v per layer from grid_U's inversion psik = -qk./(K_d2+K2) (grid_U.m:2-6),
// for the CFL speed (qg2layersw_raytrace.m:156-158); layout [c + n*r].
template <int NL, class Sink>
__device__ __forceinline__ void qg_vel_spectra_to(int64_t idx, const double2* qk, QGDev g, Sink out) {
  const int n = g.n;
  const int64_t nn = (int64_t)n * n;
  if (idx >= nn) return;
  const int sh_ = __ffs(n) - 1;  // n is a power of two
  const int c = (int)idx & (n - 1), r = (int)idx >> sh_;
  const int kmax = n / 2 - 1, nkx = 2 * kmax + 1;
  const int64_t nhalf = (int64_t)nkx * (kmax + 1);
  const int kx = signed_k(r, n), ky = signed_k(c, n);
  const bool inband = (kx >= -kmax && kx <= kmax && ky >= -kmax && ky <= kmax);
  int hx = kx, hy = ky;
  bool cj = false;
  if (ky < 0 || (ky == 0 && kx < 0)) { hx = -kx; hy = -ky; cj = true; }
  const double kxs = (double)hx * g.kscale, kys = (double)hy * g.kscale;
  const double den = g.K_d2 + (kxs * kxs + kys * kys);
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    cd u = cmk(0.0, 0.0), v = cmk(0.0, 0.0);
    if (inband) {
      const cd q = ld(qk, l * nhalf + (int64_t)(hx + kmax) * (kmax + 1) + hy);
      const cd ps = cmk(-q.x / den, -q.y / den);
      u = cmk(kys * ps.y, -(kys * ps.x));  // (-1i*ky).*psik
      v = ik(kxs, ps);
      if (hx == 0 && hy == 0) { u.y = 0.0; v.y = 0.0; }
      if (cj) { u.y = -u.y; v.y = -v.y; }
    }
    out(l, idx, pack2(u, v));
  }
}
template <int NL>
__device__ __forceinline__ void qg_vel_spectra_at(int64_t idx, const double2* qk, QGDev g, double2* Z) {
  qg_vel_spectra_to<NL>(idx, qk, g, GlobalPlanes{Z, (int64_t)g.n * g.n});
}

template <int NL>
__global__ void __launch_bounds__(256) qg_vel_spectra_kernel(const double2* qk, QGDev g, double2* Z) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  qg_vel_spectra_at<NL>(idx, qk, g, Z);
}

// max over the grid of (u + shear)^2 + v^2 (all layers) into *out (as the
// bit pattern of a non-negative double, so integer max == double max).
__global__ void qg_max_speed2_kernel(const double2* T, int64_t cnt, double shear, unsigned long long* out) {
  __shared__ double red[256];
  double m = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 z = T[i];
    const double u = z.x + shear, v = z.y;
    const double s2 = u * u + v * v;
    m = s2 > m ? s2 : m;
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicMax(out, (unsigned long long)__double_as_longlong(red[0]));
}

// Fused mode (swrt_api.hip qg_post): the post-step spectra of one qk in ONE
// launch — the Jacobian inputs, layer 1's u+iv and layer 0's grid_U, by the
// three kernels' own element functions (same values) — which also clears
// the CFL max for qg_jacobian_max_kernel.
template <int NL>
__global__ void __launch_bounds__(256) qg_post_spectra_kernel(const double2* qk, QGDev g, int64_t nhalf,
                                                              double2* Zjac, double2* Zuv1, double2* Zsnap,
                                                              unsigned long long* dmax) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx == 0) *dmax = 0ull;
  qg_jac_spectra_at<NL>(idx, qk, g, Zjac);
  if constexpr (NL == 2) qg_vel_spectra_at<1>(idx, qk + nhalf, g, Zuv1);
  spectra_at(idx, qk, g.n, 1, g.K_d2, g.kscale, 0, Zsnap, g.n / 2, 1);
}

// qg_post_spectra_kernel fused with the first pass of the batched inverse
// 2-D FFT: workgroup r builds row r (ky contiguous) of every post-step plane
// in LDS with the same element functions, runs the NB inverse row FFTs side
// by side (n/4 lanes each, fft_stages_one_buffer) and writes the pass's
// output (plane t, row r at out[t*n*n + r*n]) — bit for bit what the
// spectra launch + in-place pass write, without the planes' round trip
// through memory.  blockDim = NB*n/4 <= 1024, dynamic LDS NB*n double2.
template <int NL>
__global__ void __launch_bounds__(1024) qg_post_rows_kernel(const double2* qk, QGDev g, int64_t nhalf, int logn,
                                                            const double2* tw, double2* out,
                                                            unsigned long long* dmax) {
  constexpr int NB = 2 * NL + (NL - 1) + 3;
  extern __shared__ double2 rows[];
  const int n = g.n;
  const int64_t nn = (int64_t)n * n;
  const int r = blockIdx.x;
  if (r == 0 && threadIdx.x == 0) *dmax = 0ull;
  for (int e = threadIdx.x; e < 2 * n; e += blockDim.x) {
    const int64_t idx = (int64_t)(e < n ? e : e - n) + (int64_t)n * r;
    if (e < n) {
      qg_jac_spectra_to<NL>(idx, qk, g, LdsRowPlanes{rows, n});
    } else {
      if constexpr (NL == 2) qg_vel_spectra_to<1>(idx, qk + nhalf, g, LdsRowPlanes{rows + 2 * NL * n, n});
      spectra_to(idx, qk, n, 1, g.K_d2, g.kscale, 0, LdsRowPlanes{rows + (2 * NL + NL - 1) * n, n}, n / 2, 1);
    }
  }
  __syncthreads();
  const int q = n >> 2;
  fft_stages_one_buffer(rows + (threadIdx.x / q) * n, threadIdx.x % q, n, logn, tw, 1);
  for (int e = threadIdx.x; e < NB * n; e += blockDim.x)
    out[(int64_t)(e / n) * nn + (int64_t)r * n + (e % n)] = rows[e];
}

// The same for two layers, two workgroups per row (blockIdx = 2r + h): h = 0
// builds and transforms the four Jacobian-input planes, h = 1 layer 1's
// u+iv and layer 0's grid_U planes (output planes 4..7).  blockDim = n (four
// vectors of n/4 lanes), dynamic LDS 4n double2: half the footprint of the
// one-workgroup form (profiles/r03_v4_qg/README.md).
__global__ void __launch_bounds__(1024) qg_post_rows_split_kernel(const double2* qk, QGDev g, int64_t nhalf,
                                                                  int logn, const double2* tw, double2* out,
                                                                  unsigned long long* dmax) {
  extern __shared__ double2 rows[];
  const int n = g.n;
  const int64_t nn = (int64_t)n * n;
  const int r = blockIdx.x >> 1, h = blockIdx.x & 1;
  const int q = n >> 2, t = threadIdx.x;
  if (blockIdx.x == 0 && t == 0) *dmax = 0ull;
  const int64_t idx = (int64_t)t + (int64_t)n * r;
  if (h == 0) {
    qg_jac_spectra_to<2>(idx, qk, g, LdsRowPlanes{rows, n});
  } else {
    qg_vel_spectra_to<1>(idx, qk + nhalf, g, LdsRowPlanes{rows, n});
    spectra_to(idx, qk, n, 1, g.K_d2, g.kscale, 0, LdsRowPlanes{rows + n, n}, n / 2, 1);
  }
  __syncthreads();
  fft_stages_one_buffer(rows + (t / q) * n, t % q, n, logn, tw, 1);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int e = t + k * n;
    out[(int64_t)(4 * h + k) * nn + (int64_t)r * n + t] = rows[e];
  }
}

// qg_jacobian_kernel + qg_max_speed2_kernel over the same grid points:
// J1 + i J2, and max (u + shear)^2 + v^2 over the nl u+iv planes at `uv`.
// Grid-stride (kQgMaxPer points per thread), the max reduced by wave
// shuffles and one LDS pass, one atomic per block: the one-point-per-thread
// form with a block-wide LDS tree took 16.5 us at 512^2 (1.8 TB/s).
constexpr int kQgMaxPer = 4;
__global__ void __launch_bounds__(256) qg_jacobian_max_kernel(const double2* T, int nl, int64_t nn, double2* Zj,
                                                              const double2* uv, double shear,
                                                              unsigned long long* dmax) {
  __shared__ double red[256 / 64];
  double m = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += stride) {
    double J[2] = {0.0, 0.0};
    for (int l = 0; l < nl; ++l) {
      const double2 P = T[(2 * l) * nn + i], Q = T[(2 * l + 1) * nn + i];
      J[l] = P.x * Q.y - P.y * Q.x;
    }
    Zj[i] = make_double2(J[0], J[1]);
    for (int l = 0; l < nl; ++l) {
      const double2 z = uv[l * nn + i];
      const double u = z.x + shear, v = z.y;
      const double s2 = u * u + v * v;
      m = s2 > m ? s2 : m;
    }
  }
  for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    double b = red[0];
    for (int w = 1; w < 256 / 64; ++w) b = fmax(b, red[w]);
    atomicMax(dmax, (unsigned long long)__double_as_longlong(b));
  }
}

}  // namespace swrt
