// swrt_spectral.hpp — exact spectral evaluator (E2 / SURVEY K3).
//
// Generalises the exact Fourier kick of scratch/fourier_interpolate_test.m:
// 92-136 (psi = sum A cos(Kx + Ly + phi)) to a dense coefficient grid
//     psi(x, y) = sum_{i,j} Re( C[i,j] * exp(1i*(kx_i*x + ky_j*y)) ),
//     kx_i = (kx0 + i)*s, ky_j = (ky0 + j)*s,
// which covers the half-plane spectral layout of g2k (C = 2*psik, the
// ky = 0 / kx < 0 half-line zeroed, DC real) and the full-plane amp/phase
// field of the scratch test (C = A*exp(1i*phi)).  U = -psi_y, V = psi_x,
// u_x = -psi_xy, u_y = -psi_yy, v_x = psi_xx, v_y = psi_xy.
//
// One lane per packet; all lanes read the same coefficient at the same time
// (wave-uniform scalar loads) and each lane walks a row with the phase
// recurrence e <- e*exp(1i*s*x) (re-seeded
// with sincos at the start of every row), accumulating the five row sums
//   A0 = sum Im z, A1 = sum kx Im z, B0 = sum Re z, B1 = sum kx Re z,
//   B2 = sum kx^2 Re z   (z = C*e)
// that the ky weights then combine: psi_x -= A1, psi_y -= ky*A0,
// psi_xx -= B2, psi_xy -= ky*B1, psi_yy -= ky^2*B0.
// FP-VALU bound (≈14 flops per mode per packet); T = double or float
// (the fp32 tolerance study of config 5).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swrt {

struct ModeGrid {
  const double2* C;  // nkx x nky column-major (i fastest): row j = fixed ky
  const int2* rows;  // per row: [first, last+1) of the nonzero coefficients
  int nkx, nky;
  double kx0, ky0, s;
};

constexpr int kSpecThreads = 256;

template <typename T>
struct cplx {
  T re, im;
};

// Five derivative sums of psi at (x, y).  Every lane of a wavefront walks the
// same coefficient at the same time, so the coefficient loads are
// wave-uniform (scalar loads through the scalar cache: no LDS staging, no
// barriers); zero head/tail segments of each row are skipped.
constexpr int kSpecChains = 4;  // independent phase recurrences per row (ILP)

template <typename T>
__device__ __forceinline__ void spectral_sums(const ModeGrid& g, double x, double y, double out[5]) {
  T px = 0, py = 0, pxx = 0, pxy = 0, pyy = 0;
  double sr, cr;
  sincos(kSpecChains * g.s * x, &sr, &cr);
  const T rr = (T)cr, ri = (T)sr;  // exp(1i*kSpecChains*s*x): stride of one chain
  for (int j = 0; j < g.nky; ++j) {
    const int2 rg = g.rows[j];
    if (rg.x >= rg.y) continue;
    const double ky = (g.ky0 + j) * g.s;
    // chain c walks i = rg.x + c, rg.x + c + kSpecChains, ...
    T er[kSpecChains], ei[kSpecChains], kx[kSpecChains];
    T A0[kSpecChains], A1[kSpecChains], B0[kSpecChains], B1[kSpecChains], B2[kSpecChains];
#pragma unroll
    for (int c = 0; c < kSpecChains; ++c) {
      double s0, c0;
      sincos((g.kx0 + rg.x + c) * g.s * x + ky * y, &s0, &c0);
      er[c] = (T)c0;
      ei[c] = (T)s0;
      kx[c] = (T)((g.kx0 + rg.x + c) * g.s);
      A0[c] = A1[c] = B0[c] = B1[c] = B2[c] = 0;
    }
    const T ds = (T)(kSpecChains * g.s);
    const double2* row = g.C + (size_t)j * g.nkx;
    {
      // this sum has no reference rounding order to reproduce: let FMAs form
#pragma clang fp contract(fast)
      for (int i = rg.x; i < rg.y; i += kSpecChains) {
#pragma unroll
        for (int c = 0; c < kSpecChains; ++c) {
          // past the span end the coefficient is read as 0 (the row stays in bounds)
          const double2 cd = (i + c < rg.y) ? row[i + c] : make_double2(0.0, 0.0);
          const T cre = (T)cd.x, cim = (T)cd.y;
          const T zr = cre * er[c] - cim * ei[c];
          const T zi = cre * ei[c] + cim * er[c];
          A0[c] += zi;
          A1[c] += kx[c] * zi;
          B0[c] += zr;
          B1[c] += kx[c] * zr;
          B2[c] += (kx[c] * kx[c]) * zr;
          const T nr = er[c] * rr - ei[c] * ri;
          ei[c] = er[c] * ri + ei[c] * rr;
          er[c] = nr;
          kx[c] += ds;
        }
      }
    }
    T a0 = 0, a1 = 0, b0 = 0, b1 = 0, b2 = 0;
#pragma unroll
    for (int c = 0; c < kSpecChains; ++c) {
      a0 += A0[c]; a1 += A1[c]; b0 += B0[c]; b1 += B1[c]; b2 += B2[c];
    }
    const T kyT = (T)ky;
    px -= a1;
    py -= kyT * a0;
    pxx -= b2;
    pxy -= kyT * b1;
    pyy -= (kyT * kyT) * b0;
  }
  out[0] = px;
  out[1] = py;
  out[2] = pxx;
  out[3] = pxy;
  out[4] = pyy;
}

// U, grad U (6 x n, same order as swrt_eval) from the five psi derivatives.
__device__ __forceinline__ void psi_to_flow(const double d[5], double I[6]) {
  I[0] = -d[1];  // u = -psi_y
  I[1] = d[0];   // v = psi_x
  I[2] = -d[3];  // u_x = -psi_xy
  I[3] = -d[4];  // u_y = -psi_yy
  I[4] = d[2];   // v_x = psi_xx
  I[5] = d[3];   // v_y = psi_xy
}

template <typename T>
__global__ void __launch_bounds__(kSpecThreads) spectral_eval_kernel(ModeGrid g, const double* x,
                                                                     const double* y, int64_t n,
                                                                     double* out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  double d[5];
  spectral_sums<T>(g, x[p], y[p], d);
  double I[6];
  psi_to_flow(d, I);
#pragma unroll
  for (int q = 0; q < 6; ++q) out[(int64_t)q * n + p] = I[q];
}

// ode_symplectic.m:13-37 with the exact spectral kick (the scheme of
// scratch/fourier_interpolate_test.m:73-114): drift, exact U and
// (grad U)^T k at x1, kick, drift.  State N x 2 column-major.
template <typename T>
__global__ void __launch_bounds__(kSpecThreads) spectral_leapfrog_kernel(ModeGrid g, double* xs,
                                                                         double* ks, int64_t n,
                                                                         double dt, int nsteps,
                                                                         double f2, double gH) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  double x0 = xs[p], y0 = xs[n + p], k0 = ks[p], l0 = ks[n + p];
  const double half = dt / 2;
  // drift increment of the current k: shared by a step's closing drift and
  // the next step's opening drift (same k, same bits)
  double hcx, hcy;
  {
    const double w = sqrt(f2 + gH * (k0 * k0 + l0 * l0));
    hcx = half * (gH * k0 / w);
    hcy = half * (gH * l0 / w);
  }
  for (int s = 0; s < nsteps; ++s) {
    const double x1 = x0 + hcx;
    const double y1 = y0 + hcy;
    double d[5], I[6];
    spectral_sums<T>(g, x1, y1, d);
    psi_to_flow(d, I);
    const double x2 = x1 + dt * I[0];
    const double y2 = y1 + dt * I[1];
    const double k2 = k0 - dt * (I[2] * k0 + I[4] * l0);
    const double l2 = l0 - dt * (I[3] * k0 + I[5] * l0);
    const double w = sqrt(f2 + gH * (k2 * k2 + l2 * l2));
    hcx = half * (gH * k2 / w);
    hcy = half * (gH * l2 / w);
    x0 = x2 + hcx;
    y0 = y2 + hcy;
    k0 = k2;
    l0 = l2;
  }
  xs[p] = x0; xs[n + p] = y0; ks[p] = k0; ks[n + p] = l0;
}

}  // namespace swrt
