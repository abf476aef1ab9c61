// swrt_rsw.hpp — the RSW background of step_packet_xka on the GPU.
//
// Replaces ray_trace_sw/raytrace_sw.m:16-52: g2k of the grid state
// [u v eta], the geostrophic projection
//   zetak  = 1i*(kx.*vk - ky.*uk)                      (:29)
//   etagk  = (f*etak - zetak).*f./(f^2 + gH0*K2)       (:25,30)
//   ugk    = -1i*ky.*(gH0/f*etagk), vgk = 1i*kx.*(...) (:34-35)
// the four i*k gradients (:38-41) and seven k2g (:44-52), H = 1 + etag.
// Integer wavenumbers (L = 2*pi, raytrace_sw.m:84).  The forward spectrum of
// the three state planes is read straight at each output wavenumber's
// half-plane representative (g2k's crop + fulspec's completion in one pass),
// and the seven real outputs go through four complex inverse transforms,
// paired as ug + i vg, ugx + i ugy, vgx + i vgy, etag.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swrt_fft.hpp"

namespace swrt {

// F: forward FFT2 of the 3 state planes, layout [c + n*r] per block (r: kx FFT
// index, c: ky FFT index), unnormalised.  Z: 4 output spectra, same layout.
__global__ void rsw_spectra_kernel(const double2* F, int n, double f, double gH0, double ks, double2* Z) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nn = (int64_t)n * n;
  if (idx >= nn) return;
  const int sh_ = __ffs(n) - 1;  // n is a power of two
  const int c = (int)idx & (n - 1), r = (int)idx >> sh_;
  const int kmax = n / 2 - 1;
  const int kx = signed_k(r, n), ky = signed_k(c, n);
  double2 z[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) z[q] = make_double2(0.0, 0.0);
  if (kx >= -kmax && kx <= kmax && ky >= -kmax && ky <= kmax) {
    int hx = kx, hy = ky;
    bool cj = false;
    if (ky < 0 || (ky == 0 && kx < 0)) { hx = -kx; hy = -ky; cj = true; }
    // g2k.m:8: fftshift(fft2(fg))/nx^2 at (hx, hy)
    const int64_t src = (int64_t)hy + (int64_t)n * (hx < 0 ? hx + n : hx);
    const double nn_d = (double)n * (double)n;
    const double2 U = F[src], V = F[nn + src], E = F[2 * nn + src];
    const double2 uk = make_double2(U.x / nn_d, U.y / nn_d);
    const double2 vk = make_double2(V.x / nn_d, V.y / nn_d);
    const double2 ek = make_double2(E.x / nn_d, E.y / nn_d);
    // raytrace_sw.m:16 integer wavenumbers (L = 2*pi: ks = 1.0 exactly); any other L scales them
    const double kxd = (double)hx * ks, kyd = (double)hy * ks;
    const double K2 = kxd * kxd + kyd * kyd;
    const double sig2 = f * f + gH0 * K2;                                     // :25
    const double2 w = make_double2(kxd * vk.x - kyd * uk.x, kxd * vk.y - kyd * uk.y);
    const double2 zeta = make_double2(-w.y, w.x);                             // :29
    const double2 eg = make_double2(((f * ek.x - zeta.x) * f) / sig2, ((f * ek.y - zeta.y) * f) / sig2);  // :30
    const double g = gH0 / f;
    const double2 ge = make_double2(g * eg.x, g * eg.y);
    const double2 ug = mul_mik(kyd, ge);                                      // :34
    const double2 vg = mul_ik(kxd, ge);                                       // :35
    double2 a[7] = {ug, vg, mul_ik(kxd, ug), mul_ik(kyd, ug), mul_ik(kxd, vg), mul_ik(kyd, vg), eg};
    if (hx == 0 && hy == 0) {
#pragma unroll
      for (int t = 0; t < 7; ++t) a[t].y = 0.0;  // only DC's real part reaches k2g's real output
    }
    if (cj) {
#pragma unroll
      for (int t = 0; t < 7; ++t) a[t].y = -a[t].y;
    }
    z[0] = make_double2(a[0].x - a[1].y, a[0].y + a[1].x);
    z[1] = make_double2(a[2].x - a[3].y, a[2].y + a[3].x);
    z[2] = make_double2(a[4].x - a[5].y, a[4].y + a[5].x);
    z[3] = a[6];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) Z[q * nn + idx] = z[q];
}

// Inverse transforms (layout [x + n*y]) -> the 7 column-major planes of
// swrt_xka_set_fields: u, v, u_x, u_y, v_x, v_y, H = 1 + etag (:45).
__global__ void rsw_unpack_kernel(const double2* T, int64_t nn, double* planes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nn) return;
  const double2 z0 = T[i], z1 = T[nn + i], z2 = T[2 * nn + i], z3 = T[3 * nn + i];
  planes[i] = z0.x;
  planes[nn + i] = z0.y;
  planes[2 * nn + i] = z1.x;
  planes[3 * nn + i] = z1.y;
  planes[4 * nn + i] = z2.x;
  planes[5 * nn + i] = z2.y;
  planes[6 * nn + i] = 1.0 + z3.x;
}

// Node records back to the 7 column-major planes (swrt_xka_get_fields).
__global__ void unpack_xka_kernel(const double* nodes, int nx, int npad, double* planes) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nn = (int64_t)nx * nx;
  if (idx >= nn) return;
  const int ig = (int)(idx % nx), jg = (int)(idx / nx);
  const double* s = nodes + ((int64_t)(ig + kPadLo) * npad + (jg + kPadLo)) * kXkaRec;
  planes[idx] = s[0];
  planes[nn + idx] = s[1];
  planes[2 * nn + idx] = s[4];
  planes[3 * nn + idx] = s[5];
  planes[4 * nn + idx] = s[6];
  planes[5 * nn + idx] = s[7];
  planes[6 * nn + idx] = s[2];
}

}  // namespace swrt
