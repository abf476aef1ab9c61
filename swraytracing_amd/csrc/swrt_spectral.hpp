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
// (LDS broadcasts of a block-staged stream, SpecStream) and each lane walks a
// row with the phase recurrence e <- e*exp(1i*s*x) (re-seeded with sincos at
// the start of every row), accumulating the five row sums
//   A0 = sum Im z, A1 = sum kx Im z, B0 = sum Re z, B1 = sum kx Re z,
//   B2 = sum kx^2 Re z   (z = C*e)
// that the ky weights then combine: psi_x -= A1, psi_y -= ky*A0,
// psi_xx -= B2, psi_xy -= ky*B1, psi_yy -= ky^2*B0.
// FP-VALU bound (15 instructions, 22 flop per mode per packet); the kernels
// take T = double or float (float: packed math, the fp32 tolerance study of
// config 5).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swrt {

struct ModeGrid {
  const double2* C;  // nkx x nky column-major (i fastest): row j = fixed ky
  // row j's nonzero span zero-padded to whole groups of kSpecChains modes,
  // starting at Cd[Cd_row[j]] (the array padded past its end for SpecStream)
  const double2* Cd;
  const int* Cd_row;
  const int2* rows;  // per row: [first, last+1) of the nonzero coefficients
  // fp32 copy for the packed-math kernel: row j's span in groups of 4 modes,
  // each group two float4 {re_m, re_m+1, im_m, im_m+1} (m = first + 4g, +2),
  // zero past the span; row j starts at float4 index Cf_row[j]
  const float4* Cf;
  const int* Cf_row;
  int nkx, nky;
  double kx0, ky0, s;
};

constexpr int kSpecThreads = 256;

// Five derivative sums of psi at (x, y).  Every lane of the block walks the
// same coefficient at the same time (SpecStream); zero head/tail segments of
// each row are skipped.
constexpr int kSpecChains = 4;  // independent phase recurrences per row (ILP)

// The coefficient stream through LDS.  The rows' group-padded spans (Cd for
// fp64: 4 double2 per group of 4 modes; Cf for fp32: 2 float4) are one
// contiguous array of 16-B slots that every lane of every wave walks in the
// same order.  The block stages it in chunks of kSpecChunk slots, double
// buffered: while the waves sum chunk k from one buffer, each thread holds
// its share of chunk k+1 in registers (loaded at the previous switch) and
// writes it into the other buffer at the next switch — one barrier per
// chunk, and every coefficient read is an LDS broadcast (all lanes, one
// address).  Before, the waves read the coefficients with scalar loads that
// waited on the L2 every group (the 3.7 MB fp64 spectrum does not fit the
// scalar cache): ~half the VALU issue slots went idle.
constexpr int kSpecChunk = 512;                              // slots (8 KB) per chunk
constexpr int kSpecPer = kSpecChunk / kSpecThreads;         // slots per thread per chunk

struct SpecStream {
  const uint4* src;  // the slot array (padded past the end by two chunks)
  uint4* buf;        // __shared__ [2][kSpecChunk]
  int base;          // slot index of the chunk in buf[cur]
  int cur;
  uint4 pre[kSpecPer];

  __device__ __forceinline__ void begin(const void* slots, uint4* lds) {
    src = reinterpret_cast<const uint4*>(slots);
    buf = lds;
    base = 0;
    cur = 0;
    __syncthreads();  // the previous pass's readers are done with both buffers
#pragma unroll
    for (int q = 0; q < kSpecPer; ++q) buf[q * kSpecThreads + threadIdx.x] = src[q * kSpecThreads + threadIdx.x];
#pragma unroll
    for (int q = 0; q < kSpecPer; ++q) pre[q] = src[kSpecChunk + q * kSpecThreads + threadIdx.x];
    __syncthreads();
  }
  // slot s (wave-uniform, s >= base): make sure its chunk is in buf[cur]
  __device__ __forceinline__ const uint4* at(int s) {
    while (s >= base + kSpecChunk) {  // uniform; at most once per group in practice
      uint4* nb = buf + (cur ^ 1) * kSpecChunk;
#pragma unroll
      for (int q = 0; q < kSpecPer; ++q) nb[q * kSpecThreads + threadIdx.x] = pre[q];
      __syncthreads();
      cur ^= 1;
      base += kSpecChunk;
#pragma unroll
      for (int q = 0; q < kSpecPer; ++q) pre[q] = src[base + kSpecChunk + q * kSpecThreads + threadIdx.x];
    }
    return buf + cur * kSpecChunk + (s - base);
  }
};

__device__ __forceinline__ void spectral_sums(const ModeGrid& g, double x, double y, SpecStream& st,
                                              double out[5]) {
  double px = 0, py = 0, pxx = 0, pxy = 0, pyy = 0;
  double rr, ri;
  sincos(kSpecChains * g.s * x, &ri, &rr);  // exp(1i*kSpecChains*s*x): stride of one chain
  for (int j = 0; j < g.nky; ++j) {
    const int2 rg = g.rows[j];
    if (rg.x >= rg.y) continue;
    const double ky = (g.ky0 + j) * g.s;
    // chain c walks i = rg.x + c, rg.x + c + kSpecChains, ...
    double er[kSpecChains], ei[kSpecChains], kx[kSpecChains];
    double A0[kSpecChains], A1[kSpecChains], B0[kSpecChains], B1[kSpecChains], B2[kSpecChains];
#pragma unroll
    for (int c = 0; c < kSpecChains; ++c) {
      sincos((g.kx0 + rg.x + c) * g.s * x + ky * y, &ei[c], &er[c]);
      kx[c] = (g.kx0 + rg.x + c) * g.s;
      A0[c] = A1[c] = B0[c] = B1[c] = B2[c] = 0;
    }
    const double ds = kSpecChains * g.s;
    // row j's span, zero-padded to whole groups of kSpecChains modes
    const int s0 = g.Cd_row[j];
    const int ngroups = (rg.y - rg.x + kSpecChains - 1) / kSpecChains;
    {
      // this sum has no reference rounding order to reproduce: let FMAs form
#pragma clang fp contract(fast)
      for (int gi = 0; gi < ngroups; ++gi) {
        const double2* cc = reinterpret_cast<const double2*>(st.at(s0 + kSpecChains * gi));
#pragma unroll
        for (int c = 0; c < kSpecChains; ++c) {
          const double cre = cc[c].x, cim = cc[c].y;
          const double zr = cre * er[c] - cim * ei[c];
          const double zi = cre * ei[c] + cim * er[c];
          A0[c] += zi;
          A1[c] += kx[c] * zi;
          B0[c] += zr;
          B1[c] += kx[c] * zr;
          B2[c] += (kx[c] * kx[c]) * zr;
          const double nr = er[c] * rr - ei[c] * ri;
          ei[c] = er[c] * ri + ei[c] * rr;
          er[c] = nr;
          kx[c] += ds;
        }
      }
    }
    double a0 = 0, a1 = 0, b0 = 0, b1 = 0, b2 = 0;
#pragma unroll
    for (int c = 0; c < kSpecChains; ++c) {
      a0 += A0[c]; a1 += A1[c]; b0 += B0[c]; b1 += B1[c]; b2 += B2[c];
    }
    px -= a1;
    py -= ky * a0;
    pxx -= b2;
    pxy -= ky * b1;
    pyy -= (ky * ky) * b0;
  }
  out[0] = px;
  out[1] = py;
  out[2] = pxx;
  out[3] = pxy;
  out[4] = pyy;
}

// fp32 form of spectral_sums on packed math: the four phase chains run as two
// pairs, each pair's recurrence and sums one v_pk_mul/fma/add_f32 per two
// chains, with the coefficients pre-converted and pre-paired on the host
// (two modes per SGPR pair: no per-mode conversion).  Same sums as the
// generic form up to fp32 rounding order (the fp32 leg is a tolerance study).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void spectral_sums_pk(const ModeGrid& g, double x, double y, SpecStream& st,
                                                 double out[5]) {
  float px = 0, py = 0, pxx = 0, pxy = 0, pyy = 0;
  double sr, cr;
  sincos(kSpecChains * g.s * x, &sr, &cr);
  const f32x2 rr = {(float)cr, (float)cr}, ri = {(float)sr, (float)sr};
  const float dsf = (float)(kSpecChains * g.s);
  const f32x2 ds = {dsf, dsf};
  for (int j = 0; j < g.nky; ++j) {
    const int2 rg = g.rows[j];
    if (rg.x >= rg.y) continue;
    const double ky = (g.ky0 + j) * g.s;
    f32x2 er[2], ei[2], kx[2], A0[2], A1[2], B0[2], B1[2], B2[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = 2 * p + h;
        double s0, c0;
        sincos((g.kx0 + rg.x + c) * g.s * x + ky * y, &s0, &c0);
        er[p][h] = (float)c0;
        ei[p][h] = (float)s0;
        kx[p][h] = (float)((g.kx0 + rg.x + c) * g.s);
      }
      A0[p] = A1[p] = B0[p] = B1[p] = B2[p] = f32x2{0.f, 0.f};
    }
    const int s0 = g.Cf_row[j];
    const int ngroups = (rg.y - rg.x + kSpecChains - 1) / kSpecChains;
    {
#pragma clang fp contract(fast)
      for (int gi = 0; gi < ngroups; ++gi) {
        const float4* cc = reinterpret_cast<const float4*>(st.at(s0 + 2 * gi));
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const float4 cq = cc[p];
          const f32x2 cre = {cq.x, cq.y}, cim = {cq.z, cq.w};
          const f32x2 zr = cre * er[p] - cim * ei[p];
          const f32x2 zi = cre * ei[p] + cim * er[p];
          A0[p] += zi;
          A1[p] += kx[p] * zi;
          B0[p] += zr;
          B1[p] += kx[p] * zr;
          B2[p] += (kx[p] * kx[p]) * zr;
          const f32x2 nr = er[p] * rr - ei[p] * ri;
          ei[p] = er[p] * ri + ei[p] * rr;
          er[p] = nr;
          kx[p] += ds;
        }
      }
    }
    const f32x2 a0 = A0[0] + A0[1], a1 = A1[0] + A1[1], b0 = B0[0] + B0[1], b1 = B1[0] + B1[1],
                b2 = B2[0] + B2[1];
    const float kyT = (float)ky;
    px -= a1.x + a1.y;
    py -= kyT * (a0.x + a0.y);
    pxx -= b2.x + b2.y;
    pxy -= kyT * (b1.x + b1.y);
    pyy -= (kyT * kyT) * (b0.x + b0.y);
  }
  out[0] = px;
  out[1] = py;
  out[2] = pxx;
  out[3] = pxy;
  out[4] = pyy;
}

template <typename T>
__device__ __forceinline__ void spectral_sums_t(const ModeGrid& g, double x, double y, uint4* lds, double out[5]) {
  SpecStream st;
  if constexpr (sizeof(T) == 4) {
    st.begin(g.Cf, lds);
    spectral_sums_pk(g, x, y, st, out);
  } else {
    st.begin(g.Cd, lds);
    spectral_sums(g, x, y, st, out);
  }
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
  // lanes past n evaluate packet n-1 and store nothing: no divergent exit
  // before the mode loops, whose coefficient loads then stay scalar
  const int64_t p0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = p0 < n ? p0 : n - 1;
  __shared__ uint4 lds[2 * kSpecChunk];
  double d[5];
  spectral_sums_t<T>(g, x[p], y[p], lds, d);
  double I[6];
  psi_to_flow(d, I);
  if (p0 >= n) return;
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
  // lanes past n step packet n-1 and store nothing (see spectral_eval_kernel)
  const int64_t p0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = p0 < n ? p0 : n - 1;
  __shared__ uint4 lds[2 * kSpecChunk];
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
    spectral_sums_t<T>(g, x1, y1, lds, d);
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
  if (p0 >= n) return;
  xs[p] = x0; xs[n + p] = y0; ks[p] = k0; ks[n + p] = l0;
}

}  // namespace swrt
