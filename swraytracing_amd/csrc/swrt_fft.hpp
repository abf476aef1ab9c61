// swrt_fft.hpp — field preparation on the GPU (g2k / fulspec / k2g / grid_U).
//
// Replaces MATLAB's fft2/ifft2/fftshift in qg_flow_ray_trace/{g2k,k2g,fulspec}.m
// and the spectral algebra of grid_U.m / SpectralScheme.m:12-35.  A 2-D
// transform is two passes of a batched 1-D radix-4 Stockham FFT (one n/4-lane
// workgroup per length-n vector in one LDS buffer), the second reading the
// first's columns (no transpose pass).  Runs once per snapshot / PDE step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swrt {

// Batched length-n complex FFT over contiguous vectors data[b*n + i].
// tw[k] = exp(-2*pi*i*k/n), k < n.  inverse: conjugate twiddles, no scaling.
// Stockham autosort in radix-4 stages (r4_butterfly) and, for odd log2 n, a
// last radix-2 stage; a radix-2 stage with stride s, half-length m = n/(2s):
//   y[q + s*2p] = a + b,  y[q + s*(2p+1)] = (a - b) * w^(p*s),
//   a = x[q + s*p], b = x[q + s*(p+m)].
//
// TIN (the second pass of a 2-D transform, fused with the transpose between
// the passes): vector i of batch b is read down the column in[b*n*n + i + n*j]
// and written contiguously to out[b*n*n + i*n + j] — the same values as a
// transpose followed by an in-place pass, without the transpose's round trip
// through memory.  Blocks are mapped so that consecutive columns run on the
// same XCD at the same time (block k of XCD x = blockIdx % 8 takes vector
// x*nvec/8 + k): the 8 columns of each 128-B line are read by neighbouring
// workgroups through the same L2.
// One radix-4 Stockham butterfly (stride s = 4^(logs/2), quarter-length
// m = n/(4s), b = q + s*p):  a_j = x[b + j*n/4],
//   y_k = DFT4(a)_k * w^(k*p*s)  goes to  x'[q + s*(4p + k)];  returns q + 4sp.
// w1..w3 = tw[k*p*s], conjugated for the inverse.
__device__ __forceinline__ int r4_butterfly_w(const double2* xa, int b, int quarter, int s, int logs, double2 w1,
                                              double2 w2, double2 w3, int inverse, double2 y[4]) {
  const int q = b & (s - 1);
  const int p = b >> logs;
  const double2 a0 = xa[b], a1 = xa[b + quarter], a2 = xa[b + 2 * quarter], a3 = xa[b + 3 * quarter];
  const double2 t0 = make_double2(a0.x + a2.x, a0.y + a2.y), t1 = make_double2(a0.x - a2.x, a0.y - a2.y);
  const double2 t2 = make_double2(a1.x + a3.x, a1.y + a3.y), u = make_double2(a1.x - a3.x, a1.y - a3.y);
  // (a1 - a3) * (-i) forward, * (+i) inverse
  const double2 t3 = inverse ? make_double2(-u.y, u.x) : make_double2(u.y, -u.x);
  const double2 b1 = make_double2(t1.x + t3.x, t1.y + t3.y), b2 = make_double2(t0.x - t2.x, t0.y - t2.y);
  const double2 b3 = make_double2(t1.x - t3.x, t1.y - t3.y);
  y[0] = make_double2(t0.x + t2.x, t0.y + t2.y);
  y[1] = make_double2(b1.x * w1.x - b1.y * w1.y, b1.x * w1.y + b1.y * w1.x);
  y[2] = make_double2(b2.x * w2.x - b2.y * w2.y, b2.x * w2.y + b2.y * w2.x);
  y[3] = make_double2(b3.x * w3.x - b3.y * w3.y, b3.x * w3.y + b3.y * w3.x);
  return q + 4 * s * p;
}
__device__ __forceinline__ int r4_butterfly(const double2* xa, int b, int quarter, int s, int logs,
                                            const double2* tw, int inverse, double2 y[4]) {
  const int e = (b >> logs) * s;
  double2 w1 = tw[e], w2 = tw[2 * e], w3 = tw[3 * e];
  if (inverse) { w1.y = -w1.y; w2.y = -w2.y; w3.y = -w3.y; }
  return r4_butterfly_w(xa, b, quarter, s, logs, w1, w2, w3, inverse, y);
}

// All stages of one length-n vector in ONE LDS buffer xa, blockDim == n/4
// per vector: each lane holds its butterfly's four values in registers
// between the read and the write of a stage; b = the lane's butterfly
// (0..n/4-1).  The barriers are the whole workgroup's: several vectors of one
// length may run side by side.  Ends after a __syncthreads (xa holds the
// result).  The twiddles are read from the global table (L2-resident): an
// LDS copy of it made these kernels faster alone but the driver step slower,
// its LDS footprint crowding the packet kernel they run beside
// (profiles/r03_v4_qg/README.md).
__device__ __forceinline__ void fft_stages_one_buffer(double2* xa, int b, int n, int logn, const double2* tw,
                                                      int inverse) {
  const int quarter = n >> 2, half = n >> 1;
  // the next radix-4 stage's twiddles are loaded before this stage's LDS
  // work, so their latency hides behind it (unconditional: e <= b < n/4
  // keeps 3e inside the table for every stage)
  int e = b;
  double2 n1 = tw[e], n2 = tw[2 * e], n3 = tw[3 * e];
  int s = 1, logs = 0;
  for (; logs + 2 <= logn; logs += 2, s <<= 2) {
    double2 w1 = n1, w2 = n2, w3 = n3;
    e = (b >> (logs + 2)) << (logs + 2);
    n1 = tw[e];
    n2 = tw[2 * e];
    n3 = tw[3 * e];
    if (inverse) { w1.y = -w1.y; w2.y = -w2.y; w3.y = -w3.y; }
    double2 y[4];
    const int o = r4_butterfly_w(xa, b, quarter, s, logs, w1, w2, w3, inverse, y);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) xa[o + k * s] = y[k];
    __syncthreads();
  }
  if (logs < logn) {  // last stage radix 2: s = n/2, p = 0, twiddle 1
    const double2 a0 = xa[b], c0 = xa[b + half], a1 = xa[b + quarter], c1 = xa[b + quarter + half];
    __syncthreads();
    xa[b] = make_double2(a0.x + c0.x, a0.y + c0.y);
    xa[b + half] = make_double2(a0.x - c0.x, a0.y - c0.y);
    xa[b + quarter] = make_double2(a1.x + c1.x, a1.y + c1.y);
    xa[b + quarter + half] = make_double2(a1.x - c1.x, a1.y - c1.y);
    __syncthreads();
  }
}

// MODE 1: radix-4 stages (+ one radix-2 stage for odd log2 n), ping-pong
// LDS; 2: the same in one LDS buffer per vector, C vectors per workgroup of
// C*n/4 lanes (n <= 1024), dynamic LDS C*(n+1) double2.
template <bool TIN, int MODE>
__global__ void __launch_bounds__(1024) fft_vec_kernel(const double2* in, double2* data, int n, int logn,
                                                      const double2* tw, int inverse, int nvec) {
  extern __shared__ double2 sbuf[];
  double2* xa = sbuf;
  double2* ya = MODE == 2 ? sbuf : sbuf + n;
  double2* v;
  if constexpr (MODE == 2) {
    // C = blockDim/(n/4) vectors per workgroup (1, 2 or 4; nvec % (8C) == 0
    // for TIN), n/4 lanes each, four elements per lane; every load issued
    // before the first wait.  LDS: C vectors at stride n + 1 (the C columns
    // of one row land in distinct banks).
    const int quarter = n >> 2, t = threadIdx.x, C = (int)blockDim.x / quarter;
    const int ld = n + 1;
    const int col = t / quarter, b = t - col * quarter;
    double2 r[4];
    int vec0;
    if constexpr (TIN) {
      // groups of C adjacent columns; consecutive groups on one XCD (above)
      const int ng = nvec / C;
      vec0 = ((int)(blockIdx.x & 7) * (ng >> 3) + (int)(blockIdx.x >> 3)) * C;
      const int bb = vec0 >> logn, i0 = vec0 & (n - 1);
      const double2* src = in + ((size_t)bb << (2 * logn)) + i0;
      const int c = t % C, j0 = t / C;  // lanes C*j .. C*j + C-1 read row j's C columns
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = src[(size_t)(j0 + k * quarter) * n + c];
#pragma unroll
      for (int k = 0; k < 4; ++k) sbuf[c * ld + j0 + k * quarter] = r[k];
    } else {
      vec0 = (int)blockIdx.x * C;
      const double2* src = data + (size_t)(vec0 + col) * n;
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = src[b + k * quarter];
#pragma unroll
      for (int k = 0; k < 4; ++k) sbuf[col * ld + b + k * quarter] = r[k];
    }
    __syncthreads();
    double2* x = sbuf + col * ld;
    fft_stages_one_buffer(x, b, n, logn, tw, inverse);
    v = data + (size_t)(vec0 + col) * n;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[b + k * quarter] = x[b + k * quarter];
    return;
  }
  if constexpr (TIN) {
    const int vec = (int)(blockIdx.x & 7) * (nvec >> 3) + (int)(blockIdx.x >> 3);
    const int b = vec >> logn, i = vec & (n - 1);
    const double2* src = in + ((size_t)b << (2 * logn)) + i;
    for (int j = threadIdx.x; j < n; j += blockDim.x) xa[j] = src[(size_t)j * n];
    v = data + (size_t)vec * n;
  } else {
    v = data + (size_t)blockIdx.x * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) xa[i] = v[i];
  }
  __syncthreads();
  int s = 1, logs = 0;
  {
    const int quarter = n >> 2;
    for (; logs + 2 <= logn; logs += 2, s <<= 2) {
      for (int b = threadIdx.x; b < quarter; b += blockDim.x) {
        double2 y[4];
        const int o = r4_butterfly(xa, b, quarter, s, logs, tw, inverse, y);
#pragma unroll
        for (int k = 0; k < 4; ++k) ya[o + k * s] = y[k];
      }
      __syncthreads();
      double2* t = xa; xa = ya; ya = t;
    }
  }
  const int half = n >> 1;
  for (; logs < logn; ++logs, s <<= 1) {
    const int m = half >> logs;  // half-length of the current sub-transform
    for (int b = threadIdx.x; b < half; b += blockDim.x) {
      const int q = b & (s - 1);
      const int p = b >> logs;
      const double2 a = xa[q + s * p];
      const double2 c = xa[q + s * (p + m)];
      double2 w = tw[p * s];
      if (inverse) w.y = -w.y;
      const double2 d = make_double2(a.x - c.x, a.y - c.y);
      ya[q + s * (2 * p)] = make_double2(a.x + c.x, a.y + c.y);
      ya[q + s * (2 * p + 1)] = make_double2(d.x * w.x - d.y * w.y, d.x * w.y + d.y * w.x);
    }
    __syncthreads();
    double2* t = xa; xa = ya; ya = t;
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) v[i] = xa[i];
}


// The forward transform of J (qgsw_raytrace.m:282-283 / qg2layersw_raytrace.m:
// 313-315) with the Jacobian computed in its first pass's load: vector y of
// J1 + i J2, J_l = psix.*qy - psiy.*qx from the inverse transforms
// T[2l] = psi_x + i psi_y, T[2l+1] = q_x + i q_y (layout [x + n*y]),
// transformed along x into Zj's row y — the values qg_jacobian_max_kernel
// writes, through the same per-vector FFT.  Also the CFL max of
// (u + shear)^2 + v^2 over the nl u+iv planes at uv (one atomic per block).
// R = blockDim/(n/4) rows per workgroup (n <= 1024), dynamic LDS R*n double2;
// every point load issued before the first wait.
template <int NL>
__global__ void __launch_bounds__(1024) fft_jacobian_rows_kernel(const double2* T, int n, int logn,
                                                                 const double2* uv, double shear,
                                                                 unsigned long long* dmax, const double2* tw,
                                                                 double2* Zj) {
  extern __shared__ double2 sbuf[];
  __shared__ unsigned long long bmax;  // bits of a non-negative double: integer max == double max
  const int quarter = n >> 2, t = threadIdx.x, R = (int)blockDim.x / quarter;
  const int rr = t / quarter, b = t - rr * quarter;
  double2* x = sbuf + rr * n;
  if (t == 0) bmax = 0ull;
  const int64_t nn = (int64_t)n * n;
  const int64_t row = ((int64_t)blockIdx.x * R + rr) * n;
  // the lane's four points, every load issued before the first wait
  double2 P[4][NL], Q[4][NL], Z[4][NL];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = row + b + k * quarter;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      P[k][l] = T[(2 * l) * nn + i];
      Q[k][l] = T[(2 * l + 1) * nn + i];
      Z[k][l] = uv[l * nn + i];
    }
  }
  __syncthreads();  // bmax cleared
  double m = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double J[2] = {0.0, 0.0};
#pragma unroll
    for (int l = 0; l < NL; ++l) J[l] = P[k][l].x * Q[k][l].y - P[k][l].y * Q[k][l].x;
    x[b + k * quarter] = make_double2(J[0], J[1]);
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const double u = Z[k][l].x + shear, v = Z[k][l].y;
      const double s2 = u * u + v * v;
      m = s2 > m ? s2 : m;
    }
  }
  atomicMax(&bmax, (unsigned long long)__double_as_longlong(m));  // LDS atomic
  __syncthreads();
  if (t == 0) atomicMax(dmax, bmax);
  fft_stages_one_buffer(x, b, n, logn, tw, 0);
#pragma unroll
  for (int k = 0; k < 4; ++k) Zj[row + b + k * quarter] = x[b + k * quarter];
}

// Two-layer fused mode: the second pass of the post-step inverse transforms
// fused with what reads its first five planes (n <= 1024).  Workgroup (y, h):
//   h = 0: the column pass (along x) of the four Jacobian-input planes 0-3 at
//          y, J1 + i J2 from them (the values fft_jacobian_rows_kernel
//          forms from the pass's output) and the forward pass of J along x
//          into Zj's row y;
//   h = 1: the column pass of planes 4-7 at y, the CFL max of
//          (u + shear)^2 + v^2 over planes 4, 5 (layer 1's and layer 0's
//          u + iv) and planes 5-7 (layer 0's grid_U, the snapshot) written
//          to `out` in the pass's layout [x + n*y].
// Planes 0-4 of the inverse transform never go to memory (20 MB at 512^2,
// and the Jacobian pass's 25 MB of reads).  Same per-vector FFTs and element
// operations in the same order as the column pass + fft_jacobian_rows_kernel:
// the same bits.  Block b: XCD b % 8 walks a contiguous range of y, both
// halves of one y adjacent, so the 8 columns of each 128-B line are read by
// workgroups of one XCD (one L2).  blockDim = n (4 vectors of n/4 lanes),
// dynamic LDS 4*(n+1) double2.  Zj must not alias `in` (other workgroups are
// still reading their columns).
__global__ void __launch_bounds__(1024) fft_cols_jacobian2_kernel(const double2* in, double2* out, double2* Zj,
                                                                  int n, int logn, double shear,
                                                                  unsigned long long* dmax, const double2* tw) {
  extern __shared__ double2 sbuf[];
  __shared__ unsigned long long bmax;
  const int quarter = n >> 2, t = threadIdx.x;
  const int ld = n + 1;
  const int64_t nn = (int64_t)n * n;
  const int xcd = (int)(blockIdx.x & 7), j = (int)(blockIdx.x >> 3);
  const int y = xcd * (n >> 3) + (j >> 1), h = j & 1;
  if (t == 0) bmax = 0ull;
  // lanes 4*jr .. 4*jr + 3 read row jr's four planes (4 loads per lane per row block)
  {
    const int c = t & 3, j0 = t >> 2;
    const double2* src = in + (int64_t)(4 * h + c) * nn + y;
    double2 r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = src[(int64_t)(j0 + k * quarter) * n];
#pragma unroll
    for (int k = 0; k < 4; ++k) sbuf[c * ld + j0 + k * quarter] = r[k];
  }
  __syncthreads();
  const int col = t / quarter, b = t - col * quarter;
  fft_stages_one_buffer(sbuf + col * ld, b, n, logn, tw, 1);
  if (h == 0) {
    // J at the lane's four x of vector 0 (in place: each x read and written by one lane)
    double2* x0 = sbuf;
    if (col == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = b + k * quarter;
        const double2 P0 = sbuf[i], Q0 = sbuf[ld + i], P1 = sbuf[2 * ld + i], Q1 = sbuf[3 * ld + i];
        x0[i] = make_double2(P0.x * Q0.y - P0.y * Q0.x, P1.x * Q1.y - P1.y * Q1.x);
      }
    }
    __syncthreads();
    // every vector runs the forward stages (the barriers are the workgroup's);
    // only vector 0 — J — is kept
    fft_stages_one_buffer(sbuf + col * ld, b, n, logn, tw, 0);
    if (col == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Zj[(int64_t)y * n + b + k * quarter] = x0[b + k * quarter];
    }
    return;
  }
  double m = 0.0;
  if (col < 2) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double2 z = sbuf[col * ld + b + k * quarter];
      const double u = z.x + shear, v = z.y;
      const double s2 = u * u + v * v;
      m = s2 > m ? s2 : m;
    }
  }
  if (col >= 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      out[(int64_t)(4 + col) * nn + (int64_t)y * n + b + k * quarter] = sbuf[col * ld + b + k * quarter];
  }
  for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
  if ((t & 63) == 0) atomicMax(&bmax, (unsigned long long)__double_as_longlong(m));  // LDS atomic
  __syncthreads();
  if (t == 0) atomicMax(dmax, bmax);
}

// out[c + n*r] = in[r + n*c] for batch of nb n x n complex matrices.
__global__ void transpose_kernel(const double2* in, double2* out, int n) {
  __shared__ double2 tile[32][33];
  const size_t boff = (size_t)blockIdx.z * n * n;
  const int r0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  for (int dy = threadIdx.y; dy < 32; dy += blockDim.y) {
    const int r = r0 + threadIdx.x, c = c0 + dy;
    if (r < n && c < n) tile[dy][threadIdx.x] = in[boff + r + (size_t)n * c];
  }
  __syncthreads();
  for (int dy = threadIdx.y; dy < 32; dy += blockDim.y) {
    const int c = c0 + threadIdx.x, r = r0 + dy;
    if (r < n && c < n) out[boff + c + (size_t)n * r] = tile[threadIdx.x][dy];
  }
}

// real column-major grid -> complex
__global__ void real_to_complex_kernel(const double* g, double2* z, int64_t cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cnt) z[i] = make_double2(g[i], 0.0);
}

// FFT-order index -> signed wavenumber for even n (Nyquist -> n/2).
__device__ __forceinline__ int signed_k(int r, int n) { return r <= n / 2 ? (r == n / 2 ? n / 2 : r) : r - n; }

// g2k.m:8-9 crop of the forward spectrum.  F (forward FFT2 of the grid) is in
// layout [c + n*r] (r: kx FFT index, c: ky FFT index).  Output fk is the
// (2kmax+1) x (kmax+1) column-major half plane (row kx+kmax, col ky), /nx^2.
__global__ void crop_half_kernel(const double2* F, int n, double2* fk) {
  const int kmax = n / 2 - 1, nkx = 2 * kmax + 1;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)nkx * (kmax + 1)) return;
  const int row = (int)idx % nkx, col = (int)idx / nkx;
  const int kx = row - kmax, ky = col;
  const int r = kx < 0 ? kx + n : kx, c = ky;
  const double nn = (double)n * (double)n;
  const double2 v = F[c + (size_t)n * r];
  fk[idx] = make_double2(v.x / nn, v.y / nn);
}

// Complex helpers matching MATLAB's (i*k).*z and (-i*k).*z evaluation.
__device__ __forceinline__ double2 mul_ik(double k, double2 z) { return make_double2(-(k * z.y), k * z.x); }
__device__ __forceinline__ double2 mul_mik(double k, double2 z) { return make_double2(k * z.y, -(k * z.x)); }

// Build the full Hermitian spectra (fulspec.m:10-19 + ifftshift) of the six
// derivative fields (grid_U.m:2-9 / SpectralScheme.m:16-25), packed two real
// fields per complex transform: Z0 = u + i v, Z1 = u_x + i u_y,
// Z2 = v_x + i v_y, and (if with_psi) Z3 = psi.  Output layout [c + n*r]
// (ky FFT index c contiguous), each Zk an n*n block.
// mode 0: psik = fk (SpectralScheme path); mode 1: psik = -qk./(K_d2 + K2).
// The half plane is read at fk[(kx + kmax)*sx + ky*sy]: (1, 2kmax+1) for the
// host's column-major layout, (kmax+1, 1) for the QG state's ky-fastest one.
// Where the spectra element functions put plane `pl` of full-spectrum index
// idx: an n*n block per plane in global memory, or one row per plane in LDS
// (the row-fused first FFT pass) — same values either way.
struct GlobalPlanes {
  double2* Z;
  int64_t nn;
  __device__ __forceinline__ void operator()(int pl, int64_t idx, double2 v) const { Z[pl * nn + idx] = v; }
};
struct LdsRowPlanes {
  double2* row;  // plane pl's row at row + pl*n
  int n;
  __device__ __forceinline__ void operator()(int pl, int64_t idx, double2 v) const {
    row[pl * n + ((int)idx & (n - 1))] = v;
  }
};

// spectra_to in two halves, so a kernel can issue the loads of several
// elements before any arithmetic: spectra_fetch reads the half-plane
// coefficient of full-spectrum index idx (and where it came from),
// spectra_emit turns it into the packed plane values.
struct SpecIn {
  double2 q;
  int hx, hy;
  bool cj, inband;
};
__device__ __forceinline__ SpecIn spectra_fetch(int64_t idx, const double2* fk, int n, int sx, int sy) {
  const int sh_ = __ffs(n) - 1;  // n is a power of two
  const int c = (int)idx & (n - 1), r = (int)idx >> sh_;
  const int kmax = n / 2 - 1;
  const int kx = signed_k(r, n), ky = signed_k(c, n);
  SpecIn in;
  in.inband = (kx >= -kmax && kx <= kmax && ky >= -kmax && ky <= kmax);
  // Half-plane representative (kx', ky' >= 0 side) and whether to conjugate.
  in.hx = kx;
  in.hy = ky;
  in.cj = false;
  if (ky < 0 || (ky == 0 && kx < 0)) { in.hx = -kx; in.hy = -ky; in.cj = true; }
  in.q = in.inband ? fk[(int64_t)(in.hx + kmax) * sx + (int64_t)in.hy * sy] : make_double2(0.0, 0.0);
  return in;
}
template <class Sink>
__device__ __forceinline__ void spectra_emit(const SpecIn& in, int64_t idx, int mode, double K_d2, double kscale,
                                             int with_psi, Sink out) {
  double2 z[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) z[q] = make_double2(0.0, 0.0);
  if (in.inband) {
    const double2 q = in.q;
    const double kxs = (double)in.hx * kscale, kys = (double)in.hy * kscale;
    double2 ps;
    if (mode == 0) {
      ps = q;
    } else {
      const double den = K_d2 + (kxs * kxs + kys * kys);
      ps = make_double2(-q.x / den, -q.y / den);
    }
    const double2 u = mul_mik(kys, ps);
    const double2 v = mul_ik(kxs, ps);
    double2 a[7] = {u, v, mul_ik(kxs, u), mul_ik(kys, u), mul_ik(kxs, v), mul_ik(kys, v), ps};
    if (in.hx == 0 && in.hy == 0) {
      // DC: only its real part reaches the real output of k2g.
#pragma unroll
      for (int t = 0; t < 7; ++t) a[t].y = 0.0;
    }
    if (in.cj) {
#pragma unroll
      for (int t = 0; t < 7; ++t) a[t].y = -a[t].y;
    }
    // pack: Z = A + i*B
    z[0] = make_double2(a[0].x - a[1].y, a[0].y + a[1].x);
    z[1] = make_double2(a[2].x - a[3].y, a[2].y + a[3].x);
    z[2] = make_double2(a[4].x - a[5].y, a[4].y + a[5].x);
    z[3] = a[6];
  }
  out(0, idx, z[0]);
  out(1, idx, z[1]);
  out(2, idx, z[2]);
  if (with_psi) out(3, idx, z[3]);
}
template <class Sink>
__device__ __forceinline__ void spectra_to(int64_t idx, const double2* fk, int n, int mode, double K_d2, double kscale,
                                           int with_psi, Sink out, int sx, int sy) {
  if (idx >= (int64_t)n * n) return;
  spectra_emit(spectra_fetch(idx, fk, n, sx, sy), idx, mode, K_d2, kscale, with_psi, out);
}
__device__ __forceinline__ void spectra_at(int64_t idx, const double2* fk, int n, int mode, double K_d2, double kscale,
                                           int with_psi, double2* Z, int sx, int sy) {
  spectra_to(idx, fk, n, mode, K_d2, kscale, with_psi, GlobalPlanes{Z, (int64_t)n * n}, sx, sy);
}

__global__ void spectra_kernel(const double2* fk, int n, int mode, double K_d2, double kscale,
                               int with_psi, double2* Z, int sx, int sy) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  spectra_at(idx, fk, n, mode, K_d2, kscale, with_psi, Z, sx, sy);
}

// spectra_kernel fused with the first (row) pass of the inverse 2-D FFT:
// workgroup r builds row r of the nb grid_U planes in LDS with spectra_to
// and runs their inverse row FFTs side by side (n/4 lanes each,
// fft_stages_one_buffer), writing what the spectra launch followed by the
// in-place row pass writes — the same element function and per-vector FFT,
// so the same bits (qg_post_rows_kernel's construction, for a grid_U alone:
// swrt_set_field_qk / swrt_snapshot_qk / the unfused swrt_qg_snapshot).
// blockDim nb*n/4 <= 1024, dynamic LDS nb*n double2.
__global__ void __launch_bounds__(1024) spectra_rows_kernel(const double2* fk, int n, int mode, double K_d2,
                                                            double kscale, int with_psi, int sx, int sy, int logn,
                                                            const double2* tw, double2* out) {
  extern __shared__ double2 rows[];
  const int nb = with_psi ? 4 : 3;
  const int64_t nn = (int64_t)n * n;
  const int r = blockIdx.x;
  // a lane's elements (at most 2: blockDim >= 3n/4): both loads in flight before either's arithmetic
  const int e0 = threadIdx.x, e1 = threadIdx.x + blockDim.x;
  const SpecIn in0 = spectra_fetch((int64_t)e0 + (int64_t)n * r, fk, n, sx, sy);
  SpecIn in1;
  if (e1 < n) in1 = spectra_fetch((int64_t)e1 + (int64_t)n * r, fk, n, sx, sy);
  if (e0 < n) spectra_emit(in0, (int64_t)e0 + (int64_t)n * r, mode, K_d2, kscale, with_psi, LdsRowPlanes{rows, n});
  if (e1 < n) spectra_emit(in1, (int64_t)e1 + (int64_t)n * r, mode, K_d2, kscale, with_psi, LdsRowPlanes{rows, n});
  __syncthreads();
  const int q = n >> 2;
  fft_stages_one_buffer(rows + (threadIdx.x / q) * n, threadIdx.x % q, n, logn, tw, 1);
  for (int e = threadIdx.x; e < nb * n; e += blockDim.x)
    out[(int64_t)(e / n) * nn + (int64_t)r * n + (e % n)] = rows[e];
}

// After the inverse 2-D transform Z is in layout [r + n*c] (x contiguous):
// unpack to six column-major planes (+ psi plane).
__global__ void unpair_kernel(const double2* Z, int n, int with_psi, double* planes, double* psi) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nn = (int64_t)n * n;
  if (idx >= nn) return;
  const double2 z0 = Z[idx], z1 = Z[nn + idx], z2 = Z[2 * nn + idx];
  planes[idx] = z0.x;
  planes[nn + idx] = z0.y;
  planes[2 * nn + idx] = z1.x;
  planes[3 * nn + idx] = z1.y;
  planes[4 * nn + idx] = z2.x;
  planes[5 * nn + idx] = -z1.x;  // v_y = -u_x exactly (see pack_pairs_kernel)
  if (with_psi) psi[idx] = Z[3 * nn + idx].x;
}

// fulspec.m:10-19 + ifftshift of ONE field: full Hermitian spectrum in layout
// [c + n*r] (ky FFT index contiguous).  DC keeps its real part only.
__global__ void fulspec_kernel(const double2* fk, int n, double2* Z, int sx, int sy) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nn = (int64_t)n * n;
  if (idx >= nn) return;
  const int sh_ = __ffs(n) - 1;  // n is a power of two
  const int c = (int)idx & (n - 1), r = (int)idx >> sh_;
  const int kmax = n / 2 - 1;
  const int kx = signed_k(r, n), ky = signed_k(c, n);
  double2 z = make_double2(0.0, 0.0);
  if (kx >= -kmax && kx <= kmax && ky >= -kmax && ky <= kmax) {
    int hx = kx, hy = ky;
    bool cj = false;
    if (ky < 0 || (ky == 0 && kx < 0)) { hx = -kx; hy = -ky; cj = true; }
    z = fk[(int64_t)(hx + kmax) * sx + (int64_t)hy * sy];
    if (hx == 0 && hy == 0) z.y = 0.0;
    if (cj) z.y = -z.y;
  }
  Z[idx] = z;
}

// Fused unpair + pack: the inverse transforms T0 = u + i v, T1 = u_x + i u_y,
// T2 = v_x + i v_y (layout [x + n*y]) -> interior node records (y fastest,
// 48 B each) through a 16x16 LDS tile, so both the reads (along x) and the
// record writes (along y) are contiguous.  u gets `shear` (grid_U.m:11).
// v_y is stored as -u_x, bit for bit: the flow of a streamfunction is
// divergence-free, and grid_U.m:8-9's separate transform of i ky vk equals
// -(i kx uk) up to the transform's roundoff.  The exact identity lets the
// packet kernels carry five stencil sums instead of six (swrt_tile.hpp).
// The periodic ghost records (2 below, npad - n - 2 above in each direction,
// kPadTot = 5: 2 + 3) are written by the same thread as copies of
// their interior node, so no halo pass follows.  A node x sits at padded
// row x + 2, and at x + 2 - n (x >= n - 2) and x + 2 + n (x < npad - n - 2).
__global__ void __launch_bounds__(256) pack_pairs_kernel(const double2* T, int n, int npad, double shear,
                                                         double* nodes) {
  __shared__ double2 tile[3][16][17];
  const int64_t nn = (int64_t)n * n;
  const int x0 = blockIdx.x * 16, y0 = blockIdx.y * 16;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
  for (int k = 0; k < 3; ++k) tile[k][ty][tx] = T[k * nn + (x0 + tx) + (int64_t)n * (y0 + ty)];
  __syncthreads();
  // write: thread (tx, ty) -> node x = x0 + ty, y = y0 + tx
  const double2 a = tile[0][tx][ty], b = tile[1][tx][ty], c = tile[2][tx][ty];
  const double rec[6] = {a.x + shear, a.y, b.x, b.y, c.x, -b.x};
  const int x = x0 + ty, y = y0 + tx, hi = npad - n - 2;
  // padded rows/columns holding node x (y): x + 2, and its ghost images
  const int px[3] = {x + 2, x >= n - 2 ? x + 2 - n : -1, x < hi ? x + 2 + n : -1};
  const int py[3] = {y + 2, y >= n - 2 ? y + 2 - n : -1, y < hi ? y + 2 + n : -1};
  for (int i = 0; i < 3; ++i) {
    if (px[i] < 0) continue;
    for (int j = 0; j < 3; ++j) {
      if (py[j] < 0) continue;
      double* dst = nodes + ((int64_t)px[i] * npad + py[j]) * 6;
#pragma unroll
      for (int f = 0; f < 6; ++f) dst[f] = rec[f];
    }
  }
}

// The column pass of grid_U's inverse 2-D FFT fused with pack_pairs_kernel:
// workgroup g takes CY adjacent columns y of all three planes of the row pass
// output (Z, layout [plane][r][y]), runs their 3*CY inverse column FFTs side
// by side (n/4 lanes each, fft_stages_one_buffer: the column pass's own
// per-vector arithmetic) and writes the node records {u + shear, v, u_x, u_y,
// v_x, -u_x} of those columns, with their periodic ghost images, straight
// from LDS — the values fft_vec_kernel<true> + pack_pairs_kernel write, bit
// for bit, without the 12.6 MB round trip of the transformed planes (512^2).
// Loads: lanes c, c+1, ... of one plane read a row's CY adjacent columns
// (contiguous); consecutive groups run on one XCD (its L2 shares the rows'
// 128-B lines).  Stores: the CY records of one x are contiguous (y fastest),
// and consecutive lanes store consecutive 16-B chunks of them.
// blockDim 3*CY*n/4 <= 1024, dynamic LDS 3*CY*(n+1) double2, n/CY % 8 == 0.
template <int CY>
__global__ void __launch_bounds__(1024) fft_cols_pack_kernel(const double2* Z, int n, int logn, const double2* tw,
                                                             int npad, double shear, double* nodes) {
  extern __shared__ double2 sbuf[];
  const int quarter = n >> 2, t = threadIdx.x, ld = n + 1;
  const int64_t nn = (int64_t)n * n;
  const int ng = n / CY;
  const int g = (int)(blockIdx.x & 7) * (ng >> 3) + (int)(blockIdx.x >> 3);
  const int y0 = g * CY;
  {
    // lane -> (plane, column c, rows j0 + k*quarter)
    const int per = CY * quarter, pl = t / per, u = t - pl * per;
    const int c = u % CY, j0 = u / CY;
    const double2* src = Z + pl * nn + y0 + c;
    double2 r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = src[(int64_t)(j0 + k * quarter) * n];
    double2* dst = sbuf + (pl * CY + c) * ld;
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[j0 + k * quarter] = r[k];
  }
  __syncthreads();
  fft_stages_one_buffer(sbuf + (t / quarter) * ld, t % quarter, n, logn, tw, 1);
  const int hi = npad - n - 2;
  // chunk f = (x, r): the r-th 16 B of row x's CY contiguous records (record
  // cy = r / 3, part m = r % 3: {u + shear, v}, {u_x, u_y}, {v_x, -u_x}), so
  // consecutive lanes store consecutive 16 B of a row
  constexpr int RW = 3 * CY;
  for (int f = t; f < n * RW; f += blockDim.x) {
    const int x = f / RW, r = f - x * RW, cy = r / 3, m = r - 3 * cy, y = y0 + cy;
    const double2 b = sbuf[(1 * CY + cy) * ld + x];
    double2 v;
    if (m == 0) {
      const double2 a = sbuf[(0 * CY + cy) * ld + x];
      v = make_double2(a.x + shear, a.y);
    } else if (m == 1) {
      v = b;
    } else {
      v = make_double2(sbuf[(2 * CY + cy) * ld + x].x, -b.x);
    }
    const int px[3] = {x + 2, x >= n - 2 ? x + 2 - n : -1, x < hi ? x + 2 + n : -1};
    const int py[3] = {y + 2, y >= n - 2 ? y + 2 - n : -1, y < hi ? y + 2 + n : -1};
    for (int i = 0; i < 3; ++i) {
      if (px[i] < 0) continue;
      for (int j = 0; j < 3; ++j) {
        if (py[j] < 0) continue;
        reinterpret_cast<double2*>(nodes + ((int64_t)px[i] * npad + py[j]) * 6)[m] = v;
      }
    }
  }
}

// psi plane of the packed transform T3 (layout [x + n*y]).
__global__ void psi_plane_kernel(const double2* T3, double* psi, int64_t cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cnt) psi[i] = T3[i].x;
}

// Half-plane relayout: kx-fastest (host, column-major) <-> ky-fastest (QG state).
__global__ void halfplane_relayout_kernel(const double2* in, double2* out, int nkx, int nky, int to_ky_fastest,
                                          int nlayers) {
  const int64_t nh = (int64_t)nkx * nky;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= nh * nlayers) return;
  const int64_t l = idx / nh, e = idx % nh;
  if (to_ky_fastest) {  // e = ky + nky*row (write contiguous)
    const int ky = (int)(e % nky), row = (int)(e / nky);
    out[l * nh + e] = in[l * nh + row + (int64_t)nkx * ky];
  } else {              // e = row + nkx*ky
    const int row = (int)(e % nkx), ky = (int)(e / nkx);
    out[l * nh + e] = in[l * nh + ky + (int64_t)nky * row];
  }
}

// swrt_qg_export: a half plane copied out and `tail` stored right after it
// (the owner driver's one broadcast buffer: qk's top layer, then dt)
__global__ void export_half_kernel(const double2* src, double* dst, int64_t nh, double tail) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nh) {
    const double2 v = src[i];
    dst[2 * i] = v.x;
    dst[2 * i + 1] = v.y;
  } else if (i == nh) {
    dst[2 * nh] = tail;
  }
}

__global__ void real_part_kernel(const double2* Z, double* out, int64_t cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cnt) out[i] = Z[i].x;
}

}  // namespace swrt
