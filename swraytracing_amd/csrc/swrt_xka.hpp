// swrt_xka.hpp — wave-action packet stepping over an RSW background.
//
// Replaces ray_trace_sw/step_packet_xka.m (+ cg_sw.m).  The reference builds
// the packet-dependent fields U.u + C.x, U.v + C.y, grad(omega), div(C) on the
// whole nx x ny grid for every packet and step (cg_sw.m:15-32, O(nx^2) per
// packet-step) and then interpolates them.  Here each of those node values is
// formed per stencil tap from the node's (u, v, H, u_x, u_y, v_x, v_y) with the
// same scalar operations in the same order, so the interpolated values are
// bit-identical while the cost drops to O(36) per interpolation.
//
// Node record: 8 doubles {u, v, H, 0, u_x, u_y, v_x, v_y} (64 B) in the same
// halo-padded x-major / y-contiguous layout as the QG snapshot nodes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swrt_kernels.hpp"
#include "swrt_tile.hpp"

namespace swrt {

constexpr int kXkaRec = 8;

struct XkaArgs {
  const double* nodes;
  int nx, npad;
  double dx, dy, inv_dx, inv_dy, px, py, inv_px, inv_py;
  double C0sq, f, f2, dt, bump;
  double* st;          // 5 x n: x, y, k, l, a (column blocks) — the output, slot p
  const double* st_in; // the input state (== st: in place)
  const int* src;      // non-NULL: slot p's packet is input slot src[p] (a re-binning read
                       // through by the launch that follows it; st_in != st)
  int64_t n;
  int nsteps;
  int64_t save_every;
  double* hist;        // frames of 5 x n (NULL: none)
  int64_t step0;       // global index of this launch's first step (frames: (step0+s+1) % save_every == 0)
  const int* perm;     // input slot -> caller's packet index (history frames); NULL: identity
  int* perm_out;       // non-NULL (with src): the output slots' permutation, perm[src[p]]
};

// Per-tap dispersion of cg_sw.m:16-26: w = sqrt(f^2 + gH*K2), cx = gH*k/w,
// cy = gH*l/w, and rw = RN(1/w) for the gradient quotients.  FAST: the short
// sequences of drift_inc (sqrt_rn_normal, one rcp_rn_normal, Markstein
// quotients div_rn_z) — the same bits as IEEE sqrt and division while the
// radicand lies in [2^-767, 2^1000] (tests/test_divconst.py,
// swrt_check_arith); a tap outside sets `bad` and the caller redoes the whole
// interpolation with the compiler's IEEE operations (FAST = false; never
// taken for physical fields, gH >= 0).
struct XkaDisp {
  double w, rw, cx, cy;
};
template <bool FAST>
__device__ __forceinline__ XkaDisp xka_disp(double f2, double gH, double K2, double k, double l, bool& bad) {
  XkaDisp d;
  const double r = f2 + gH * K2;
  if constexpr (FAST) {
    bad |= !(r >= 0x1p-767 && r <= 0x1p+1000);
    d.w = sqrt_rn_normal(r);
    d.rw = rcp_rn_normal(d.w);
    d.cx = div_rn_z(gH * k, d.w, d.rw);
    d.cy = div_rn_z(gH * l, d.w, d.rw);
  } else {
    d.w = sqrt(r);
    d.rw = 0.0;
    d.cx = gH * k / d.w;
    d.cy = gH * l / d.w;
  }
  return d;
}
// a / w and a / (2w) with the tap's dispersion (RN(1/(2w)) = RN(1/w)/2 exactly)
template <bool FAST>
__device__ __forceinline__ double xka_divw(double a, const XkaDisp& d) {
  if constexpr (FAST) return div_rn_z(a, d.w, d.rw);
  else return a / d.w;
}
template <bool FAST>
__device__ __forceinline__ double xka_div2w(double a, const XkaDisp& d) {
  if constexpr (FAST) return div_rn_z(a, 2 * d.w, 0.5 * d.rw);
  else return a / (2 * d.w);
}

struct XkaStencil {
  int ic, jc;
  double wx[kNT], wy[kNT];
};

__device__ __forceinline__ void xka_stencil(const XkaArgs& a, double x, double y, XkaStencil& s) {
  double ax, ay;
  s.ic = cell_frac(x, a.dx, a.inv_dx, a.px, a.inv_px, a.nx, a.nx, ax);
  s.jc = cell_frac(y, a.dy, a.inv_dy, a.py, a.inv_py, a.nx, a.nx, ay);
  lagrange_w(ax, a.bump, s.wx);
  lagrange_w(ay, a.bump, s.wy);
}

// Tap sources of the stencil sums: the global node array, or a tile's
// window in LDS (chunk-major: chunk c of window node e at win[c*WN + e],
// chunks {u, v}, {H, 0}, {u_x, u_y}, {v_x, v_y}).  Same values either way.
struct XkaGlobalTaps {
  const double* base;  // the stencil's first tap (ic-2, jc-2) in the padded node array
  int npad;
  __device__ __forceinline__ const double2* at(int i, int j) const {
    return reinterpret_cast<const double2*>(base + ((size_t)i * npad + j) * kXkaRec);
  }
  __device__ __forceinline__ double2 uv(int i, int j) const { return at(i, j)[0]; }
  __device__ __forceinline__ double H(int i, int j) const { return at(i, j)[1].x; }
  __device__ __forceinline__ double2 g0(int i, int j) const { return at(i, j)[2]; }
  __device__ __forceinline__ double2 g1(int i, int j) const { return at(i, j)[3]; }
};
template <int WS, int WN>
struct XkaLdsTaps {
  const double2* p;  // the stencil's first tap in the window
  __device__ __forceinline__ double2 uv(int i, int j) const { return p[0 * WN + i * WS + j]; }
  __device__ __forceinline__ double H(int i, int j) const { return p[1 * WN + i * WS + j].x; }
  __device__ __forceinline__ double2 g0(int i, int j) const { return p[2 * WN + i * WS + j]; }
  __device__ __forceinline__ double2 g1(int i, int j) const { return p[3 * WN + i * WS + j]; }
};

// interpolate(x, y, U.u + C.x) and interpolate(x, y, U.v + C.y)
// (step_packet_xka.m:42-52) with C from cg_sw.m:15-26 formed per tap.  Rows
// are not unrolled (6 taps each): the fully unrolled 4 RK stages + gradients
// held 348 VGPRs, one wave per SIMD.
template <bool FAST, class Taps>
__device__ __forceinline__ bool xka_velocity_t(const XkaArgs& a, const XkaStencil& s, const Taps& tp, double k,
                                               double l, double K2, double& Iu, double& Iv) {
  double su = 0.0, sv = 0.0;
  bool bad = false;
  // the row weights shift through registers (a run-time index into s.wx
  // would put the array in scratch)
  double wxs[kNT];
#pragma unroll
  for (int q = 0; q < kNT; ++q) wxs[q] = s.wx[q];
#pragma unroll 1
  for (int i = 0; i < kNT; ++i) {
    const double wxi = wxs[0];
#pragma unroll
    for (int q = 0; q + 1 < kNT; ++q) wxs[q] = wxs[q + 1];
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
      const double2 uv = tp.uv(i, j);
      const double H = tp.H(i, j);
      const double gH = a.C0sq * H;                   // cg_sw.m:16
      // w (cg_sw.m:22), cx, cy (cg_sw.m:25-26)
      const XkaDisp d = xka_disp<FAST>(a.f2, gH, K2, k, l, bad);
      const double wij = wxi * s.wy[j];
      su = su + wij * (uv.x + d.cx);
      sv = sv + wij * (uv.y + d.cy);
    }
  }
  Iu = su;
  Iv = sv;
  return bad;
}
template <class Taps>
__device__ __forceinline__ void xka_velocity_s(const XkaArgs& a, const XkaStencil& s, const Taps& tp, double k,
                                               double l, double K2, double& Iu, double& Iv) {
  if (xka_velocity_t<true>(a, s, tp, k, l, K2, Iu, Iv)) xka_velocity_t<false>(a, s, tp, k, l, K2, Iu, Iv);
}

// The 7 interpolations at the new position (step_packet_xka.m:59-65):
// u_x, u_y, v_x, v_y, gradomega.x, gradomega.y, divC.
template <bool FAST, class Taps>
__device__ __forceinline__ bool xka_gradients_t(const XkaArgs& a, const XkaStencil& s, const Taps& tp, double k,
                                                double l, double K2, double out[7]) {
  const double kf = k * a.f, lf = l * a.f;        // k*f, l*f (cg_sw.m:29)
  const double fK2 = a.f * K2, mfK2 = (-a.f) * K2;  // f*(k^2+l^2), -f*(k^2+l^2) (cg_sw.m:30-31)
  bool bad = false;
#pragma unroll
  for (int q = 0; q < 7; ++q) out[q] = 0.0;
  double wxs[kNT];  // (as in xka_velocity_t)
#pragma unroll
  for (int q = 0; q < kNT; ++q) wxs[q] = s.wx[q];
#pragma unroll 1
  for (int i = 0; i < kNT; ++i) {
    const double wxi = wxs[0];
#pragma unroll
    for (int q = 0; q + 1 < kNT; ++q) wxs[q] = wxs[q + 1];
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
      const double2 uv = tp.uv(i, j);
      const double H = tp.H(i, j);
      const double2 g0 = tp.g0(i, j), g1 = tp.g1(i, j);  // (u_x, u_y), (v_x, v_y)
      const double gH = a.C0sq * H;
      const XkaDisp d = xka_disp<FAST>(a.f2, gH, K2, k, l, bad);
      const double divC = xka_divw<FAST>(((kf * uv.y - lf * uv.x) - d.cx * d.cx) - d.cy * d.cy, d);  // cg_sw.m:29
      const double gwx = xka_div2w<FAST>(fK2 * uv.y, d);   // cg_sw.m:30: / (2*w)
      const double gwy = xka_div2w<FAST>(mfK2 * uv.x, d);  // cg_sw.m:31
      const double wij = wxi * s.wy[j];
      out[0] = out[0] + wij * g0.x;
      out[1] = out[1] + wij * g0.y;
      out[2] = out[2] + wij * g1.x;
      out[3] = out[3] + wij * g1.y;
      out[4] = out[4] + wij * gwx;
      out[5] = out[5] + wij * gwy;
      out[6] = out[6] + wij * divC;
    }
  }
  return bad;
}
template <class Taps>
__device__ __forceinline__ void xka_gradients_s(const XkaArgs& a, const XkaStencil& s, const Taps& tp, double k,
                                                double l, double K2, double out[7]) {
  if (xka_gradients_t<true>(a, s, tp, k, l, K2, out)) xka_gradients_t<false>(a, s, tp, k, l, K2, out);
}

// The interpolations from the global node array (the per-packet kernel).
struct XkaGlobalField {
  __device__ __forceinline__ void vel(const XkaArgs& a, double x, double y, double k, double l, double K2,
                                      double& u, double& v) const {
    XkaStencil s;
    xka_stencil(a, x, y, s);
    const XkaGlobalTaps tp{a.nodes + ((size_t)s.ic * a.npad + s.jc) * kXkaRec, a.npad};
    xka_velocity_s(a, s, tp, k, l, K2, u, v);
  }
  __device__ __forceinline__ void grad(const XkaArgs& a, double x, double y, double k, double l, double K2,
                                       double g[7]) const {
    XkaStencil s;
    xka_stencil(a, x, y, s);
    const XkaGlobalTaps tp{a.nodes + ((size_t)s.ic * a.npad + s.jc) * kXkaRec, a.npad};
    xka_gradients_s(a, s, tp, k, l, K2, g);
  }
};

// ... or from a tile's LDS window when the stencil lies inside it (the
// margin M covers the packet's motion within the launch), else globally.
template <int T, int M, int WS, int WN>
struct XkaTileField {
  const double2* win;
  int ox, oy;
  __device__ __forceinline__ bool inside(const XkaStencil& s, int nx, int& node0) const {
    int dx_ = s.ic - ox, dy_ = s.jc - oy;
    if (dx_ >= nx / 2) dx_ -= nx;
    if (dx_ < -nx / 2) dx_ += nx;
    if (dy_ >= nx / 2) dy_ -= nx;
    if (dy_ < -nx / 2) dy_ += nx;
    node0 = (dx_ + M) * WS + (dy_ + M);
    return dx_ >= -M && dx_ < T + M && dy_ >= -M && dy_ < T + M;
  }
  __device__ __forceinline__ void vel(const XkaArgs& a, double x, double y, double k, double l, double K2,
                                      double& u, double& v) const {
    XkaStencil s;
    xka_stencil(a, x, y, s);
    int node0;
    if (inside(s, a.nx, node0)) {
      xka_velocity_s(a, s, XkaLdsTaps<WS, WN>{win + node0}, k, l, K2, u, v);
    } else {
      const XkaGlobalTaps tp{a.nodes + ((size_t)s.ic * a.npad + s.jc) * kXkaRec, a.npad};
      xka_velocity_s(a, s, tp, k, l, K2, u, v);
    }
  }
  __device__ __forceinline__ void grad(const XkaArgs& a, double x, double y, double k, double l, double K2,
                                       double g[7]) const {
    XkaStencil s;
    xka_stencil(a, x, y, s);
    int node0;
    if (inside(s, a.nx, node0)) {
      xka_gradients_s(a, s, XkaLdsTaps<WS, WN>{win + node0}, k, l, K2, g);
    } else {
      const XkaGlobalTaps tp{a.nodes + ((size_t)s.ic * a.npad + s.jc) * kXkaRec, a.npad};
      xka_gradients_s(a, s, tp, k, l, K2, g);
    }
  }
};

// (a + 2b + 2c + d)/6 in MATLAB's left-to-right order; /6 = (/2 exact)/3.
__device__ __forceinline__ double rk4_mean(double a, double b, double c, double d) {
  return div_const<3>((((a + 2 * b) + 2 * c) + d) * 0.5);
}

// step_packet_xka.m:38-91 for packet p (state slot p), a.nsteps steps.
template <class Field>
__device__ __forceinline__ void xka_advance(const XkaArgs& a, const Field& fld, int64_t p) {
  const int64_t n = a.n;
  const int64_t pi = a.src ? (int64_t)a.src[p] : p;  // input slot
  double x = a.st_in[pi], y = a.st_in[n + pi], k = a.st_in[2 * n + pi], l = a.st_in[3 * n + pi],
         ac = a.st_in[4 * n + pi];
  const int64_t o = a.perm ? (int64_t)a.perm[pi] : pi;  // the caller's packet index
  if (a.perm_out) a.perm_out[p] = (int)o;
  const double dt = a.dt;
  for (int s = 0; s < a.nsteps; ++s) {
    const double K2 = k * k + l * l;  // cg_sw.m:22 (k^2+l^2)
    double u, v;
    fld.vel(a, x, y, k, l, K2, u, v);
    const double x1 = dt * u, y1 = dt * v;
    fld.vel(a, x + x1 * 0.5, y + y1 * 0.5, k, l, K2, u, v);
    const double x2 = dt * u, y2 = dt * v;
    fld.vel(a, x + x2 * 0.5, y + y2 * 0.5, k, l, K2, u, v);
    const double x3 = dt * u, y3 = dt * v;
    fld.vel(a, x + x3, y + y3, k, l, K2, u, v);
    const double x4 = dt * u, y4 = dt * v;
    const double X = x + rk4_mean(x1, x2, x3, x4);  // step_packet_xka.m:54-55
    const double Y = y + rk4_mean(y1, y2, y3, y4);
    double g[7];
    fld.grad(a, X, Y, k, l, K2, g);
    const double uxi = g[0], uyi = g[1], vxi = g[2], vyi = g[3], oxi = g[4], oyi = g[5], dci = g[6];
    // step_packet_xka.m:69-82
    const double k1 = dt * (((-uxi) * k - vxi * l) - oxi);
    const double l1 = dt * (((-uyi) * k - vyi * l) - oyi);
    const double k2 = dt * (((-uxi) * (k + k1 * 0.5) - vxi * (l + l1 * 0.5)) - oxi);
    const double l2 = dt * (((-uyi) * (k + k1 * 0.5) - vyi * (l + l1 * 0.5)) - oyi);
    const double k3 = dt * (((-uxi) * (k + k2 * 0.5) - vxi * (l + l2 * 0.5)) - oxi);
    const double l3 = dt * (((-uyi) * (k + k2 * 0.5) - vyi * (l + l2 * 0.5)) - oyi);
    const double k4 = dt * (((-uxi) * (k + k3) - vxi * (l + l3)) - oxi);
    const double l4 = dt * (((-uyi) * (k + k3) - vyi * (l + l3)) - oyi);
    const double Kn = k + rk4_mean(k1, k2, k3, k4);
    const double Ln = l + rk4_mean(l1, l2, l3, l4);
    // step_packet_xka.m:86-91
    const double a1 = dt * ((-ac) * dci);
    const double a2 = dt * ((-(ac + a1 * 0.5)) * dci);
    const double a3 = dt * ((-(ac + a2 * 0.5)) * dci);
    const double a4 = dt * ((-(ac + a3)) * dci);
    ac = ac + rk4_mean(a1, a2, a3, a4);
    x = X;
    y = Y;
    k = Kn;
    l = Ln;
    const int64_t sg = a.step0 + s + 1;  // global steps done; launches need not align with save_every
    if (a.hist != nullptr && (sg % a.save_every) == 0) {  // frames in the caller's packet order
      double* h = a.hist + (sg / a.save_every - 1) * 5 * n;
      h[o] = x; h[n + o] = y; h[2 * n + o] = k; h[3 * n + o] = l; h[4 * n + o] = ac;
    }
  }
  a.st[p] = x; a.st[n + p] = y; a.st[2 * n + p] = k; a.st[3 * n + p] = l; a.st[4 * n + p] = ac;
}

// One lane per packet, interpolations from the global node array.
__global__ void __launch_bounds__(256) xka_kernel(XkaArgs a) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.n) return;
  xka_advance(a, XkaGlobalField{}, p);
}

// LDS-tiled form over spatially binned packets (swrt_xka_step): one
// workgroup per T x T-cell tile stages the tile's window of node records —
// the tile, the stencil reach and an M-cell margin, rows padded to a 12
// (mod 16) stride — into LDS, then its lanes step the tile's packets with
// every tap of an in-window stencil read from LDS (5 interpolations x 36 taps
// per packet-step; the per-packet kernel gathered them from L1/L2, which
// bounded it).  A stencil outside the window reads global memory.  Same
// operations in the same order: the same bits.
template <int T, int M, int NT>
__global__ void __launch_bounds__(NT) xka_tile_kernel(XkaArgs a, const int* starts, int ntx) {
  constexpr int W = T + 5 + 2 * M;
  constexpr int WS = W + ((12 - W % 16) + 16) % 16;
  constexpr int WN = W * WS;
  __shared__ double2 win[4 * WN];
  int pbeg, pend;  // clamped to [0, n] (wg_work_range)
  const int tile = wg_work_range(starts, a.n, pbeg, pend);
  if (pbeg == pend) return;  // uniform: no barrier is skipped by part of the block
  const int ox = (tile / ntx) * T, oy = (tile % ntx) * T;
  const int nx = a.nx;
  for (int e = threadIdx.x; e < W * W; e += NT) {
    const int wi = e / W, wj = e % W;
    int gx = (ox - M - 2 + wi) % nx; gx += gx < 0 ? nx : 0;
    int gy = (oy - M - 2 + wj) % nx; gy += gy < 0 ? nx : 0;
    const double2* src = reinterpret_cast<const double2*>(a.nodes + ((size_t)(gx + kPadLo) * a.npad + (gy + kPadLo)) * kXkaRec);
    const double2 c0 = src[0], c1 = src[1], c2 = src[2], c3 = src[3];
    const int d = wi * WS + wj;
    win[0 * WN + d] = c0;
    win[1 * WN + d] = c1;
    win[2 * WN + d] = c2;
    win[3 * WN + d] = c3;
  }
  __syncthreads();
  const XkaTileField<T, M, WS, WN> fld{win, ox, oy};
  for (int p = pbeg + (int)threadIdx.x; p < pend; p += NT) xka_advance(a, fld, p);
}

// Spatial order for the xka lanes (swrt_xka_step): the launch after each
// re-binning reads its packets through the binned source index (XkaArgs::src)
// and writes them in binned order; the final state is scattered back to the
// caller's order through the composed permutation.  Neighbouring lanes then
// read the same few node records.  Order only: every packet is stepped by the
// same operations whatever its lane.
__global__ void xka_scatter_back_kernel(const double* st, const int* src, int64_t n, double* out) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  const int64_t p = src[d];
#pragma unroll
  for (int q = 0; q < 5; ++q) out[q * n + p] = st[q * n + d];
}

// 7 column-major planes (u, v, u_x, u_y, v_x, v_y, H) -> padded 8-double node records.
__global__ void pack_xka_kernel(const double* planes, int nx, int npad, double* nodes) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = (int64_t)npad * npad;
  if (idx >= tot) return;
  const int ip = (int)idx / npad, jp = (int)idx % npad;
  const int ig = ((ip - kPadLo) % nx + nx) % nx, jg = ((jp - kPadLo) % nx + nx) % nx;
  const int64_t plane = (int64_t)nx * nx, src = ig + (int64_t)nx * jg;
  double* d = nodes + idx * kXkaRec;
  d[0] = planes[0 * plane + src];  // u
  d[1] = planes[1 * plane + src];  // v
  d[2] = planes[6 * plane + src];  // H
  d[3] = 0.0;
  d[4] = planes[2 * plane + src];  // u_x
  d[5] = planes[3 * plane + src];  // u_y
  d[6] = planes[4 * plane + src];  // v_x
  d[7] = planes[5 * plane + src];  // v_y
}

}  // namespace swrt
