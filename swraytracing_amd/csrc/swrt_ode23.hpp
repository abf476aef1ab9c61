// swrt_ode23.hpp — device stages of the drivers' ode23 packet integrator
// (qgsw_raytrace.m:143-150, qg2layersw_raytrace.m:189-196).
//
// MATLAB's ode23 (Bogacki-Shampine 3(2), FSAL, max-norm error control)
// integrates all packets as ONE 4N-vector ODE, so the step size is a global
// decision; the host controller (swraytracing_amd/integrate.py ode23_packets)
// keeps that logic, the device does everything per packet:
//   stage 1:  F1 = odefun(t, y)             + max |F1| / max(|y|, thr)   (initial step)
//   stage 2:  F2 = odefun(t + h/2, y + F1*(h/2))
//   stage 3:  F3 = odefun(t + 3h/4, y + F2*(3h/4))
//   stage 4:  ynew = y + ((F1*(2h/9) + F2*(h/3)) + F3*(4h/9)),  F4 = odefun(tnew, ynew),
//             max |((F1 E1 + F2 E2) + F3 E3) + F4 E4| / max(max(|y|, |ynew|), thr)
// odefun (qgsw_raytrace.m:259-265): dx/dt = U + Cg*k./sqrt(f^2 + Cg^2*|k|^2),
// dk/dt = -[u_x k + v_x l, u_y k + v_y l], U and grad U from interpolate_U at
// alpha = t/tmax (same stencil code as every packet kernel).  The vectors are
// SoA over the device-ordered packets: y = {x, y} (2N) and {k, l} (2N).
// The max-norms leave the kernel as the bit pattern of a non-negative double
// through atomicMax (order independent, so the result is exact).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swrt_kernels.hpp"
#include "swrt_ode23_ctl.hpp"
#include "swrt_tile.hpp"

namespace swrt {

struct Ode23Args {
  FieldView f0, f1;
  int nslots;
  int64_t n;
  const double* yx;  // x, y   (2N)
  const double* yk;  // k, l   (2N)
  double* F[4];      // stage derivatives, 4N each: [dx; dy; dk; dl]
  double* ynx;       // ynew x, y (stage 4)
  double* ynk;       // ynew k, l
  double ts;         // stage time
  double inv_tmax;   // unused when tmax == 0 (steady)
  double tmax;
  double f2, Cg, Cg2;
  int fastdisp;      // dispersion_fast(f2): quot2_sqrt's short sequences
  double c[3];       // stage coefficients (already multiplied by h)
  // STAGE 0 (tile kernel): stages 2, 3 and 4 of one attempt fused per packet;
  // ts / c[0] are stage 2's, these stages 3 and 4's
  double ts3, ts4, c3;
  double c4[3];
  double thr;        // AbsTol / RelTol
  double bump;
  unsigned long long* dmax;
  unsigned long long* dmax_clear;  // the next max slot, zeroed for the next launch (NULL: none)
  // Speculative attempt (swrt_ode23_run): run only if gate_scale * (the
  // previous attempt's raw error max at *gate) < gate_limit — the condition
  // under which the controller certainly accepts that attempt and asks for
  // this one; otherwise every workgroup returns at once.  NULL: always run.
  const unsigned long long* gate;
  double gate_scale, gate_limit;
  const int* order;  // tile kernel: binned slots in in-tile cell order (NULL: slot order)
  // tile kernel: every workgroup's max also stored at hpart[blockIdx.x]
  // (host-mapped memory, read by swrt_ode23_run after the launch's event: no
  // copy between consecutive attempts; NULL: none)
  unsigned long long* hpart;
  // tile kernel: the share of the tiles this launch takes (swrt_share.hpp;
  // part -1: every tile, one workgroup each)
  TileShare sh;
  // STAGE 0: the attempt's coefficients {ts, c[0], ts3, c3, ts4, c4[0..2]}
  // from device memory (ode23_first_step_kernel) instead of the fields
  // above: the kernel's DC instantiation (NULL: the fields)
  const double* coef;
};

// MATLAB ode23's step-size arithmetic (o23_initial_absh, o23_step_head,
// o23_coeffs) is shared with the host controller: swrt_ode23_ctl.hpp.

// swrt_ode23_run's first attempt without a host round trip: from stage 1's
// max (the f1 launch's atomicMax slot) the initial step and the loop head,
// then the attempt's coefficients — to `coef` (read by the attempt launch
// queued behind this one) and, with {raw bits, absh, h, tnew} ahead of
// them, to host-mapped `shown`, against which the host checks its own
// computation of the same.  `clear`/`nclear`: max slots zeroed on the way
// (a split run's part-1 slots; no memset launch in front of the first
// attempt).  One lane; plain vector stores.  `shown` is coherent host memory
// and the launch's own completion event carries no system-scope release: the
// values go first, then `ticket` to shown[12] by a system-scope release
// store, and the host reads them once it sees its ticket there.
__global__ void ode23_first_step_kernel(const unsigned long long* dmax, double c0, double hmax, double htspan,
                                        double hmin0, double tdir, double t0, double tfinal, double* coef,
                                        double* shown, unsigned long long* clear, int nclear,
                                        unsigned long long ticket) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int i = 0; i < nclear; ++i) clear[i] = 0ull;
  const unsigned long long bits = *dmax;
  const double raw = __longlong_as_double((long long)bits);
  double absh = o23_initial_absh(raw, c0, hmax, htspan, hmin0);
  double h, tnew;
  (void)o23_step_head(absh, hmax, hmin0, tdir, t0, tfinal, h, tnew);
  double cf[8];
  o23_coeffs(t0, h, tnew, cf);
  for (int i = 0; i < 8; ++i) coef[i] = cf[i];
  shown[0] = raw;
  shown[1] = absh;
  shown[2] = h;
  shown[3] = tnew;
  for (int i = 0; i < 8; ++i) shown[4 + i] = cf[i];
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(shown + 12), ticket, __ATOMIC_RELEASE,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void ode_rhs(const Ode23Args& a, const double ys[4], double fo[4]) {
  const double alpha = a.tmax != 0.0 ? a.ts / a.tmax : 0.0;  // interpolate_U(..., t/tmax, ...)
  double I[kRec];
  eval_flow(a.f0, a.f1, a.nslots, alpha, ys[0], ys[1], a.bump, I);
  const double k1 = ys[2], k2 = ys[3];
  double c1, c2;  // Cg*k./sqrt(f^2 + Cg^2|k|^2)
  quot2_sqrt(a.f2 + a.Cg2 * (k1 * k1 + k2 * k2), a.Cg * k1, a.Cg * k2, a.fastdisp, c1, c2);
  fo[0] = I[0] + c1;
  fo[1] = I[1] + c2;
  fo[2] = -(I[2] * k1 + I[4] * k2);
  fo[3] = -(I[3] * k1 + I[5] * k2);
}

__device__ __forceinline__ void block_max_to(double m, unsigned long long* out) {
  __shared__ double red[256];
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicMax(out, (unsigned long long)__double_as_longlong(red[0]));
}

template <int STAGE>
__global__ void __launch_bounds__(256) ode23_stage_kernel(Ode23Args a) {
  if (a.dmax_clear && blockIdx.x == 0 && threadIdx.x == 0) *a.dmax_clear = 0ull;
  if (a.gate && !(a.gate_scale * __longlong_as_double((long long)*a.gate) < a.gate_limit)) return;
  const int64_t p = xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const int64_t n = a.n;
  double m = 0.0;
  if (p < n) {
    const double y[4] = {a.yx[p], a.yx[n + p], a.yk[p], a.yk[n + p]};
    double ys[4];
    if constexpr (STAGE == 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) ys[c] = y[c];
    } else if constexpr (STAGE == 2 || STAGE == 3) {
      const double* Fp = a.F[STAGE - 2];  // F1 for stage 2, F2 for stage 3
#pragma unroll
      for (int c = 0; c < 4; ++c) ys[c] = y[c] + Fp[c * n + p] * a.c[0];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        ys[c] = y[c] + (((a.F[0][c * n + p] * a.c[0]) + a.F[1][c * n + p] * a.c[1]) + a.F[2][c * n + p] * a.c[2]);
      a.ynx[p] = ys[0]; a.ynx[n + p] = ys[1];
      a.ynk[p] = ys[2]; a.ynk[n + p] = ys[3];
    }
    double fo[4];
    ode_rhs(a, ys, fo);
    double* Fo = a.F[STAGE - 1];
#pragma unroll
    for (int c = 0; c < 4; ++c) Fo[c * n + p] = fo[c];
    if constexpr (STAGE == 1) {
      // norm(f0 ./ max(abs(y), threshold), inf)
#pragma unroll
      for (int c = 0; c < 4; ++c) m = fmax(m, fabs(fo[c]) / fmax(fabs(y[c]), a.thr));
    } else if constexpr (STAGE == 4) {
      constexpr double E1 = -5.0 / 72.0, E2 = 1.0 / 12.0, E3 = 1.0 / 9.0, E4 = -1.0 / 8.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double fe = ((a.F[0][c * n + p] * E1 + a.F[1][c * n + p] * E2) + a.F[2][c * n + p] * E3) + fo[c] * E4;
        m = fmax(m, fabs(fe) / fmax(fmax(fabs(y[c]), fabs(ys[c])), a.thr));
      }
    }
  }
  if constexpr (STAGE == 1 || STAGE == 4) block_max_to(m, a.dmax);
}

// In-tile cell order of the binned packets (one workgroup per tile, once per
// binning): a counting sort by the Z-order of the packet's cell inside its
// tile, in batches of up to 2*NT packets, written as slot indices.  The ode23
// stages then take their packets in that order, so the lanes of one
// ds_read_b128 group read neighbouring window nodes (as the leapfrog tile
// kernel's own in-tile sort does).  Order only: results do not depend on it.
// The rank of a packet within its cell comes from an LDS atomicAdd, so the
// order of packets that share a cell may differ from run to run; each
// packet's arithmetic reads only its own state and the field, and the error
// norm is a max, so every output bit is the same for any such order (the
// ode23 GPU tests compare bits across runs and against the oracle).
template <int T, int NT>
__global__ void __launch_bounds__(NT) tile_cell_order_kernel(const double* x, int64_t n, const int* starts,
                                                             int ntx, double inv_dx, int nx,
                                                             int* order) {
  constexpr int NB = T * T;
  constexpr int MAXB = 2 * NT;
  __shared__ int hist[NB];
  __shared__ int kr[MAXB];
  int pbeg, pend;
  const int tile = wg_work_range(starts, n, pbeg, pend);
  const int ox = (tile / ntx) * T, oy = (tile % ntx) * T;
  const int tid = threadIdx.x;
  for (int b0 = pbeg; b0 < pend; b0 += MAXB) {
    const int nb = min(MAXB, pend - b0);
    for (int h = tid; h < NB; h += NT) hist[h] = 0;
    __syncthreads();
    for (int i = tid; i < nb; i += NT) {
      const int64_t p = b0 + i;
      const int dx_ = min(max(ring_diff(fast_cell(x[p], inv_dx, nx), ox, nx), 0), T - 1);
      const int dy_ = min(max(ring_diff(fast_cell(x[n + p], inv_dx, nx), oy, nx), 0), T - 1);
      int key = 0;
#pragma unroll
      for (int bit = 0; (1 << bit) < T; ++bit)
        key |= ((dy_ >> bit) & 1) << (2 * bit) | ((dx_ >> bit) & 1) << (2 * bit + 1);
      kr[i] = (key << 16) | atomicAdd(&hist[key], 1);
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the NB bins by one wavefront
      constexpr int PER = (NB + 63) / 64;
      int loc[PER];
      int sum = 0;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int h = tid * PER + q;
        loc[q] = h < NB ? hist[h] : 0;
        sum += loc[q];
      }
      int incl = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off, 64);
        if (tid >= off) incl += v;
      }
      int run = incl - sum;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int h = tid * PER + q;
        if (h < NB) hist[h] = run;
        run += loc[q];
      }
    }
    __syncthreads();
    for (int i = tid; i < nb; i += NT) {
      const int v = kr[i];
      order[b0 + hist[v >> 16] + (v & 0xffff)] = b0 + i;
    }
    __syncthreads();
  }
}

// The ode23 calls' in-tile cell order applied to the packets themselves:
// tile_cell_order_kernel's counting sort, with each packet's state (x, k and
// its original index) copied to its sorted slot of the spare buffers instead
// of writing an order array.  The stages then read y and F1 and write ynew
// and F4 at contiguous slots (through order[] every 8-byte access was
// scattered: 250 MB of writes per 1e6-packet attempt for 64 MB of outputs,
// profiles/r04_ode23).  Order only: results do not depend on it (the
// in-cell order is run-dependent, as above; the packets' original indices
// travel with them, so packets_get and the history frames are in the
// original order regardless).
template <int T, int NT>
__global__ void __launch_bounds__(NT) tile_cell_sort_kernel(const double* x, const double* k, const int* perm,
                                                            int64_t n, const int* starts, int ntx,
                                                            double inv_dx, int nx, double* x_out, double* k_out,
                                                            int* perm_out) {
  constexpr int NB = T * T;
  constexpr int MAXB = 2 * NT;
  __shared__ int hist[NB];
  __shared__ int kr[MAXB];
  int pbeg, pend;
  const int tile = wg_work_range(starts, n, pbeg, pend);
  const int ox = (tile / ntx) * T, oy = (tile % ntx) * T;
  const int tid = threadIdx.x;
  for (int b0 = pbeg; b0 < pend; b0 += MAXB) {
    const int nb = min(MAXB, pend - b0);
    for (int h = tid; h < NB; h += NT) hist[h] = 0;
    __syncthreads();
    for (int i = tid; i < nb; i += NT) {
      const int64_t p = b0 + i;
      const int dx_ = min(max(ring_diff(fast_cell(x[p], inv_dx, nx), ox, nx), 0), T - 1);
      const int dy_ = min(max(ring_diff(fast_cell(x[n + p], inv_dx, nx), oy, nx), 0), T - 1);
      int key = 0;
#pragma unroll
      for (int bit = 0; (1 << bit) < T; ++bit)
        key |= ((dy_ >> bit) & 1) << (2 * bit) | ((dx_ >> bit) & 1) << (2 * bit + 1);
      kr[i] = (key << 16) | atomicAdd(&hist[key], 1);
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the NB bins by one wavefront
      constexpr int PER = (NB + 63) / 64;
      int loc[PER];
      int sum = 0;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int h = tid * PER + q;
        loc[q] = h < NB ? hist[h] : 0;
        sum += loc[q];
      }
      int incl = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off, 64);
        if (tid >= off) incl += v;
      }
      int run = incl - sum;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int h = tid * PER + q;
        if (h < NB) hist[h] = run;
        run += loc[q];
      }
    }
    __syncthreads();
    for (int i = tid; i < nb; i += NT) {
      const int v = kr[i];
      const int64_t src = b0 + i, dst = b0 + hist[v >> 16] + (v & 0xffff);
      x_out[dst] = x[src];
      x_out[n + dst] = x[n + src];
      k_out[dst] = k[src];
      k_out[n + dst] = k[n + src];
      perm_out[dst] = perm[src];
    }
    __syncthreads();
  }
}

// The same four stages over spatially binned packets, one workgroup per
// T x T-cell tile (half-tile workgroups at the end of each XCD band) with the
// field window of both snapshots in LDS — the leapfrog tile kernel's window:
// rows padded to a 12 (mod 16) stride, the five-sum layout for
// divergence-free slots (V5) — and the packets taken in in-tile cell order
// (a.order) mapped onto the ds_read_b128 lane groups.  The packets move well
// under the M-cell margin within one PDE interval; a packet outside it takes
// the global gather.  Same arithmetic as ode23_stage_kernel, so the same bits.
// interpolate_U's alpha = t/tmax at stage time ts
__device__ __forceinline__ double alpha_of(const Ode23Args& a, double ts) { return a.tmax != 0.0 ? ts / a.tmax : 0.0; }

// odefun at ys from the tile's LDS window (or global memory outside it)
template <bool TWO, int T, int M, int WS, int WNP, bool V5>
__device__ __forceinline__ void tile_rhs(const Ode23Args& a, const double2* win, int ox, int oy, int nx,
                                         double alpha, const double ys[4], double fo[4]) {
  // odefun at (ts, ys): interpolate_U from the window (or global memory)
  Stencil sc;
  stencil_at(a.f0, ys[0], ys[1], a.bump, sc);
  const int dx_ = ring_diff(sc.ic, ox, nx), dy_ = ring_diff(sc.jc, oy, nx);
  double I[kRec], J[kRec];
  if (dx_ >= -M && dx_ < T + M && dy_ >= -M && dy_ < T + M) {
    if constexpr (V5)
      gather5_lds<TWO, WS, WNP>(win, (dx_ + M) * WS + (dy_ + M), sc, I, J);
    else
      gather6_lds<TWO, WS, WNP>(win, (dx_ + M) * WS + (dy_ + M), sc, I, J);
  } else {
    gather6_lean<TWO>(a.f0.nodes, a.f1.nodes, a.f0.npad, sc, I, J);
  }
  if constexpr (TWO) {
    const double oma = 1 - alpha;
#pragma unroll
    for (int q = 0; q < kRec; ++q) I[q] = oma * I[q] + alpha * J[q];
  }
  const double k1 = ys[2], k2 = ys[3];
  double c1, c2;  // Cg*k./sqrt(f^2 + Cg^2|k|^2)
  quot2_sqrt(a.f2 + a.Cg2 * (k1 * k1 + k2 * k2), a.Cg * k1, a.Cg * k2, a.fastdisp, c1, c2);
  fo[0] = I[0] + c1;
  fo[1] = I[1] + c2;
  fo[2] = -(I[2] * k1 + I[4] * k2);
  fo[3] = -(I[3] * k1 + I[5] * k2);
}

// DC (STAGE 0): the attempt's coefficients from a.coef (a separate
// instantiation: the first attempt of swrt_ode23_run only, so the others keep
// their coefficients in the kernel arguments' scalar registers)
template <int STAGE, bool TWO, int T, int M, int NT, bool V5, bool DC = false>
__global__ void __launch_bounds__(NT, 4) tile_ode23_kernel(Ode23Args a, const int* starts, int ntx) {
  constexpr int W = T + 5 + 2 * M;
  constexpr int WS = W + ((12 - W % 16) + 16) % 16;  // LDS row stride (nodes)
  constexpr int WNP = W * WS;
  constexpr int NCH = TWO ? (V5 ? 5 : 6) : 3;
  __shared__ double2 win[NCH * WNP];
  __shared__ double red[NT / 64];
  if (a.dmax_clear && blockIdx.x == 0 && threadIdx.x == 0) *a.dmax_clear = 0ull;
  if (a.gate && !(a.gate_scale * __longlong_as_double((long long)*a.gate) < a.gate_limit)) return;
  int pbeg, pend;
  TileShare sh = a.sh;
  if (sh.part < 0) sh.ntiles = (int)gridDim.x;
  const int tile = wg_work_range(starts, nullptr, a.n, sh, pbeg, pend);
  const int ox = (tile / ntx) * T, oy = (tile % ntx) * T;
  const int nx = a.f0.nx;
  stage_window_regs<TWO, T, M, NT, WS, V5>(a.f0, a.f1, ox, oy, win);
  __syncthreads();
  const int64_t n = a.n;
  const double alpha = a.tmax != 0.0 ? a.ts / a.tmax : 0.0;
  const int lane_rank = b128_lane_rank(threadIdx.x & 63);
  const int cnt = pend - pbeg;
  double m = 0.0;
  for (int r0 = (int)(threadIdx.x & ~63u); r0 < cnt; r0 += NT) {
    const int r = r0 + lane_rank;
    if (r >= cnt) continue;
    const int64_t p = a.order ? a.order[pbeg + r] : pbeg + r;
    const double y[4] = {a.yx[p], a.yx[n + p], a.yk[p], a.yk[n + p]};
    double ys[4];
    if constexpr (STAGE == 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) ys[c] = y[c];
    } else if constexpr (STAGE == 2 || STAGE == 3) {
      const double* Fp = a.F[STAGE - 2];
#pragma unroll
      for (int c = 0; c < 4; ++c) ys[c] = y[c] + Fp[c * n + p] * a.c[0];
    } else if constexpr (STAGE == 4) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        ys[c] = y[c] + (((a.F[0][c * n + p] * a.c[0]) + a.F[1][c * n + p] * a.c[1]) + a.F[2][c * n + p] * a.c[2]);
      a.ynx[p] = ys[0]; a.ynx[n + p] = ys[1];
      a.ynk[p] = ys[2]; a.ynk[n + p] = ys[3];
    }
    double fo[4];
    if constexpr (STAGE == 0) {
      // the attempt's coefficients
      double cf[8] = {a.ts, a.c[0], a.ts3, a.c3, a.ts4, a.c4[0], a.c4[1], a.c4[2]};
      if constexpr (DC) {  // uniform values: kept in scalar registers (vector ones spilled)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const unsigned long long v = reinterpret_cast<const unsigned long long*>(a.coef)[i];
          const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
          const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
          cf[i] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
        }
      }
      // stages 2, 3, 4 of the attempt in one pass (a rolled loop: one copy of
      // the gather, so registers stay at the single-stage count).  The sums
      // that combine the stage derivatives are carried in registers, added
      // to as each derivative appears, in the reference's order:
      //   s4 = (F1*c4[0] + F2*c4[1]) [+ F3*c4[2] at stage 4],
      //   fe = ((F1*E1 + F2*E2) + F3*E3) + F4*E4,
      // so F1 is read once and the stage-2/3 derivatives never go to memory
      // (only F4 does: the next step's F1, FSAL) — the same bits as the
      // separate stages, which store and re-read them.
      constexpr double E1 = -5.0 / 72.0, E2 = 1.0 / 12.0, E3 = 1.0 / 9.0, E4 = -1.0 / 8.0;
      double s4[4], fe[4];
#pragma unroll 1
      for (int sg = 0; sg < 3; ++sg) {
        // The packet's index re-materialised per stage: without the barrier
        // the compiler hoisted the per-packet 64-bit addresses (y, F1, F4,
        // ynew) out of the loop and kept them live across the gather — 76 B
        // per lane spilled to scratch and re-loaded every stage, most of the
        // launch's HBM writes (profiles/r04_ode23_pmc).  Recomputing them
        // costs a few integer instructions per stage.
        int64_t q = p;
        asm volatile("" : "+v"(q));
        double ts;
        // y is re-read per stage (an L2 hit) rather than held across the
        // gather: 8 VGPRs fewer at the loop's peak
        const double yv[4] = {a.yx[q], a.yx[n + q], a.yk[q], a.yk[n + q]};
        if (sg == 0) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const double f1 = a.F[0][c * n + q];
            ys[c] = yv[c] + f1 * cf[1];
            s4[c] = f1 * cf[5];
            fe[c] = f1 * E1;
          }
          ts = cf[0];
        } else if (sg == 1) {
#pragma unroll
          for (int c = 0; c < 4; ++c) ys[c] = yv[c] + fo[c] * cf[3];
          ts = cf[2];
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) ys[c] = yv[c] + (s4[c] + fo[c] * cf[7]);
          a.ynx[q] = ys[0]; a.ynx[n + q] = ys[1];
          a.ynk[q] = ys[2]; a.ynk[n + q] = ys[3];
          ts = cf[4];
        }
        tile_rhs<TWO, T, M, WS, WNP, V5>(a, win, ox, oy, nx, alpha_of(a, ts), ys, fo);
        if (sg == 0) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            s4[c] = s4[c] + fo[c] * cf[6];
            fe[c] = fe[c] + fo[c] * E2;
          }
        } else if (sg == 1) {
#pragma unroll
          for (int c = 0; c < 4; ++c) fe[c] = fe[c] + fo[c] * E3;
        }
      }
      int64_t q = p;
      asm volatile("" : "+v"(q));
#pragma unroll
      for (int c = 0; c < 4; ++c) a.F[3][c * n + q] = fo[c];
      const double yv[4] = {a.yx[q], a.yx[n + q], a.yk[q], a.yk[n + q]};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double e = fe[c] + fo[c] * E4;
        m = fmax(m, fabs(e) / fmax(fmax(fabs(yv[c]), fabs(ys[c])), a.thr));
      }
      continue;
    }
    tile_rhs<TWO, T, M, WS, WNP, V5>(a, win, ox, oy, nx, alpha, ys, fo);
    double* Fo = a.F[STAGE > 0 ? STAGE - 1 : 0];  // (STAGE 0 returned above)
#pragma unroll
    for (int c = 0; c < 4; ++c) Fo[c * n + p] = fo[c];
    if constexpr (STAGE == 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) m = fmax(m, fabs(fo[c]) / fmax(fabs(y[c]), a.thr));
    } else if constexpr (STAGE == 4) {
      constexpr double E1 = -5.0 / 72.0, E2 = 1.0 / 12.0, E3 = 1.0 / 9.0, E4 = -1.0 / 8.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double fe = ((a.F[0][c * n + p] * E1 + a.F[1][c * n + p] * E2) + a.F[2][c * n + p] * E3) + fo[c] * E4;
        m = fmax(m, fabs(fe) / fmax(fmax(fabs(y[c]), fabs(ys[c])), a.thr));
      }
    }
  }
  if constexpr (STAGE == 0 || STAGE == 1 || STAGE == 4) {
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      double b = red[0];
      for (int w = 1; w < NT / 64; ++w) b = fmax(b, red[w]);
      const unsigned long long bits = (unsigned long long)__double_as_longlong(b);
      atomicMax(a.dmax, bits);
      // system scope: the host reads it after the launch's own completion event
      if (a.hpart) __hip_atomic_store(a.hpart + blockIdx.x, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace swrt
