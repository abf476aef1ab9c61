// swrt_persist.hpp — persistent, software-pipelined LDS tile kernel.
//
// Same arithmetic and results as tile_leapfrog_kernel (bit-identical), with
// the per-tile fixed costs taken off the critical path: one 1024-lane
// workgroup per CU walks a contiguous (XCD-local) run of tiles and
//   * stages the NEXT tile's field window into the second of two LDS buffers
//     with LDS-DMA (global_load_lds_dwordx4: no VGPR round trip) while it
//     computes the current tile,
//   * counting-sorts the next tile's packets by cell and prefetches their
//     state into registers right after the current tile, so the next tile
//     starts computing immediately after one barrier.
// LDS: 2 windows x 6 chunks x 640 nodes x 16 B = 120 KB + sort arrays.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swrt_kernels.hpp"
#include "swrt_tile.hpp"

#ifndef SWRT_PERSIST_PF
#define SWRT_PERSIST_PF 2  // packets per lane taken through the sort/prefetch pipeline
#endif

namespace swrt {

template <bool TWO, int T, int M, int NT>
__global__ void __launch_bounds__(NT, 1) tile_persist_kernel(TileArgs ta, int tiles_per_wg) {
  using G = WinGeom<T, M>;
  constexpr int W = G::W;
  constexpr int WNP = G::WNP;
  constexpr int NCH = TWO ? 6 : 3;
  constexpr int NB = T * T + 1;
  constexpr int PF = SWRT_PERSIST_PF;
  constexpr int MAXB = PF * NT;  // packets per tile taken through the pipeline
  __shared__ double2 win[2][NCH * WNP];
  __shared__ int hist[NB];
  __shared__ int kr[MAXB];
  __shared__ int order[MAXB];
  __shared__ int nbr[9];

  const StepArgs& a = ta.s;
  const int tid = threadIdx.x;
  const int nx = a.f0.nx, npad = a.f0.npad;
  const int ntiles = ta.ntx * ta.ntx;
  const int wg = (int)xcd_block(blockIdx.x, gridDim.x);
  const int t_begin = wg * tiles_per_wg;
  const int t_end = min(ntiles, t_begin + tiles_per_wg);
  if (t_begin >= t_end) return;  // uniform per workgroup
  if (tid < 9) nbr[tid] = 0;

  // prefetched state of this lane's (up to 2) packets of the upcoming tile
  double px0[PF], py0[PF], pk0[PF], pl0[PF];
  int porig[PF], pcnt = 0;

  // counting sort of tile t's first min(MAXB, count) packets by cell, then
  // prefetch this lane's packets in sorted order.  Contains barriers.
  auto sort_and_prefetch = [&](int t) {
    const int tx = t / ta.ntx, ty = t % ta.ntx;
    const int ox = tx * T, oy = ty * T;
    const int b0 = ta.starts[t];
    const int nb = min(MAXB, ta.starts[t + 1] - b0);
    for (int h = tid; h < NB; h += NT) hist[h] = 0;
    __syncthreads();
    for (int i = tid; i < nb; i += NT) {
      const int64_t p = b0 + i;
      const int ic = fast_cell(a.x[p], a.f0.inv_dx, nx);
      const int jc = fast_cell(a.x[a.n + p], a.f0.inv_dx, nx);
      const int dx_ = ring_diff(ic, ox, nx), dy_ = ring_diff(jc, oy, nx);
      const int key = (dx_ >= 0 && dx_ < T && dy_ >= 0 && dy_ < T) ? dx_ * T + dy_ : T * T;
      const int r = atomicAdd(&hist[key], 1);
      kr[i] = (key << 16) | r;
    }
    __syncthreads();
    if (tid < 64) {
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
      order[hist[v >> 16] + (v & 0xffff)] = i;
    }
    __syncthreads();
    pcnt = 0;
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int r = tid + q * NT;
      if (r < nb) {
        const int64_t pi = b0 + order[r];
        px0[q] = a.x[pi];
        py0[q] = a.x[a.n + pi];
        pk0[q] = a.k[pi];
        pl0[q] = a.k[a.n + pi];
        porig[q] = a.perm[pi];
        pcnt = q + 1;
      }
    }
  };

  // advance one packet (state in registers) over a.nsteps steps with tile
  // (ox, oy)'s window `w`; writes it to output slot po.
  auto advance_packet = [&](double x0, double y0, double k0, double l0, int orig, int64_t po, int tx,
                            int ty, const double2* w) {
    const int ox = tx * T, oy = ty * T;
    for (int st = 0; st < a.nsteps; ++st) {
      const int64_t sg = a.s0 + st;
      double om = sqrt(a.f2 + a.gH * (k0 * k0 + l0 * l0));
      const double x1 = x0 + a.half * (a.gH * k0 / om);
      const double y1 = y0 + a.half * (a.gH * l0 / om);
      Stencil sc;
      stencil_at(a.f0, x1, y1, a.bump, sc);
      const int dx_ = ring_diff(sc.ic, ox, nx), dy_ = ring_diff(sc.jc, oy, nx);
      double I[kRec], J[kRec];
      if (dx_ >= -M && dx_ < T + M && dy_ >= -M && dy_ < T + M) {
        gather6_lds<TWO, W, WNP>(w, (dx_ + M) * W + (dy_ + M), sc, I, J);
      } else {
        gather6<TWO>(a.f0.nodes, a.f1.nodes, npad, sc, I, J);
      }
      if constexpr (TWO) {
        const double alpha = a.alpha0 + (double)sg * a.dalpha;
        const double oma = 1 - alpha;
#pragma unroll
        for (int q = 0; q < kRec; ++q) I[q] = oma * I[q] + alpha * J[q];
      }
      const double x2 = x1 + a.dt * I[0];
      const double y2 = y1 + a.dt * I[1];
      const double k2 = k0 - a.dt * (I[2] * k0 + I[4] * l0);
      const double l2 = l0 - a.dt * (I[3] * k0 + I[5] * l0);
      om = sqrt(a.f2 + a.gH * (k2 * k2 + l2 * l2));
      x0 = x2 + a.half * (a.gH * k2 / om);
      y0 = y2 + a.half * (a.gH * l2 / om);
      k0 = k2;
      l0 = l2;
      if (a.hist_x != nullptr && ((sg + 1) % a.save_every) == 0) {
        const int64_t fr = a.frame0 + (sg + 1) / a.save_every - 1;
        double* hx = a.hist_x + fr * 2 * a.n;
        double* hk = a.hist_k + fr * 2 * a.n;
        hx[orig] = x0; hx[a.n + orig] = y0;
        hk[orig] = k0; hk[a.n + orig] = l0;
      }
    }
    ta.x_out[po] = x0; ta.x_out[a.n + po] = y0;
    ta.k_out[po] = k0; ta.k_out[a.n + po] = l0;
    ta.perm_out[po] = orig;
    if (ta.next_keys != nullptr) {
      const int ic = fast_cell(x0, a.f0.inv_dx, nx);
      const int jc = fast_cell(y0, a.f0.inv_dx, nx);
      const int ntx_ = ta.ntx;
      const int ntx2 = ic / T, nty2 = jc / T;
      ta.next_keys[po] = ntx2 * ntx_ + nty2;
      const int ddx = ring_diff(ntx2, tx, ntx_), ddy = ring_diff(nty2, ty, ntx_);
      int nb_idx = -1;
      if (ddx >= -1 && ddx <= 1 && ddy >= -1 && ddy <= 1)
        nb_idx = (ddx + 1) * 3 + (ddy + 1);
      else
        atomicAdd(&ta.next_counts[ntx2 * ntx_ + nty2], 1);
      return nb_idx;
    }
    return -1;
  };

  // prologue: first window + first sort
  stage_window_dma<TWO, T, M>(a, (t_begin / ta.ntx) * T, (t_begin % ta.ntx) * T, win[0]);
  sort_and_prefetch(t_begin);

  for (int t = t_begin; t < t_end; ++t) {
    const int it = t - t_begin;
    const int tx = t / ta.ntx, ty = t % ta.ntx;
    const int b0 = ta.starts[t];
    const int cnt = ta.starts[t + 1] - b0;
    // consume the prefetched state into locals first, so the compiler's
    // vmcnt wait for them precedes the next tile's DMA issue
    double sx[PF], sy[PF], sk[PF], sl[PF];
    int so[PF];
    const int mycnt = pcnt;
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      sx[q] = px0[q]; sy[q] = py0[q]; sk[q] = pk0[q]; sl[q] = pl0[q]; so[q] = porig[q];
    }
    // every wave waits for its own DMA (and its prefetch loads) before the
    // barrier, so the whole window of t is in LDS after it
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 1 < t_end)
      stage_window_dma<TWO, T, M>(a, ((t + 1) / ta.ntx) * T, ((t + 1) % ta.ntx) * T, win[(it + 1) & 1]);
    const double2* w = win[it & 1];
    int nbi[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      nbi[q] = -1;
      if (q < mycnt) nbi[q] = advance_packet(sx[q], sy[q], sk[q], sl[q], so[q], b0 + tid + q * NT, tx, ty, w);
    }
    // packets beyond the pipelined MAXB (very dense tiles): unsorted, in place
    for (int r = MAXB + tid; r < cnt; r += NT) {
      const int64_t pi = b0 + r;
      const int v = advance_packet(a.x[pi], a.x[a.n + pi], a.k[pi], a.k[a.n + pi], a.perm[pi], pi, tx, ty, w);
      if (v >= 0) atomicAdd(&nbr[v], 1);
    }
    if (ta.next_keys != nullptr) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
#pragma unroll
        for (int b = 0; b < 9; ++b) {
          const unsigned long long m = __ballot(nbi[q] == b);
          if (m != 0ull && (tid & 63) == (int)__builtin_ctzll(m)) atomicAdd(&nbr[b], (int)__popcll(m));
        }
      }
      __syncthreads();
      if (tid < 9) {
        if (nbr[tid] != 0) {
          const int n_ = ta.ntx;
          const int gx = ((tx + tid / 3 - 1) % n_ + n_) % n_, gy = ((ty + tid % 3 - 1) % n_ + n_) % n_;
          atomicAdd(&ta.next_counts[gx * n_ + gy], nbr[tid]);
        }
        nbr[tid] = 0;
      }
    }
    if (t + 1 < t_end) sort_and_prefetch(t + 1);  // barriers: the next reset/reads are ordered
  }
}

}  // namespace swrt
