// swrt_tile.hpp — LDS-tiled fused leapfrog (the throughput kernel).
//
// Packets are counting-sorted by T x T-cell spatial tile (swrt_bin.hpp).  One
// workgroup owns one tile per launch:
//   1. it stages the tile's field window — (T + 5 + 2M)^2 nodes, i.e. the
//      tile, the 6x6 stencil reach and an M-cell drift margin — for one or
//      two snapshots into LDS (chunk-major: chunk c of node e at
//      lds[c*WN + e], 16 B each, so lanes reading neighbouring nodes hit
//      different LDS banks);
//   2. on the first launch after a re-binning it counting-sorts the tile's
//      packets by their cell inside the tile (LDS histogram + scan) so that
//      the 16-lane groups of a ds_read_b128 read equal (broadcast) or
//      adjacent nodes; later launches find them in that order already (each
//      launch writes its outputs in the order it processed them);
//   3. each lane advances one packet: the 36-tap gathers come from LDS, or —
//      for a packet that drifted beyond the margin since the last re-binning —
//      from the global node array (same arithmetic, same result);
//   4. outputs are written in the in-tile sorted order to the other state
//      buffer (double-buffered), carrying the permutation along.
// Arithmetic is identical to leapfrog_kernel (same Stencil / weights / blend
// / order), so results are bit-identical to the oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swrt_kernels.hpp"

namespace swrt {

struct TileArgs {
  StepArgs s;            // fields, physics, history (s.x/s.k/s.perm are the inputs)
  double* x_out;
  double* k_out;
  int* perm_out;
  const int* starts;     // ntiles + 1 packet offsets of the tiles
  const int* order;      // non-NULL: band position -> tile (bin_scan_kernel's longest-first order)
  int ntx;               // tiles per side
  int* next_keys;        // non-NULL: write each output packet's tile (next binning) ...
  int* next_counts;      // ... and add it to the per-tile counts (zeroed by the host)
  int sort_cells;        // 1: counting-sort each tile's packets by cell first; 0: the input
                         // is already in cell order (written so by the previous launch)
  const int* src;        // non-NULL (sort launches only): binned slot p holds input packet
                         // src[p] (indirect re-binning); NULL: slot p holds packet p
  double sort_lead;      // in-tile sort key: position + sort_lead * (group velocity)
  // the band slots this launch takes (share_slot): all of them, or one
  // part's share of a split launch
  TileShare sh;
  // Multi-interval launch (ivmode, swrt_advance_intervals): nint consecutive
  // PDE intervals of s.nsteps steps each; interval i blends snapshots iv[i]
  // and iv[i+1] with alpha = alpha0 + st*dalpha (st = step within the
  // interval) at step size ivdt[i].  A workgroup owns its tile's packets for
  // the whole launch: it re-stages the window between intervals and the
  // later intervals read the previous one's output in place.
  // All snapshots share s.f0's grid; only their node arrays differ.
  int ivmode;
  int nint;
  const double* ivn[kMaxIntervals + 1];
  double ivdt[kMaxIntervals];
};

// Interval views by constant-index selects: a runtime index into the
// by-value kernel argument would copy the whole argument to scratch.
__device__ __forceinline__ const double* iv_nodes(const TileArgs& ta, int i) {
  const double* p = ta.ivn[0];
#pragma unroll
  for (int j = 1; j <= kMaxIntervals; ++j)
    if (i == j) p = ta.ivn[j];
  return p;
}
__device__ __forceinline__ double iv_dt(const TileArgs& ta, int i) {
  double d = ta.ivdt[0];
#pragma unroll
  for (int j = 1; j < kMaxIntervals; ++j)
    if (i == j) d = ta.ivdt[j];
  return d;
}

// Workgroup -> (tile, packet range).  XCD-aware (xcd_block): XCD x walks one
// contiguous band of tiles; `order` (bin_scan_kernel) lists each band's tiles
// longest first; a part launch takes its share's slots (share_slot).  The
// range is clamped to [0, n]: a corrupted binning becomes an empty or short
// range (and the scan's own check, bin_scan_kernel, reports it as an error),
// never a loop over foreign memory.
__device__ __forceinline__ int wg_work_range(const int* starts, const int* order, int64_t n, const TileShare& sh,
                                             int& pbeg, int& pend) {
  int tile = share_slot(sh, (int)blockIdx.x);
  if (order != nullptr) tile = order[tile];  // the tile at this band slot
  const int nn = (int)n;
  pbeg = min(max(starts[tile], 0), nn);
  pend = min(max(starts[tile + 1], pbeg), nn);
  return tile;
}
// one workgroup per tile (gridDim = the tiles), no tile order
__device__ __forceinline__ int wg_work_range(const int* starts, int64_t n, int& pbeg, int& pend) {
  TileShare sh;
  sh.ntiles = (int)gridDim.x;
  return wg_work_range(starts, nullptr, n, sh, pbeg, pend);
}

__device__ __forceinline__ int wg_work(const TileArgs& ta, int& pbeg, int& pend) {
  return wg_work_range(ta.starts, ta.order, ta.s.n, ta.sh, pbeg, pend);
}

// a - b on the periodic ring of n cells, mapped to [-n/2, n/2)
__device__ __forceinline__ int ring_diff(int a, int b, int n) {
  int d = a - b;
  if (d >= n / 2) d -= n;
  if (d < -n / 2) d += n;
  return d;
}

// ds_read_b128 serves a wave64 in four 16-lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} and the same +32 (MI355X_MICROARCH.md §LDS); only lanes
// of one group can conflict.  Rank of lane `lane` within its wave's run of 64
// cell-sorted packets, so that each group takes 16 consecutive packets (few
// distinct, near-adjacent nodes) instead of three scattered runs of 4-8.
__device__ __forceinline__ int b128_lane_rank(int lane) {
  const int h = lane & 32, t = lane & 31;
  int k;
  if (t < 4) k = t;
  else if (t < 12) k = 16 + (t - 4);
  else if (t < 16) k = 4 + (t - 12);
  else if (t < 20) k = 24 + (t - 16);
  else if (t < 28) k = 8 + (t - 20);
  else k = t;
  return h + k;
}

// Six-sum form (host-given fields): the weights kept per path, and — for one
// snapshot — the next tap's reads issued before this tap's arithmetic, as in
// gather5_lds below (with two snapshots the 12 reads in flight would spill).
template <bool TWO>
struct Tap6 {
  double2 a0, a1, a2, b0, b1, b2;
};
template <bool TWO, int WN>
__device__ __forceinline__ void tap6_read(const double2* p, int e, Tap6<TWO>& t) {
  t.a0 = p[0 * WN + e];
  t.a1 = p[1 * WN + e];
  t.a2 = p[2 * WN + e];
  if constexpr (TWO) {
    t.b0 = p[3 * WN + e];
    t.b1 = p[4 * WN + e];
    t.b2 = p[5 * WN + e];
  }
}
template <bool TWO, int W, int WN>
__device__ __forceinline__ void gather6_lds(const double2* lds, int node0, const Stencil& s,
                                            double o0[kRec], double o1[kRec]) {
#pragma unroll
  for (int f = 0; f < kRec; ++f) { o0[f] = -0.0; o1[f] = -0.0; }
  const double2* p = lds + node0;
  double wx[kNT], wy[kNT];
#pragma unroll
  for (int q = 0; q < kNT; ++q) {
    wx[q] = s.wx[q];
    wy[q] = s.wy[q];
    asm volatile("" : "+v"(wx[q]));
    asm volatile("" : "+v"(wy[q]));
  }
  if constexpr (TWO) {
#pragma unroll
    for (int i = 0; i < kNT; ++i) {
#pragma unroll
      for (int j = 0; j < kNT; ++j) {
        const int e = i * W + j;
        const double wij = wx[i] * wy[j];
        const double2 a0 = p[0 * WN + e], a1 = p[1 * WN + e], a2 = p[2 * WN + e];
        o0[0] = o0[0] + wij * a0.x; o0[1] = o0[1] + wij * a0.y;
        o0[2] = o0[2] + wij * a1.x; o0[3] = o0[3] + wij * a1.y;
        o0[4] = o0[4] + wij * a2.x; o0[5] = o0[5] + wij * a2.y;
        const double2 b0 = p[3 * WN + e], b1 = p[4 * WN + e], b2 = p[5 * WN + e];
        o1[0] = o1[0] + wij * b0.x; o1[1] = o1[1] + wij * b0.y;
        o1[2] = o1[2] + wij * b1.x; o1[3] = o1[3] + wij * b1.y;
        o1[4] = o1[4] + wij * b2.x; o1[5] = o1[5] + wij * b2.y;
      }
    }
    return;
  }
  Tap6<TWO> cur, nxt;
  tap6_read<TWO, WN>(p, 0, cur);
#pragma unroll
  for (int t = 0; t < kNT * kNT; ++t) {
    const int i = t / kNT, j = t % kNT;
    if (t + 1 < kNT * kNT) tap6_read<TWO, WN>(p, ((t + 1) / kNT) * W + (t + 1) % kNT, nxt);
    if constexpr (!TWO) __builtin_amdgcn_sched_barrier(0);
    const double wij = wx[i] * wy[j];
    o0[0] = o0[0] + wij * cur.a0.x; o0[1] = o0[1] + wij * cur.a0.y;
    o0[2] = o0[2] + wij * cur.a1.x; o0[3] = o0[3] + wij * cur.a1.y;
    o0[4] = o0[4] + wij * cur.a2.x; o0[5] = o0[5] + wij * cur.a2.y;
    if constexpr (TWO) {
      o1[0] = o1[0] + wij * cur.b0.x; o1[1] = o1[1] + wij * cur.b0.y;
      o1[2] = o1[2] + wij * cur.b1.x; o1[3] = o1[3] + wij * cur.b1.y;
      o1[4] = o1[4] + wij * cur.b2.x; o1[5] = o1[5] + wij * cur.b2.y;
    }
    if constexpr (!TWO) __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < kNT * kNT) cur = nxt;
  }
}

// gather6_lds for fields with v_y == -u_x bit for bit (Slot::div_free):
// five sums per snapshot from the V5 window, the same per-field order, and
// the v_y sum as the exact negation of the u_x sum (negation commutes with
// rounding), so the results are those of gather6_lds on the same nodes.
//
// Software-pipelined: tap t+1's window reads are issued before tap t's
// arithmetic, and scheduling barriers keep that order, so a wave waits only
// for reads issued one tap earlier (lgkmcnt 5..9 instead of draining to 0
// every few reads).  The weights pass through an empty asm so the compiler
// cannot hoist the 36 products wx_i*wy_j out of this path and the global
// fallback's (both compute them): 36 hoisted products held 72 VGPRs and left
// no room for the reads in flight.  Same operations, same order, same bits.
template <bool TWO>
struct Tap5 {
  double2 a0, a1, c, b0, b1;
};
template <bool TWO, int WN>
__device__ __forceinline__ void tap5_read(const double2* p, int e, Tap5<TWO>& t) {
  t.a0 = p[0 * WN + e];
  t.a1 = p[1 * WN + e];
  if constexpr (TWO) {
    t.c = p[2 * WN + e];
    t.b0 = p[3 * WN + e];
    t.b1 = p[4 * WN + e];
  } else {
    t.c.x = reinterpret_cast<const double*>(p + 2 * WN + e)[0];
  }
}
//
// PF (prefetch depth, default 1): tap t+PF's reads are issued before tap t's
// arithmetic, from a ring of PF+1 tap buffers (fully unrolled: registers).
// The sparse-tile launches (few packets per tile, at most two waves per SIMD,
// 256 VGPRs per wave) run PF = 3: a lone wave per SIMD then waits on reads
// issued three taps earlier instead of one.  Same operations, same bits.
template <bool TWO, int W, int WN, bool FMA = false, int PF = 1>
__device__ __forceinline__ void gather5_lds(const double2* lds, int node0, const Stencil& s,
                                            double o0[kRec], double o1[kRec]) {
  static_assert(PF >= 1 && PF <= 4, "prefetch depth");
  constexpr int NTAP = kNT * kNT;
#pragma unroll
  for (int f = 0; f < 5; ++f) { o0[f] = -0.0; o1[f] = -0.0; }
  const double2* p = lds + node0;
  double wx[kNT], wy[kNT];
#pragma unroll
  for (int q = 0; q < kNT; ++q) {
    wx[q] = s.wx[q];
    wy[q] = s.wy[q];
    asm volatile("" : "+v"(wx[q]));
    asm volatile("" : "+v"(wy[q]));
  }
  Tap5<TWO> ring[PF + 1];
#pragma unroll
  for (int t = 0; t < PF; ++t) tap5_read<TWO, WN>(p, (t / kNT) * W + t % kNT, ring[t]);
#pragma unroll
  for (int t = 0; t < NTAP; ++t) {
    const int i = t / kNT, j = t % kNT;
    if (t + PF < NTAP) tap5_read<TWO, WN>(p, ((t + PF) / kNT) * W + (t + PF) % kNT, ring[(t + PF) % (PF + 1)]);
    __builtin_amdgcn_sched_barrier(0);
    const Tap5<TWO>& cur = ring[t % (PF + 1)];
    const double wij = wx[i] * wy[j];
    o0[0] = madd<FMA>(o0[0], wij, cur.a0.x); o0[1] = madd<FMA>(o0[1], wij, cur.a0.y);
    o0[2] = madd<FMA>(o0[2], wij, cur.a1.x); o0[3] = madd<FMA>(o0[3], wij, cur.a1.y);
    o0[4] = madd<FMA>(o0[4], wij, cur.c.x);
    if constexpr (TWO) {
      o1[0] = madd<FMA>(o1[0], wij, cur.b0.x); o1[1] = madd<FMA>(o1[1], wij, cur.b0.y);
      o1[2] = madd<FMA>(o1[2], wij, cur.b1.x); o1[3] = madd<FMA>(o1[3], wij, cur.b1.y);
      o1[4] = madd<FMA>(o1[4], wij, cur.c.y);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  o0[5] = -o0[2];
  o1[5] = -o1[2];
}

// Stage tile (ox, oy)'s window into LDS, chunk-major (chunk c of node e at
// win[c*WN + e]): node (wi, wj) <-> global node (ox-M-2+wi, oy-M-2+wj) mod nx.
// Register staging: each lane copies whole 48-B records, 3 or 6 loads back
// to back (measured faster than LDS-DMA of the chunk-major image, whose 16-B
// pieces are 48 B apart in HBM).  The caller publishes with a barrier.
// V5 (fields with v_y == -u_x exactly): 5 chunks for two snapshots —
// {u,v}0 {ux,uy}0 {vx0,vx1} {u,v}1 {ux,uy}1 — or 3 for one, whose third
// holds {vx, vy} of which only vx is read.
template <bool TWO, int T, int M, int NT, int WS = T + 5 + 2 * M, bool V5 = false>
__device__ __forceinline__ void stage_window_regs(const FieldView& f0, const FieldView& f1, int ox, int oy,
                                                  double2* win) {
  constexpr int W = T + 5 + 2 * M;
  constexpr int WN = W * WS;  // chunk size (rows of WS >= W nodes)
  const int nx = f0.nx, npad = f0.npad;
  for (int e = threadIdx.x; e < W * W; e += NT) {
    const int wi = e / W, wj = e % W;
    int gx = (ox - M - 2 + wi) % nx; gx += gx < 0 ? nx : 0;
    int gy = (oy - M - 2 + wj) % nx; gy += gy < 0 ? nx : 0;
    const size_t src = ((size_t)(gx + kPadLo) * npad + (gy + kPadLo)) * kRec;
    const int d = wi * WS + wj;
    const double2* s0 = reinterpret_cast<const double2*>(f0.nodes + src);
    if constexpr (V5 && TWO) {
      const double2* s1 = reinterpret_cast<const double2*>(f1.nodes + src);
      const double2 a0 = s0[0], a1 = s0[1], a2 = s0[2], b0 = s1[0], b1 = s1[1], b2 = s1[2];
      win[0 * WN + d] = a0;
      win[1 * WN + d] = a1;
      win[2 * WN + d] = make_double2(a2.x, b2.x);
      win[3 * WN + d] = b0;
      win[4 * WN + d] = b1;
    } else {
      win[0 * WN + d] = s0[0];
      win[1 * WN + d] = s0[1];
      win[2 * WN + d] = s0[2];
      if constexpr (TWO) {
        const double2* s1 = reinterpret_cast<const double2*>(f1.nodes + src);
        win[3 * WN + d] = s1[0];
        win[4 * WN + d] = s1[1];
        win[5 * WN + d] = s1[2];
      }
    }
  }
}

#ifdef SWRT_PHASE_TIMING
// diagnostic build only: per-workgroup wall-clock stamps (100 MHz) of the
// phases, read back by swrt_debug_phases; never compiled into the product.
__device__ unsigned long long swrt_phase_dbg[16384 * 8];
#define SWRT_STAMP(slot)                                                            \
  do {                                                                              \
    if (tid == 0) swrt_phase_dbg[blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define SWRT_STAMP(slot) \
  do {                   \
  } while (0)
#endif

#ifndef SWRT_TILE_MIN_WAVES
#define SWRT_TILE_MIN_WAVES 4
#endif

// FMA (opt-in gather mode 1, V5 windows only): the stencil sums and the
// snapshot blend as fused multiply-adds — tolerance parity, not bits.
// PF: the five-sum gather's prefetch depth (gather5_lds); MINW: the waves per
// SIMD the register budget is sized for (4: 128 VGPRs; the sparse-tile
// instantiation, 256 threads with PF 3, takes 2: 256 VGPRs).
template <bool TWO, int T, int M, int NT, bool V5 = false, bool FMA = false, int PF = 1,
          int MINW = SWRT_TILE_MIN_WAVES>
__global__ void __launch_bounds__(NT, MINW) tile_leapfrog_kernel(TileArgs ta) {
  static_assert(!FMA || V5, "the FMA gather exists for the five-sum window only");
  constexpr int W = T + 5 + 2 * M;  // window side in nodes
  // row stride = 12 (mod 16) nodes: any 4x4 block of window nodes falls on
  // 16 distinct ds_read_b128 bank quads (node n -> quad (n mod 16)), so lanes
  // of one 16-lane group reading a few neighbouring nodes never conflict
  constexpr int WS = W + ((12 - W % 16) + 16) % 16;
  constexpr int WNP = W * WS;       // nodes per chunk
  constexpr int NCH = TWO ? (V5 ? 5 : 6) : 3;  // 16-B chunks per node
  constexpr int NB = T * T + 1;     // in-tile cell bins + "elsewhere"
  constexpr int MAXB = 2 * NT;      // packets sorted per batch
  __shared__ double2 win[NCH * WNP];
  __shared__ int hist[NB];
  __shared__ int kr[MAXB];          // key << 16 | rank
  __shared__ int order[MAXB];
  __shared__ int nbr[9];            // next-binning counts of the 3x3 neighbour tiles
#ifdef SWRT_PHASE_TIMING
  __shared__ int nfall;             // diagnostic: packet-steps that took the global gather
  __shared__ unsigned simds;        // diagnostic: SIMD id (2 bits) of every wave of the workgroup
#endif

  const StepArgs& a = ta.s;
  const int tid = threadIdx.x;
  int pbeg, pend;
  const int tile = wg_work(ta, pbeg, pend);
  const int tx = tile / ta.ntx, ty = tile % ta.ntx;
  const int nx = a.f0.nx, npad = a.f0.npad;
  const int ox = tx * T, oy = ty * T;  // tile origin (cells)
  if (tid < 9) nbr[tid] = 0;
#ifdef SWRT_PHASE_TIMING
  if (tid == 0) nfall = 0;
  if (tid == 0) simds = 0;
#endif
  SWRT_STAMP(0);
#ifdef SWRT_PHASE_TIMING
  if (tid == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    swrt_phase_dbg[blockIdx.x * 8 + 7] = ((unsigned long long)xcc << 32) | hw;
    swrt_phase_dbg[blockIdx.x * 8 + 6] = (unsigned long long)(pend - pbeg);
  }
  __syncthreads();
  if ((tid & 63) == 0) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    atomicOr(&simds, ((hw >> 4) & 3u) << (2 * (tid >> 6)));
  }
  __syncthreads();
  if (tid == 0) swrt_phase_dbg[blockIdx.x * 8 + 6] |= (unsigned long long)simds << 32;
#endif

  const int lane_rank = b128_lane_rank(tid & 63);
  const int nint = ta.ivmode ? ta.nint : 1;
  for (int ivl = 0; ivl < nint; ++ivl) {
  // interval ivl of a multi-interval launch (TileArgs::ivmode): its snapshot
  // pair and step size; the later intervals take the previous one's output
  // in place, already in cell order
  FieldView fa = a.f0, fb = a.f1;
  if (ta.ivmode) {
    fa.nodes = iv_nodes(ta, ivl);
    fb.nodes = iv_nodes(ta, ivl + 1);
  }
  const double dt = ta.ivmode ? iv_dt(ta, ivl) : a.dt;
  const double half = ta.ivmode ? 0.5 * dt : a.half;
  const bool first = ivl == 0;
  const double* xin = first ? a.x : ta.x_out;
  const double* kin = first ? a.k : ta.k_out;
  const int* pin = first ? a.perm : ta.perm_out;
  const int sortc = first ? ta.sort_cells : 0;
  const int* srcp = first ? ta.src : nullptr;
  int* nkeys = ivl == nint - 1 ? ta.next_keys : nullptr;
  const int64_t sbase = a.s0 + (int64_t)ivl * a.nsteps;
  if (!first) __syncthreads();  // every wave is done with the previous window

  // 1. stage the window
  stage_window_regs<TWO, T, M, NT, WS, V5>(fa, fb, ox, oy, win);
  if (!sortc) {
    __syncthreads();  // publish the window
    SWRT_STAMP(1);
  }
  for (int b0 = pbeg; b0 < pend; b0 += MAXB) {
    const int nb = min(MAXB, pend - b0);
    if (sortc) {
    // 2. in-tile counting sort by the cell of the current position
    for (int h = tid; h < NB; h += NT) hist[h] = 0;
    __syncthreads();  // (also publishes the window on the first batch)
    if (b0 == pbeg) SWRT_STAMP(1);
    for (int i = tid; i < nb; i += NT) {
      const int64_t p = srcp ? srcp[b0 + i] : b0 + i;
      // sort key position: the packet drifted by its group velocity to the
      // middle of the steps this order serves (x0 + sort_lead*gH*k/omega).
      // Packets of one cell separate at up to 2|cg| (k points every way), so
      // keys of the launch-start cell go stale within a cycle; the lead
      // keeps the lane groups compact over the whole cycle (LDS bank-conflict
      // model, tools/conflict_model.py: 1.40 -> 1.22 LDS cycles per access).
      // Order only: results do not depend on it.
      double xs = xin[p], ys = xin[a.n + p];
      if (ta.sort_lead != 0.0) {
        const double kx = kin[p], ky = kin[a.n + p];
        const double s = ta.sort_lead * a.gH / sqrt(a.f2 + a.gH * (kx * kx + ky * ky));
        xs += s * kx;
        ys += s * ky;
      }
      const int ic = fast_cell(xs, a.f0.inv_dx, nx);
      const int jc = fast_cell(ys, a.f0.inv_dx, nx);
      // cells predicted beyond the tile sort at its edge
      const int dx_ = min(max(ring_diff(ic, ox, nx), 0), T - 1);
      const int dy_ = min(max(ring_diff(jc, oy, nx), 0), T - 1);
      // Z-order of the cell within the tile (T = 16): a run of 16 consecutive
      // packets (one ds_read_b128 lane group) stays inside a 2x2 or 4x4 block
      // of cells — with the 12 (mod 16) row stride a conflict-free read
      // (measured: bank-conflict cycles -36 %, LDS busy -15 %)
      int key;
      if constexpr (T == 16) {
        key = (dx_ >= 0 && dx_ < T && dy_ >= 0 && dy_ < T)
                  ? ((dy_ & 1) | ((dx_ & 1) << 1) | ((dy_ & 2) << 1) | ((dx_ & 2) << 2) |
                     ((dy_ & 4) << 2) | ((dx_ & 4) << 3) | ((dy_ & 8) << 3) | ((dx_ & 8) << 4))
                  : T * T;
      } else {  // the same interleave for any power-of-two T
        key = 0;
#pragma unroll
        for (int b = 0; (1 << b) < T; ++b) key |= (((dy_ >> b) & 1) << (2 * b)) | (((dx_ >> b) & 1) << (2 * b + 1));
      }
      const int r = atomicAdd(&hist[key], 1);
      kr[i] = (key << 16) | r;
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of NB bins by one wavefront
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
      order[hist[v >> 16] + (v & 0xffff)] = srcp ? srcp[b0 + i] : b0 + i;  // input slot
    }
    __syncthreads();
    }  // sort_cells
    if (b0 == pbeg) SWRT_STAMP(2);

    // 3. advance the packets in sorted order (lane -> rank remapped for the
    //    ds_read_b128 lane groups; every rank of the batch is still taken once)
    for (int r0 = tid & ~63; r0 < nb; r0 += NT) {
      const int r = r0 + lane_rank;
      if (r >= nb) continue;
      const int64_t pi = sortc ? order[r] : b0 + r;
      const int64_t po = b0 + r;
      double x0 = xin[pi], y0 = xin[a.n + pi];
      double k0 = kin[pi], l0 = kin[a.n + pi];
      const int orig = pin[pi];
      // half-step drift of the current k, half * gH*k/omega(k)
      // (ode_symplectic.m:10-16): the second drift of a step and the first
      // drift of the next one use the same k (k0 = k2), hence the same
      // value — computed once per step, bit-identical to computing it twice.
      double hcx, hcy;
      drift_inc(k0, l0, a.f2, a.gH, half, a.fastdisp, hcx, hcy);
      // the blend's step index as a double, counted up by exact additions
      // (integers < 2^53): (double)sg without an int64 conversion per step
      double sgd = (double)(ta.ivmode ? (int64_t)0 : sbase);
      for (int st = 0; st < a.nsteps; ++st) {
        const int64_t sg = sbase + st;
        const double alpha = a.alpha0 + sgd * a.dalpha;
        sgd = sgd + 1.0;
        const double x1 = x0 + hcx;
        const double y1 = y0 + hcy;
        Stencil sc;
        stencil_at(a.f0, x1, y1, a.bump, sc);
        const int dx_ = ring_diff(sc.ic, ox, nx), dy_ = ring_diff(sc.jc, oy, nx);
        double I[kRec], J[kRec];
        const bool inwin = dx_ >= -M && dx_ < T + M && dy_ >= -M && dy_ < T + M;
#ifdef SWRT_PHASE_TIMING
        if (!inwin) atomicAdd(&nfall, 1);
#endif
        if (inwin) {
          if constexpr (V5)
            gather5_lds<TWO, WS, WNP, FMA, PF>(win, (dx_ + M) * WS + (dy_ + M), sc, I, J);
          else
            gather6_lds<TWO, WS, WNP>(win, (dx_ + M) * WS + (dy_ + M), sc, I, J);
        } else {
          gather6_lean<TWO, FMA>(fa.nodes, fb.nodes, npad, sc, I, J);
        }
        if constexpr (TWO) {
          const double oma = 1 - alpha;
          // V5 fields have v_y == -u_x in both snapshots (and both gathers
          // sum them in the same order), so the blended v_y is exactly the
          // negated blended u_x: negation commutes with every rounding
#pragma unroll
          for (int q = 0; q < (V5 ? 5 : kRec); ++q) I[q] = madd<FMA>(oma * I[q], alpha, J[q]);
          if constexpr (V5) I[5] = -I[2];
        }
        const double x2 = x1 + dt * I[0];
        const double y2 = y1 + dt * I[1];
        const double k2 = k0 - dt * (I[2] * k0 + I[4] * l0);
        const double l2 = l0 - dt * (I[3] * k0 + I[5] * l0);
        drift_inc(k2, l2, a.f2, a.gH, half, a.fastdisp, hcx, hcy);
        x0 = x2 + hcx;
        y0 = y2 + hcy;
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
      if (nkeys != nullptr) {  // fused histogram for the next re-binning
        const int ic = fast_cell(x0, a.f0.inv_dx, nx);
        const int jc = fast_cell(y0, a.f0.inv_dx, nx);
        const int ntx_ = ta.ntx;
        const int ntx2 = ic / T, nty2 = jc / T;
        nkeys[po] = ntx2 * ntx_ + nty2;
        const int ddx = ring_diff(ntx2, tx, ntx_), ddy = ring_diff(nty2, ty, ntx_);
        // Most packets stay in this tile: they cost nothing here, the tile's
        // own count is (packets in the tile) - (movers), settled at the end.
        // A mover takes one LDS atomic for a 3x3 neighbour (or one global
        // atomic beyond) and one on the stayers' correction nbr[4].
        if (ddx != 0 || ddy != 0) {
          atomicAdd(&nbr[4], -1);
          if (ddx >= -1 && ddx <= 1 && ddy >= -1 && ddy <= 1)
            atomicAdd(&nbr[(ddx + 1) * 3 + (ddy + 1)], 1);
          else
            atomicAdd(&ta.next_counts[ntx2 * ntx_ + nty2], 1);
        }
      }
    }
    __syncthreads();  // LDS sort arrays are reused by the next batch
    if (b0 == pbeg) SWRT_STAMP(3);
  }
  }  // intervals
  if (ta.next_keys != nullptr) {
    __syncthreads();
    const int v = tid < 9 ? nbr[tid] + (tid == 4 ? pend - pbeg : 0) : 0;
    if (v != 0) {
      const int n_ = ta.ntx;
      const int gx = ((tx + tid / 3 - 1) % n_ + n_) % n_, gy = ((ty + tid % 3 - 1) % n_ + n_) % n_;
      atomicAdd(&ta.next_counts[gx * n_ + gy], v);
    }
  }
  SWRT_STAMP(4);
#ifdef SWRT_PHASE_TIMING
  __syncthreads();
  if (tid == 0) swrt_phase_dbg[blockIdx.x * 8 + 5] = (unsigned long long)nfall;
#endif
}

}  // namespace swrt
