// swrt_bin.hpp — spatial binning of packets (locality for the stencil gather).
//
// Packets are independent, so their order in device memory is free: every
// `rebin_every` steps they are counting-sorted by spatial tile (TILE x TILE
// cells, tiles in row-major order) so that the lanes of a wavefront, the
// waves of a workgroup and the workgroups of one XCD gather from the same
// few cache lines of the field.  A permutation array keeps each packet's
// original index; downloads and history frames are written in the original
// order, so results are independent of the binning (and bit-identical).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swrt_kernels.hpp"

namespace swrt {

struct BinGeom {
  double dx, px, py, inv_px, inv_py, inv_dx;
  int nx;
  int tile;     // cells per tile side
  int ntx;      // tiles per side
};

__device__ __forceinline__ int tile_of(const BinGeom& g, double x, double y) {
  const int cx = fast_cell(x, g.inv_dx, g.nx);
  const int cy = fast_cell(y, g.inv_dx, g.nx);
  return (cx / g.tile) * g.ntx + (cy / g.tile);
}

// Pass 1: key per packet + histogram (LDS-aggregated, one global atomic per
// (block, occupied bin)).  Each block handles kBinPerThread packets per
// thread so the per-block LDS histogram clear is amortised.
constexpr int kMaxBins = 16384;
constexpr int kBinPerThread = 4;

__global__ void __launch_bounds__(256) bin_count_kernel(BinGeom g, const double* x, int64_t n,
                                                        int nbins, int* keys, int* counts) {
  extern __shared__ int hist[];
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) hist[b] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * blockDim.x * kBinPerThread;
  for (int q = 0; q < kBinPerThread; ++q) {
    const int64_t p = base + (int64_t)q * blockDim.x + threadIdx.x;
    if (p < n) {
      const int key = tile_of(g, x[p], x[n + p]);
      keys[p] = key;
      atomicAdd(&hist[key], 1);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    const int c = hist[b];
    if (c) atomicAdd(&counts[b], c);
  }
}

constexpr int kOrderBuckets = 16;  // workgroup rounds told apart by the tile order

// Pass 2: exclusive scan of counts -> cursor (single workgroup, nbins <= 16384).
// Also clears counts (each thread its own bins, after reading them) so the next
// fused count in the tile kernel starts from zero without a memset launch.
// Guard: the counts must be >= 0 and sum to n (the packets binned).  If not
// — a corrupted count — the scan writes an empty binning (every start 0, every
// cursor n: the scatter skips every packet, the tile launches get empty
// ranges) and raises *err (host-visible memory), which the host turns into
// SWRT_ERR_STATE at its next synchronisation.  So a bad binning is an error,
// never a launch over foreign packet ranges.
// order != NULL (nbins % 8 == 0): the tile order of the LDS-tiled launches
// (tile_order_of).  Each of the 8 XCD bands of nbins/8 consecutive tiles is
// listed longest first — by the rounds ceil(count / lanes) its workgroup of
// `lanes` threads runs (one packet per lane per round), spatial order within
// a round count — so a band's long tiles start first and its tail is made of
// the short ones (longest-processing-time-first list scheduling).  A stable
// counting sort per band by one wavefront (ballots).
__global__ void __launch_bounds__(1024) bin_scan_kernel(int* counts, int nbins, int* cursor,
                                                        int* starts, int64_t n, int* err, int* order = nullptr,
                                                        int lanes = 512) {
  __shared__ int part[1024];
  const int per = (nbins + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  int s = 0;
  int neg = 0;
  for (int i = 0; i < per; ++i) {
    const int b = b0 + i;
    if (b < nbins) {
      const int c = counts[b];
      neg |= c < 0;
      s += c;
    }
  }
  part[threadIdx.x] = s;
  neg = __syncthreads_or(neg);
  // Hillis-Steele inclusive scan over the 1024 partials
  for (int off = 1; off < 1024; off <<= 1) {
    const int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  if (neg || (int64_t)part[1023] != n) {
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
      cursor[b] = (int)n;
      starts[b] = 0;
      counts[b] = 0;
    }
    if (threadIdx.x == 0) {
      starts[nbins] = 0;
      // coherent host memory, read after events that carry no system-scope release
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (order != nullptr)
      for (int b = threadIdx.x; b < nbins; b += blockDim.x) order[b] = b;
    return;
  }
  int run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int i = 0; i < per; ++i) {
    const int b = b0 + i;
    if (b < nbins) {
      cursor[b] = run;
      starts[b] = run;
      run += counts[b];
      counts[b] = 0;
    }
  }
  if (threadIdx.x == 1023) starts[nbins] = part[1023];
  if (order == nullptr) return;
  __syncthreads();  // every start written (workgroup scope)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (nbins % 8 != 0) {
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) order[b] = b;
    return;
  }
  if (wave >= 8) return;
  const int tpx = nbins / 8, base = wave * tpx;
  const uint64_t below = (1ull << lane) - 1;
  int cnt[kOrderBuckets];
#pragma unroll
  for (int v = 0; v < kOrderBuckets; ++v) cnt[v] = 0;
  for (int c0 = 0; c0 < tpx; c0 += 64) {
    const int i = c0 + lane;
    const int r = i < tpx ? min((starts[base + i + 1] - starts[base + i] + lanes - 1) / lanes, kOrderBuckets - 1) : -1;
#pragma unroll
    for (int v = 0; v < kOrderBuckets; ++v) cnt[v] += __popcll(__ballot(r == v));
  }
  int acc = 0;
#pragma unroll
  for (int v = kOrderBuckets - 1; v >= 0; --v) {  // longest first
    const int c = cnt[v];
    cnt[v] = acc;
    acc += c;
  }
  for (int c0 = 0; c0 < tpx; c0 += 64) {
    const int i = c0 + lane;
    const int r = i < tpx ? min((starts[base + i + 1] - starts[base + i] + lanes - 1) / lanes, kOrderBuckets - 1) : -1;
#pragma unroll
    for (int v = 0; v < kOrderBuckets; ++v) {
      const uint64_t m = __ballot(r == v);
      if (r == v) order[base + cnt[v] + __popcll(m & below)] = base + i;
      cnt[v] += __popcll(m);
    }
  }
}

// Pass 3: scatter.  Each block ranks its packets per bin in LDS, reserves one
// contiguous range per occupied bin with a single global atomic, then writes.
// INDEX: write only the source index of every destination slot (src[d] = p,
// 4 B instead of the 36 B packet): the next tile launch reads its packets
// through it and writes them in binned order itself.
template <bool INDEX>
__global__ void __launch_bounds__(256) bin_scatter_kernel(const double* x, const double* k,
                                                          const int* perm, const int* keys, int64_t n,
                                                          int nbins, int* cursor, double* x2,
                                                          double* k2, int* perm2, int* src) {
  extern __shared__ int sh[];
  int* cnt = sh;            // nbins
  int* base = sh + nbins;   // nbins
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * blockDim.x * kBinPerThread;
  int key[kBinPerThread], local[kBinPerThread];
#pragma unroll
  for (int q = 0; q < kBinPerThread; ++q) {
    const int64_t p = b0 + (int64_t)q * blockDim.x + threadIdx.x;
    key[q] = 0;
    local[q] = 0;
    if (p < n) {
      key[q] = keys[p];
      local[q] = atomicAdd(&cnt[key[q]], 1);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    const int c = cnt[b];
    if (c) base[b] = atomicAdd(&cursor[b], c);
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kBinPerThread; ++q) {
    const int64_t p = b0 + (int64_t)q * blockDim.x + threadIdx.x;
    if (p < n) {
      const int64_t d = (int64_t)base[key[q]] + local[q];
      if (d < 0 || d >= n) continue;  // an empty binning after a failed scan check (bin_scan_kernel)
      if constexpr (INDEX) {
        src[d] = (int)p;
        continue;
      }
      x2[d] = x[p];
      x2[n + d] = x[n + p];
      k2[d] = k[p];
      k2[n + d] = k[n + p];
      perm2[d] = perm[p];
    }
  }
}

__global__ void iota_kernel(int* perm, int64_t n) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) perm[p] = (int)p;
}

// Binned (device) order -> original order; outputs N x 2 column-major with
// leading dimension ld >= n (the second column at xo + ld).
__global__ void unpermute_kernel(const double* x, const double* k, const int* perm, int64_t n, int64_t ld,
                                 double* xo, double* ko) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int64_t d = perm[p];
  xo[d] = x[p];
  xo[ld + d] = x[n + p];
  ko[d] = k[p];
  ko[ld + d] = k[n + p];
}

}  // namespace swrt
