// swrt_diag.hpp — on-device diagnostics of the packet ensemble.
//
// analysis/load_data.m:33-52,63: omega = sqrt(f^2 + Cg^2*dot(k,k,2)) per
// packet and frame, histcounts over given edges (energy = centre * counts),
// and the mean omega per frame.  Runs on the device-resident packets, so a
// diagnostic frame costs one pass over k instead of a trajectory download.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swrt {

constexpr int kHistThreads = 256;
constexpr int kMaxHistBins = 4096;

// histcounts(w, edges): bin i holds edges[i] <= w < edges[i+1]; the last bin
// also holds w == edges[nb] (MATLAB / numpy semantics); others not counted.
__device__ __forceinline__ int hist_bin(double w, const double* edges, int nb) {
  if (!(w >= edges[0]) || !(w <= edges[nb])) return -1;
  if (w == edges[nb]) return nb - 1;
  int lo = 0, hi = nb;  // edges[lo] <= w < edges[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (w >= edges[mid]) lo = mid; else hi = mid;
  }
  return lo;
}

// Per-block LDS histogram -> global 64-bit counts; per-block omega sums into
// `partial` (summed in block order by omega_sum_kernel: deterministic).
__global__ void __launch_bounds__(kHistThreads) omega_hist_kernel(const double* k, int64_t n, double f2,
                                                                  double Cg2, const double* edges, int nb,
                                                                  unsigned long long* counts,
                                                                  double* partial) {
  __shared__ unsigned int h[kMaxHistBins];
  __shared__ double red[kHistThreads];
  __shared__ double sedges[kMaxHistBins + 1];
  for (int b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  for (int b = threadIdx.x; b <= nb; b += blockDim.x) sedges[b] = edges[b];
  __syncthreads();
  double s = 0.0;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const double k1 = k[p], k2 = k[n + p];
    const double w = sqrt(f2 + Cg2 * (k1 * k1 + k2 * k2));  // load_data.m:33
    s += w;
    const int b = hist_bin(w, sedges, nb);
    if (b >= 0) atomicAdd(&h[b], 1u);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = blockDim.x / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&counts[b], (unsigned long long)h[b]);
}

__global__ void omega_sum_kernel(const double* partial, int nblk, double* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < nblk; ++i) s += partial[i];
    *out = s;
  }
}

}  // namespace swrt
