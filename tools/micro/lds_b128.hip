// Microbenchmark: ds_read_b128 bank-conflict behaviour for lane->address
// patterns (calibrates the tile kernel's gather model).  Each block: 256
// threads, 64 KB LDS of double2; every lane reads node addr(pattern, lane)
// 4096 times (offset by a loop-varying stride that keeps the pattern).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ int addr_of(int pat, int lane, int wave) {
  switch (pat) {
    case 0: return 0;                        // all lanes one node: broadcast
    case 1: return lane;                     // 64 consecutive nodes
    case 2: return lane >> 2;                // 4 lanes per node, 16 consecutive nodes
    case 3: return (lane >> 2) * 16;         // 16 nodes, all in one bank quad (stride 16)
    case 4: return lane * 16;                // 64 nodes, same bank quad
    case 5: {                                // 16 consecutive packets per ds_read_b128 group, 4 per node
      const int t = lane & 31;
      int g;  // group of the lane in {0-3,12-15,20-27} -> 0, {4-11,16-19,28-31} -> 1
      g = (t < 4 || (t >= 12 && t < 16) || (t >= 20 && t < 28)) ? 0 : 1;
      g += (lane >> 5) * 2;
      return g * 4 + (lane & 3);             // each group: 4 distinct consecutive nodes
    }
    case 6: return (lane >> 3);              // 8 lanes per node, 8 consecutive nodes
    default: return (lane * 7) & 63;
  }
}

__global__ void __launch_bounds__(256) lds_kernel(double* out, int pat, int iters) {
  __shared__ double2 buf[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) buf[i] = make_double2(i, -i);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int a = addr_of(pat, lane, wave);
  double2 acc = make_double2(0, 0);
  for (int it = 0; it < iters; ++it) {
    const int base = (it * 64) & 2047;  // multiple of 64 nodes: same bank mapping
    const double2 v = buf[base + a];
    acc.x += v.x;
    acc.y += v.y;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y;
}

int main(int argc, char** argv) {
  const int pat = argc > 1 ? atoi(argv[1]) : 0;
  const int blocks = 1024, iters = 4096;
  double* d;
  hipMalloc(&d, sizeof(double) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  lds_kernel<<<blocks, 256>>>(d, pat, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) lds_kernel<<<blocks, 256>>>(d, pat, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("pattern %d: %.3f ms per launch\n", pat, ms / 5);
  hipFree(d);
  return 0;
}
