// swrt_share.hpp — workgroup -> tile mapping of the LDS-tiled launches,
// shared by the device (swrt_tile.hpp wg_work_range) and the host's
// packet-buffer hazard checker (swrt_hazard.hpp), so the checker models the
// tiles a launch actually takes.  Host/device functions only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace swrt {

// XCD-aware block order: the dispatcher deals blocks round-robin over the 8
// XCDs (b and b+8 share one); remap so each XCD walks one contiguous range of
// the (spatially binned) packet array and its L2 holds one band of the field.
// Bijective for any grid size (cdna_hip_programming.md §5 "XCD swizzle").
__host__ __device__ inline int64_t xcd_block(int64_t b, int64_t nblk) {
  const int64_t q = nblk / 8, r = nblk % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// ---- tile-to-part mapping (the "share rule") -------------------------------
// A split launch (swrt_set_packet_streams 2) runs as part launches on
// different streams that are not joined between calls; they may only ever
// touch disjoint tiles of one binning.  ONE function maps workgroup b of a
// part launch to the band slot it takes (slot s -> tile order[s] of the
// binning's longest-first order), compiled for the device (wg_work_range) and
// for the host's hazard checker (hz_tile_launch / swrt_hazard.hpp), so the
// checker models the slots a launch actually takes — any mapping, including a
// share rule that differs between launches — not a part index.
// Band position j (0 .. tpx-1, tpx = ntiles / 8) of each XCD band belongs to
//   kShareEven: part j mod S (the product rule);
//   kShareSkew (test-only, SWRT_DEBUG_SHARE_SKEW; S = 2): part 1 iff
//     j mod 3 == 2, i.e. part 0 takes two thirds — round 4's uneven split,
//     which raced when applied at one launch only (profiles/r04_stream_split).
enum { kShareEven = 0, kShareSkew = 1 };
struct TileShare {
  int ntiles = 0;  // band slots of the binning
  int part = -1;   // -1: one launch over every slot (gridDim = ntiles)
  int parts = 1;   // S
  int rule = kShareEven;
};
// k-th band position of part p
__host__ __device__ inline int share_pos(int rule, int S, int p, int k) {
  if (rule == kShareSkew) return p == 0 ? 3 * (k >> 1) + (k & 1) : 3 * k + 2;
  return S * k + p;
}
// workgroups of the launch (8 XCD bands x the part's positions per band)
__host__ __device__ inline int share_grid(const TileShare& sh) {
  if (sh.part < 0) return sh.ntiles;
  const int tpx = sh.ntiles / 8;
  if (sh.rule == kShareSkew) return 8 * (sh.part == 0 ? tpx - tpx / 3 : tpx / 3);
  return 8 * (tpx / sh.parts);
}
// band slot of workgroup b
__host__ __device__ inline int share_slot(const TileShare& sh, int b) {
  if (sh.part < 0) return (int)xcd_block(b, sh.ntiles);
  return (int)xcd_block((int64_t)share_pos(sh.rule, sh.parts, sh.part, b / 8) * 8 + b % 8, sh.ntiles);
}

}  // namespace swrt
