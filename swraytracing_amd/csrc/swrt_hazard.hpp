// swrt_hazard.hpp — debug-only happens-before checker of the packet buffers
// (host code; swrt_debug_set(ctx, SWRT_DEBUG_HAZARD_CHECK, 1) or the
// environment variable SWRT_HAZARD_CHECK=1 turns it on).
//
// The LDS-tiled leapfrog runs each launch as S = 2 part launches on two
// streams (swrt_set_packet_streams): the packet stream and an extra one.
// Between re-binnings the parts touch disjoint packet ranges, and the extra
// streams' work is joined back into the packet stream only where something
// reads every packet (join_b).  That protocol lives in comments in
// swrt_api.hip; this checker makes it testable.  It mirrors every stream
// operation that touches a packet buffer on the host, with one vector clock
// per stream (DJIT+ style):
//   * an operation on stream s advances s's own clock component;
//   * hipEventRecord(ev, s) captures s's clock, hipStreamWaitEvent(s2, ev)
//     joins it into s2's clock; a host synchronisation joins the synchronised
//     stream's clock into the host clock, which every later operation
//     inherits;
//   * each access names a buffer, a kind (read / write / atomic add) and a
//     region: the whole buffer, or a set of band slots of binning epoch e —
//     the slots the launch's workgroups actually take, enumerated with the
//     device's own mapping (swrt_share.hpp share_slot), i.e. the packets of
//     those tiles of the binning made at epoch e (and the history frames'
//     entries of those packets).  Two regions overlap unless both belong to
//     the same epoch and their slot sets are disjoint: whatever share rule a
//     launch uses, only slots proven disjoint count as disjoint.
// An access conflicts with an earlier one on an overlapping region unless
// both read (or both add atomically); a conflicting pair must be ordered:
// the earlier access's stream clock at that access <= the later stream's
// clock component for it.  The first unordered pair is reported and the
// launch that would make it is refused (swrt_api.hip returns SWRT_ERR_STATE
// before enqueuing anything), so a detected race never runs.
#pragma once
#include <stdint.h>
#include <stdio.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "swrt_share.hpp"

namespace swrt {

constexpr int kHzStreams = 3;  // 0 = packet stream, 1 = the extra packet stream, 2 = any other stream

struct HzClock {
  uint64_t v[kHzStreams] = {};
  void join(const HzClock& o) {
    for (int i = 0; i < kHzStreams; ++i) v[i] = v[i] > o.v[i] ? v[i] : o.v[i];
  }
};

struct HzRegion {
  int64_t epoch = 0;
  std::shared_ptr<const std::vector<uint64_t>> slots;  // bit s: band slot s; null: the whole buffer
  std::string desc;
  static HzRegion all() { return HzRegion{}; }
  // the band slots of the launch `sh` (every workgroup b < share_grid(sh))
  static HzRegion of_share(int64_t e, const TileShare& sh) {
    auto bits = std::make_shared<std::vector<uint64_t>>((sh.ntiles + 63) / 64, 0ull);
    const int grid = share_grid(sh);
    for (int b = 0; b < grid; ++b) {
      const int t = share_slot(sh, b);
      if (t >= 0 && t < sh.ntiles) (*bits)[t >> 6] |= 1ull << (t & 63);
    }
    HzRegion r;
    r.epoch = e;
    r.slots = bits;
    r.desc = sh.part < 0 ? std::string("every tile") :
             "part " + std::to_string(sh.part) + "/" + std::to_string(sh.parts) +
             (sh.rule == kShareSkew ? " (skewed share)" : "") + " (" + std::to_string(grid) + " tiles)";
    return r;
  }
  bool whole() const { return !slots; }
};

inline bool hz_overlap(const HzRegion& a, const HzRegion& b) {
  if (a.whole() || b.whole()) return true;
  if (a.epoch != b.epoch || a.slots->size() != b.slots->size()) return true;
  for (size_t i = 0; i < a.slots->size(); ++i)
    if ((*a.slots)[i] & (*b.slots)[i]) return true;
  return false;
}

// a is contained in b
inline bool hz_within(const HzRegion& a, const HzRegion& b) {
  if (b.whole()) return true;
  if (a.whole() || a.epoch != b.epoch || a.slots->size() != b.slots->size()) return false;
  for (size_t i = 0; i < a.slots->size(); ++i)
    if ((*a.slots)[i] & ~(*b.slots)[i]) return false;
  return true;
}

enum HzKind { kHzRead = 0, kHzWrite = 1, kHzAtomic = 2 };

struct HzAccess {
  int stream;
  uint64_t t;
  int kind;
  HzRegion r;
  const char* what;
};

struct HazardChecker {
  bool on = false;
  HzClock vc[kHzStreams];
  HzClock host;
  std::map<const void*, HzClock> events;
  std::map<const void*, std::vector<HzAccess>> bufs;
  std::map<const void*, std::string> names;
  int64_t epoch = 0;  // binning generation (advanced by every re-binning / new ensemble)
  int64_t checks = 0;  // accesses checked (diagnostic)
  std::string err;

  // start one operation on stream s; returns its time on s
  uint64_t op(int s) {
    vc[s].join(host);
    return ++vc[s].v[s];
  }
  void record(const void* ev, int s) { events[ev] = vc[s]; }
  void wait(int s, const void* ev) {
    auto it = events.find(ev);
    if (it != events.end()) vc[s].join(it->second);
  }
  // the host waited for every operation queued on s so far
  void sync(int s) { host.join(vc[s]); }
  void sync_all() {
    for (auto& c : vc) host.join(c);
  }
  // every buffer's accesses completed (host synchronised with every stream
  // that touched them): forget them (buffers may be freed and reallocated)
  void quiesce() {
    sync_all();
    bufs.clear();
  }
  void name(const void* buf, const std::string& n) { names[buf] = n; }

  static const char* kind_name(int k) { return k == kHzRead ? "read" : k == kHzWrite ? "write" : "atomic add"; }
  std::string region_name(const HzRegion& r) const {
    if (r.whole()) return "all packets";
    return r.desc + " of binning " + std::to_string(r.epoch);
  }
  std::string buf_name(const void* b) const {
    auto it = names.find(b);
    if (it != names.end()) return it->second;
    char tmp[32];
    snprintf(tmp, sizeof tmp, "%p", b);
    return tmp;
  }

  // Check one access of operation (s, t) and record it; false (err set) on a
  // conflict with an earlier access not ordered before it.
  bool access(int s, uint64_t t, const void* buf, int kind, HzRegion r, const char* what) {
    if (buf == nullptr) return true;
    std::vector<HzAccess>& acc = bufs[buf];
    for (const HzAccess& p : acc) {
      ++checks;
      if (!hz_overlap(p.r, r)) continue;
      if (p.kind == kind && kind != kHzWrite) continue;  // read/read, atomic/atomic
      if (p.stream == s || vc[s].v[p.stream] >= p.t) continue;
      err = std::string("packet-buffer hazard: ") + kind_name(kind) + " of " + buf_name(buf) + " (" +
            region_name(r) + ") by " + what + " on stream " + std::to_string(s) + " is not ordered after the " +
            kind_name(p.kind) + " (" + region_name(p.r) + ") by " + p.what + " on stream " + std::to_string(p.stream);
      return false;
    }
    // prune what this access subsumes: a write orders every later conflicting
    // access behind it (or is itself reported against it); a read replaces the
    // same stream's earlier read of the same region
    std::vector<HzAccess> keep;
    keep.reserve(acc.size() + 1);
    for (const HzAccess& p : acc) {
      const bool covered = hz_within(p.r, r);
      if (kind == kHzWrite && covered) continue;
      if (kind != kHzWrite && p.kind == kind && p.stream == s && covered) continue;
      keep.push_back(p);
    }
    keep.push_back(HzAccess{s, t, kind, r, what});
    acc.swap(keep);
    return true;
  }
};

}  // namespace swrt
