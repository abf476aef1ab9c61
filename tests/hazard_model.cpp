// CPU test of the packet-buffer hazard checker (swraytracing_amd/csrc/
// swrt_hazard.hpp): replays the multi-stream launch protocol of swrt_api.hip
// (tile_launch / launch_tiles / join_b / rebin) in the abstract — buffers are
// tags, launches are accesses over the band slots the device mapping gives
// each part (swrt_share.hpp share_slot, the same function the kernels run)
// — and prints one line per scenario: "<name> ok" when the checker's verdict
// is the expected one.  Built (hipcc, host code only) and run by
// tests/test_hazard_model.py; no GPU.
#include <cstdio>
#include <string>
#include <vector>

#include "../swraytracing_amd/csrc/swrt_hazard.hpp"

using namespace swrt;

namespace {

struct Proto {
  HazardChecker h;
  int bufX[3] = {0, 1, 2};  // the three packet buffers (x stands for x, k, perm)
  int in = 0, out = 1, park = 2;
  int src = 10, counts = 11, fork = 20, join[3] = {21, 22, 23};
  int pending = 0;
  bool legacy = false;
  int ntiles = 64;  // 8 XCD bands x 8 band positions
  const void* B(int i) { return reinterpret_cast<const void*>(static_cast<intptr_t>(0x1000 + 16 * i)); }

  bool join_b() {
    for (int i = 0; i < pending; ++i) {
      h.record(B(join[i]), i + 1);
      h.wait(0, B(join[i]));
    }
    pending = 0;
    return true;
  }
  // re-binning on the packet stream (indirect: only the source index)
  bool rebin(bool do_join = true) {
    if (do_join) join_b();
    const uint64_t t = h.op(0);
    bool ok = h.access(0, t, B(bufX[in]), kHzRead, HzRegion::all(), "rebin") &&
              h.access(0, t, B(counts), kHzWrite, HzRegion::all(), "rebin") &&
              h.access(0, t, B(src), kHzWrite, HzRegion::all(), "rebin");
    ++h.epoch;
    return ok;
  }
  // one tile launch as S parts (share rule `rule`); sort = the first launch
  // after a re-binning
  bool launch(int S, bool sort, bool count_next = false, int rule = kShareEven) {
    if (S > 1) {
      h.record(B(fork), 0);
      for (int i = 1; i < S; ++i) h.wait(i, B(fork));
    }
    for (int p = 0; p < S; ++p) {
      const uint64_t t = h.op(p);
      const HzRegion r = HzRegion::of_share(h.epoch, S > 1 ? TileShare{ntiles, p, S, rule} : TileShare{ntiles, -1, 1, 0});
      bool ok = h.access(p, t, B(bufX[in]), kHzRead, sort ? HzRegion::all() : r, "part") &&
                (!sort || h.access(p, t, B(src), kHzRead, r, "part")) &&
                h.access(p, t, B(bufX[out]), kHzWrite, r, "part") &&
                (!count_next || h.access(p, t, B(counts), kHzAtomic, HzRegion::all(), "part"));
      if (!ok) return false;
    }
    pending = S - 1;
    if (sort && pending && !legacy) {  // park the gathered-from buffer
      const int x = in;
      in = out;
      out = park;
      park = x;
    } else {
      const int x = in;
      in = out;
      out = x;
    }
    return true;
  }
  // a per-packet launch over every packet on the packet stream
  bool whole(bool do_join) {
    if (do_join) join_b();
    const uint64_t t = h.op(0);
    return h.access(0, t, B(bufX[in]), kHzWrite, HzRegion::all(), "whole launch");
  }
};

int fails = 0;
void expect(const char* name, bool got, bool want, const Proto& p) {
  if (got == want) {
    std::printf("%s ok\n", name);
  } else {
    std::printf("%s FAILED (checker %s)%s%s\n", name, got ? "silent" : "reported", got ? "" : ": ",
                got ? "" : p.h.err.c_str());
    ++fails;
  }
}

}  // namespace

int main() {
  {  // the shared mapping: every slot taken exactly once by the parts of a launch, for both rules
    bool ok = true;
    for (int rule : {kShareEven, kShareSkew})
      for (int nt : {64, 72, 1024}) {
        if (rule == kShareEven && nt % 16) continue;  // the library splits evenly only when 16 | ntiles
        std::vector<int> seen(nt, 0);
        for (int p = 0; p < 2; ++p) {
          const TileShare sh{nt, p, 2, rule};
          for (int b = 0; b < share_grid(sh); ++b) ++seen[share_slot(sh, b)];
        }
        for (int v : seen) ok = ok && v == 1;
      }
    std::vector<int> all(100, 0);
    for (int b = 0; b < 100; ++b) ++all[share_slot(TileShare{100, -1, 1, 0}, b)];
    for (int v : all) ok = ok && v == 1;
    expect("share_partitions_slots", ok, true, Proto());
  }
  {  // round 4's hang: the cycle-ending launch takes a skewed share -> reported
    Proto p;
    bool ok = p.rebin();
    for (int l = 0; l < 3 && ok; ++l) ok = p.launch(2, l == 0);
    expect("even_launches_silent", ok, true, p);
    ok = p.launch(2, false, true, kShareSkew);
    expect("skewed_cycle_end_reported", ok, false, p);
    std::printf("  message: %s\n", p.h.err.c_str());
  }
  {  // a skewed share used by every launch of a binning is a consistent mapping: silent
    Proto p;
    bool ok = true;
    for (int cyc = 0; cyc < 2 && ok; ++cyc) {
      ok = ok && p.rebin();
      for (int l = 0; l < 4 && ok; ++l) ok = p.launch(2, l == 0, l == 3, kShareSkew);
    }
    expect("consistent_skew_silent", ok, true, p);
  }
  for (int S : {2}) {
    const std::string sfx = "_s" + std::to_string(S);
    {  // the library's protocol over three re-binning cycles: silent
      Proto p;
      bool ok = true;
      for (int cyc = 0; cyc < 3 && ok; ++cyc) {
        ok = ok && p.rebin();
        for (int l = 0; l < 4 && ok; ++l) ok = p.launch(S, l == 0, l == 3);
      }
      expect(("protocol_third_buffer" + sfx).c_str(), ok, true, p);
    }
    {  // legacy ordering: the launch after the sort launch is reported
      Proto p;
      p.legacy = true;
      bool ok = p.rebin() && p.launch(S, true);
      expect(("sort_launch_parts_ok" + sfx).c_str(), ok, true, p);
      ok = p.launch(S, false);
      expect(("legacy_park_reported" + sfx).c_str(), ok, false, p);
      std::printf("  message: %s\n", p.h.err.c_str());
    }
    {  // a whole launch after split calls must join first
      Proto p;
      bool ok = p.rebin() && p.launch(S, true) && p.launch(S, false);
      expect(("split_calls" + sfx).c_str(), ok, true, p);
      Proto q = p;
      expect(("whole_launch_without_join_reported" + sfx).c_str(), q.whole(false), false, q);
      expect(("whole_launch_after_join" + sfx).c_str(), p.whole(true), true, p);
    }
    {  // a re-binning must join the extra streams first
      Proto p;
      bool ok = p.rebin() && p.launch(S, true) && p.launch(S, false, true);
      Proto q = p;
      expect(("rebin_without_join_reported" + sfx).c_str(), q.rebin(false), false, q);
      expect(("rebin_after_join" + sfx).c_str(), ok && p.rebin(true), true, p);
    }
  }
  {  // host synchronisation orders everything before it
    Proto p;
    bool ok = p.rebin() && p.launch(2, true) && p.launch(2, false);
    for (int s = 0; s < kHzStreams; ++s) p.h.sync(s);
    p.pending = 0;
    expect("whole_launch_after_host_sync", ok && p.whole(false), true, p);
  }
  std::printf("%s\n", fails ? "FAILED" : "ALL OK");
  return fails ? 1 : 0;
}
