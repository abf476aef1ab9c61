// swrt_clock.cpp — the observed-shader-clock arithmetic of swrt_clock_ghz,
// host-only (no device): swrt_api.hip hands it the probe waves' stamps, the
// CPU tests hand it synthetic ones (tests/test_clock_pairs.py).
//
// Each probe wave recorded {s_memtime (shader cycles), s_memrealtime (100 MHz),
// CU id}.  The cycle counters of different CUs are not aligned, so a clock is
// only formed from ONE CU's first start stamp and last end stamp; the result
// is the median over the CUs stamped at both ends.  When no CU ran both a start
// and an end wave (e.g. another process's kernels held the CUs while the probes
// ran — ranks sharing one GPU), there is no clock: SWRT_ERR_STATE, which
// bench.py reports as an unobserved clock (null), never as a failed run.
#include <algorithm>
#include <cstdint>
#include <map>
#include <utility>
#include <vector>

#include "../../include/swrt.h"

extern "C" int swrt_clock_ghz_stamps(const uint64_t* stamps, int64_t waves, double realtime_hz, double* ghz_out,
                                     double* spread_out) {
  if (!stamps || waves < 1 || !(realtime_hz > 0) || !ghz_out) return SWRT_ERR_ARG;
  try {
    const uint64_t* s = stamps;              // start waves: {cycles, realtime, cu} each
    const uint64_t* e = stamps + waves * 3;  // end waves
    // per CU: its first start stamp and its last end stamp
    std::map<uint64_t, std::pair<int64_t, int64_t>> cu;  // id -> (start wave, end wave)
    for (int64_t i = 0; i < waves; ++i) {
      auto& p = cu.emplace(s[3 * i + 2], std::make_pair(int64_t(-1), int64_t(-1))).first->second;
      if (p.first < 0 || s[3 * i + 1] < s[3 * p.first + 1]) p.first = i;
    }
    for (int64_t j = 0; j < waves; ++j) {
      auto it = cu.find(e[3 * j + 2]);
      if (it != cu.end() && (it->second.second < 0 || e[3 * j + 1] > e[3 * it->second.second + 1]))
        it->second.second = j;
    }
    std::vector<double> ghz;
    for (const auto& kv : cu) {
      const int64_t i = kv.second.first, j = kv.second.second;
      if (i < 0 || j < 0 || e[3 * j + 1] <= s[3 * i + 1] || e[3 * j] <= s[3 * i]) continue;
      const double sec = (double)(e[3 * j + 1] - s[3 * i + 1]) / realtime_hz;
      ghz.push_back((double)(e[3 * j] - s[3 * i]) / sec / 1e9);
    }
    if (ghz.empty()) return SWRT_ERR_STATE;
    std::sort(ghz.begin(), ghz.end());
    const double med = ghz[ghz.size() / 2];
    *ghz_out = med;
    // spread of the per-CU clocks: (p90 - p10) / median over the CUs paired
    if (spread_out) *spread_out = (ghz[(ghz.size() * 9) / 10] - ghz[ghz.size() / 10]) / med;
    return SWRT_OK;
  } catch (...) {
    return SWRT_ERR_ALLOC;
  }
}
