// swrt_api.hip — the C ABI (include/swrt.h) over the gfx950 kernels.
//
// Host-side orchestration only: device buffers owned by the context, one HIP
// stream per context, every call synchronous to the host and exception-free
// across the ABI boundary.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "../../include/swrt.h"
#include "swrt_bin.hpp"
#include "swrt_fft.hpp"
#include "swrt_kernels.hpp"
#include "swrt_tile.hpp"
#include "swrt_qg.hpp"
#include "swrt_ode23.hpp"
#include "swrt_xka.hpp"
#include "swrt_rsw.hpp"
#include "swrt_spectral.hpp"
#include "swrt_hazard.hpp"
#include "swrt_diag.hpp"

using namespace swrt;

namespace {

constexpr int kMaxStepsPerLaunch = 64;  // bound one launch's run time
// a host copy of an attempt workgroup's error max not yet written (no max of
// non-negative doubles, NaN included, has this bit pattern)
constexpr unsigned long long kHpartEmpty = ~0ull;
constexpr int kXkaMargin = 3;           // xka_tile_kernel: drift margin (cells) of a tile's window
#ifndef SWRT_TILE
#define SWRT_TILE 16
#endif
#ifndef SWRT_MARGIN
#define SWRT_MARGIN 3
#endif
#ifndef SWRT_SORT_LEAD
#define SWRT_SORT_LEAD 1
#endif
#ifndef SWRT_TILE_THREADS
#define SWRT_TILE_THREADS 512
#endif
constexpr int kTile = SWRT_TILE;                // LDS tile kernel: cells per tile side
constexpr int kMargin = SWRT_MARGIN;            // LDS tile kernel: drift margin (cells)
constexpr int kTileThreads = SWRT_TILE_THREADS;
// Sparse-tile launches: below SWRT_SPARSE_BELOW packets per 16x16 tile on
// average (a strong-scaling shard: ~120 at 1.25e5 packets on 512^2) a
// 512-thread workgroup has one or two busy waves, one per SIMD, each capped
// at 128 VGPRs by the dense launch's 4-waves-per-SIMD budget and waiting on
// LDS reads issued one tap earlier, and its idle waves hold their registers
// until the workgroup ends.  The sparse form is the same kernel with 256
// threads per workgroup, a 256-VGPR budget and the gather's reads issued
// three taps ahead (gather5_lds PF): same arithmetic, same bits.  Packets
// alone it measured the same as the dense shape at 1.25e5 and 2.5e5 and 4 %
// slower at 5e5 (profiles/r04_v1/ab_*.json); beside the replicated PDE at
// the 8-GPU shard (1.25e5) the driver step is 2.5 % shorter, the PDE's
// kernels finding the slots the idle waves no longer hold
// (profiles/r04_sparse_driver): on below 192 packets per tile (1.25e5 on
// 512^2, not 2.5e5).
#ifndef SWRT_SPARSE_BELOW
#define SWRT_SPARSE_BELOW 192
#endif
constexpr int kSparseBelow = SWRT_SPARSE_BELOW;
#ifndef SWRT_SPARSE_THREADS
#define SWRT_SPARSE_THREADS 256
#endif
#ifndef SWRT_SPARSE_PREFETCH
#define SWRT_SPARSE_PREFETCH 3
#endif
#ifndef SWRT_SPARSE_MINW
#define SWRT_SPARSE_MINW 2
#endif
constexpr int kSparseThreads = SWRT_SPARSE_THREADS;
constexpr int kSparsePrefetch = SWRT_SPARSE_PREFETCH;
constexpr int kSparseMinWaves = SWRT_SPARSE_MINW;  // waves per SIMD the sparse shape's registers are sized for

struct Slot {
  double* nodes = nullptr;  // padded interleaved records
  double* psi = nullptr;    // filtered psi plane (swrt_set_field_psi)
  int64_t nx = 0;
  int64_t npad = 0;
  int64_t ny_period = 0;
  double L = 0.0;
  bool set = false;
  bool has_psi = false;
  bool div_free = false;    // every node's v_y is exactly -u_x (five-sum kernels apply)
  uint64_t wgen = 0;        // write generation: a new value at every write of the nodes (ctx slot_wgen)
  // cross-stream order (they travel with the buffers through swaps and renames):
  hipEvent_t uev = nullptr;  // last context-stream use (packet kernels, field writes)
  hipEvent_t uref = nullptr; // the event that marks that use: uev, or the stop event attached to
                             // the call's last packet launch (context-wide, re-recorded by later
                             // launches: waiting on it waits for a later point, never an earlier one)
  hipEvent_t wev = nullptr;  // last QG-stream write (swrt_qg_snapshot)
  bool upend = false, wpend = false;
};

// device-resident QG PDE state (swrt_qg.hpp)
struct QGState {
  bool init = false;
  QGDev g{};
  int64_t nhalf = 0, nn = 0;
  double2* qk = nullptr;       // nl * nhalf
  double2* qk_prev = nullptr;  // prev_qk of the last step
  double2* Qm1 = nullptr;      // Qn_minus(:,:,1) / (:,:,:,1)
  double2* Qm2 = nullptr;
  double2* E1 = nullptr;       // expLdt  (2 layers): 4 per wavenumber
  double2* E2 = nullptr;       // expL2dt
  double2* Z = nullptr;        // max(2*nl, 3) * nn transform scratch
  double2* T = nullptr;
  unsigned long long* dmax = nullptr;
  // The CFL read-back (dmax -> pinned host memory + an event): a FIFO of two,
  // so a speculative step's speed can be queued behind the committed one's.
  double* hmax = nullptr;      // pinned host copies of dmax, two slots
  hipEvent_t ev = nullptr;     // recorded after the copy into hmax[0]
  hipEvent_t ev_b = nullptr;   // ... into hmax[1]
  int sp_head = 0;             // slot of the next read-back
  int sp_count = 0;            // read-backs pending (0..2), the oldest at (sp_head - sp_count) & 1
  // Speculative step (swrt_qg_step_speculative): computed into the spare
  // buffers from the committed state, which stays untouched until
  // swrt_qg_resolve accepts it (pointer swaps) or drops it.
  double2* qk_spare = nullptr;
  double2* Qm1_spare = nullptr;
  double2* Qm2_spare = nullptr;
  bool spec = false;
  double spec_dt = 0.0, spec_t = 0.0;
  int64_t spec_steps = 0;
  const double2* post_of = nullptr;  // the qk whose post-step transforms PZ/PT hold
  bool post_jrows = false;     // phase 1 ran fft_cols_jacobian2_kernel: J's first forward pass is in PT[0, nn)
  const double2* Fj = nullptr; // where qg_post left the spectrum of J (the update's input)
  bool Fj_rows = false;        // Fj is J after its first forward pass only: the update runs the last
                               // (qg_update_cols_kernel) and renames the tendency history
  bool spec_rot = false;       // the pending speculative step stored only its tendency (Qm1_spare)
  bool spec_rb = false;        // the pending speculative step's CFL read-back is still queued (not popped by
                               // swrt_qg_max_speed_result): a reject drops it only then
  int spec_rb_slot = 0;        // ... its FIFO slot
  // fused mode: the post-step transforms of the current qk — the next step's
  // Jacobian spectrum (PT[0, nn) after its forward FFT), the CFL speed
  // (dmax) and layer 0's grid_U (the snapshot) — from ONE batched inverse
  // 2-D FFT, computed once per qk on first use
  double2* PZ = nullptr;
  double2* PT = nullptr;
  bool post_valid = false;      // both phases of qg_post done for post_of (valid for the current qk when
  bool post_inv_valid = false;  // post_of == qk); post_inv_valid: its first phase (the inverse transforms)
  double exp_dt = -1.0;        // dt of the current E1/E2
  int64_t steps = 0;
  double t = 0.0;
  bool has_prev = false;
};

struct Timing {
  std::vector<hipEvent_t> ev;  // pairs
  size_t used = 0;             // events used (2 per launch)
  double folded_ms = 0.0;      // elapsed of pairs already folded (ring recycled)
  int64_t folded_n = 0;
};
constexpr size_t kMaxEvents = 2048;

}  // namespace

struct swrt_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  Slot slot[SWRT_MAX_SLOTS];
  // The QG PDE (swrt_qg_*) runs on its own stream so the next PDE step, its
  // CFL speed and snapshot overlap the packet launch reading the previous
  // snapshots.  A snapshot into a slot whose buffer a queued packet launch
  // still reads takes an idle buffer from `spares` instead (renaming): a
  // multi-interval launch reads up to 5 snapshots while the PDE writes the
  // next group's.
  hipStream_t qstream = nullptr;
  bool qg_sep = true;
  bool qg_fused = true;  // swrt_qg_set_fused
  int qg_jfuse = 1;  // fused mode, 2 layers, no packets beside: the column pass fused with the Jacobian (SWRT_DEBUG_QG_JFUSE)
  int qg_update_cols = 1;  // fused mode, no packets beside: J's last forward pass inside the update (SWRT_DEBUG_QG_UPDATE_COLS)
  std::vector<Slot> spares;
  // packets (device order = spatially binned; perm maps to the original index)
  double* dx = nullptr;  // 2N
  double* dk = nullptr;  // 2N
  int* perm = nullptr;   // N
  double* dx2 = nullptr;  // scatter targets of the binning pass
  double* dk2 = nullptr;
  int* perm2 = nullptr;
  // third packet buffers: the output of the launch after a source-gather
  // sort launch split over several streams (see tile_launch)
  double* dx3 = nullptr;
  double* dk3 = nullptr;
  int* perm3 = nullptr;
  int* keys = nullptr;   // N
  int* src_idx = nullptr;   // N: source slot of each binned slot (indirect re-binning)
  bool src_pending = false;  // the next tile launch reads its packets through src_idx
  int* bins = nullptr;   // counts | cursor | starts (kMaxBins + 1) | tile order  (4 * kMaxBins + 1)
  int kernel = 0;        // 0 auto, 1 per-packet global gather, 2 LDS tile kernel
  int nbins = 0;         // bins of the current binning
  int64_t n = 0;
  int64_t cap = 0;
  int64_t rebin_every = 4;  // steps between spatial re-binning (0: never)
  int64_t tile = 0;         // cells per tile side (0: automatic)
  int64_t steps_since_bin = 0;
  bool bin_valid = false;
  bool keys_fresh = false;  // keys/counts of the current state came from the last tile launch
  int64_t key_nx = 0;       // ... on the grid the launch read (its first snapshot's nx and dx: the keys
  double key_dx = 0.0;      //     depend on those only, not on the field values — new snapshots keep them valid)
  bool counts_zero = false;  // bins' count block is all zero (cleared by the last scan)
  bool sort_lead = SWRT_SORT_LEAD;  // in-tile sort keys lead by the group-velocity drift
  int gather_mode = 0;      // 0: stencil sums mul then add (bit-exact); 1: fused multiply-add (tolerance)
  int sparse_mode = 0;      // sparse-tile launches: 0 auto (below kSparseBelow packets per tile), 1 never, 2 always
  // Two packet streams (swrt_set_packet_streams 2, the default): each
  // LDS-tiled leapfrog launch runs as 2 part launches — the even and the odd
  // band positions of every XCD band — on `stream` and the extra stream
  // sx[0].  Within a re-binning cycle the parts touch disjoint packet ranges,
  // so one part's launch k overlaps the other's launch k+1 (one part's tail
  // under the other's body).  The extra stream's work is joined back into
  // `stream` (join_b) before anything else reads the packets.
  static constexpr int kMaxPacketStreams = 2;
  int packet_streams = 2;           // default: two (measured +2-4 %, bit-identical); 1 = one launch per step
  hipStream_t sx[kMaxPacketStreams - 1] = {};  // the extra packet streams
  hipEvent_t jx[kMaxPacketStreams - 1] = {};   // their join events
  hipStream_t stream0 = nullptr;  // the packet stream (`stream` outside OnQGStream)
  hipEvent_t fork_ev = nullptr;
  int b_pending = 0;              // extra streams holding packet work not yet ordered before stream's
  int bin_tile = 0;         // cells per tile side of the current binning
  int bin_lanes = 0;        // ... and the workgroup width its tile order was ranked for (tile_threads)
  bool cells_sorted = false;  // packets of every tile are in cell order (a tile launch wrote them)
  // history
  double* hx = nullptr;
  double* hk = nullptr;
  int64_t hframes = 0;
  int64_t hcap = 0;  // doubles allocated per history buffer (frames x 2 x n)
  int64_t steps_done = 0;  // global step counter since history reset (for save cadence)
  // scratch
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  double2* tw = nullptr;
  int tw_n = 0;
  // wave-action (step_packet_xka) background and state
  double* xka_nodes = nullptr;
  int64_t xka_nx = 0;
  double xka_dx = 0.0, xka_dy = 0.0;
  double* xka_state = nullptr;  // 5n
  double* xka_state2 = nullptr; // 5n: the state in binned order
  int* xka_keys = nullptr;      // n
  int* xka_src = nullptr;       // n: binned slot -> packet
  int* xka_src2 = nullptr;      // n: a re-binning's slot -> previous slot
  int* xka_perm2 = nullptr;     // n: composed permutation (ping-pong with xka_src)
  int* xka_bins = nullptr;      // counts | cursor | starts of the xka binning
  int64_t xka_cap = 0;
  double* xka_hist = nullptr;
  int64_t xka_hcap = 0;  // doubles allocated
  // exact spectral evaluator (dense coefficient grid)
  double2* modes = nullptr;
  int2* mode_rows = nullptr;
  int64_t mode_cap = 0;
  int64_t rows_cap = 0;
  double2* modes_d = nullptr;  // group-padded spans (ModeGrid::Cd)
  int* modes_d_row = nullptr;
  float4* modes_f = nullptr;   // fp32 packed-pair copy (ModeGrid::Cf)
  int* modes_f_row = nullptr;
  int64_t modes_f_cap = 0;     // float4 allocated
  int64_t modes_f_rcap = 0;
  ModeGrid mg{};
  bool modes_set = false;
  int64_t mode_active = 0;  // coefficients inside the per-row nonzero spans
  QGState qg;
  // ode23 stage buffers (cap-sized, device packet order)
  double* oF[4] = {nullptr, nullptr, nullptr, nullptr};
  int* o_order = nullptr;      // ode23 tile kernel: in-tile cell order of the binned slots
  int64_t o_order_cap = 0;
  bool o_order_valid = false;  // computed for the current binning
  bool o_sorted = false;       // the packets themselves are in the in-tile cell order of the current binning
  int o_since_bin = 0;         // ode23 calls since the last one that re-binned
                               // (swrt_ode23_f1's tile_cell_sort_kernel): the stages take them in slot order
  double* o_ynx = nullptr;
  double* o_ynk = nullptr;
  // a third state set (x, k, F) for swrt_ode23_run's speculative attempt
  double* o_spx = nullptr;
  double* o_spk = nullptr;
  double* o_spF = nullptr;
  int64_t o_cap = 0;
  // three max slots used in turn: each ode23 launch zeroes the next one for
  // the next launch (no memset launch between attempts); each is read back
  // through its pinned o_hmax slot, o_ev marking the copy
  unsigned long long* o_dmax = nullptr;
  int o_dmax_cur = 0;
  unsigned long long* o_hmax = nullptr;
  hipEvent_t o_ev[3] = {nullptr, nullptr, nullptr};
  hipEvent_t o_evb[3] = {nullptr, nullptr, nullptr};  // ... of part 1 (split attempts, on sx[0])
  // swrt_ode23_run's attempts store every workgroup's max here (host-mapped,
  // [part][slot][workgroup], kMaxBins per slot): read after the launch's
  // event, no copy queued between consecutive attempts
  unsigned long long* o_hpart = nullptr;
  unsigned long long* o_hpart_d = nullptr;
  // swrt_ode23_run's first attempt: its coefficients from the device's own
  // step-size computation (ode23_first_step_kernel), and the host-mapped copy
  // {raw, absh, h, tnew, coefficients} the host checks its computation against
  // (coherent; shown[12]: the launch's ticket, stored after the values)
  double* o_coef = nullptr;
  double* o_shown = nullptr;
  double* o_shown_d = nullptr;
  uint64_t o_ticket = 0;  // the last first-step launch's ticket
  // SWRT_ODE23_MARKERS=1 (environment, A/B runs): swrt_ode23_run's launches
  // as before round 6's last change — an event marker after the first-step
  // kernel and after the chained first attempt's part 0, a join recorded on
  // the extra stream at the end of a split call, and the host waiting for
  // each launch's event before reading its maxima
  bool o23_markers = false;
  // the next swrt_ode23_run's stage 1, queued at the end of this one
  // (swrt_ode23_chain_next): armed with the slots the next call reads as its
  // slots 0 / 1; `queued` holds what it was computed from, and any API call
  // that may touch the packets drops it (GUARD_BEGIN)
  struct O23Chain {
    bool want = false;
    int sa = -1, sb = -1;
    bool queued = false;
    int dmax_slot = 0;
    const double* nodes[2] = {nullptr, nullptr};
    uint64_t wgen[2] = {0, 0};
    double alpha = 0.0, f = 0.0, Cg = 0.0, thr = 0.0, bump = 0.0;
    int64_t taken = 0;  // calls that took it (SWRT_DEBUG_ODE23_CHAINED)
    // the next call's first attempt, queued behind its stage 1 from the
    // device's own step size for t0 = 0, tfinal = tmax and `rtol`
    // (ode23_chain_first): its max slot, each part's workgroups, the split
    bool first_q = false;
    int first_slot = -1;
    unsigned first_wg[2] = {0, 0};
    bool split = false;
    uint64_t first_ticket = 0;
    double rtol = 0.0, tfinal = 0.0, tmax = 0.0;
    int64_t first_taken = 0;  // calls that took it (SWRT_DEBUG_ODE23_FIRST_CHAINED)
  } o_chain;
  // the chained first attempt's part 1 is queued on sx[0] and not joined
  // (b_pending stays 0, so the QG calls between two intervals do not join
  // it): a call that drops the chain, or an ode23 call that does not take the
  // attempt, joins it first (chain_join)
  bool chain_b = false;
  hipEvent_t chain_ev[2] = {nullptr, nullptr};
  bool chain_first = true;  // SWRT_ODE23_CHAIN_FIRST=0 (environment, A/B runs): stage 1 alone is chained
  // the packet stream got work since the last split launch's part 0 that the
  // next split launch's part 1 (on sx[0]) must follow: that launch forks (an
  // event marker, ~7 us of idle on each stream).  Only consecutive split
  // launches of swrt_advance / swrt_advance_intervals with nothing in between
  // skip it: part p of a binning owns the same tiles at every launch, so
  // stream order alone orders a part's launches (launch_tiles).
  // SWRT_FORK_ALWAYS=1 (environment, A/B runs): fork at every split launch.
  bool s0_dirty = true;
  bool fork_always = false;
  uint64_t slot_wgen = 0;  // Slot::wgen source
  Timing timing;
  int timing_every = 1;     // bracket every k-th leapfrog launch with HIP events (0: off)
  int64_t launch_count = 0;
  // set only around a timed packet launch: the dispatch itself stamps them
  // (hipExtLaunchKernel), so they bracket the kernel and nothing else
  hipEvent_t kev0 = nullptr, kev1 = nullptr;
  // stop event attached to every untimed packet launch (launch_k), and the
  // stop event of the last stream operation of the current API call if that
  // was a packet launch (else nullptr): SlotUse marks the slots' use with it
  // instead of recording a separate marker, which cost ~11 us of idle GPU
  // between dependent packet launches (tools/gap_probe.py)
  hipEvent_t use_ev = nullptr;
  hipEvent_t tail_ev = nullptr;
  // debug knobs (swrt_debug_set): the packet-buffer hazard checker
  // (swrt_hazard.hpp), a spin kernel queued on every extra packet stream
  // before each of its part launches (adversarial overlap of consecutive
  // calls), and the pre-third-buffer ordering after a source-gather sort
  // launch (test-only: reintroduces the race the checker must catch)
  HazardChecker hz;
  int debug_spin_us = 0;
  bool debug_legacy_park = false;
  bool debug_share_skew = false;  // test-only: the cycle-ending launch takes an uneven share (checker on only)
  int debug_corrupt_count = 0;    // test-only: added to one tile count before the next scan (once)
  // device-raised errors (host-visible pinned memory): [0] the binning scan's
  // count check failed (bin_scan_kernel) — read after host synchronisations
  int* dev_err = nullptr;
  int* dev_err_d = nullptr;
  bool packets_lost = false;  // a failed binning left the packet state undefined (until swrt_packets_set)
  bool in_hook = false;       // an ode23 hook is running (swrt_ode23_run_hooked): packet calls are refused
  // swrt_snapshot_qk (snapshots from a half plane another context exported):
  // transform scratch, the staged host half plane, the cross-stream events
  double2* xq_Z = nullptr;
  double2* xq_T = nullptr;
  double2* xq_fk = nullptr;
  int64_t xq_nx = 0;
  bool xq_init = false;   // slot writes may come from the QG stream (slot_events)
  hipEvent_t xev[2] = {nullptr, nullptr};
  O23Stats o23_last;          // the last swrt_ode23_run's controller counts
  int64_t o23_first_taken = 0, o23_guesses_taken = 0;  // ... summed over runs (SWRT_DEBUG_ODE23_*)
  int64_t o23_split_runs = 0;  // runs whose attempts ran as two part launches (SWRT_DEBUG_ODE23_SPLIT_RUNS)
  // shader-clock probe (swrt_clock_stamp): 2 stamps x kClockWaves waves x
  // {s_memtime, s_memrealtime, XCC id}
  unsigned long long* clk = nullptr;
};

namespace {
constexpr size_t kMaxSpares = 8;  // renamed snapshot buffers per context

// the work recorded in `ev` has not finished yet
bool event_pending(hipEvent_t ev) {
  const hipError_t e = hipEventQuery(ev);
  (void)hipGetLastError();  // hipErrorNotReady is a status, not an error
  return e == hipErrorNotReady;
}

// Run a swrt_qg_* call on the QG stream: every helper launches on c->stream.
struct OnQGStream {
  swrt_ctx* c;
  hipStream_t saved;
  explicit OnQGStream(swrt_ctx* c_) : c(c_), saved(c_->stream) {
    if (c->qg_sep) c->stream = c->qstream;
  }
  ~OnQGStream() { c->stream = saved; }
};

// A context-stream call that reads or writes the field slots: wait for the
// QG-stream snapshots written into them, then mark them used by this call.
// Slot-use events are only needed while a QG stream may write slots beside
// the packet launches (swrt_qg_init on a separate stream); without one a
// packet launch carries no event at all (each costs ~5 us of idle GPU at the
// launch boundary, tools/gap_probe.py).
bool slot_events(const swrt_ctx* c) { return c->qg_sep && (c->qg.init || c->xq_init); }

// The packet stream waits for the QG stream's pending snapshot writes before
// the first kernel that reads a slot.  Deferred (swrt_advance / _intervals):
// the wait is placed by slot_writes_wait() just before the first packet
// launch, so a re-binning at the start of the call (packet buffers only)
// runs while the PDE chain is still producing the snapshot.
constexpr unsigned kAllSlots = (1u << SWRT_MAX_SLOTS) - 1;
constexpr unsigned kSlots01 = 3u;  // the ode23 calls read slots 0 and 1 only

void slot_writes_wait(swrt_ctx* c, unsigned mask = kAllSlots) {
  if (!c->qg_sep) return;
  for (int i = 0; i < SWRT_MAX_SLOTS; ++i)
    if (Slot& s = c->slot[i]; (mask >> i & 1u) && s.wpend) {
      (void)hipStreamWaitEvent(c->stream, s.wev, 0);
      s.wpend = false;
      c->s0_dirty = true;
    }
}

struct SlotUse {
  swrt_ctx* c;
  // wait_mask: the slots whose pending QG-stream writes this call's reads wait
  // for (the ode23 calls read slots 0 and 1 only: a hook's snapshot into slot
  // 2 keeps running beside their attempts)
  explicit SlotUse(swrt_ctx* c_, bool defer_writes = false, unsigned wait_mask = kAllSlots) : c(c_) {
    c->tail_ev = nullptr;
    if (!defer_writes) slot_writes_wait(c, wait_mask);
  }
  ~SlotUse() {
    if (!slot_events(c)) return;
    for (Slot& s : c->slot) {
      if (!s.nodes) continue;
      if (c->tail_ev) {
        s.uref = c->tail_ev;
        s.upend = true;
      } else if (hipEventRecord(s.uev, c->stream) == hipSuccess) {
        s.uref = s.uev;
        s.upend = true;
      }
    }
    c->tail_ev = nullptr;
  }
};
}  // namespace

namespace {

int fail(swrt_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(ctx, expr)                                                                   \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return fail(ctx, SWRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));    \
  } while (0)

// GUARD_BEGIN also orders any pending second-stream packet work before the
// call (join_b); the split-launch entry points use GUARD_BEGIN_KEEP_SPLIT.
#define HIPCHK_RC(expr)       \
  do {                        \
    const int rc_ = (expr);   \
    if (rc_) return rc_;      \
  } while (0)
// GUARD_BEGIN drops a queued ode23 chain (the packets may change); the calls
// that never touch the packets (QG, clock) use GUARD_BEGIN_KEEP_CHAIN.
// A call that may touch the packets is refused inside an ode23 hook
// (swrt_ode23_run_hooked): it would race the interval's attempts in flight.
#define HOOK_REFUSE \
  if (c->in_hook) return fail(c, SWRT_ERR_STATE, "this call may touch the packets: not allowed inside an ode23 hook");
#define GUARD_BEGIN_KEEP_SPLIT                  \
  HOOK_REFUSE                                   \
  try {                                         \
    {                                           \
      const int crc_ = chain_drop(c);           \
      if (crc_) return crc_;                    \
    }
#define GUARD_BEGIN_KEEP_CHAIN    \
  try {                           \
    {                             \
      const int jrc_ = join_b(c); \
      if (jrc_) return jrc_;      \
      hz_api(c);                  \
      c->s0_dirty = true;         \
    }
#define GUARD_BEGIN              \
  HOOK_REFUSE                    \
  GUARD_BEGIN_KEEP_CHAIN         \
  {                              \
    const int crc_ = chain_drop(c); \
    if (crc_) return crc_;       \
  }
#define GUARD_END(ctx)                                                \
  }                                                                   \
  catch (const std::bad_alloc&) {                                     \
    return fail(ctx, SWRT_ERR_ALLOC, "host allocation failed");       \
  }                                                                   \
  catch (...) {                                                       \
    return fail(ctx, SWRT_ERR_STATE, "unexpected C++ exception");     \
  }

// Order the extra streams' queued packet work before the packet stream's next work.
int join_b(swrt_ctx* c) {
  if (!c || !c->b_pending) return SWRT_OK;
  for (int i = 0; i < c->b_pending; ++i) {
    HIPCHK(c, hipEventRecord(c->jx[i], c->sx[i]));
    HIPCHK(c, hipStreamWaitEvent(c->stream0, c->jx[i], 0));
    if (c->hz.on) {
      c->hz.record(c->jx[i], i + 1);
      c->hz.wait(0, c->jx[i]);
    }
  }
  c->b_pending = 0;
  return SWRT_OK;
}

// Order a chained first attempt's part 1 (sx[0]) before the packet stream's
// next work: the attempt is dropped, or its call runs another.
int chain_join(swrt_ctx* c) {
  if (!c->chain_b) return SWRT_OK;
  c->chain_b = false;
  HIPCHK(c, hipEventRecord(c->jx[0], c->sx[0]));
  HIPCHK(c, hipStreamWaitEvent(c->stream0, c->jx[0], 0));
  if (c->hz.on) {
    c->hz.record(c->jx[0], 1);
    c->hz.wait(0, c->jx[0]);
  }
  return SWRT_OK;
}

// A queued ode23 chain dropped (the packets may change).
int chain_drop(swrt_ctx* c) {
  c->o_chain.queued = false;
  c->o_chain.first_q = false;
  return chain_join(c);
}

// Hazard checker (swrt_hazard.hpp): the packet-state buffers of the context.
template <typename F>
void hz_each_buffer(swrt_ctx* c, F fn) {
  for (const void* b : {(const void*)c->dx, (const void*)c->dk, (const void*)c->perm, (const void*)c->dx2,
                        (const void*)c->dk2, (const void*)c->perm2, (const void*)c->dx3, (const void*)c->dk3,
                        (const void*)c->perm3, (const void*)c->keys, (const void*)c->src_idx, (const void*)c->bins,
                        (const void*)(c->bins ? c->bins + kMaxBins : nullptr),
                        (const void*)(c->bins ? c->bins + 2 * kMaxBins : nullptr),
                        (const void*)(c->bins ? c->bins + 3 * kMaxBins + 1 : nullptr), (const void*)c->hx,
                        (const void*)c->hk})
    if (b) fn(b);
}

// Every other API call runs on the packet stream after join_b: to the checker
// it reads and writes every packet buffer there (conservative: a call that
// lost its join is reported by the next part launch).
void hz_api(swrt_ctx* c) {
  if (!c || !c->hz.on) return;
  const uint64_t t = c->hz.op(0);
  hz_each_buffer(c, [&](const void* b) { (void)c->hz.access(0, t, b, kHzWrite, HzRegion::all(), "an API call"); });
}

// The host synchronised the packet stream after join_b: everything queued on
// any packet stream before has completed.
void hz_synced(swrt_ctx* c) {
  if (c->hz.on) c->hz.sync(0);
}

// After a host synchronisation with the packet stream: an error the device
// raised since (bin_scan_kernel's count check) becomes SWRT_ERR_STATE here,
// and the packet state — advanced by launches over an empty binning — is
// marked lost until the next swrt_packets_set.
int dev_err_check(swrt_ctx* c) {
  if (!c->dev_err || !c->dev_err[0]) return SWRT_OK;
  c->dev_err[0] = 0;
  c->packets_lost = true;
  c->bin_valid = false;
  c->keys_fresh = false;
  c->src_pending = false;
  c->o_order_valid = false;
  c->o_sorted = false;
  return fail(c, SWRT_ERR_STATE,
              "packet binning corrupted: the tile counts do not sum to the packets (device check in "
              "bin_scan_kernel); no packet kernel ran over the bad ranges, but the packet state is lost — "
              "swrt_packets_set again");
}

// The packet state stays refused after a corrupted binning until
// swrt_packets_set (every entry point that reads the packets checks).
int lost_check(swrt_ctx* c) {
  if (c->packets_lost)
    return fail(c, SWRT_ERR_STATE, "the packet state was lost to a corrupted binning (swrt_packets_set again)");
  return SWRT_OK;
}

// Wait for the extra packet streams (host side).
int sync_sx(swrt_ctx* c) {
  for (int i = 0; i < swrt_ctx::kMaxPacketStreams - 1; ++i)
    if (c->sx[i]) {
      HIPCHK(c, hipStreamSynchronize(c->sx[i]));
      if (c->hz.on) c->hz.sync(i + 1);
    }
  c->b_pending = 0;
  c->chain_b = false;
  return SWRT_OK;
}

bool is_pow2(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }

int ensure_scratch(swrt_ctx* c, size_t bytes) {
  if (c->scratch_bytes >= bytes) return SWRT_OK;
  if (c->scratch) (void)hipFree(c->scratch);
  c->scratch = nullptr;
  c->scratch_bytes = 0;
  HIPCHK(c, hipMalloc(&c->scratch, bytes));
  c->scratch_bytes = bytes;
  return SWRT_OK;
}

int ensure_twiddles(swrt_ctx* c, int n) {
  if (c->tw_n == n) return SWRT_OK;
  if (c->tw) {
    HIPCHK(c, hipDeviceSynchronize());  // the other stream may still read them
    (void)hipFree(c->tw);
  }
  c->tw = nullptr;
  std::vector<double2> h(n);  // k < n: the radix-4 stages read w^(3*p*s) < w^(3n/4)
  for (int k = 0; k < n; ++k) {
    // exp(-2*pi*i*k/n); long double for the argument reduction
    const long double th = -2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)n;
    h[k] = make_double2((double)cosl(th), (double)sinl(th));
  }
  HIPCHK(c, hipMalloc(&c->tw, sizeof(double2) * n));
  HIPCHK(c, hipMemcpyAsync(c->tw, h.data(), sizeof(double2) * n, hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->tw_n = n;
  return SWRT_OK;
}

int ensure_slot(swrt_ctx* c, int slot, int64_t nx) {
  Slot& s = c->slot[slot];
  const int64_t npad = nx + kPadTot;
  if (s.nodes && s.nx == nx) return SWRT_OK;
  if (s.nodes) HIPCHK(c, hipDeviceSynchronize());  // a queued launch on either stream may read it
  if (s.nodes) (void)hipFree(s.nodes);
  if (s.psi) (void)hipFree(s.psi);
  s.nodes = nullptr;
  s.psi = nullptr;
  s.set = false;
  HIPCHK(c, hipMalloc(&s.nodes, sizeof(double) * kRec * npad * npad));
  s.nx = nx;
  s.npad = npad;
  return SWRT_OK;
}

int check_slot_args(swrt_ctx* c, int slot, int64_t nx) {
  if (!c) return SWRT_ERR_ARG;
  if (slot < 0 || slot >= SWRT_MAX_SLOTS) return fail(c, SWRT_ERR_ARG, "slot out of range");
  if (nx < 8 || nx > 4096 || (nx & 1)) return fail(c, SWRT_ERR_ARG, "nx must be even, 8..4096");
  return SWRT_OK;
}

FieldView view_of(const Slot& s) {
  FieldView v;
  v.nodes = s.nodes;
  v.nx = (int)s.nx;
  v.npad = (int)s.npad;
  v.dx = s.L / (double)s.nx;
  v.px = (double)s.nx;
  v.py = (double)s.ny_period;
  v.inv_px = 1.0 / v.px;
  v.inv_py = 1.0 / v.py;
  v.ipx = (int)s.nx;
  v.ipy = (int)s.ny_period;
  v.inv_dx = 1.0 / v.dx;
  return v;
}

inline unsigned nblocks(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// Pack 6 device planes (already in scratch) into the slot's node array.
int pack_slot(swrt_ctx* c, int slot, const double* dplanes, double shear) {
  Slot& s = c->slot[slot];
  const int64_t tot = s.npad * s.npad;
  hipLaunchKernelGGL(pack_nodes_kernel, dim3(nblocks(tot, 256)), dim3(256), 0, c->stream, dplanes,
                     (int)s.nx, (int)s.npad, shear, s.nodes);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}

// FFT kernel variant (swrt_fft.hpp): radix 4 in one LDS buffer with n/4
// lanes for n <= 1024, else radix 4 ping-pong with 128 lanes.  At 512^2 x 2
// layers (8-vector inverse + 1-vector forward 2-D transforms per step) the
// one-buffer form takes the PDE step from 0.078 (radix 2, 256 lanes) / 0.077
// (radix 4 ping-pong) to 0.073 ms (profiles/r02_v21_fft_mode_ab.log).
// Vectors per workgroup of the one-buffer form (rows per workgroup of the
// Jacobian pass): two when the transforms run alone (the PDE step 0.080 vs
// 0.081 ms with four and 0.083 with one), one while packet launches run
// beside them on their own stream (driver step 0.288 vs 0.293 ms with two and
// 0.295 with four: small workgroups fit the slots packet workgroups free,
// profiles/r03_v4_qg/README.md).  Batches that do not divide fall back to one.
int fft_group(const swrt_ctx* c, int n, int nvec, bool tin) {
  const int C = (c->qg_sep && c->n > 0) ? 1 : 2;
  if (C * (n / 4) > 1024 || nvec % (tin ? 8 * C : C) != 0) return 1;
  return C;
}

template <bool TIN>
void launch_fft(swrt_ctx* c, const double2* in, double2* out, int n, int logn, int nvec, int inverse) {
  if (n <= 1024) {
    const int C = fft_group(c, n, nvec, TIN);
    hipLaunchKernelGGL((fft_vec_kernel<TIN, 2>), dim3((unsigned)(nvec / C)), dim3(C * n / 4),
                       sizeof(double2) * C * (n + 1), c->stream, in, out, n, logn, c->tw, inverse, nvec);
  } else
    hipLaunchKernelGGL((fft_vec_kernel<TIN, 1>), dim3((unsigned)nvec), dim3(128), sizeof(double2) * 2 * n, c->stream,
                       in, out, n, logn, c->tw, inverse, nvec);
}

int run_fft_pass(swrt_ctx* c, double2* Z, int n, int nb, int inverse) {
  int logn = 0;
  while ((1 << logn) < n) ++logn;
  const int64_t nvec = (int64_t)n * nb;
  launch_fft<false>(c, Z, Z, n, logn, (int)nvec, inverse);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}

int run_transpose(swrt_ctx* c, const double2* in, double2* out, int n, int nb) {
  dim3 grid((n + 31) / 32, (n + 31) / 32, nb);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(32, 8), 0, c->stream, in, out, n);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}

// 2-D transform of nb n x n blocks: a pass along the contiguous index of Z (in
// place), then a pass along the other index reading Z's columns and writing
// `out` transposed ([r + n*c] for Z in [c + n*r]).  Z keeps the first pass.
int transform_2d(swrt_ctx* c, double2* Z, double2* out, int n, int nb, int inverse) {
  int rc;
  if ((rc = run_fft_pass(c, Z, n, nb, inverse))) return rc;
  const int64_t nvec = (int64_t)n * nb;
  if (nvec % 8) {  // tiny grids: the XCD mapping needs 8 | nvec
    if ((rc = run_transpose(c, Z, out, n, nb))) return rc;
    return run_fft_pass(c, out, n, nb, inverse);
  }
  int logn = 0;
  while ((1 << logn) < n) ++logn;
  launch_fft<true>(c, Z, out, n, logn, (int)nvec, inverse);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}

// Inverse 2-D transform of nb spectra in layout [c + n*r] (ky contiguous);
// result in layout [r + n*c] (x contiguous) in `out`.
int inverse_2d(swrt_ctx* c, double2* Z, double2* out, int n, int nb) { return transform_2d(c, Z, out, n, nb, 1); }

// Shared tail of set_field_psi / set_field_qk / swrt_qg_snapshot: fk half
// plane in device memory, read at fk[(kx + kmax)*sx + ky*sy].
int fields_from_halfplane(swrt_ctx* c, int slot, const double2* dfk, int n, int mode, double K_d2,
                          double kscale, double shear, int with_psi, double2* Z, double2* T, int sx, int sy) {
  int rc;
  const int64_t nn = (int64_t)n * n;
  const int nb = with_psi ? 4 : 3;
  Slot& s0 = c->slot[slot];
  if (!with_psi && n % 16 == 0 && 3 * 2 * n / 4 <= 1024 && (n / 2) % 8 == 0) {
    // the spectra built by the row pass (spectra_rows_kernel), the column
    // pass fused with the pack into the node records (fft_cols_pack_kernel):
    // two launches, the values of the four below
    int logn = 0;
    while ((1 << logn) < n) ++logn;
    hipLaunchKernelGGL(spectra_rows_kernel, dim3((unsigned)n), dim3(3 * n / 4), sizeof(double2) * 3 * n, c->stream,
                       dfk, n, mode, K_d2, kscale, 0, sx, sy, logn, (const double2*)c->tw, Z);
    HIPCHK(c, hipGetLastError());
    hipLaunchKernelGGL(fft_cols_pack_kernel<2>, dim3((unsigned)(n / 2)), dim3(3 * 2 * n / 4),
                       sizeof(double2) * 3 * 2 * (n + 1), c->stream, (const double2*)Z, n, logn,
                       (const double2*)c->tw, (int)s0.npad, shear, s0.nodes);
    HIPCHK(c, hipGetLastError());
    s0.has_psi = false;
    s0.div_free = true;  // v_y = -u_x, as pack_pairs_kernel
    return SWRT_OK;
  }
  if (nb * n / 4 <= 1024 && ((int64_t)n * nb) % 8 == 0) {
    // the spectra built row by row in LDS by the first inverse pass
    // (spectra_rows_kernel: the same values as the separate launches below,
    // one 12.6 MB round trip less at 512^2), then the column pass
    int logn = 0;
    while ((1 << logn) < n) ++logn;
    hipLaunchKernelGGL(spectra_rows_kernel, dim3((unsigned)n), dim3(nb * n / 4), sizeof(double2) * nb * n, c->stream,
                       dfk, n, mode, K_d2, kscale, with_psi, sx, sy, logn, (const double2*)c->tw, Z);
    HIPCHK(c, hipGetLastError());
    launch_fft<true>(c, Z, T, n, logn, n * nb, 1);
    HIPCHK(c, hipGetLastError());
  } else {
    hipLaunchKernelGGL(spectra_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, dfk, n, mode,
                       K_d2, kscale, with_psi, Z, sx, sy);
    HIPCHK(c, hipGetLastError());
    if ((rc = inverse_2d(c, Z, T, n, nb))) return rc;
  }
  // T now holds the packed fields in [x + n*y]
  Slot& s = c->slot[slot];
  if (with_psi && !s.psi) HIPCHK(c, hipMalloc(&s.psi, sizeof(double) * nn));
  if (n % 16 == 0) {
    hipLaunchKernelGGL(pack_pairs_kernel, dim3(n / 16, n / 16), dim3(256), 0, c->stream, T, n, (int)s.npad, shear,
                       s.nodes);
    HIPCHK(c, hipGetLastError());
    if (with_psi) {
      hipLaunchKernelGGL(psi_plane_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, T + 3 * nn, s.psi, nn);
      HIPCHK(c, hipGetLastError());
    }
  } else {  // tiny grids: unpair into planes (reuse Z), then pack
    double* planes = reinterpret_cast<double*>(Z);
    hipLaunchKernelGGL(unpair_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, T, n, with_psi,
                       planes, with_psi ? s.psi : nullptr);
    HIPCHK(c, hipGetLastError());
    if ((rc = pack_slot(c, slot, planes, shear))) return rc;
  }
  s.has_psi = with_psi != 0;
  s.div_free = true;  // pack_pairs_kernel / unpair_kernel write v_y = -u_x
  return SWRT_OK;
}

bool use_tile_kernel(const swrt_ctx* c);
// the intervals of one multi-interval tile launch (swrt_advance_intervals)
struct IvLaunch {
  int nint;
  FieldView views[kMaxIntervals + 1];
  double dts[kMaxIntervals];
  bool div_free;
};
int tile_launch(swrt_ctx* c, const StepArgs& a, bool count_next, const IvLaunch* iv = nullptr);

// Launch a packet kernel on the context stream; inside a timed launch the
// start/stop events take the kernel's own begin/end timestamps.
template <typename F, typename... Args>
void launch_k(swrt_ctx* c, F kernel, dim3 grid, dim3 block, Args... args) {
  hipEvent_t stop = c->kev1 ? c->kev1 : (slot_events(c) ? c->use_ev : nullptr);
  hipExtLaunchKernelGGL(kernel, grid, block, 0, c->stream, c->kev0, stop, 0, args...);
  c->tail_ev = stop;
}

// Ensembles below this run every tile launch on one stream: the split's
// fork/join costs more than the overlap returns (profiles/r03_streams_ab:
// 3e4 packets 3.0 vs 3.4e9, 1e4 at 256^2 1.8 vs 2.8e9; 6.25e4 even; 1.25e5
// +3 %, 2.5e5 +6 %, 5e5 +4 %, 1e6 +3.7 %).
constexpr int64_t kMultiStreamFrom = 65536;

// ode23 calls per spatial re-binning (ode23_f1_queue)
#ifndef SWRT_ODE23_REBIN
#define SWRT_ODE23_REBIN 2  // every 1 / 2 / 4 calls: 1.843-1.845 / 1.824-1.830 / 1.878-1.892 ms per driver interval (profiles/r05_ode23)
#endif
constexpr int kOde23RebinEvery = SWRT_ODE23_REBIN;

// The LDS-tiled launch of TileArgs t: one launch over every tile, or (two
// packet streams) two part launches, each a share of every XCD band's tiles
// (swrt_share.hpp), the second on the extra stream after everything queued
// on the packet stream so far (this call's re-binning, memsets and history
// growth).  A timed pair brackets the first part's start and the last
// part's end.
//
// Hazard checker: the accesses of the launch's parts (part p on stream p),
// forked from the packet stream when split, each over the band slots its
// workgroups take — enumerated with the device's own mapping (share_slot),
// so a launch whose tile-to-stream mapping differs from the previous
// launch's is seen to touch the other stream's tiles.  Checked on a copy of
// the checker state, committed only if every access is ordered: a hazard
// refuses the launch before anything is queued.
int hz_tile_launch(swrt_ctx* c, const TileArgs& t, const TileShare* parts, int nparts, bool zero_counts,
                   bool fork = true) {
  HazardChecker h = c->hz;
  if (zero_counts) {  // the next-binning counts' memset, on the packet stream before the parts
    const uint64_t tm = h.op(0);
    if (!h.access(0, tm, t.next_counts, kHzWrite, HzRegion::all(), "the next-binning counts' memset"))
      return fail(c, SWRT_ERR_STATE, h.err);
  }
  if (nparts > 1 && fork) {
    h.record(c->fork_ev, 0);
    for (int i = 1; i < nparts; ++i) h.wait(i, c->fork_ev);
  }
  const StepArgs& a = t.s;
  for (int p = 0; p < nparts; ++p) {
    const uint64_t tp = h.op(p);
    const HzRegion r = HzRegion::of_share(h.epoch, parts[p]);
    const char* what = t.src ? "a part of the sort launch after a re-binning" : "a part launch";
    // the sort launch after an indirect re-binning gathers its input through
    // src_idx from any slot of the input buffers
    const HzRegion rin = t.src ? HzRegion::all() : r;
    bool ok = h.access(p, tp, a.x, kHzRead, rin, what) && h.access(p, tp, a.k, kHzRead, rin, what) &&
              h.access(p, tp, a.perm, kHzRead, rin, what) && h.access(p, tp, t.src, kHzRead, r, what) &&
              h.access(p, tp, t.starts, kHzRead, HzRegion::all(), what) &&
              h.access(p, tp, t.order, kHzRead, HzRegion::all(), what) &&
              h.access(p, tp, t.x_out, kHzWrite, r, what) && h.access(p, tp, t.k_out, kHzWrite, r, what) &&
              h.access(p, tp, t.perm_out, kHzWrite, r, what) &&
              h.access(p, tp, t.next_keys, kHzWrite, r, what) &&
              h.access(p, tp, t.next_counts, kHzAtomic, HzRegion::all(), what) &&
              h.access(p, tp, a.hist_x, kHzWrite, r, what) && h.access(p, tp, a.hist_k, kHzWrite, r, what);
    if (!ok) return fail(c, SWRT_ERR_STATE, h.err);
  }
  c->hz = std::move(h);
  return SWRT_OK;
}

// debug: a kernel that sleeps ~4 us per iteration (every wave returns)
__global__ void debug_spin_kernel(int iters) {
  for (int i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
}

// debug (SWRT_DEBUG_CORRUPT_COUNT): add `delta` to one tile's count before a
// scan, as a corrupted binning would
__global__ void debug_corrupt_count_kernel(int* counts, int tile, int delta) {
  if (threadIdx.x == 0) counts[tile] += delta;
}

// Shader-clock probe (swrt_clock_stamp): kClockWaves one-wave workgroups
// (several per CU) each record the shader-cycle counter (s_memtime), the
// 100 MHz real-time counter (s_memrealtime) and the CU they ran on (XCD, SE,
// SH, CU ids).  A start and an end stamp of the SAME CU bracket a timed
// region: cycles / seconds = the clock that CU ran at over it
// (MI355X_MICROARCH.md, "DVFS give-back" item 6); s_memtime counters of
// different CUs are not aligned, so only same-CU pairs are used.  Plain
// vector stores, a buffer of its own.
constexpr int kClockWaves = 1024;
constexpr double kRealTimeHz = 100e6;
__global__ void clock_stamp_kernel(unsigned long long* out) {
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x + 0] = t;
    out[3 * blockIdx.x + 1] = r;
    // CU identity: XCD | SE | SH | CU (the wave/SIMD bits masked off)
    out[3 * blockIdx.x + 2] = ((unsigned long long)(xcc & 0xf) << 16) | ((hw >> 8) & 0xffffu);
  }
}

// zero_counts: clear t.next_counts (the next binning's counts) first, on the
// packet stream — after the hazard check, so a refused launch queues nothing.
template <typename F>
int launch_tiles(swrt_ctx* c, F kernel, int nt, TileArgs t, bool zero_counts) {
  const int ntiles = t.ntx * t.ntx;
  const int S = c->n >= kMultiStreamFrom ? c->packet_streams : 1;
  // test-only (SWRT_DEBUG_SHARE_SKEW): the launch that ends a re-binning
  // cycle takes an uneven share — a mapping that differs from the previous
  // launch's, round 4's race; only ever run with the checker on, which
  // refuses it (swrt_debug_set enforces that)
  const bool skew = c->debug_share_skew && t.next_keys != nullptr;
  if (skew && !c->hz.on) return fail(c, SWRT_ERR_STATE, "the skewed share runs only under the hazard checker");
  const bool multi = S == 2 && c->stream == c->stream0 && c->sx[0] != nullptr &&
                     (skew ? ntiles % 8 == 0 && ntiles / 8 >= 3 : ntiles % 16 == 0);
  if (!multi) {
    // one launch over every tile on the packet stream: it reads and writes
    // packets that the extra stream's part launch of an earlier call may
    // still be writing
    t.sh = TileShare{ntiles, -1, 1, kShareEven};
    HIPCHK_RC(join_b(c));
    if (c->hz.on) HIPCHK_RC(hz_tile_launch(c, t, &t.sh, 1, zero_counts));
    if (zero_counts) HIPCHK(c, hipMemsetAsync(t.next_counts, 0, sizeof(int) * ntiles, c->stream));
    launch_k(c, kernel, dim3((unsigned)share_grid(t.sh)), dim3(nt), t);
    c->s0_dirty = true;  // every tile on the packet stream
    return SWRT_OK;
  }
  const TileShare sh[2] = {TileShare{ntiles, 0, 2, skew ? kShareSkew : kShareEven},
                           TileShare{ntiles, 1, 2, skew ? kShareSkew : kShareEven}};
  // the fork: only when the packet stream has had other work since the last
  // split launch (s0_dirty), the counts' memset included; the hazard checker
  // models exactly the orderings the launch queues
  const bool fork = c->s0_dirty || zero_counts || skew || c->fork_always;
  if (c->hz.on) HIPCHK_RC(hz_tile_launch(c, t, sh, 2, zero_counts, fork));
  if (zero_counts) HIPCHK(c, hipMemsetAsync(t.next_counts, 0, sizeof(int) * ntiles, c->stream));
  // Part p takes the same slots at every launch of a binning (the product
  // rule, kShareEven): a stream's consecutive part launches own the same
  // tiles, so stream order alone orders them, and stream 0's next launch may
  // start while stream 1's previous one still runs.  A launch with another
  // mapping races it unless joined first — the checker, which enumerates the
  // slots each part takes, refuses it (round 4's hang, profiles/r04_stream_split).
  if (fork) {
    HIPCHK(c, hipEventRecord(c->fork_ev, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->sx[0], c->fork_ev, 0));
  }
  c->s0_dirty = false;
  t.sh = sh[0];
  hipExtLaunchKernelGGL(kernel, dim3((unsigned)share_grid(sh[0])), dim3(nt), 0, c->stream, c->kev0, nullptr, 0, t);
  if (c->debug_spin_us > 0)
    hipLaunchKernelGGL(debug_spin_kernel, dim3(1), dim3(64), 0, c->sx[0], (c->debug_spin_us + 3) / 4);
  t.sh = sh[1];
  hipExtLaunchKernelGGL(kernel, dim3((unsigned)share_grid(sh[1])), dim3(nt), 0, c->sx[0], nullptr, c->kev1, 0, t);
  c->b_pending = 1;
  c->tail_ev = nullptr;  // slot uses are marked after the join (swrt_advance)
  return SWRT_OK;
}

// Before a per-packet leapfrog launch (packets updated in place on the packet
// stream): order the extra stream's part launches of an earlier call first
// (swrt_set_locality(0, ..) after split launches lands here), and tell the
// hazard checker.
int leap_launch_prep(swrt_ctx* c, const StepArgs& a) {
  HIPCHK_RC(join_b(c));
  c->s0_dirty = true;
  if (!c->hz.on) return SWRT_OK;
  HazardChecker& h = c->hz;
  const uint64_t t = h.op(0);
  const char* what = "the per-packet leapfrog launch";
  const bool ok = h.access(0, t, a.x, kHzWrite, HzRegion::all(), what) &&
                  h.access(0, t, a.k, kHzWrite, HzRegion::all(), what) &&
                  h.access(0, t, a.perm, kHzRead, HzRegion::all(), what) &&
                  h.access(0, t, a.hist_x, kHzWrite, HzRegion::all(), what) &&
                  h.access(0, t, a.hist_k, kHzWrite, HzRegion::all(), what);
  return ok ? SWRT_OK : fail(c, SWRT_ERR_STATE, h.err);
}

// Time every timing_every-th leapfrog launch with a pair of HIP events.
int timed_launch(swrt_ctx* c, const StepArgs& a, unsigned grid, bool count_next, const IvLaunch* iv = nullptr) {
  const bool timed = c->timing_every > 0 && (c->launch_count++ % c->timing_every) == 0;
  if (!timed) {
    if (use_tile_kernel(c)) return tile_launch(c, a, count_next, iv);
    HIPCHK_RC(leap_launch_prep(c, a));
    c->keys_fresh = false;
    if (a.nslots == 2)
      hipLaunchKernelGGL(leapfrog_kernel<true>, dim3(grid), dim3(256), 0, c->stream, a);
    else
      hipLaunchKernelGGL(leapfrog_kernel<false>, dim3(grid), dim3(256), 0, c->stream, a);
    c->tail_ev = nullptr;
    HIPCHK(c, hipGetLastError());
    return SWRT_OK;
  }
  // timing events (pairs), grown on demand; fold into a running sum when full
  if (c->timing.used + 2 > kMaxEvents) {
    if (int rc = sync_sx(c)) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (size_t i = 0; i + 1 < c->timing.used; i += 2) {
      float ms = 0.f;
      HIPCHK(c, hipEventElapsedTime(&ms, c->timing.ev[i], c->timing.ev[i + 1]));
      c->timing.folded_ms += ms;
      c->timing.folded_n += 1;
    }
    c->timing.used = 0;
  }
  if (c->timing.used + 2 > c->timing.ev.size()) {
    for (int e = 0; e < 64; ++e) {
      hipEvent_t ev;
      HIPCHK(c, hipEventCreate(&ev));
      c->timing.ev.push_back(ev);
    }
  }
  c->kev0 = c->timing.ev[c->timing.used];
  c->kev1 = c->timing.ev[c->timing.used + 1];
  c->timing.used += 2;
  int rc = SWRT_OK;
  if (use_tile_kernel(c)) {
    rc = tile_launch(c, a, count_next, iv);
  } else if ((rc = leap_launch_prep(c, a)) == SWRT_OK) {
    c->keys_fresh = false;
    if (a.nslots == 2)
      launch_k(c, leapfrog_kernel<true>, dim3(grid), dim3(256), a);
    else
      launch_k(c, leapfrog_kernel<false>, dim3(grid), dim3(256), a);
  }
  c->kev0 = c->kev1 = nullptr;
  if (rc) return rc;
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}

// Longest-first tile order of the LDS-tiled launches, written by every
// re-binning's scan (bin_scan_kernel) beside the tile starts.
int* tile_order_of(swrt_ctx* c) { return c->bins + 3 * kMaxBins + 1; }

bool use_tile_kernel(const swrt_ctx* c) {
  if (c->rebin_every <= 0) return false;
  if (c->kernel == 2) return true;
  return c->kernel == 0 && c->slot[0].nx >= 2 * kTile;
}

// The sparse-tile launch shape (kSparseThreads threads, prefetch depth
// kSparsePrefetch) for the two-snapshot five-sum launches over `ntiles` tiles.
bool sparse_tiles(const swrt_ctx* c, int64_t ntiles) {
  if (c->sparse_mode == 1) return false;
  if (c->sparse_mode == 2) return true;
  return c->n < (int64_t)kSparseBelow * ntiles;
}

// Threads per workgroup of the LDS-tiled leapfrog launch over `ntiles` tiles
// of snapshots that are (v5) two divergence-free slots: ONE decision for the
// launch (tile_launch) and for the re-binning's longest-first tile order,
// which ranks tiles by the rounds of this many lanes their workgroup runs.
int tile_threads(const swrt_ctx* c, bool v5_two, int64_t ntiles) {
  return v5_two && sparse_tiles(c, ntiles) ? kSparseThreads : kTileThreads;
}

// slots sa .. sa+nslots-1 are two divergence-free snapshots (the five-sum kernels)
bool two_v5(const swrt_ctx* c, int nslots, int sa) {
  bool v5 = nslots >= 2;
  for (int i = 0; i < nslots && v5; ++i) v5 = c->slot[sa + i].div_free;
  return v5;
}

int tile_cells(const swrt_ctx* c, int64_t nx) {
  if (use_tile_kernel(c)) return kTile;
  if (c->tile > 0) return (int)std::min<int64_t>(c->tile, nx);
  // default: 8x8-cell tiles, coarser on big grids so bins stay <= 4096
  int t = 8;
  while ((nx + t - 1) / t > 64) t *= 2;
  return t;
}

// Counting-sort the packets by spatial tile of slot 0's grid (swrt_bin.hpp).
// indirect: only build the source index of the binned order (c->src_idx);
// the tile launch that follows reads through it and writes the packets in
// binned order (saves moving 36 B per packet twice).  Callers other than the
// leapfrog loop need the packets moved (indirect = false).  lanes: the
// workgroup width of the launches this binning serves (tile_threads), by
// which the scan ranks the tile order.
int rebin(swrt_ctx* c, bool indirect, int tile = 0, int lanes = kTileThreads) {
  if (int rc = join_b(c)) return rc;  // the second stream's half launches wrote packets this pass reads
  c->s0_dirty = true;  // a new binning: the next split launch forks
  const Slot& s = c->slot[0];
  const FieldView v = view_of(s);
  BinGeom g;
  g.dx = v.dx; g.px = v.px; g.py = v.py; g.inv_px = v.inv_px; g.inv_py = v.inv_py; g.inv_dx = v.inv_dx;
  g.nx = v.nx;
  g.tile = tile > 0 ? tile : tile_cells(c, s.nx);
  g.ntx = (int)((s.nx + g.tile - 1) / g.tile);
  const int nbins = g.ntx * g.ntx;
  if (nbins > kMaxBins) return fail(c, SWRT_ERR_ARG, "too many spatial bins (raise tile size)");
  const int64_t n = c->n;
  const unsigned grid = nblocks(n, 256 * kBinPerThread);
  const bool keys_valid = c->keys_fresh && c->bin_valid && nbins == c->nbins && c->key_nx == v.nx && c->key_dx == v.dx;
  if (c->hz.on) {  // count, scan and scatter on the packet stream
    HazardChecker& h = c->hz;
    const uint64_t t = h.op(0);
    const char* what = "a re-binning";
    const HzRegion all = HzRegion::all();
    bool ok = h.access(0, t, c->dx, kHzRead, all, what) && h.access(0, t, c->dk, kHzRead, all, what) &&
              h.access(0, t, c->perm, kHzRead, all, what) &&
              h.access(0, t, c->keys, keys_valid ? kHzRead : kHzWrite, all, what) &&
              h.access(0, t, c->bins, kHzWrite, all, what) && h.access(0, t, c->bins + kMaxBins, kHzWrite, all, what) &&
              h.access(0, t, c->bins + 2 * kMaxBins, kHzWrite, all, what) &&
              h.access(0, t, tile_order_of(c), kHzWrite, all, what);
    if (indirect)
      ok = ok && h.access(0, t, c->src_idx, kHzWrite, all, what);
    else
      ok = ok && h.access(0, t, c->dx2, kHzWrite, all, what) && h.access(0, t, c->dk2, kHzWrite, all, what) &&
           h.access(0, t, c->perm2, kHzWrite, all, what);
    if (!ok) return fail(c, SWRT_ERR_STATE, h.err);
    ++h.epoch;  // a new partition of the packets into tiles
  }
  if (!keys_valid) {
    // No memset when the last scan zeroed exactly these counts (the same bin
    // count, no counting launch since): every second ode23 interval's
    // re-binning then starts with the count.  Counts past the last scan's
    // bins may hold an older, larger binning's counting launch
    // (profiles/r06_ode23/README.md), hence the equal bin count.
    if (!(c->counts_zero && c->nbins == nbins)) HIPCHK(c, hipMemsetAsync(c->bins, 0, sizeof(int) * nbins, c->stream));
    hipLaunchKernelGGL(bin_count_kernel, dim3(grid), dim3(256), sizeof(int) * nbins, c->stream, g, c->dx, n,
                       nbins, c->keys, c->bins);
    HIPCHK(c, hipGetLastError());
  }
  c->keys_fresh = false;
  if (c->debug_corrupt_count != 0) {  // test-only: one corrupted count, once
    hipLaunchKernelGGL(debug_corrupt_count_kernel, dim3(1), dim3(64), 0, c->stream, c->bins, nbins / 2,
                       c->debug_corrupt_count);
    c->debug_corrupt_count = 0;
  }
  hipLaunchKernelGGL(bin_scan_kernel, dim3(1), dim3(1024), 0, c->stream, c->bins, nbins, c->bins + kMaxBins,
                     c->bins + 2 * kMaxBins, n, c->dev_err_d, tile_order_of(c), lanes);
  HIPCHK(c, hipGetLastError());
  c->counts_zero = true;
  c->bin_tile = g.tile;
  c->bin_lanes = lanes;
  if (indirect) {
    hipLaunchKernelGGL(bin_scatter_kernel<true>, dim3(grid), dim3(256), 2 * sizeof(int) * nbins, c->stream,
                       c->dx, c->dk, c->perm, c->keys, n, nbins, c->bins + kMaxBins, c->dx2, c->dk2, c->perm2,
                       c->src_idx);
  } else {
    hipLaunchKernelGGL(bin_scatter_kernel<false>, dim3(grid), dim3(256), 2 * sizeof(int) * nbins, c->stream,
                       c->dx, c->dk, c->perm, c->keys, n, nbins, c->bins + kMaxBins, c->dx2, c->dk2, c->perm2,
                       nullptr);
    std::swap(c->dx, c->dx2);
    std::swap(c->dk, c->dk2);
    std::swap(c->perm, c->perm2);
  }
  HIPCHK(c, hipGetLastError());
  c->src_pending = indirect;
  c->o_order_valid = false;
  c->o_sorted = false;
  c->steps_since_bin = 0;
  c->bin_valid = true;
  c->cells_sorted = false;
  c->nbins = nbins;
  return SWRT_OK;
}

int tile_launch(swrt_ctx* c, const StepArgs& a, bool count_next, const IvLaunch* iv) {
  TileArgs t;
  t.s = a;
  t.ivmode = iv != nullptr;
  t.nint = iv ? iv->nint : 1;
  if (iv) {
    for (int i = 0; i <= iv->nint; ++i) t.ivn[i] = iv->views[i].nodes;
    for (int i = 0; i < iv->nint; ++i) t.ivdt[i] = iv->dts[i];
  }
  t.x_out = c->dx2;
  t.k_out = c->dk2;
  t.perm_out = c->perm2;
  t.starts = c->bins + 2 * kMaxBins;
  t.order = tile_order_of(c);
  if (c->bin_tile != kTile) return fail(c, SWRT_ERR_STATE, "the binning is not the LDS-tiled kernel's");
  t.ntx = (int)((a.f0.nx + kTile - 1) / kTile);
  const int ntiles = t.ntx * t.ntx;
  t.next_keys = nullptr;
  t.next_counts = nullptr;
  t.sort_cells = c->cells_sorted ? 0 : 1;
  t.src = nullptr;
  // sort keys lead by half the steps until the next sort (swrt_tile.hpp)
  t.sort_lead = c->sort_lead ? 0.5 * a.dt * (double)std::max<int64_t>(1, c->rebin_every) : 0.0;
  if (c->src_pending) {  // first launch after an indirect re-binning (always a sort launch)
    t.src = c->src_idx;
    t.sort_cells = 1;
  }
  bool zero = false;  // the counts' memset, queued by launch_tiles after its hazard check
  if (count_next && ntiles == c->nbins) {
    zero = !c->counts_zero;
    t.next_keys = c->keys;
    t.next_counts = c->bins;
  }
  const bool fma = c->gather_mode == 1;
  if (a.nslots == 2) {
    if (iv ? iv->div_free : two_v5(c, 2, 0)) {
      if (tile_threads(c, true, ntiles) == kSparseThreads) {
        if (fma)
          HIPCHK_RC(launch_tiles(c, tile_leapfrog_kernel<true, kTile, kMargin, kSparseThreads, true, true, kSparsePrefetch, kSparseMinWaves>, kSparseThreads, t, zero));
        else
          HIPCHK_RC(launch_tiles(c, tile_leapfrog_kernel<true, kTile, kMargin, kSparseThreads, true, false, kSparsePrefetch, kSparseMinWaves>, kSparseThreads, t, zero));
      } else if (fma) {
        HIPCHK_RC(launch_tiles(c, tile_leapfrog_kernel<true, kTile, kMargin, kTileThreads, true, true>, kTileThreads, t, zero));
      } else {
        HIPCHK_RC(launch_tiles(c, tile_leapfrog_kernel<true, kTile, kMargin, kTileThreads, true>, kTileThreads, t, zero));
      }
    } else {
      HIPCHK_RC(launch_tiles(c, tile_leapfrog_kernel<true, kTile, kMargin, kTileThreads>, kTileThreads, t, zero));
    }
  } else {
    if (c->slot[0].div_free && fma)
      HIPCHK_RC(launch_tiles(c, tile_leapfrog_kernel<false, kTile, kMargin, kTileThreads, true, true>, kTileThreads, t, zero));
    else if (c->slot[0].div_free)
      HIPCHK_RC(launch_tiles(c, tile_leapfrog_kernel<false, kTile, kMargin, kTileThreads, true>, kTileThreads, t, zero));
    else
      HIPCHK_RC(launch_tiles(c, tile_leapfrog_kernel<false, kTile, kMargin, kTileThreads>, kTileThreads, t, zero));
  }
  HIPCHK(c, hipGetLastError());
  c->src_pending = false;
  if (t.next_keys != nullptr) {
    c->counts_zero = false;
    c->key_nx = a.f0.nx;  // the view this launch bins by (a multi-interval launch: slot i0's)
    c->key_dx = a.f0.dx;
  }
  if (t.src != nullptr && c->b_pending && !c->debug_legacy_park) {
    // The first launch after an indirect re-binning reads its input through
    // src_idx from any slot of dx while its parts run on two streams; the
    // next launch's parts would overwrite dx at their own tiles' slots before
    // the other part has read them.  The next launches write the third
    // buffers instead and dx is parked there until the next re-binning
    // (which orders every stream's work first).
    double* x = c->dx; double* k = c->dk; int* pm = c->perm;
    c->dx = c->dx2; c->dk = c->dk2; c->perm = c->perm2;
    c->dx2 = c->dx3; c->dk2 = c->dk3; c->perm2 = c->perm3;
    c->dx3 = x; c->dk3 = k; c->perm3 = pm;
  } else {
    std::swap(c->dx, c->dx2);
    std::swap(c->dk, c->dk2);
    std::swap(c->perm, c->perm2);
  }
  c->keys_fresh = t.next_keys != nullptr;
  c->cells_sorted = true;  // written in (the input's or this launch's) cell order
  return SWRT_OK;
}

// the re-binning of a leapfrog call over slots sa .. sa+nslots-1, when due
int leap_rebin_if_due(swrt_ctx* c, int nslots, int sa) {
  if (c->rebin_every <= 0) return SWRT_OK;
  const bool tiled = use_tile_kernel(c);
  const int64_t ntiles = tiled ? ((c->slot[sa].nx + kTile - 1) / kTile) * ((c->slot[sa].nx + kTile - 1) / kTile) : 0;
  const int lanes = tiled ? tile_threads(c, two_v5(c, nslots, sa), ntiles) : kTileThreads;
  if (!c->bin_valid || c->steps_since_bin >= c->rebin_every ||
      (tiled && (c->bin_tile != kTile || c->bin_lanes != lanes)))
    return rebin(c, tiled, tiled ? kTile : 0, lanes);
  return SWRT_OK;
}

int run_advance(swrt_ctx* c, double dt, int64_t nsteps, double f, double gH, int nslots,
                double alpha0, double dalpha, double bump, int64_t save_every, int sa = 0) {
  StepArgs a;
  a.f0 = view_of(c->slot[sa]);
  a.f1 = nslots == 2 ? view_of(c->slot[sa + 1]) : a.f0;
  a.nslots = nslots;
  a.n = c->n;
  a.dt = dt;
  a.half = dt / 2;
  a.f2 = f * f;
  a.fastdisp = dispersion_fast(a.f2);
  a.gH = gH;
  a.alpha0 = alpha0;
  a.dalpha = dalpha;
  a.bump = bump;
  a.save_every = save_every > 0 ? save_every : 1;
  a.hist_x = save_every > 0 ? c->hx : nullptr;
  a.hist_k = save_every > 0 ? c->hk : nullptr;
  a.frame0 = c->hframes;
  const unsigned grid = nblocks(c->n, 256);
  int64_t s0 = 0;
  while (s0 < nsteps) {
    int64_t chunk = std::min<int64_t>(kMaxStepsPerLaunch, nsteps - s0);
    if (c->rebin_every > 0) {
      if (int rc = leap_rebin_if_due(c, nslots, sa)) return rc;
      chunk = std::min<int64_t>(chunk, c->rebin_every - c->steps_since_bin);
    }
    a.x = c->dx;
    a.k = c->dk;
    a.perm = c->perm;
    a.s0 = s0;
    a.nsteps = (int)chunk;
    // the launch that ends at a re-binning point also counts the next bins
    const bool count_next = c->rebin_every > 0 && c->steps_since_bin + chunk >= c->rebin_every;
    slot_writes_wait(c);  // after the re-binning: it reads no slot
    int rc = timed_launch(c, a, grid, count_next);
    if (rc) return rc;
    c->steps_since_bin += chunk;
    s0 += chunk;
  }
  return SWRT_OK;
}

// nint PDE intervals of nsub steps each, interval i blending slots i, i+1 at
// step size hs[i]: whole intervals per tile launch (up to kMaxIntervals, never
// across a re-binning), else one interval at a time through run_advance.
int run_advance_intervals(swrt_ctx* c, int nint, const double* hs, int64_t nsub, double f, double gH,
                          double alpha0, double dalpha, double bump, int64_t save_every) {
  const bool fused = use_tile_kernel(c) && c->rebin_every > 0 && c->rebin_every % nsub == 0 &&
                     nsub <= kMaxStepsPerLaunch;
  const int64_t fpi = save_every > 0 ? nsub / save_every : 0;  // frames per interval
  int i0 = 0;
  while (i0 < nint) {
    int k = 0;
    if (fused) {
      if (int rc = leap_rebin_if_due(c, std::min(nint - i0, kMaxIntervals) + 1, i0)) return rc;
      k = (int)std::min<int64_t>({(int64_t)(nint - i0), (c->rebin_every - c->steps_since_bin) / nsub,
                                  (int64_t)kMaxIntervals});
    }
    if (k < 1) {  // one interval on its own (it may straddle a re-binning)
      int rc = run_advance(c, hs[i0], nsub, f, gH, 2, alpha0, dalpha, bump, save_every, i0);
      if (rc) return rc;
      c->hframes += fpi;
      i0 += 1;
      continue;
    }
    IvLaunch iv;
    iv.nint = k;
    iv.div_free = true;
    for (int i = 0; i <= k; ++i) {
      iv.views[i] = view_of(c->slot[i0 + i]);
      iv.div_free = iv.div_free && c->slot[i0 + i].div_free;
    }
    for (int i = 0; i < k; ++i) iv.dts[i] = hs[i0 + i];
    StepArgs a;
    a.f0 = iv.views[0];
    a.f1 = iv.views[1];
    a.nslots = 2;
    a.n = c->n;
    a.dt = hs[i0];
    a.half = hs[i0] / 2;
    a.f2 = f * f;
    a.fastdisp = dispersion_fast(a.f2);
    a.gH = gH;
    a.alpha0 = alpha0;
    a.dalpha = dalpha;
    a.bump = bump;
    a.save_every = save_every > 0 ? save_every : 1;
    a.hist_x = save_every > 0 ? c->hx : nullptr;
    a.hist_k = save_every > 0 ? c->hk : nullptr;
    a.frame0 = c->hframes;
    a.x = c->dx;
    a.k = c->dk;
    a.perm = c->perm;
    a.s0 = 0;
    a.nsteps = (int)nsub;
    const bool count_next = c->steps_since_bin + k * nsub >= c->rebin_every;
    slot_writes_wait(c);  // after the re-binning: it reads no slot
    int rc = timed_launch(c, a, nblocks(c->n, 256), count_next, &iv);
    if (rc) return rc;
    c->steps_since_bin += k * nsub;
    c->hframes += k * fpi;
    i0 += k;
  }
  return SWRT_OK;
}

// grow the history frames (keeps the existing ones).  The capacity is kept in
// doubles, not frames: a frame is 2 x n doubles and n changes with every
// swrt_packets_set, so a frame count sized for a smaller ensemble must not
// pass the check.
int ensure_history(swrt_ctx* c, int64_t new_frames) {
  const int64_t per = 2 * c->n;
  const int64_t need = (c->hframes + new_frames) * per;
  if (new_frames <= 0 || need <= c->hcap) return SWRT_OK;
  if (int rc = join_b(c)) return rc;  // the second stream may still write frames into the old buffers
  c->s0_dirty = true;
  const int64_t ncap = std::max<int64_t>(need, 2 * c->hcap);
  double *nx_ = nullptr, *nk_ = nullptr;
  HIPCHK(c, hipMalloc(&nx_, sizeof(double) * ncap));
  if (hipMalloc(&nk_, sizeof(double) * ncap) != hipSuccess) {
    (void)hipFree(nx_);
    return fail(c, SWRT_ERR_ALLOC, "history allocation failed");
  }
  if (c->hframes > 0) {
    HIPCHK(c, hipMemcpyAsync(nx_, c->hx, sizeof(double) * per * c->hframes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(nk_, c->hk, sizeof(double) * per * c->hframes, hipMemcpyDeviceToDevice, c->stream));
  }
  // the old buffers may still be read or written by queued work
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hz_synced(c);
  if (c->hz.on) {
    c->hz.bufs.erase(c->hx);
    c->hz.bufs.erase(c->hk);
    c->hz.name(nx_, "history x frames");
    c->hz.name(nk_, "history k frames");
  }
  if (c->hx) (void)hipFree(c->hx);
  if (c->hk) (void)hipFree(c->hk);
  c->hx = nx_;
  c->hk = nk_;
  c->hcap = ncap;
  return SWRT_OK;
}

}  // namespace

extern "C" {

int swrt_version(void) { return 100; }

int swrt_create(int device, swrt_ctx** out) {
  if (!out) return SWRT_ERR_ARG;
  *out = nullptr;
  swrt_ctx* c = nullptr;
  try {
    c = new swrt_ctx();
  } catch (...) {
    return SWRT_ERR_ALLOC;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    delete c;
    return SWRT_ERR_HIP;
  }
  c->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SWRT_ERR_HIP;
  }
  // the QG stream at the highest priority: its short dependent kernels are
  // dispatched ahead of the waiting workgroups of a packet launch (measured
  // neither faster nor slower than the default priority)
  int prio_least = 0, prio_greatest = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
  const int prio = prio_greatest;
  bool ok = hipStreamCreateWithPriority(&c->qstream, hipStreamNonBlocking, prio) == hipSuccess;
  for (Slot* s = c->slot; s != c->slot + SWRT_MAX_SLOTS; ++s)
    ok = ok && hipEventCreateWithFlags(&s->uev, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&s->wev, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&c->use_ev, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) == hipSuccess &&
       hipStreamCreateWithFlags(&c->sx[0], hipStreamNonBlocking) == hipSuccess;
  for (hipEvent_t& e : c->jx) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  for (hipEvent_t& e : c->chain_ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->dev_err, sizeof(int) * 4, hipHostMallocMapped | hipHostMallocCoherent) ==
                 hipSuccess &&
       hipHostGetDevicePointer((void**)&c->dev_err_d, c->dev_err, 0) == hipSuccess;
  if (c->dev_err) std::memset(c->dev_err, 0, sizeof(int) * 4);
  c->stream0 = c->stream;
  if (const char* e = getenv("SWRT_HAZARD_CHECK")) c->hz.on = atoi(e) != 0;
  if (const char* e = getenv("SWRT_ODE23_CHAIN_FIRST")) c->chain_first = atoi(e) != 0;
  if (const char* e = getenv("SWRT_FORK_ALWAYS")) c->fork_always = atoi(e) != 0;
  if (const char* e = getenv("SWRT_ODE23_MARKERS")) c->o23_markers = atoi(e) != 0;
  if (!ok) {
    swrt_destroy(c);
    return SWRT_ERR_HIP;
  }
  *out = c;
  return SWRT_OK;
}

void swrt_destroy(swrt_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (hipStream_t s : c->sx)
    if (s) (void)hipStreamSynchronize(s);
  if (c->qstream) (void)hipStreamSynchronize(c->qstream);
  auto free_slot = [](Slot& s) {
    if (s.nodes) (void)hipFree(s.nodes);
    if (s.psi) (void)hipFree(s.psi);
    if (s.uev) (void)hipEventDestroy(s.uev);
    if (s.wev) (void)hipEventDestroy(s.wev);
  };
  for (auto& s : c->slot) free_slot(s);
  if (c->use_ev) (void)hipEventDestroy(c->use_ev);
  for (auto& s : c->spares) free_slot(s);
  for (void* p : {(void*)c->dx, (void*)c->dk, (void*)c->perm, (void*)c->dx2, (void*)c->dk2,
                  (void*)c->perm2, (void*)c->dx3, (void*)c->dk3, (void*)c->perm3, (void*)c->keys,
                  (void*)c->src_idx, (void*)c->bins})
    if (p) (void)hipFree(p);
  if (c->hx) (void)hipFree(c->hx);
  if (c->hk) (void)hipFree(c->hk);
  if (c->clk) (void)hipFree(c->clk);
  if (c->dev_err) (void)hipHostFree(c->dev_err);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->tw) (void)hipFree(c->tw);
  for (void* p : {(void*)c->xka_state2, (void*)c->xka_keys, (void*)c->xka_src, (void*)c->xka_bins,
                  (void*)c->xka_src2, (void*)c->xka_perm2})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->xka_nodes, (void*)c->xka_state, (void*)c->xka_hist, (void*)c->modes,
                  (void*)c->mode_rows, (void*)c->modes_f, (void*)c->modes_f_row, (void*)c->modes_d,
                  (void*)c->modes_d_row})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->qg.qk, (void*)c->qg.qk_prev, (void*)c->qg.Qm1, (void*)c->qg.Qm2, (void*)c->qg.E1,
                  (void*)c->qg.E2, (void*)c->qg.Z, (void*)c->qg.T, (void*)c->qg.dmax, (void*)c->qg.PZ,
                  (void*)c->qg.PT, (void*)c->qg.qk_spare, (void*)c->qg.Qm1_spare, (void*)c->qg.Qm2_spare})
    if (p) (void)hipFree(p);
  if (c->qg.hmax) (void)hipHostFree(c->qg.hmax);
  if (c->o_hmax) (void)hipHostFree(c->o_hmax);
  if (c->o_hpart) (void)hipHostFree(c->o_hpart);
  if (c->o_shown) (void)hipHostFree(c->o_shown);
  if (c->o_coef) (void)hipFree(c->o_coef);
  for (hipEvent_t e : c->o_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->o_evb)
    if (e) (void)hipEventDestroy(e);
  if (c->qg.ev) (void)hipEventDestroy(c->qg.ev);
  if (c->qg.ev_b) (void)hipEventDestroy(c->qg.ev_b);
  if (c->o_order) (void)hipFree(c->o_order);
  for (void* p : {(void*)c->xq_Z, (void*)c->xq_T, (void*)c->xq_fk})
    if (p) (void)hipFree(p);
  for (hipEvent_t e : c->xev)
    if (e) (void)hipEventDestroy(e);
  for (void* p : {(void*)c->o_spx, (void*)c->o_spk, (void*)c->o_spF})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->oF[0], (void*)c->oF[1], (void*)c->oF[2], (void*)c->oF[3], (void*)c->o_ynx,
                  (void*)c->o_ynk, (void*)c->o_dmax})
    if (p) (void)hipFree(p);
  for (auto e : c->timing.ev) (void)hipEventDestroy(e);
  if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
  for (hipEvent_t e : c->chain_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->jx)
    if (e) (void)hipEventDestroy(e);
  if (c->qstream) (void)hipStreamDestroy(c->qstream);
  for (hipStream_t s : c->sx)
    if (s) (void)hipStreamDestroy(s);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* swrt_last_error(const swrt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int swrt_set_field_grid(swrt_ctx* c, int slot, const double* fields6, int64_t nx, double L,
                        int64_t ny_period) {
  int rc = check_slot_args(c, slot, nx);
  if (rc) return rc;
  GUARD_BEGIN
  SlotUse slot_use(c);
  if (!fields6) return fail(c, SWRT_ERR_ARG, "fields6 is NULL");
  if (!(L > 0)) return fail(c, SWRT_ERR_ARG, "L must be > 0");
  if (ny_period == 0) ny_period = nx;
  if (ny_period % nx) return fail(c, SWRT_ERR_ARG, "ny_period must be a multiple of nx");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_slot(c, slot, nx))) return rc;
  const size_t bytes = sizeof(double) * 6 * nx * nx;
  if ((rc = ensure_scratch(c, bytes))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->scratch, fields6, bytes, hipMemcpyHostToDevice, c->stream));
  if ((rc = pack_slot(c, slot, (const double*)c->scratch, 0.0))) return rc;
  // host-given fields take the five-sum kernels only if v_y == -u_x bit for bit
  bool div_free = true;
  {
    const int64_t plane = nx * nx;
    const uint64_t* ux = reinterpret_cast<const uint64_t*>(fields6 + 2 * plane);
    const uint64_t* vy = reinterpret_cast<const uint64_t*>(fields6 + 5 * plane);
    for (int64_t i = 0; i < plane && div_free; ++i) div_free = vy[i] == (ux[i] ^ 0x8000000000000000ull);
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  Slot& s = c->slot[slot];
  s.div_free = div_free;
  s.L = L;
  s.ny_period = ny_period;
  s.has_psi = false;
  s.set = true;
  s.wgen = ++c->slot_wgen;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_set_field_psi(swrt_ctx* c, int slot, const double* psi_grid, int64_t nx, double L) {
  int rc = check_slot_args(c, slot, nx);
  if (rc) return rc;
  GUARD_BEGIN
  SlotUse slot_use(c);
  if (!psi_grid) return fail(c, SWRT_ERR_ARG, "psi_grid is NULL");
  if (!is_pow2(nx)) return fail(c, SWRT_ERR_ARG, "nx must be a power of two for the GPU FFT");
  if (!(L > 0)) return fail(c, SWRT_ERR_ARG, "L must be > 0");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_slot(c, slot, nx))) return rc;
  if ((rc = ensure_twiddles(c, (int)nx))) return rc;
  const int n = (int)nx;
  const int64_t nn = nx * nx;
  const int kmax = n / 2 - 1;
  const int64_t nhalf = (int64_t)(2 * kmax + 1) * (kmax + 1);
  // scratch: Z (4 nn complex) | T (4 nn complex) | fk (nhalf complex) | raw (nn double)
  const size_t zb = sizeof(double2) * 4 * nn;
  const size_t bytes = 2 * zb + sizeof(double2) * nhalf + sizeof(double) * nn;
  if ((rc = ensure_scratch(c, bytes))) return rc;
  char* base = (char*)c->scratch;
  double2* Z = (double2*)base;
  double2* T = (double2*)(base + zb);
  double2* fk = (double2*)(base + 2 * zb);
  double* raw = (double*)(base + 2 * zb + sizeof(double2) * nhalf);
  HIPCHK(c, hipMemcpyAsync(raw, psi_grid, sizeof(double) * nn, hipMemcpyHostToDevice, c->stream));
  // g2k: forward FFT2 of the real grid (layout [r + n*c], r = x index)
  hipLaunchKernelGGL(real_to_complex_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, raw,
                     Z, nn);
  HIPCHK(c, hipGetLastError());
  if ((rc = transform_2d(c, Z, T, n, 1, 0))) return rc;  // along x, then y; T: [c + n*r]
  hipLaunchKernelGGL(crop_half_kernel, dim3(nblocks(nhalf, 256)), dim3(256), 0, c->stream, T, n, fk);
  HIPCHK(c, hipGetLastError());
  if ((rc = fields_from_halfplane(c, slot, fk, n, 0, 0.0, 1.0, 0.0, 1, Z, T, 1, 2 * (n / 2 - 1) + 1))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  Slot& s = c->slot[slot];
  s.L = L;
  s.ny_period = nx;
  s.set = true;
  s.wgen = ++c->slot_wgen;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_set_field_qk(swrt_ctx* c, int slot, const double* qk_interleaved, int64_t nx, double L,
                      double K_d2, double shear, double k_scale, int64_t ny_period) {
  int rc = check_slot_args(c, slot, nx);
  if (rc) return rc;
  GUARD_BEGIN
  SlotUse slot_use(c);
  if (!qk_interleaved) return fail(c, SWRT_ERR_ARG, "qk is NULL");
  if (!is_pow2(nx)) return fail(c, SWRT_ERR_ARG, "nx must be a power of two for the GPU FFT");
  if (!(L > 0)) return fail(c, SWRT_ERR_ARG, "L must be > 0");
  if (ny_period == 0) ny_period = nx;
  if (ny_period % nx) return fail(c, SWRT_ERR_ARG, "ny_period must be a multiple of nx");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_slot(c, slot, nx))) return rc;
  if ((rc = ensure_twiddles(c, (int)nx))) return rc;
  const int n = (int)nx;
  const int64_t nn = nx * nx;
  const int kmax = n / 2 - 1;
  const int64_t nhalf = (int64_t)(2 * kmax + 1) * (kmax + 1);
  const size_t zb = sizeof(double2) * 3 * nn;
  const size_t bytes = 2 * zb + sizeof(double2) * nhalf;
  if ((rc = ensure_scratch(c, bytes))) return rc;
  char* base = (char*)c->scratch;
  double2* Z = (double2*)base;
  double2* T = (double2*)(base + zb);
  double2* fk = (double2*)(base + 2 * zb);
  HIPCHK(c, hipMemcpyAsync(fk, qk_interleaved, sizeof(double2) * nhalf, hipMemcpyHostToDevice,
                           c->stream));
  if ((rc = fields_from_halfplane(c, slot, fk, n, 1, K_d2, k_scale, shear, 0, Z, T, 1, 2 * kmax + 1))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  Slot& s = c->slot[slot];
  s.L = L;
  s.ny_period = ny_period;
  s.set = true;
  s.wgen = ++c->slot_wgen;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_set_field_q(swrt_ctx* c, int slot, const double* q_grid, int64_t nx, double L, double K_d2,
                     double shear, double k_scale, int64_t ny_period) {
  int rc = check_slot_args(c, slot, nx);
  if (rc) return rc;
  GUARD_BEGIN
  SlotUse slot_use(c);
  if (!q_grid) return fail(c, SWRT_ERR_ARG, "q_grid is NULL");
  if (!is_pow2(nx)) return fail(c, SWRT_ERR_ARG, "nx must be a power of two for the GPU FFT");
  if (!(L > 0)) return fail(c, SWRT_ERR_ARG, "L must be > 0");
  if (ny_period == 0) ny_period = nx;
  if (ny_period % nx) return fail(c, SWRT_ERR_ARG, "ny_period must be a multiple of nx");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_slot(c, slot, nx))) return rc;
  if ((rc = ensure_twiddles(c, (int)nx))) return rc;
  const int n = (int)nx;
  const int64_t nn = nx * nx;
  const int kmax = n / 2 - 1;
  const int64_t nhalf = (int64_t)(2 * kmax + 1) * (kmax + 1);
  // scratch: Z (3 nn complex) | T (3 nn complex) | fk (nhalf complex) | raw (nn double)
  const size_t zb = sizeof(double2) * 3 * nn;
  if ((rc = ensure_scratch(c, 2 * zb + sizeof(double2) * nhalf + sizeof(double) * nn))) return rc;
  char* base = (char*)c->scratch;
  double2* Z = (double2*)base;
  double2* T = (double2*)(base + zb);
  double2* fk = (double2*)(base + 2 * zb);
  double* raw = (double*)(base + 2 * zb + sizeof(double2) * nhalf);
  HIPCHK(c, hipMemcpyAsync(raw, q_grid, sizeof(double) * nn, hipMemcpyHostToDevice, c->stream));
  // qk = g2k(q) (g2k.m:8-9), exactly swrt_g2k's transform, kept on the device
  hipLaunchKernelGGL(real_to_complex_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, raw, Z, nn);
  HIPCHK(c, hipGetLastError());
  if ((rc = transform_2d(c, Z, T, n, 1, 0))) return rc;
  hipLaunchKernelGGL(crop_half_kernel, dim3(nblocks(nhalf, 256)), dim3(256), 0, c->stream, T, n, fk);
  HIPCHK(c, hipGetLastError());
  // grid_U(qk) (grid_U.m:1-18): the same path as swrt_set_field_qk
  if ((rc = fields_from_halfplane(c, slot, fk, n, 1, K_d2, k_scale, shear, 0, Z, T, 1, 2 * kmax + 1))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  Slot& s = c->slot[slot];
  s.L = L;
  s.ny_period = ny_period;
  s.set = true;
  s.wgen = ++c->slot_wgen;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_g2k(swrt_ctx* c, const double* fg, int64_t nx, double* fk_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!fg || !fk_out) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  if (nx < 8 || nx > 4096 || !is_pow2(nx)) return fail(c, SWRT_ERR_ARG, "nx must be a power of two, 8..4096");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_twiddles(c, (int)nx))) return rc;
  const int n = (int)nx;
  const int64_t nn = nx * nx;
  const int kmax = n / 2 - 1;
  const int64_t nhalf = (int64_t)(2 * kmax + 1) * (kmax + 1);
  const size_t zb = sizeof(double2) * nn;
  if ((rc = ensure_scratch(c, 2 * zb + sizeof(double2) * nhalf + sizeof(double) * nn))) return rc;
  char* base = (char*)c->scratch;
  double2* Z = (double2*)base;
  double2* T = (double2*)(base + zb);
  double2* fk = (double2*)(base + 2 * zb);
  double* raw = (double*)(base + 2 * zb + sizeof(double2) * nhalf);
  HIPCHK(c, hipMemcpyAsync(raw, fg, sizeof(double) * nn, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(real_to_complex_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, raw, Z, nn);
  HIPCHK(c, hipGetLastError());
  if ((rc = transform_2d(c, Z, T, n, 1, 0))) return rc;
  hipLaunchKernelGGL(crop_half_kernel, dim3(nblocks(nhalf, 256)), dim3(256), 0, c->stream, T, n, fk);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(fk_out, fk, sizeof(double2) * nhalf, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_k2g(swrt_ctx* c, const double* fk_in, int64_t nx, double* fg_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!fk_in || !fg_out) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  if (nx < 8 || nx > 4096 || !is_pow2(nx)) return fail(c, SWRT_ERR_ARG, "nx must be a power of two, 8..4096");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_twiddles(c, (int)nx))) return rc;
  const int n = (int)nx;
  const int64_t nn = nx * nx;
  const int kmax = n / 2 - 1;
  const int64_t nhalf = (int64_t)(2 * kmax + 1) * (kmax + 1);
  const size_t zb = sizeof(double2) * nn;
  if ((rc = ensure_scratch(c, 2 * zb + sizeof(double2) * nhalf + sizeof(double) * nn))) return rc;
  char* base = (char*)c->scratch;
  double2* Z = (double2*)base;
  double2* T = (double2*)(base + zb);
  double2* fk = (double2*)(base + 2 * zb);
  double* raw = (double*)(base + 2 * zb + sizeof(double2) * nhalf);
  HIPCHK(c, hipMemcpyAsync(fk, fk_in, sizeof(double2) * nhalf, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(fulspec_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, fk, n, Z, 1, 2 * kmax + 1);
  HIPCHK(c, hipGetLastError());
  if ((rc = inverse_2d(c, Z, T, n, 1))) return rc;
  hipLaunchKernelGGL(real_part_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, T, raw, nn);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(fg_out, raw, sizeof(double) * nn, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_field_div_free(swrt_ctx* c, int slot) {
  if (!c) return SWRT_ERR_ARG;
  if (slot < 0 || slot >= SWRT_MAX_SLOTS || !c->slot[slot].set)
    return fail(c, SWRT_ERR_STATE, "slot not set");
  return c->slot[slot].div_free ? 1 : 0;
}

int swrt_get_field_grid(swrt_ctx* c, int slot, double* out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  SlotUse slot_use(c);
  if (slot < 0 || slot >= SWRT_MAX_SLOTS || !c->slot[slot].set)
    return fail(c, SWRT_ERR_STATE, "slot not set");
  if (!out) return fail(c, SWRT_ERR_ARG, "out is NULL");
  HIPCHK(c, hipSetDevice(c->device));
  Slot& s = c->slot[slot];
  const int64_t nn = s.nx * s.nx;
  int rc;
  if ((rc = ensure_scratch(c, sizeof(double) * 6 * nn))) return rc;
  hipLaunchKernelGGL(unpack_nodes_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, s.nodes,
                     (int)s.nx, (int)s.npad, (double*)c->scratch);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, c->scratch, sizeof(double) * 6 * nn, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_get_psi_grid(swrt_ctx* c, int slot, double* out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  SlotUse slot_use(c);
  if (slot < 0 || slot >= SWRT_MAX_SLOTS || !c->slot[slot].set || !c->slot[slot].has_psi)
    return fail(c, SWRT_ERR_STATE, "slot has no psi grid (use swrt_set_field_psi)");
  if (!out) return fail(c, SWRT_ERR_ARG, "out is NULL");
  HIPCHK(c, hipSetDevice(c->device));
  Slot& s = c->slot[slot];
  HIPCHK(c, hipMemcpyAsync(out, s.psi, sizeof(double) * s.nx * s.nx, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_interpolate(swrt_ctx* c, const double* F, int64_t nx, int64_t nyF, double dx, double dy,
                     double bump, const double* x, const double* y, int64_t n, double* out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (n < 0) return fail(c, SWRT_ERR_ARG, "n < 0");
  if (n == 0) return SWRT_OK;
  if (!F || !x || !y || !out) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  if (nx < 6 || nyF < nx) return fail(c, SWRT_ERR_ARG, "need nx >= 6 and nyF >= nx");
  if (!(dx > 0) || !(dy > 0)) return fail(c, SWRT_ERR_ARG, "dx, dy must be > 0");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t fb = sizeof(double) * nx * nx;  // only the first nx columns are read
  const size_t bytes = fb + sizeof(double) * 3 * n;
  int rc;
  if ((rc = ensure_scratch(c, bytes))) return rc;
  double* dF = (double*)c->scratch;
  double* dxp = dF + nx * nx;
  double* dyp = dxp + n;
  double* dout = dyp + n;
  HIPCHK(c, hipMemcpyAsync(dF, F, fb, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dxp, x, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dyp, y, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  const double py = (double)nyF;
  hipLaunchKernelGGL(interp1_kernel, dim3(nblocks(n, 256)), dim3(256), 0, c->stream, dF, (int)nx, py,
                     1.0 / py, dx, dy, bump, dxp, dyp, n, dout);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, dout, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_eval(swrt_ctx* c, const double* x, const double* y, int64_t n, int nslots, double alpha,
              double bump, double* out6) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  SlotUse slot_use(c);
  if (n < 0) return fail(c, SWRT_ERR_ARG, "n < 0");
  if (n == 0) return SWRT_OK;
  if (!x || !y || !out6) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  if (nslots != 1 && nslots != 2) return fail(c, SWRT_ERR_ARG, "nslots must be 1 or 2");
  for (int s = 0; s < nslots; ++s)
    if (!c->slot[s].set) return fail(c, SWRT_ERR_STATE, "field slot not set");
  if (nslots == 2 && (c->slot[1].nx != c->slot[0].nx || c->slot[1].L != c->slot[0].L ||
                      c->slot[1].ny_period != c->slot[0].ny_period))
    return fail(c, SWRT_ERR_ARG, "slots 0 and 1 have different grids");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_scratch(c, sizeof(double) * 8 * n))) return rc;
  double* dxp = (double*)c->scratch;
  double* dyp = dxp + n;
  double* dout = dyp + n;
  HIPCHK(c, hipMemcpyAsync(dxp, x, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dyp, y, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  FieldView f0 = view_of(c->slot[0]);
  FieldView f1 = nslots == 2 ? view_of(c->slot[1]) : f0;
  hipLaunchKernelGGL(eval_kernel, dim3(nblocks(n, 256)), dim3(256), 0, c->stream, f0, f1, nslots,
                     alpha, bump, dxp, dyp, n, dout);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out6, dout, sizeof(double) * 6 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_packets_set(swrt_ctx* c, const double* x, const double* k, int64_t n) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (n < 0 || n > INT32_MAX) return fail(c, SWRT_ERR_ARG, "n out of range (0..2^31-1)");
  if (n > 0 && (!x || !k)) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  HIPCHK(c, hipSetDevice(c->device));
  if (n > c->cap) {
    for (void** p : {(void**)&c->dx, (void**)&c->dk, (void**)&c->perm, (void**)&c->dx2, (void**)&c->dk2,
                     (void**)&c->perm2, (void**)&c->dx3, (void**)&c->dk3, (void**)&c->perm3, (void**)&c->keys,
                     (void**)&c->src_idx}) {
      if (*p) (void)hipFree(*p);
      *p = nullptr;
    }
    c->cap = 0;
    HIPCHK(c, hipMalloc(&c->dx, sizeof(double) * 2 * n));
    HIPCHK(c, hipMalloc(&c->dk, sizeof(double) * 2 * n));
    HIPCHK(c, hipMalloc(&c->dx2, sizeof(double) * 2 * n));
    HIPCHK(c, hipMalloc(&c->dk2, sizeof(double) * 2 * n));
    HIPCHK(c, hipMalloc(&c->perm, sizeof(int) * n));
    HIPCHK(c, hipMalloc(&c->perm2, sizeof(int) * n));
    HIPCHK(c, hipMalloc(&c->dx3, sizeof(double) * 2 * n));
    HIPCHK(c, hipMalloc(&c->dk3, sizeof(double) * 2 * n));
    HIPCHK(c, hipMalloc(&c->perm3, sizeof(int) * n));
    HIPCHK(c, hipMalloc(&c->keys, sizeof(int) * n));
    HIPCHK(c, hipMalloc(&c->src_idx, sizeof(int) * n));
    c->cap = n;
  }
  if (!c->bins) HIPCHK(c, hipMalloc(&c->bins, sizeof(int) * (4 * kMaxBins + 1)));
  c->n = n;
  if (n > 0) {
    HIPCHK(c, hipMemcpyAsync(c->dx, x, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->dk, k, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(iota_kernel, dim3(nblocks(n, 256)), dim3(256), 0, c->stream, c->perm, n);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->hz.on) {  // every packet stream's work is complete (joined, then synchronised)
    c->hz.quiesce();
    ++c->hz.epoch;
    const char* tags[] = {"A", "B", "C"};
    double* xs[] = {c->dx, c->dx2, c->dx3};
    double* ks[] = {c->dk, c->dk2, c->dk3};
    int* ps[] = {c->perm, c->perm2, c->perm3};
    for (int i = 0; i < 3; ++i) {
      c->hz.name(xs[i], std::string("packet x buffer ") + tags[i]);
      c->hz.name(ks[i], std::string("packet k buffer ") + tags[i]);
      c->hz.name(ps[i], std::string("permutation buffer ") + tags[i]);
    }
    c->hz.name(c->keys, "binning keys");
    c->hz.name(c->src_idx, "re-binning source index");
    c->hz.name(c->bins, "bin counts");
    c->hz.name(c->bins + kMaxBins, "bin cursors");
    c->hz.name(c->bins + 2 * kMaxBins, "tile starts");
    c->hz.name(c->bins + 3 * kMaxBins + 1, "tile order");
  }
  // a new ensemble starts a new history and needs binning before the next step
  if (c->dev_err) c->dev_err[0] = 0;  // (an error raised over the old ensemble is superseded)
  c->packets_lost = false;
  c->hframes = 0;
  c->steps_done = 0;
  c->bin_valid = false;
  c->keys_fresh = false;
  c->src_pending = false;
  c->steps_since_bin = 0;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_packets_get(swrt_ctx* c, double* x, double* k) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (c->n == 0) return SWRT_OK;
  if (!x || !k) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  if (c->packets_lost) return fail(c, SWRT_ERR_STATE, "the packet state was lost to a corrupted binning");
  HIPCHK(c, hipSetDevice(c->device));
  // un-permute into the scatter buffers, then download in original order
  hipLaunchKernelGGL(unpermute_kernel, dim3(nblocks(c->n, 256)), dim3(256), 0, c->stream, c->dx, c->dk,
                     c->perm, c->n, c->n, c->dx2, c->dk2);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(x, c->dx2, sizeof(double) * 2 * c->n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(k, c->dk2, sizeof(double) * 2 * c->n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return dev_err_check(c);
  GUARD_END(c)
}

int swrt_packets_get_device(swrt_ctx* c, double* x_dev, double* k_dev, int64_t ld) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  HIPCHK_RC(lost_check(c));  // (perm would be stale: never unpermute a lost state)
  if (c->n == 0) return SWRT_OK;
  if (!x_dev || !k_dev) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  if (ld < c->n) return fail(c, SWRT_ERR_ARG, "leading dimension below the packet count");
  HIPCHK(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(unpermute_kernel, dim3(nblocks(c->n, 256)), dim3(256), 0, c->stream, c->dx, c->dk,
                     c->perm, c->n, ld, x_dev, k_dev);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_set_timing(swrt_ctx* c, int every) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (every < 0) return fail(c, SWRT_ERR_ARG, "timing interval must be >= 0");
  c->timing_every = every;
  c->launch_count = 0;
  return SWRT_OK;
}

int swrt_set_gather_mode(swrt_ctx* c, int mode) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (mode != 0 && mode != 1) return fail(c, SWRT_ERR_ARG, "gather mode must be 0 or 1");
  c->gather_mode = mode;
  return SWRT_OK;
}

int swrt_set_packet_streams(swrt_ctx* c, int streams) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (streams != 1 && streams != 2) return fail(c, SWRT_ERR_ARG, "packet streams must be 1 or 2");
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = join_b(c)) return rc;
  for (int i = 0; i < streams - 1; ++i)
    if (!c->sx[i]) HIPCHK(c, hipStreamCreateWithFlags(&c->sx[i], hipStreamNonBlocking));
  c->packet_streams = streams;
  return SWRT_OK;
}

int swrt_set_sparse_tiles(swrt_ctx* c, int mode) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (mode < 0 || mode > 2) return fail(c, SWRT_ERR_ARG, "sparse tiles must be 0 (auto), 1 (never) or 2 (always)");
  c->sparse_mode = mode;
  c->bin_valid = false;  // the tile order of the next binning is sized for the launch shape
  c->keys_fresh = false;
  c->src_pending = false;
  return SWRT_OK;
}

int swrt_set_kernel(swrt_ctx* c, int variant) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (variant < 0 || variant > 2) return fail(c, SWRT_ERR_ARG, "kernel variant must be 0..2");
  c->kernel = variant;
  c->bin_valid = false;
  c->keys_fresh = false;
  c->src_pending = false;
  return SWRT_OK;
}

int swrt_set_locality(swrt_ctx* c, int64_t rebin_every, int64_t tile) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (rebin_every < 0 || tile < 0) return fail(c, SWRT_ERR_ARG, "negative locality parameter");
  c->rebin_every = rebin_every;
  c->tile = tile;
  c->bin_valid = false;
  c->keys_fresh = false;
  c->src_pending = false;
  return SWRT_OK;
}

int64_t swrt_packets_count(const swrt_ctx* c) { return c ? c->n : -1; }

int swrt_advance(swrt_ctx* c, double dt, int64_t nsteps, double f, double gH, int nslots,
                 double alpha0, double dalpha, double bump, int64_t save_every) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_SPLIT  // the half launches of the second packet stream stay unjoined across calls
  SlotUse slot_use(c, true);  // snapshot writes waited for before the first launch (run_advance)
  if (c->packets_lost) return fail(c, SWRT_ERR_STATE, "the packet state was lost to a corrupted binning");
  if (nsteps < 0) return fail(c, SWRT_ERR_ARG, "nsteps < 0");
  if (nslots != 1 && nslots != 2) return fail(c, SWRT_ERR_ARG, "nslots must be 1 or 2");
  if (save_every < 0) return fail(c, SWRT_ERR_ARG, "save_every < 0");
  for (int s = 0; s < nslots; ++s)
    if (!c->slot[s].set) return fail(c, SWRT_ERR_STATE, "field slot not set");
  if (nslots == 2 && (c->slot[1].nx != c->slot[0].nx || c->slot[1].L != c->slot[0].L ||
                      c->slot[1].ny_period != c->slot[0].ny_period))
    return fail(c, SWRT_ERR_ARG, "slots 0 and 1 have different grids");
  if (c->n == 0 || nsteps == 0) return SWRT_OK;
  HIPCHK(c, hipSetDevice(c->device));
  int64_t new_frames = save_every > 0 ? nsteps / save_every : 0;
  if (save_every > 0 && nsteps % save_every)
    return fail(c, SWRT_ERR_ARG, "nsteps must be a multiple of save_every");
  int rc = ensure_history(c, new_frames);
  if (rc) return rc;
  rc = run_advance(c, dt, nsteps, f, gH, nslots, alpha0, dalpha, bump, save_every);
  if (rc) return rc;
  c->hframes += new_frames;
  c->steps_done += nsteps;
  // a QG stream renames slots by their use events: mark them after the second stream's launches too
  if (slot_events(c)) HIPCHK_RC(join_b(c));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_advance_intervals(swrt_ctx* c, int nintervals, const double* dts, int64_t nsub, double f, double gH,
                           double alpha0, double dalpha, double bump, int64_t save_every) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_SPLIT  // the half launches of the second packet stream stay unjoined across calls
  SlotUse slot_use(c, true);  // snapshot writes waited for before the first launch (run_advance*)
  if (c->packets_lost) return fail(c, SWRT_ERR_STATE, "the packet state was lost to a corrupted binning");
  if (nintervals < 1 || nintervals > SWRT_MAX_SLOTS - 1)
    return fail(c, SWRT_ERR_ARG, "nintervals must be 1..SWRT_MAX_SLOTS-1");
  if (!dts) return fail(c, SWRT_ERR_ARG, "dts is NULL");
  if (nsub < 1) return fail(c, SWRT_ERR_ARG, "nsub must be >= 1");
  if (save_every < 0 || (save_every > 0 && nsub % save_every))
    return fail(c, SWRT_ERR_ARG, "save_every must divide nsub");
  for (int s = 0; s <= nintervals; ++s) {
    const Slot& sl = c->slot[s];
    if (!sl.set) return fail(c, SWRT_ERR_STATE, "field slot not set");
    if (sl.nx != c->slot[0].nx || sl.L != c->slot[0].L || sl.ny_period != c->slot[0].ny_period)
      return fail(c, SWRT_ERR_ARG, "slots have different grids");
  }
  for (int i = 0; i < nintervals; ++i)
    if (!(dts[i] > 0) || !std::isfinite(dts[i])) return fail(c, SWRT_ERR_ARG, "dts must be finite and > 0");
  if (c->n == 0) return SWRT_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const int64_t new_frames = save_every > 0 ? nintervals * (nsub / save_every) : 0;
  int rc = ensure_history(c, new_frames);
  if (rc) return rc;
  rc = run_advance_intervals(c, nintervals, dts, nsub, f, gH, alpha0, dalpha, bump, save_every);
  if (rc) return rc;
  c->steps_done += nintervals * nsub;
  // a QG stream renames slots by their use events: mark them after the second stream's launches too
  if (slot_events(c)) HIPCHK_RC(join_b(c));
  return SWRT_OK;
  GUARD_END(c)
}

int64_t swrt_history_frames(const swrt_ctx* c) { return c ? c->hframes : -1; }

int swrt_history_get(swrt_ctx* c, int64_t first, int64_t count, double* hist_x, double* hist_k) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (first < 0 || count < 0 || first + count > c->hframes)
    return fail(c, SWRT_ERR_ARG, "history frame range out of bounds");
  if (count == 0) return SWRT_OK;
  if (!hist_x || !hist_k) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t fb = sizeof(double) * 2 * c->n;
  HIPCHK(c, hipMemcpyAsync(hist_x, (char*)c->hx + fb * first, fb * count, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(hist_k, (char*)c->hk + fb * first, fb * count, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return dev_err_check(c);
  GUARD_END(c)
}

int swrt_history_reset(swrt_ctx* c) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  c->hframes = 0;
  c->steps_done = 0;
  return SWRT_OK;
}

int swrt_leapfrog(swrt_ctx* c, double* x, double* k, int64_t n, double dt, int64_t nsteps, double f,
                  double gH, int nslots, double alpha0, double dalpha, double bump,
                  int64_t save_every, double* hist_x, double* hist_k) {
  if (!c) return SWRT_ERR_ARG;
  int rc;
  if ((rc = swrt_packets_set(c, x, k, n))) return rc;
  const int64_t se = (hist_x && hist_k) ? save_every : 0;
  if ((rc = swrt_advance(c, dt, nsteps, f, gH, nslots, alpha0, dalpha, bump, se))) return rc;
  if ((rc = swrt_packets_get(c, x, k))) return rc;
  if (se > 0) {
    if ((rc = swrt_history_get(c, 0, c->hframes, hist_x, hist_k))) return rc;
  }
  return SWRT_OK;
}

}  // extern "C"

namespace {
// (Re)allocate the xka node array for an nx grid.
int xka_nodes_for(swrt_ctx* c, int64_t nx) {
  const int64_t npad = nx + kPadTot;
  if (c->xka_nx != nx) {
    if (c->xka_nodes) (void)hipFree(c->xka_nodes);
    c->xka_nodes = nullptr;
    c->xka_nx = 0;
    HIPCHK(c, hipMalloc(&c->xka_nodes, sizeof(double) * kXkaRec * npad * npad));
    c->xka_nx = nx;
  }
  return SWRT_OK;
}

// 7 device planes -> padded node records
int xka_pack(swrt_ctx* c, const double* dplanes, int64_t nx) {
  const int64_t npad = nx + kPadTot;
  hipLaunchKernelGGL(pack_xka_kernel, dim3(nblocks(npad * npad, 256)), dim3(256), 0, c->stream, dplanes, (int)nx,
                     (int)npad, c->xka_nodes);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}
}  // namespace

extern "C" {

int swrt_xka_set_fields(swrt_ctx* c, const double* fields7, int64_t nx, double dx, double dy) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!fields7) return fail(c, SWRT_ERR_ARG, "fields7 is NULL");
  if (nx < 6 || nx > 8192) return fail(c, SWRT_ERR_ARG, "nx out of range");
  if (!(dx > 0) || !(dy > 0)) return fail(c, SWRT_ERR_ARG, "dx, dy must be > 0");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = xka_nodes_for(c, nx))) return rc;
  if ((rc = ensure_scratch(c, sizeof(double) * 7 * nx * nx))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->scratch, fields7, sizeof(double) * 7 * nx * nx, hipMemcpyHostToDevice, c->stream));
  if ((rc = xka_pack(c, (const double*)c->scratch, nx))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->xka_dx = dx;
  c->xka_dy = dy;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_xka_set_rsw(swrt_ctx* c, const double* state3, int64_t nx, double f, double Cg, double L) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!state3) return fail(c, SWRT_ERR_ARG, "state3 is NULL");
  if (nx < 8 || nx > 4096 || !is_pow2(nx)) return fail(c, SWRT_ERR_ARG, "nx must be a power of two, 8..4096");
  if (!(f != 0.0) || !std::isfinite(f) || !std::isfinite(Cg) || !(L > 0))
    return fail(c, SWRT_ERR_ARG, "f must be nonzero and finite, L > 0");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_twiddles(c, (int)nx))) return rc;
  if ((rc = xka_nodes_for(c, nx))) return rc;
  const int n = (int)nx;
  const int64_t nn = nx * nx;
  const size_t zb = sizeof(double2) * nn;
  // Z: 4 spectra | T: 4 transforms | planes: 7 real (the 3 state planes first)
  if ((rc = ensure_scratch(c, 8 * zb + sizeof(double) * 7 * nn))) return rc;
  char* base = (char*)c->scratch;
  double2* Z = (double2*)base;
  double2* T = (double2*)(base + 4 * zb);
  double* planes = (double*)(base + 8 * zb);
  HIPCHK(c, hipMemcpyAsync(planes, state3, sizeof(double) * 3 * nn, hipMemcpyHostToDevice, c->stream));
  // g2k.m:8 fft2 of u, v, eta (raytrace_sw.m:26-28)
  hipLaunchKernelGGL(real_to_complex_kernel, dim3(nblocks(3 * nn, 256)), dim3(256), 0, c->stream, planes, Z, 3 * nn);
  HIPCHK(c, hipGetLastError());
  if ((rc = transform_2d(c, Z, T, n, 3, 0))) return rc;
  // projection + gradients + fulspec (raytrace_sw.m:25-41), then 4 inverse transforms
  hipLaunchKernelGGL(rsw_spectra_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, T, n, f, Cg * Cg,
                     (2.0 * M_PI) / L, Z);
  HIPCHK(c, hipGetLastError());
  if ((rc = inverse_2d(c, Z, T, n, 4))) return rc;
  hipLaunchKernelGGL(rsw_unpack_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, T, nn, planes);
  HIPCHK(c, hipGetLastError());
  if ((rc = xka_pack(c, planes, nx))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->xka_dx = L / (double)nx;
  c->xka_dy = L / (double)nx;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_xka_get_fields(swrt_ctx* c, double* fields7_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!fields7_out) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  if (!c->xka_nodes) return fail(c, SWRT_ERR_STATE, "call swrt_xka_set_fields or swrt_xka_set_rsw first");
  HIPCHK(c, hipSetDevice(c->device));
  const int64_t nx = c->xka_nx, nn = nx * nx;
  int rc;
  if ((rc = ensure_scratch(c, sizeof(double) * 7 * nn))) return rc;
  hipLaunchKernelGGL(unpack_xka_kernel, dim3(nblocks(nn, 256)), dim3(256), 0, c->stream, c->xka_nodes, (int)nx,
                     (int)(nx + kPadTot), (double*)c->scratch);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(fields7_out, c->scratch, sizeof(double) * 7 * nn, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int64_t swrt_xka_grid(const swrt_ctx* c) { return c ? c->xka_nx : -1; }

int64_t swrt_field_grid(const swrt_ctx* c, int slot) {
  if (!c || slot < 0 || slot >= SWRT_MAX_SLOTS || !c->slot[slot].set) return -1;
  return c->slot[slot].nx;
}

int64_t swrt_qg_grid(const swrt_ctx* c, int* nlayers_out) {
  if (nlayers_out) *nlayers_out = (c && c->qg.init) ? c->qg.g.nl : 0;
  if (!c || !c->qg.init) return -1;
  return c->qg.g.n;
}

int swrt_xka_step(swrt_ctx* c, double* state5, int64_t n, double C0, double f, double dt, int64_t nsteps,
                  int64_t save_every, double* hist5) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!c->xka_nodes) return fail(c, SWRT_ERR_STATE, "call swrt_xka_set_fields first");
  if (n < 0 || nsteps < 0 || save_every < 0) return fail(c, SWRT_ERR_ARG, "negative size");
  if (n == 0 || nsteps == 0) return SWRT_OK;  // nothing to advance: state5 unchanged, no frames
  if (!state5) return fail(c, SWRT_ERR_ARG, "state is NULL");
  if (hist5 && save_every > 0 && nsteps % save_every)
    return fail(c, SWRT_ERR_ARG, "nsteps must be a multiple of save_every");
  HIPCHK(c, hipSetDevice(c->device));
  if (n > c->xka_cap) {
    for (void** p : {(void**)&c->xka_state, (void**)&c->xka_state2, (void**)&c->xka_keys, (void**)&c->xka_src,
                     (void**)&c->xka_src2, (void**)&c->xka_perm2}) {
      if (*p) (void)hipFree(*p);
      *p = nullptr;
    }
    c->xka_cap = 0;
    HIPCHK(c, hipMalloc(&c->xka_state, sizeof(double) * 5 * n));
    HIPCHK(c, hipMalloc(&c->xka_state2, sizeof(double) * 5 * n));
    HIPCHK(c, hipMalloc(&c->xka_keys, sizeof(int) * n));
    HIPCHK(c, hipMalloc(&c->xka_src, sizeof(int) * n));
    HIPCHK(c, hipMalloc(&c->xka_src2, sizeof(int) * n));
    HIPCHK(c, hipMalloc(&c->xka_perm2, sizeof(int) * n));
    c->xka_cap = n;
  }
  if (!c->xka_bins) HIPCHK(c, hipMalloc(&c->xka_bins, sizeof(int) * (3 * kMaxBins + 1)));
  const int64_t frames = (hist5 && save_every > 0) ? nsteps / save_every : 0;
  if (frames * 5 * n > c->xka_hcap) {
    if (c->xka_hist) (void)hipFree(c->xka_hist);
    c->xka_hist = nullptr;
    c->xka_hcap = 0;
    HIPCHK(c, hipMalloc(&c->xka_hist, sizeof(double) * frames * 5 * n));
    c->xka_hcap = frames * 5 * n;
  }
  HIPCHK(c, hipMemcpyAsync(c->xka_state, state5, sizeof(double) * 5 * n, hipMemcpyHostToDevice, c->stream));
  XkaArgs a;
  a.nodes = c->xka_nodes;
  a.nx = (int)c->xka_nx;
  a.npad = (int)(c->xka_nx + kPadTot);
  a.dx = c->xka_dx;
  a.dy = c->xka_dy;
  a.inv_dx = 1.0 / a.dx;
  a.inv_dy = 1.0 / a.dy;
  a.px = a.py = (double)c->xka_nx;
  a.inv_px = a.inv_py = 1.0 / (double)c->xka_nx;
  a.C0sq = C0 * C0;
  a.f = f;
  a.f2 = f * f;
  a.dt = dt;
  a.bump = 1e-13;  // ray_trace_sw/interpolate.m:13
  a.st = c->xka_state;
  a.n = n;
  a.save_every = save_every > 0 ? save_every : 1;
  a.hist = frames ? c->xka_hist : nullptr;
  a.perm = nullptr;
  a.st_in = a.st;
  a.src = nullptr;
  a.perm_out = nullptr;
  // larger ensembles: step the packets in spatially binned order (8 x 8-cell
  // tiles, counting sort by index) with the LDS-tiled kernel (one workgroup
  // per tile, xka_tile_kernel), re-binned every rebin_every steps (the
  // context's locality setting) so the packets stay inside their tile's
  // window; the permutation to the caller's order is composed across
  // re-binnings and history frames are written through it
  const bool binned = n >= 4096 && c->rebin_every > 0;
  BinGeom g;
  g.dx = a.dx; g.px = a.px; g.py = a.py; g.inv_px = a.inv_px; g.inv_py = a.inv_py; g.inv_dx = a.inv_dx;
  g.nx = a.nx;
  g.tile = 8;
  while ((a.nx + g.tile - 1) / g.tile > 64) g.tile *= 2;
  g.ntx = (a.nx + g.tile - 1) / g.tile;
  const int nbins = g.ntx * g.ntx;
  const bool tiled = binned && a.nx % g.tile == 0 && g.ntx >= 2 && (g.tile == 8 || g.tile == 16);
  const unsigned bgrid = nblocks(n, 256 * kBinPerThread);
  // Binning is index-only: the scatter writes the source slot of every binned
  // slot and the launch that follows reads its packets through it into the
  // other state buffer, composing the permutation to the caller's order
  double* cur = c->xka_state;   // the state the next launch reads
  double* other = c->xka_state2;
  int* perm = nullptr;          // cur's slot -> caller's packet (nullptr: identity)
  int* perm_other = c->xka_perm2;
  const int* src = nullptr;     // pending re-binning (cur's slots, binned order)
  auto rebin_xka = [&]() -> int {
    HIPCHK(c, hipMemsetAsync(c->xka_bins, 0, sizeof(int) * nbins, c->stream));
    hipLaunchKernelGGL(bin_count_kernel, dim3(bgrid), dim3(256), sizeof(int) * nbins, c->stream, g, cur, n, nbins,
                       c->xka_keys, c->xka_bins);
    hipLaunchKernelGGL(bin_scan_kernel, dim3(1), dim3(1024), 0, c->stream, c->xka_bins, nbins,
                       c->xka_bins + kMaxBins, c->xka_bins + 2 * kMaxBins, n, c->dev_err_d, nullptr,
                       kTileThreads);
    hipLaunchKernelGGL(bin_scatter_kernel<true>, dim3(bgrid), dim3(256), 2 * sizeof(int) * nbins, c->stream,
                       cur, cur, nullptr, c->xka_keys, n, nbins, c->xka_bins + kMaxBins, nullptr, nullptr, nullptr,
                       c->xka_src2);
    HIPCHK(c, hipGetLastError());
    src = c->xka_src2;
    return SWRT_OK;
  };
  int rc;
  if (binned && (rc = rebin_xka())) return rc;
  const int64_t per_launch = tiled ? std::min<int64_t>(kMaxStepsPerLaunch, c->rebin_every) : kMaxStepsPerLaunch;
  for (int64_t s0 = 0; s0 < nsteps; s0 += per_launch) {
    if (tiled && s0 > 0 && (rc = rebin_xka())) return rc;
    a.st_in = cur;
    a.src = src;
    a.perm = perm;
    if (src) {  // out of place: into the other buffer, with the composed permutation
      int* pout = perm == nullptr ? c->xka_src : perm_other;
      a.st = other;
      a.perm_out = pout;
    } else {
      a.st = cur;
      a.perm_out = nullptr;
    }
    a.nsteps = (int)std::min<int64_t>(per_launch, nsteps - s0);
    a.step0 = s0;
    if (tiled && g.tile == 8)
      hipLaunchKernelGGL((xka_tile_kernel<8, kXkaMargin, 256>), dim3(nbins), dim3(256), 0, c->stream, a,
                         (const int*)(c->xka_bins + 2 * kMaxBins), g.ntx);
    else if (tiled)
      hipLaunchKernelGGL((xka_tile_kernel<16, kXkaMargin, 256>), dim3(nbins), dim3(256), 0, c->stream, a,
                         (const int*)(c->xka_bins + 2 * kMaxBins), g.ntx);
    else
      hipLaunchKernelGGL(xka_kernel, dim3(nblocks(n, 256)), dim3(256), 0, c->stream, a);
    HIPCHK(c, hipGetLastError());
    if (src) {
      std::swap(cur, other);
      if (perm == nullptr) {
        perm = c->xka_src;
      } else {
        std::swap(perm, perm_other);
      }
      src = nullptr;
    }
  }
  if (binned) {
    hipLaunchKernelGGL(xka_scatter_back_kernel, dim3(nblocks(n, 256)), dim3(256), 0, c->stream, cur, perm, n, other);
    HIPCHK(c, hipGetLastError());
    cur = other;
  }
  HIPCHK(c, hipMemcpyAsync(state5, cur, sizeof(double) * 5 * n, hipMemcpyDeviceToHost, c->stream));
  if (frames)
    HIPCHK(c, hipMemcpyAsync(hist5, c->xka_hist, sizeof(double) * frames * 5 * n, hipMemcpyDeviceToHost,
                             c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_spectral_set_modes(swrt_ctx* c, const double* C, int64_t nkx, int64_t nky, double kx0, double ky0,
                            double s) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!C) return fail(c, SWRT_ERR_ARG, "C is NULL");
  if (nkx <= 0 || nky <= 0 || nkx * nky > (int64_t)1 << 28) return fail(c, SWRT_ERR_ARG, "bad mode grid");
  HIPCHK(c, hipSetDevice(c->device));
  if (nkx * nky > c->mode_cap) {
    if (c->modes) (void)hipFree(c->modes);
    c->modes = nullptr;
    c->mode_cap = 0;
    HIPCHK(c, hipMalloc(&c->modes, sizeof(double2) * nkx * nky));
    c->mode_cap = nkx * nky;
  }
  if (nky > c->rows_cap) {
    if (c->mode_rows) (void)hipFree(c->mode_rows);
    c->mode_rows = nullptr;
    c->rows_cap = 0;
    HIPCHK(c, hipMalloc(&c->mode_rows, sizeof(int2) * nky));
    c->rows_cap = nky;
  }
  // nonzero span of each row (the kernel skips zero head/tail segments)
  std::vector<int2> rows(nky);
  for (int64_t j = 0; j < nky; ++j) {
    int lo = 0, hi = (int)nkx;
    while (lo < hi && C[2 * (j * nkx + lo)] == 0.0 && C[2 * (j * nkx + lo) + 1] == 0.0) ++lo;
    while (hi > lo && C[2 * (j * nkx + hi - 1)] == 0.0 && C[2 * (j * nkx + hi - 1) + 1] == 0.0) --hi;
    rows[j] = make_int2(lo, hi);
  }
  // fp32 packed-pair copy of the spans (ModeGrid::Cf): groups of 4 modes as
  // two float4 {re_m, re_m+1, im_m, im_m+1}, zero past the span end
  std::vector<int> frow(nky);
  int64_t nf = 0;
  for (int64_t j = 0; j < nky; ++j) {
    frow[j] = (int)nf;
    nf += 2 * (((int64_t)rows[j].y - rows[j].x + kSpecChains - 1) / kSpecChains);
  }
  // + zero slots: the LDS stream's chunk prefetch reads up to two chunks past
  // the last group (SpecStream; 16-B slots in both precisions)
  std::vector<float4> cf((size_t)(nf + 2 * kSpecChunk), make_float4(0.f, 0.f, 0.f, 0.f));
  for (int64_t j = 0; j < nky; ++j) {
    for (int m = rows[j].x; m < rows[j].y; ++m) {
      const int64_t r = m - rows[j].x, q = frow[j] + 2 * (r / kSpecChains) + (r % kSpecChains) / 2;
      const int h = (int)(r & 1);
      float* v = reinterpret_cast<float*>(&cf[q]);
      v[h] = (float)C[2 * (j * nkx + m)];
      v[2 + h] = (float)C[2 * (j * nkx + m) + 1];
    }
  }
  // the same groups in fp64: kSpecChains double2 per group (Cd_row = 2 * Cf_row)
  std::vector<double2> cd((size_t)(2 * nf + 2 * kSpecChunk), make_double2(0.0, 0.0));
  std::vector<int> drow(nky);
  for (int64_t j = 0; j < nky; ++j) {
    drow[j] = 2 * frow[j];
    for (int m = rows[j].x; m < rows[j].y; ++m)
      cd[(size_t)drow[j] + (m - rows[j].x)] = make_double2(C[2 * (j * nkx + m)], C[2 * (j * nkx + m) + 1]);
  }
  if ((int64_t)cd.size() > c->modes_f_cap) {
    for (void* p : {(void*)c->modes_f, (void*)c->modes_d})
      if (p) (void)hipFree(p);
    c->modes_f = nullptr;
    c->modes_d = nullptr;
    c->modes_f_cap = 0;
    HIPCHK(c, hipMalloc(&c->modes_f, sizeof(float4) * cd.size()));
    HIPCHK(c, hipMalloc(&c->modes_d, sizeof(double2) * cd.size()));
    c->modes_f_cap = (int64_t)cd.size();
  }
  if (nky > c->modes_f_rcap) {
    for (void* p : {(void*)c->modes_f_row, (void*)c->modes_d_row})
      if (p) (void)hipFree(p);
    c->modes_f_row = nullptr;
    c->modes_d_row = nullptr;
    c->modes_f_rcap = 0;
    HIPCHK(c, hipMalloc(&c->modes_f_row, sizeof(int) * nky));
    HIPCHK(c, hipMalloc(&c->modes_d_row, sizeof(int) * nky));
    c->modes_f_rcap = nky;
  }
  HIPCHK(c, hipMemcpyAsync(c->modes_d, cd.data(), sizeof(double2) * cd.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->modes_d_row, drow.data(), sizeof(int) * nky, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->modes, C, sizeof(double2) * nkx * nky, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->mode_rows, rows.data(), sizeof(int2) * nky, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->modes_f, cf.data(), sizeof(float4) * cf.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->modes_f_row, frow.data(), sizeof(int) * nky, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->mg.Cd = c->modes_d;
  c->mg.Cd_row = c->modes_d_row;
  c->mg.Cf = c->modes_f;
  c->mg.Cf_row = c->modes_f_row;
  int64_t active = 0;
  for (auto& r : rows) active += r.y - r.x;
  c->mode_active = active;
  c->mg.rows = c->mode_rows;
  c->mg.C = c->modes;
  c->mg.nkx = (int)nkx;
  c->mg.nky = (int)nky;
  c->mg.kx0 = kx0;
  c->mg.ky0 = ky0;
  c->mg.s = s;
  c->modes_set = true;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_spectral_eval(swrt_ctx* c, const double* x, const double* y, int64_t n, int precision, double* out6) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!c->modes_set) return fail(c, SWRT_ERR_STATE, "call swrt_spectral_set_modes first");
  if (precision != 64 && precision != 32) return fail(c, SWRT_ERR_ARG, "precision must be 64 or 32");
  if (n < 0) return fail(c, SWRT_ERR_ARG, "n < 0");
  if (n == 0) return SWRT_OK;
  if (!x || !y || !out6) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_scratch(c, sizeof(double) * 8 * n))) return rc;
  double* dxp = (double*)c->scratch;
  double* dyp = dxp + n;
  double* dout = dyp + n;
  HIPCHK(c, hipMemcpyAsync(dxp, x, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dyp, y, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  if (precision == 64)
    hipLaunchKernelGGL(spectral_eval_kernel<double>, dim3(nblocks(n, kSpecThreads)), dim3(kSpecThreads), 0,
                       c->stream, c->mg, dxp, dyp, n, dout);
  else
    hipLaunchKernelGGL(spectral_eval_kernel<float>, dim3(nblocks(n, kSpecThreads)), dim3(kSpecThreads), 0,
                       c->stream, c->mg, dxp, dyp, n, dout);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out6, dout, sizeof(double) * 6 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_spectral_leapfrog(swrt_ctx* c, double* x, double* k, int64_t n, double dt, int64_t nsteps, double f,
                           double gH, int precision) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (!c->modes_set) return fail(c, SWRT_ERR_STATE, "call swrt_spectral_set_modes first");
  if (precision != 64 && precision != 32) return fail(c, SWRT_ERR_ARG, "precision must be 64 or 32");
  if (n < 0 || nsteps < 0) return fail(c, SWRT_ERR_ARG, "negative size");
  if (n == 0 || nsteps == 0) return SWRT_OK;
  if (!x || !k) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_scratch(c, sizeof(double) * 4 * n))) return rc;
  double* dxp = (double*)c->scratch;
  double* dkp = dxp + 2 * n;
  HIPCHK(c, hipMemcpyAsync(dxp, x, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dkp, k, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream));
  for (int64_t s0 = 0; s0 < nsteps; s0 += kMaxStepsPerLaunch) {
    const int ns = (int)std::min<int64_t>(kMaxStepsPerLaunch, nsteps - s0);
    if (precision == 64)
      hipLaunchKernelGGL(spectral_leapfrog_kernel<double>, dim3(nblocks(n, kSpecThreads)), dim3(kSpecThreads),
                         0, c->stream, c->mg, dxp, dkp, n, dt, ns, f * f, gH);
    else
      hipLaunchKernelGGL(spectral_leapfrog_kernel<float>, dim3(nblocks(n, kSpecThreads)), dim3(kSpecThreads),
                         0, c->stream, c->mg, dxp, dkp, n, dt, ns, f * f, gH);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipMemcpyAsync(x, dxp, sizeof(double) * 2 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(k, dkp, sizeof(double) * 2 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_omega_histogram(swrt_ctx* c, double f, double Cg, const double* edges, int64_t nbins,
                         int64_t* counts_inout, double* mean_omega_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (nbins <= 0 || nbins > kMaxHistBins) return fail(c, SWRT_ERR_ARG, "nbins must be 1..4096");
  if (!edges || !counts_inout) return fail(c, SWRT_ERR_ARG, "NULL buffer");
  for (int64_t i = 0; i < nbins; ++i)
    if (!(edges[i] < edges[i + 1])) return fail(c, SWRT_ERR_ARG, "edges must increase");
  HIPCHK(c, hipSetDevice(c->device));
  const int nblk = 1024;
  const size_t bytes = sizeof(double) * (nbins + 1) + sizeof(unsigned long long) * nbins +
                       sizeof(double) * (nblk + 1);
  int rc;
  if ((rc = ensure_scratch(c, bytes))) return rc;
  double* dedges = (double*)c->scratch;
  unsigned long long* dcounts = (unsigned long long*)(dedges + nbins + 1);
  double* partial = (double*)(dcounts + nbins);
  HIPCHK(c, hipMemcpyAsync(dedges, edges, sizeof(double) * (nbins + 1), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(dcounts, 0, sizeof(unsigned long long) * nbins, c->stream));
  double mean = 0.0;
  if (c->n > 0) {
    hipLaunchKernelGGL(omega_hist_kernel, dim3(nblk), dim3(kHistThreads), 0, c->stream, c->dk, c->n, f * f,
                       Cg * Cg, dedges, (int)nbins, dcounts, partial);
    HIPCHK(c, hipGetLastError());
    hipLaunchKernelGGL(omega_sum_kernel, dim3(1), dim3(64), 0, c->stream, partial, nblk, partial + nblk);
    HIPCHK(c, hipGetLastError());
  }
  std::vector<unsigned long long> hc(nbins, 0ull);
  double sum = 0.0;
  HIPCHK(c, hipMemcpyAsync(hc.data(), dcounts, sizeof(unsigned long long) * nbins, hipMemcpyDeviceToHost, c->stream));
  if (c->n > 0)
    HIPCHK(c, hipMemcpyAsync(&sum, partial + nblk, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int64_t i = 0; i < nbins; ++i) counts_inout[i] += (int64_t)hc[i];
  if (c->n > 0) mean = sum / (double)c->n;
  if (mean_omega_out) *mean_omega_out = mean;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_check_arith(swrt_ctx* c, int64_t n, uint64_t seed, int64_t* mismatches3) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  if (n <= 0 || !mismatches3) return fail(c, SWRT_ERR_ARG, "n must be > 0, mismatches3 non-NULL");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_scratch(c, 3 * sizeof(unsigned long long)))) return rc;
  unsigned long long* d = (unsigned long long*)c->scratch;
  HIPCHK(c, hipMemsetAsync(d, 0, 3 * sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(check_arith_kernel, dim3(nblocks(n, 256)), dim3(256), 0, c->stream, n, seed, d);
  HIPCHK(c, hipGetLastError());
  unsigned long long h[3];
  HIPCHK(c, hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int q = 0; q < 3; ++q) mismatches3[q] = (int64_t)h[q];
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_synchronize(swrt_ctx* c) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = sync_sx(c)) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipStreamSynchronize(c->qstream));
  if (c->hz.on) c->hz.sync_all();
  return dev_err_check(c);
}

int swrt_debug_set(swrt_ctx* c, int key, int64_t value) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (int rc = chain_drop(c)) return rc;
  switch (key) {
    case SWRT_DEBUG_HAZARD_CHECK:
      if (value != 0 && value != 1) return fail(c, SWRT_ERR_ARG, "hazard check must be 0 or 1");
      if (value && !c->hz.on) {
        // start from a quiet device: nothing queued before is tracked
        if (int rc = swrt_synchronize(c)) return rc;
        c->hz = HazardChecker();
      }
      c->hz.on = value != 0;
      if (!c->hz.on) c->debug_share_skew = false;
      return SWRT_OK;
    case SWRT_DEBUG_SPIN_US:
      if (value < 0 || value > 100000) return fail(c, SWRT_ERR_ARG, "spin must be 0..100000 us");
      c->debug_spin_us = (int)value;
      return SWRT_OK;
    case SWRT_DEBUG_LEGACY_PARK:
      if (value != 0 && value != 1) return fail(c, SWRT_ERR_ARG, "legacy park must be 0 or 1");
      c->debug_legacy_park = value != 0;
      return SWRT_OK;
    case SWRT_DEBUG_SHARE_SKEW:
      if (value != 0 && value != 1) return fail(c, SWRT_ERR_ARG, "share skew must be 0 or 1");
      if (value && !c->hz.on) return fail(c, SWRT_ERR_STATE, "the skewed share runs only under the hazard checker");
      c->debug_share_skew = value != 0;
      return SWRT_OK;
    case SWRT_DEBUG_CORRUPT_COUNT:
      if (value < -1000000 || value > 1000000) return fail(c, SWRT_ERR_ARG, "count corruption out of range");
      c->debug_corrupt_count = (int)value;
      c->keys_fresh = false;
      c->bin_valid = false;  // the next call re-bins (and meets the corrupted count)
      return SWRT_OK;
    case SWRT_DEBUG_QG_UPDATE_COLS:
      if (value != 0 && value != 1) return fail(c, SWRT_ERR_ARG, "QG update/column-pass fusion must be 0 or 1");
      if (c->qg.spec) return fail(c, SWRT_ERR_STATE, "a speculative QG step is pending (swrt_qg_resolve first)");
      c->qg_update_cols = (int)value;
      c->qg.post_valid = false;
      return SWRT_OK;
    case SWRT_DEBUG_QG_JFUSE:
      if (value != 0 && value != 1) return fail(c, SWRT_ERR_ARG, "QG column/Jacobian fusion must be 0 or 1");
      if (c->qg.spec) return fail(c, SWRT_ERR_STATE, "a speculative QG step is pending (swrt_qg_resolve first)");
      c->qg_jfuse = (int)value;
      c->qg.post_valid = false;
      c->qg.post_inv_valid = false;
      return SWRT_OK;
    default:
      return fail(c, SWRT_ERR_ARG, "unknown debug key");
  }
}

int swrt_debug_get(swrt_ctx* c, int key, int64_t* value_out) {
  if (!c || !value_out) return SWRT_ERR_ARG;
  switch (key) {
    case SWRT_DEBUG_HAZARD_CHECK: *value_out = c->hz.on ? 1 : 0; return SWRT_OK;
    case SWRT_DEBUG_SPIN_US: *value_out = c->debug_spin_us; return SWRT_OK;
    case SWRT_DEBUG_LEGACY_PARK: *value_out = c->debug_legacy_park ? 1 : 0; return SWRT_OK;
    case SWRT_DEBUG_HAZARD_CHECKS: *value_out = c->hz.checks; return SWRT_OK;
    case SWRT_DEBUG_QG_JFUSE: *value_out = c->qg_jfuse; return SWRT_OK;
    case SWRT_DEBUG_SHARE_SKEW: *value_out = c->debug_share_skew ? 1 : 0; return SWRT_OK;
    case SWRT_DEBUG_CORRUPT_COUNT: *value_out = c->debug_corrupt_count; return SWRT_OK;
    case SWRT_DEBUG_QG_UPDATE_COLS: *value_out = c->qg_update_cols; return SWRT_OK;
    case SWRT_DEBUG_ODE23_CHAINED: *value_out = c->o_chain.taken; return SWRT_OK;
    case SWRT_DEBUG_ODE23_FIRST_TAKEN: *value_out = c->o23_first_taken; return SWRT_OK;
    case SWRT_DEBUG_ODE23_GUESSES_TAKEN: *value_out = c->o23_guesses_taken; return SWRT_OK;
    case SWRT_DEBUG_ODE23_SPLIT_RUNS: *value_out = c->o23_split_runs; return SWRT_OK;
    case SWRT_DEBUG_ODE23_FIRST_CHAINED: *value_out = c->o_chain.first_taken; return SWRT_OK;
    default: return fail(c, SWRT_ERR_ARG, "unknown debug key");
  }
}

int swrt_qg_set_fused(swrt_ctx* c, int on) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (c->qg.spec) return fail(c, SWRT_ERR_STATE, "a speculative QG step is pending (swrt_qg_resolve first)");
  if (on != 0 && on != 1) return fail(c, SWRT_ERR_ARG, "on must be 0 or 1");
  int rc = swrt_synchronize(c);
  if (rc) return rc;
  c->qg_fused = on != 0;
  c->qg.post_valid = false;
  c->qg.post_inv_valid = false;
  return SWRT_OK;
}

int swrt_qg_set_stream(swrt_ctx* c, int separate) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (c->qg.spec) return fail(c, SWRT_ERR_STATE, "a speculative QG step is pending (swrt_qg_resolve first)");
  if (separate != 0 && separate != 1) return fail(c, SWRT_ERR_ARG, "separate must be 0 or 1");
  int rc = swrt_synchronize(c);
  if (rc) return rc;
  c->qg_sep = separate != 0;
  return SWRT_OK;
}

int swrt_get_stream(swrt_ctx* c, void** out) {
  if (!c || !out) return SWRT_ERR_ARG;
  if (int rc = join_b(c)) return rc;  // work queued on it by the caller sees every packet
  c->s0_dirty = true;                   // ... and the next split launch follows that work
  *out = (void*)c->stream;
  return SWRT_OK;
}

int swrt_kernel_time(swrt_ctx* c, int reset, double* total_ms, int64_t* launches) {
  if (!c) return SWRT_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  for (hipStream_t s : c->sx)  // stop events of split launches
    if (s) HIPCHK(c, hipStreamSynchronize(s));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  double tot = c->timing.folded_ms;
  for (size_t i = 0; i + 1 < c->timing.used; i += 2) {
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->timing.ev[i], c->timing.ev[i + 1]));
    tot += ms;
  }
  HIPCHK_RC(dev_err_check(c));
  if (total_ms) *total_ms = tot;
  if (launches) *launches = c->timing.folded_n + (int64_t)(c->timing.used / 2);
  if (reset) {
    c->timing.used = 0;
    c->timing.folded_ms = 0.0;
    c->timing.folded_n = 0;
  }
  return SWRT_OK;
}

int swrt_clock_stamp(swrt_ctx* c, int which) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN  // join_b: the stamp follows every packet launch queued on any packet stream
  if (which != 0 && which != 1) return fail(c, SWRT_ERR_ARG, "which must be 0 (start) or 1 (end)");
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->clk) HIPCHK(c, hipMalloc(&c->clk, sizeof(unsigned long long) * 2 * kClockWaves * 3));
  hipLaunchKernelGGL(clock_stamp_kernel, dim3(kClockWaves), dim3(64), 0, c->stream, c->clk + which * kClockWaves * 3);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_clock_ghz(swrt_ctx* c, double* ghz_out, double* spread_out) {
  if (!c || !ghz_out) return SWRT_ERR_ARG;
  if (!c->clk) return fail(c, SWRT_ERR_STATE, "no clock stamps (swrt_clock_stamp 0 and 1 first)");
  GUARD_BEGIN_KEEP_CHAIN
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<uint64_t> h(2 * kClockWaves * 3);
  HIPCHK(c, hipMemcpyAsync(h.data(), c->clk, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hz_synced(c);
  // the pairing and median (swrt_clock.cpp, host-only, tested on synthetic stamps)
  const int rc = swrt_clock_ghz_stamps(h.data(), kClockWaves, kRealTimeHz, ghz_out, spread_out);
  if (rc == SWRT_ERR_STATE) return fail(c, rc, "no CU with both a start and an end stamp");
  if (rc) return fail(c, rc, "swrt_clock_ghz_stamps");
  return SWRT_OK;
  GUARD_END(c)
}

// ---------------------------------------------------------------------------
// QG PDE stepper (swrt_qg.hpp)
// ---------------------------------------------------------------------------
int swrt_qg_init(swrt_ctx* c, const swrt_qg_params* p, int64_t nx, const double* qk_in) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  if (!p || !qk_in) return fail(c, SWRT_ERR_ARG, "NULL argument");
  if (p->nlayers != 1 && p->nlayers != 2) return fail(c, SWRT_ERR_ARG, "nlayers must be 1 or 2");
  if (nx < 8 || nx > 4096 || !is_pow2(nx)) return fail(c, SWRT_ERR_ARG, "nx must be a power of two, 8..4096");
  if (!(p->L > 0)) return fail(c, SWRT_ERR_ARG, "L must be > 0");
  HIPCHK(c, hipSetDevice(c->device));
  QGState& q = c->qg;
  for (void* ptr : {(void*)q.qk, (void*)q.qk_prev, (void*)q.Qm1, (void*)q.Qm2, (void*)q.E1, (void*)q.E2,
                    (void*)q.Z, (void*)q.T, (void*)q.dmax, (void*)q.PZ, (void*)q.PT, (void*)q.qk_spare,
                    (void*)q.Qm1_spare, (void*)q.Qm2_spare})
    if (ptr) (void)hipFree(ptr);
  if (q.hmax) (void)hipHostFree(q.hmax);
  if (q.ev) (void)hipEventDestroy(q.ev);
  if (q.ev_b) (void)hipEventDestroy(q.ev_b);
  q = QGState{};
  const int n = (int)nx, kmax = n / 2 - 1;
  q.nhalf = (int64_t)(2 * kmax + 1) * (kmax + 1);
  q.nn = nx * nx;
  QGDev& g = q.g;
  g.n = n;
  g.nl = p->nlayers;
  g.kscale = 2.0 * 3.14159265358979323846 / p->L;
  if (p->nlayers == 1) g.kscale = 1.0;  // qgsw_raytrace.m:13-20: L = 2*pi, integer k
  g.dx = p->L / (double)n;
  g.K_d2 = p->K_d2;
  g.beta = p->beta;
  g.r_drag = p->r_drag;
  g.force_strength = p->force_strength;
  g.f = p->f;
  g.Cg = p->Cg;
  g.filter = p->filter;
  g.shear = p->nlayers == 2 ? p->shear : 0.0;
  g.nu = p->nu;
  g.hyper = p->hyper_order;
  g.r = p->r;
  const size_t hb = sizeof(double2) * q.nhalf * g.nl;
  const size_t zb = sizeof(double2) * q.nn * std::max(2 * g.nl, 3);
  HIPCHK(c, hipMalloc(&q.qk, hb));
  HIPCHK(c, hipMalloc(&q.qk_prev, hb));
  HIPCHK(c, hipMalloc(&q.Qm1, hb));
  HIPCHK(c, hipMalloc(&q.Qm2, hb));
  HIPCHK(c, hipMalloc(&q.Z, zb));
  HIPCHK(c, hipMalloc(&q.T, zb));
  HIPCHK(c, hipMalloc(&q.dmax, sizeof(unsigned long long)));
  HIPCHK(c, hipHostMalloc(&q.hmax, 2 * sizeof(double)));
  HIPCHK(c, hipEventCreateWithFlags(&q.ev, hipEventDisableTiming));
  HIPCHK(c, hipEventCreateWithFlags(&q.ev_b, hipEventDisableTiming));
  if (g.nl == 2) {
    HIPCHK(c, hipMalloc(&q.E1, sizeof(double2) * 4 * q.nhalf));
    HIPCHK(c, hipMalloc(&q.E2, sizeof(double2) * 4 * q.nhalf));
  }
  // host column-major (kx fastest) -> device ky-fastest, via qk_prev as staging
  HIPCHK(c, hipMemcpyAsync(q.qk_prev, qk_in, hb, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(halfplane_relayout_kernel, dim3(nblocks(q.nhalf * g.nl, 256)), dim3(256), 0, c->stream,
                     q.qk_prev, q.qk, 2 * kmax + 1, kmax + 1, 1, g.nl);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemsetAsync(q.Qm1, 0, hb, c->stream));
  HIPCHK(c, hipMemsetAsync(q.Qm2, 0, hb, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  q.init = true;
  if (c->qg_sep) {
    // from here on packet launches mark their slot use; everything queued on
    // the context stream so far is marked by one record per slot
    for (Slot& sl : c->slot)
      if (sl.nodes && hipEventRecord(sl.uev, on_qg.saved) == hipSuccess) {
        sl.uref = sl.uev;
        sl.upend = true;
      }
  }
  return SWRT_OK;
  GUARD_END(c)
}

namespace {
// fused g2k crop + AB3 update from the forward-transformed Jacobian F into
// qk_prev (out of place: the new qk goes to the other buffer, the old one
// becomes prev_qk)
// The AB3 update of the current qk into qk_out, the tendency history into
// Qm1_out/Qm2_out (the committed buffers, or a speculative step's spares).
int qg_update_launch(swrt_ctx* c, double dt, int abstep, const double2* F, double2* qk_out, double2* Qm1_out,
                     double2* Qm2_out) {
  QGState& q = c->qg;
  if (q.g.nl == 2)
    hipLaunchKernelGGL(qg_update_kernel<2>, dim3(nblocks(q.nhalf, 256)), dim3(256), 0, c->stream, F, q.g, dt,
                       abstep, q.E1, q.E2, (const double2*)q.qk, qk_out, (const double2*)q.Qm1,
                       (const double2*)q.Qm2, Qm1_out, Qm2_out);
  else
    hipLaunchKernelGGL(qg_update_kernel<1>, dim3(nblocks(q.nhalf, 256)), dim3(256), 0, c->stream, F, q.g, dt,
                       abstep, q.E1, q.E2, (const double2*)q.qk, qk_out, (const double2*)q.Qm1,
                       (const double2*)q.Qm2, Qm1_out, Qm2_out);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}

// Fused mode: J's last forward pass and the update in one launch from J after
// its first pass (Zr); the new tendency goes to Qn_out only (the caller
// renames the history buffers).
int qg_update_cols_launch(swrt_ctx* c, double dt, int abstep, const double2* Zr, double2* qk_out,
                          double2* Qn_out) {
  QGState& q = c->qg;
  const int n = q.g.n;
  int logn = 0;
  while ((1 << logn) < n) ++logn;
  const size_t lds = sizeof(double2) * 2 * (size_t)(n + 1);
  if (q.g.nl == 2)
    hipLaunchKernelGGL(qg_update_cols_kernel<2>, dim3((unsigned)(n / 2)), dim3((unsigned)(n / 2)), lds, c->stream,
                       Zr, q.g, logn, (const double2*)c->tw, dt, abstep, q.E1, q.E2, (const double2*)q.qk, qk_out,
                       (const double2*)q.Qm1, (const double2*)q.Qm2, Qn_out);
  else
    hipLaunchKernelGGL(qg_update_cols_kernel<1>, dim3((unsigned)(n / 2)), dim3((unsigned)(n / 2)), lds, c->stream,
                       Zr, q.g, logn, (const double2*)c->tw, dt, abstep, q.E1, q.E2, (const double2*)q.qk, qk_out,
                       (const double2*)q.Qm1, (const double2*)q.Qm2, Qn_out);
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}

// The kernel sequence of one QG step (update of qgsw_raytrace.m:270-286 /
// qg2layersw_raytrace.m:309-323 + the AB3 step): spectra -> inverse 2-D FFT ->
// Jacobian -> forward 2-D FFT -> fused g2k crop + AB3 update into qk_prev.
int qg_step_launches(swrt_ctx* c, double dt, int abstep) {
  QGState& q = c->qg;
  const int n = q.g.n, nl = q.g.nl;
  int rc;
  if (nl == 2)
    hipLaunchKernelGGL(qg_jac_spectra_kernel<2>, dim3(nblocks(q.nn, 256)), dim3(256), 0, c->stream, q.qk, q.g, q.Z);
  else
    hipLaunchKernelGGL(qg_jac_spectra_kernel<1>, dim3(nblocks(q.nn, 256)), dim3(256), 0, c->stream, q.qk, q.g, q.Z);
  HIPCHK(c, hipGetLastError());
  if ((rc = inverse_2d(c, q.Z, q.T, n, 2 * nl))) return rc;
  double2* Zj = q.Z;  // J1 + i J2, grid layout (x contiguous)
  hipLaunchKernelGGL(qg_jacobian_kernel, dim3(nblocks(q.nn, 256)), dim3(256), 0, c->stream, q.T, nl, q.nn, Zj);
  HIPCHK(c, hipGetLastError());
  if ((rc = transform_2d(c, Zj, q.T, n, 1, 0))) return rc;  // along x, then y: [ky + n*kx]
  return qg_update_launch(c, dt, abstep, q.T, q.qk_prev, q.Qm1, q.Qm2);
}

// Post-step transforms of the current qk (fused mode), see QGState::PZ.
// Every transform is the one the unfused calls make (same spectra kernels,
// same per-vector FFT), so results are bit-identical to them.  Two phases:
// the inverse transforms (all a snapshot needs) and the Jacobian + CFL max
// + forward transform of J (what the speed and the next step need), so a
// snapshot's pack — and the packet launch waiting for it — need not queue
// behind the second phase.
int qg_post_inverse(swrt_ctx* c) {
  QGState& q = c->qg;
  if (q.post_inv_valid && q.post_of == q.qk) return SWRT_OK;
  q.post_valid = false;
  q.post_of = q.qk;
  const int n = q.g.n, nl = q.g.nl;
  const int nb = 2 * nl + (nl - 1) + 3;  // Jacobian inputs | layer-1 u+iv | layer-0 grid_U (u+iv first)
  if (!q.PZ) {
    HIPCHK(c, hipMalloc(&q.PZ, sizeof(double2) * nb * q.nn));
    HIPCHK(c, hipMalloc(&q.PT, sizeof(double2) * nb * q.nn));
  }
  int rc;
  if ((rc = ensure_twiddles(c, n))) return rc;
  const dim3 grid((unsigned)nblocks(q.nn, 256)), block(256);
  // Jacobian inputs | layer-1 u+iv | swrt_qg_snapshot(which 0, layer 0)'s
  // grid_U spectra (grid_U.m inversion, ky-fastest half plane) — one launch
  double2* uv = q.PZ + 2 * nl * q.nn;
  if (nb * n / 4 <= 1024) {
    // spectra fused into the first inverse pass (qg_post_rows_kernel), then
    // the column pass — the same values as the three launches below
    int logn = 0;
    while ((1 << logn) < n) ++logn;
    const size_t lds = sizeof(double2) * nb * n;
    if (nl == 2)
      hipLaunchKernelGGL(qg_post_rows_split_kernel, dim3(2 * (unsigned)n), dim3(n), sizeof(double2) * 4 * n,
                         c->stream, (const double2*)q.qk, q.g, q.nhalf, logn, (const double2*)c->tw, q.PZ, q.dmax);
    else
      hipLaunchKernelGGL(qg_post_rows_kernel<1>, dim3((unsigned)n), dim3(nb * n / 4), lds, c->stream,
                         (const double2*)q.qk, q.g, q.nhalf, logn, (const double2*)c->tw, q.PZ, q.dmax);
    HIPCHK(c, hipGetLastError());
    // (not beside packets: its four-plane 512-lane workgroups then wait for
    // packet workgroups to retire — driver step +2 %, 8-GPU shard +10 %,
    // profiles/r04_qg_ab — where the separate column pass runs one plane per
    // 128-lane workgroup)
    if (nl == 2 && n % 8 == 0 && c->qg_jfuse == 1 && !(c->qg_sep && c->n > 0)) {
      // the column pass fused with the Jacobian, the CFL max and J's first
      // forward pass (swrt_fft.hpp): planes 0-4 stay on chip; J -> PT[0, nn)
      hipLaunchKernelGGL(fft_cols_jacobian2_kernel, dim3(2 * (unsigned)n), dim3(n), sizeof(double2) * 4 * (n + 1),
                         c->stream, (const double2*)q.PZ, q.PT, q.PT, n, logn, q.g.shear, q.dmax,
                         (const double2*)c->tw);
      q.post_jrows = true;
    } else {
      launch_fft<true>(c, q.PZ, q.PT, n, logn, nb * n, 1);
      q.post_jrows = false;
    }
    HIPCHK(c, hipGetLastError());
  } else {
    if (nl == 2)
      hipLaunchKernelGGL(qg_post_spectra_kernel<2>, grid, block, 0, c->stream, (const double2*)q.qk, q.g, q.nhalf,
                         q.PZ, uv, uv + q.nn, q.dmax);
    else
      hipLaunchKernelGGL(qg_post_spectra_kernel<1>, grid, block, 0, c->stream, (const double2*)q.qk, q.g, q.nhalf,
                         q.PZ, uv, uv, q.dmax);
    HIPCHK(c, hipGetLastError());
    if ((rc = inverse_2d(c, q.PZ, q.PT, n, nb))) return rc;
    q.post_jrows = false;
  }
  q.post_inv_valid = true;
  return SWRT_OK;
}

int qg_post(swrt_ctx* c) {
  QGState& q = c->qg;
  if (q.post_valid && q.post_of == q.qk) return SWRT_OK;
  int rc;
  if ((rc = qg_post_inverse(c))) return rc;
  const int n = q.g.n, nl = q.g.nl;
  const dim3 block(256);
  // Jacobian and the CFL speed over every layer's u + i v (layer 1, then
  // layer 0: contiguous); the spectrum of J then lands in PT[0, nn)
  const double2* uvT = q.PT + 2 * nl * q.nn;
  q.Fj = q.PT;
  q.Fj_rows = false;
  // J's last forward pass is left to the update (qg_update_cols_kernel) —
  // not beside packets: PDE alone -7 %, but the driver step +1.3 % with the
  // QG stream beside packet launches (profiles/r04_update_cols), as for
  // fft_cols_jacobian2_kernel
  const bool cols =
      n >= 16 && c->qg_update_cols == 1 && !(c->qg_sep && c->n > 0);
  if (q.post_jrows) {
    // J's first pass came with the inverse column pass: its second pass only
    if (cols) {
      q.Fj_rows = true;  // J's first pass is in PT[0, nn)
    } else {
      int logn = 0;
      while ((1 << logn) < n) ++logn;
      launch_fft<true>(c, q.PT, q.PZ, n, logn, n, 0);
      HIPCHK(c, hipGetLastError());
      q.Fj = q.PZ;
    }
  } else if (n <= 1024) {
    // J computed in the load of the forward transform's first pass (same
    // values, same per-vector FFT as the separate kernel + transform_2d)
    int logn = 0;
    while ((1 << logn) < n) ++logn;
    const int R = fft_group(c, n, n, false);  // rows per workgroup
    const dim3 jg((unsigned)(n / R)), jb((unsigned)(R * n / 4));
    const size_t jl = sizeof(double2) * R * n;
    if (nl == 2)
      hipLaunchKernelGGL(fft_jacobian_rows_kernel<2>, jg, jb, jl, c->stream, (const double2*)q.PT, n, logn, uvT,
                         q.g.shear, q.dmax, (const double2*)c->tw, q.PZ);
    else
      hipLaunchKernelGGL(fft_jacobian_rows_kernel<1>, jg, jb, jl, c->stream, (const double2*)q.PT, n, logn, uvT,
                         q.g.shear, q.dmax, (const double2*)c->tw, q.PZ);
    HIPCHK(c, hipGetLastError());
    if (cols) {
      q.Fj = q.PZ;
      q.Fj_rows = true;
    } else {
      launch_fft<true>(c, q.PZ, q.PT, n, logn, n, 0);
      HIPCHK(c, hipGetLastError());
    }
  } else {
    const dim3 jgrid((unsigned)nblocks(q.nn, 256 * kQgMaxPer));
    hipLaunchKernelGGL(qg_jacobian_max_kernel, jgrid, block, 0, c->stream, (const double2*)q.PT, nl, q.nn, q.PZ,
                       uvT, q.g.shear, q.dmax);
    HIPCHK(c, hipGetLastError());
    if ((rc = transform_2d(c, q.PZ, q.PT, n, 1, 0))) return rc;
  }
  q.post_valid = true;
  return SWRT_OK;
}

}  // namespace

int swrt_qg_step(swrt_ctx* c, double dt, int64_t nsteps) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  QGState& q = c->qg;
  if (!q.init) return fail(c, SWRT_ERR_STATE, "swrt_qg_init not called");
  if (c->qg.spec) return fail(c, SWRT_ERR_STATE, "a speculative QG step is pending (swrt_qg_resolve first)");
  if (!(dt > 0) || nsteps < 0) return fail(c, SWRT_ERR_ARG, "dt must be > 0, nsteps >= 0");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  const int n = q.g.n, nl = q.g.nl;
  if ((rc = ensure_twiddles(c, n))) return rc;
  for (int64_t s = 0; s < nsteps; ++s) {
    if (nl == 2 && dt != q.exp_dt) {
      hipLaunchKernelGGL(qg2_exp_kernel, dim3(nblocks(q.nhalf, 256)), dim3(256), 0, c->stream, q.g, dt, q.E1, q.E2);
      HIPCHK(c, hipGetLastError());
      q.exp_dt = dt;
    }
    const int abstep = q.steps == 0 ? 1 : (q.steps == 1 ? 2 : 3);
    if (c->qg_fused) {
      if ((rc = qg_post(c))) return rc;
      if (q.Fj_rows) {
        // the tendency over Qm2 (read first by the same lane), then renamed:
        // Qm2 <- Qm1, Qm1 <- Qn
        if ((rc = qg_update_cols_launch(c, dt, abstep, q.Fj, q.qk_prev, q.Qm2))) return rc;
        std::swap(q.Qm1, q.Qm2);
      } else {
        rc = qg_update_launch(c, dt, abstep, q.Fj, q.qk_prev, q.Qm1, q.Qm2);
      }
    } else {
      rc = qg_step_launches(c, dt, abstep);
    }
    if (rc) return rc;
    q.post_valid = false;
    q.post_inv_valid = false;
    std::swap(q.qk, q.qk_prev);
    q.steps += 1;
    q.t = q.t + dt;
    q.has_prev = true;
  }
  return SWRT_OK;
  GUARD_END(c)
}

namespace {
int qg_speed_launch(swrt_ctx* c);
}  // namespace

int swrt_qg_step_speculative(swrt_ctx* c, double dt) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  QGState& q = c->qg;
  if (!q.init) return fail(c, SWRT_ERR_STATE, "swrt_qg_init not called");
  if (q.spec) return fail(c, SWRT_ERR_STATE, "a speculative QG step is already pending");
  if (!c->qg_fused) return fail(c, SWRT_ERR_STATE, "speculative steps need the fused post-step transforms");
  if (!(dt > 0)) return fail(c, SWRT_ERR_ARG, "dt must be > 0");
  if (q.g.nl == 2 && dt != q.exp_dt)
    return fail(c, SWRT_ERR_STATE, "a speculative step takes the dt of the exponential propagators in place");
  if (q.sp_count >= 2) return fail(c, SWRT_ERR_STATE, "two CFL read-backs already pending");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_twiddles(c, q.g.n))) return rc;
  const size_t hb = sizeof(double2) * (size_t)q.g.nl * (size_t)q.nhalf;
  for (double2** b : {&q.qk_spare, &q.Qm1_spare, &q.Qm2_spare})
    if (!*b) HIPCHK(c, hipMalloc(b, hb));
  const int abstep = q.steps == 0 ? 1 : (q.steps == 1 ? 2 : 3);
  if ((rc = qg_post(c))) return rc;  // of the committed qk (valid when the caller read its speed)
  q.spec_rot = q.Fj_rows;
  if (q.spec_rot)  // the tendency only; the committed Qm1 becomes Qm2 on acceptance
    rc = qg_update_cols_launch(c, dt, abstep, q.Fj, q.qk_spare, q.Qm1_spare);
  else
    rc = qg_update_launch(c, dt, abstep, q.Fj, q.qk_spare, q.Qm1_spare, q.Qm2_spare);
  if (rc) return rc;
  // the post-step transforms and CFL read-back of the speculative qk
  double2* committed = q.qk;
  q.qk = q.qk_spare;
  const int rb_slot = q.sp_head;
  rc = qg_speed_launch(c);
  q.qk = committed;
  if (rc) return rc;
  q.spec_rb = true;
  q.spec_rb_slot = rb_slot;
  q.spec = true;
  q.spec_dt = dt;
  q.spec_steps = q.steps + 1;
  q.spec_t = q.t + dt;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_qg_resolve(swrt_ctx* c, int accept) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  QGState& q = c->qg;
  if (!q.spec) return fail(c, SWRT_ERR_STATE, "no speculative QG step pending");
  if (accept) {
    // the committed qk becomes the previous one, the speculative one current
    double2* old_prev = q.qk_prev;
    q.qk_prev = q.qk;
    q.qk = q.qk_spare;
    q.qk_spare = old_prev;
    if (q.spec_rot) {
      // Qm2 <- the committed Qm1, Qm1 <- the speculative tendency; the old
      // Qm2 is the next spare
      double2* old_m2 = q.Qm2;
      q.Qm2 = q.Qm1;
      q.Qm1 = q.Qm1_spare;
      q.Qm1_spare = old_m2;
    } else {
      std::swap(q.Qm1, q.Qm1_spare);
      std::swap(q.Qm2, q.Qm2_spare);
    }
    q.steps = q.spec_steps;
    q.t = q.spec_t;
    q.has_prev = true;
  } else {
    // its CFL read-back (the newest pending) is dropped unless the caller
    // already popped it; PZ/PT hold its post-step transforms, so the
    // committed qk's are recomputed on use
    if (q.spec_rb) {
      q.sp_head ^= 1;
      q.sp_count -= 1;
    }
  }
  q.spec = false;
  q.spec_rb = false;
  return SWRT_OK;
  GUARD_END(c)
}

namespace {
// dmax -> the next FIFO slot of pinned host memory, and its event
int qg_speed_copy(swrt_ctx* c) {
  QGState& q = c->qg;
  const int slot = q.sp_head;
  HIPCHK(c, hipMemcpyAsync(q.hmax + slot, q.dmax, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipEventRecord(slot ? q.ev_b : q.ev, c->stream));
  q.sp_head ^= 1;
  q.sp_count += 1;
  return SWRT_OK;
}

// grid_U speed of the current qk -> device max -> pinned host copy + event
int qg_speed_launch(swrt_ctx* c) {
  QGState& q = c->qg;
  int rc;
  const int n = q.g.n, nl = q.g.nl;
  if (q.sp_count >= 2) return fail(c, SWRT_ERR_STATE, "two CFL read-backs already pending");
  if (c->qg_fused) {  // the speed comes with the post-step transforms
    if ((rc = qg_post(c))) return rc;
    return qg_speed_copy(c);
  }
  if ((rc = ensure_twiddles(c, n))) return rc;
  if (nl == 2)
    hipLaunchKernelGGL(qg_vel_spectra_kernel<2>, dim3(nblocks(q.nn, 256)), dim3(256), 0, c->stream, q.qk, q.g, q.Z);
  else
    hipLaunchKernelGGL(qg_vel_spectra_kernel<1>, dim3(nblocks(q.nn, 256)), dim3(256), 0, c->stream, q.qk, q.g, q.Z);
  HIPCHK(c, hipGetLastError());
  if ((rc = inverse_2d(c, q.Z, q.T, n, nl))) return rc;
  q.post_valid = false;  // dmax is overwritten (and the first phase clears it)
  q.post_inv_valid = false;
  HIPCHK(c, hipMemsetAsync(q.dmax, 0, sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(qg_max_speed2_kernel, dim3(256), dim3(256), 0, c->stream, q.T, q.nn * nl, q.g.shear, q.dmax);
  HIPCHK(c, hipGetLastError());
  return qg_speed_copy(c);
}

// the oldest pending read-back (FIFO)
int qg_speed_wait(swrt_ctx* c, double* U0_out) {
  QGState& q = c->qg;
  const int slot = (q.sp_head - q.sp_count) & 1;
  HIPCHK(c, hipEventSynchronize(slot ? q.ev_b : q.ev));
  q.sp_count -= 1;
  if (q.spec && q.spec_rb && slot == q.spec_rb_slot) q.spec_rb = false;  // the speculative step's, consumed
  *U0_out = std::sqrt(q.hmax[slot]);  // bits of a non-negative double: the max of (u+shear)^2 + v^2
  return SWRT_OK;
}
}  // namespace

int swrt_qg_max_speed(swrt_ctx* c, double* U0_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  QGState& q = c->qg;
  if (!q.init) return fail(c, SWRT_ERR_STATE, "swrt_qg_init not called");
  if (!U0_out) return fail(c, SWRT_ERR_ARG, "NULL output");
  if (c->qg.spec) return fail(c, SWRT_ERR_STATE, "a speculative QG step is pending (swrt_qg_resolve first)");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = qg_speed_launch(c))) return rc;
  while (q.sp_count > 0)  // the last one popped is this call's (earlier pending ones are superseded)
    if ((rc = qg_speed_wait(c, U0_out))) return rc;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_qg_max_speed_async(swrt_ctx* c) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  if (!c->qg.init) return fail(c, SWRT_ERR_STATE, "swrt_qg_init not called");
  if (c->qg.spec) return fail(c, SWRT_ERR_STATE, "a speculative QG step is pending (swrt_qg_resolve first)");
  HIPCHK(c, hipSetDevice(c->device));
  return qg_speed_launch(c);
  GUARD_END(c)
}

int swrt_qg_max_speed_result(swrt_ctx* c, double* U0_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  if (c->qg.sp_count == 0) return fail(c, SWRT_ERR_STATE, "no swrt_qg_max_speed_async pending");
  if (!U0_out) return fail(c, SWRT_ERR_ARG, "NULL output");
  return qg_speed_wait(c, U0_out);
  GUARD_END(c)
}

int swrt_qg_get(swrt_ctx* c, double* qk_out, double* t_out, int64_t* steps_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  QGState& q = c->qg;
  if (!q.init) return fail(c, SWRT_ERR_STATE, "swrt_qg_init not called");
  HIPCHK(c, hipSetDevice(c->device));
  if (qk_out) {
    const int kmax = q.g.n / 2 - 1;
    double2* tmp = q.Z;  // relayout to the host's kx-fastest order
    hipLaunchKernelGGL(halfplane_relayout_kernel, dim3(nblocks(q.nhalf * q.g.nl, 256)), dim3(256), 0, c->stream,
                       q.qk, tmp, 2 * kmax + 1, kmax + 1, 0, q.g.nl);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(qk_out, tmp, sizeof(double2) * q.nhalf * q.g.nl, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (t_out) *t_out = q.t;
  if (steps_out) *steps_out = q.steps;
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_qg_get_q(swrt_ctx* c, double* q_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  QGState& q = c->qg;
  if (!q.init) return fail(c, SWRT_ERR_STATE, "swrt_qg_init not called");
  if (!q_out) return fail(c, SWRT_ERR_ARG, "NULL output");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  const int n = q.g.n, nl = q.g.nl;
  if ((rc = ensure_twiddles(c, n))) return rc;
  for (int l = 0; l < nl; ++l) {
    hipLaunchKernelGGL(fulspec_kernel, dim3(nblocks(q.nn, 256)), dim3(256), 0, c->stream, q.qk + l * q.nhalf, n,
                       q.Z + l * q.nn, n / 2, 1);
    HIPCHK(c, hipGetLastError());
  }
  if ((rc = inverse_2d(c, q.Z, q.T, n, nl))) return rc;
  double* planes = reinterpret_cast<double*>(q.Z);
  hipLaunchKernelGGL(real_part_kernel, dim3(nblocks(q.nn * nl, 256)), dim3(256), 0, c->stream, q.T, planes,
                     q.nn * nl);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(q_out, planes, sizeof(double) * q.nn * nl, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SWRT_OK;
  GUARD_END(c)
}

namespace {
// A snapshot written on the QG stream (c->stream = the QG stream, OnQGStream):
// a slot buffer still read by a queued packet launch is renamed (an idle
// spare takes its place), else the write waits for the slot's last reader.
int qg_slot_acquire(swrt_ctx* c, int slot) {
  if (!c->qg_sep) return SWRT_OK;
  if (c->slot[slot].upend && event_pending(c->slot[slot].uref)) {
    int pick = -1;
    for (size_t i = 0; i < c->spares.size() && pick < 0; ++i)
      if (!c->spares[i].upend || !event_pending(c->spares[i].uref)) pick = (int)i;
    if (pick < 0 && c->spares.size() < kMaxSpares) {
      Slot sp;
      HIPCHK(c, hipEventCreateWithFlags(&sp.uev, hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&sp.wev, hipEventDisableTiming));
      c->spares.push_back(sp);
      pick = (int)c->spares.size() - 1;
    }
    if (pick >= 0) std::swap(c->slot[slot], c->spares[pick]);  // else wait for the slot's own reader
  }
  if (c->slot[slot].upend) HIPCHK(c, hipStreamWaitEvent(c->stream, c->slot[slot].uref, 0));
  return SWRT_OK;
}

// ... and done: a new write generation; the packet stream's next reader waits
// for the write's event (slot_writes_wait)
int qg_slot_written(swrt_ctx* c, int slot) {
  Slot& s = c->slot[slot];
  s.set = true;
  s.wgen = ++c->slot_wgen;
  if (c->qg_sep) {
    HIPCHK(c, hipEventRecord(s.wev, c->stream));
    s.wpend = true;
  }
  return SWRT_OK;
}

// swrt_qg_snapshot, or (spec) the same snapshot of the pending speculative
// step's qk: its post-step transforms (swrt_qg_step_speculative) hold layer
// 0's grid_U planes, which a snapshot after accepting the step would pack
// unchanged — so the pack can run before the CFL rule has decided.
int qg_snapshot_impl(swrt_ctx* c, int slot, int which, int layer, int64_t ny_period, bool spec) {
  OnQGStream on_qg(c);
  QGState& q = c->qg;
  if (!q.init) return fail(c, SWRT_ERR_STATE, "swrt_qg_init not called");
  if (spec) {
    if (!q.spec) return fail(c, SWRT_ERR_STATE, "no speculative QG step pending");
    if (!c->qg_fused || which != 0 || layer != 0 || q.g.n % 16 || !q.post_inv_valid || q.post_of != q.qk_spare)
      return fail(c, SWRT_ERR_STATE, "a speculative snapshot needs the fused transforms of the pending step (layer 0)");
  } else if (c->qg.spec) {
    return fail(c, SWRT_ERR_STATE, "a speculative QG step is pending (swrt_qg_resolve first)");
  }
  if (which != 0 && which != 1) return fail(c, SWRT_ERR_ARG, "which must be 0 (current) or 1 (previous)");
  if (which == 1 && !q.has_prev) return fail(c, SWRT_ERR_STATE, "no previous qk before the first step");
  if (layer < 0 || layer >= q.g.nl) return fail(c, SWRT_ERR_ARG, "layer out of range");
  const int64_t nx = q.g.n;
  int rc = check_slot_args(c, slot, nx);
  if (rc) return rc;
  if (ny_period == 0) ny_period = nx;
  if (ny_period % nx) return fail(c, SWRT_ERR_ARG, "ny_period must be a multiple of nx");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = qg_slot_acquire(c, slot))) return rc;
  if ((rc = ensure_slot(c, slot, nx))) return rc;
  if ((rc = ensure_twiddles(c, (int)nx))) return rc;
  Slot& s = c->slot[slot];
  if (c->qg_fused && which == 0 && layer == 0 && nx % 16 == 0) {
    // layer 0's grid_U of the current qk is part of the post-step transforms
    // (of the speculative qk: already computed, checked above)
    if (!spec && (rc = qg_post_inverse(c))) return rc;
    const double2* T = q.PT + (3 * q.g.nl - 1) * q.nn;
    hipLaunchKernelGGL(pack_pairs_kernel, dim3(nx / 16, nx / 16), dim3(256), 0, c->stream, T, (int)nx, (int)s.npad,
                       q.g.shear, s.nodes);
    HIPCHK(c, hipGetLastError());
    s.has_psi = false;
    s.div_free = true;
  } else {
    const double2* src = (which == 0 ? q.qk : q.qk_prev) + layer * q.nhalf;
    if ((rc = fields_from_halfplane(c, slot, src, (int)nx, 1, q.g.K_d2, q.g.kscale, q.g.shear, 0, q.Z, q.T,
                                    (int)(nx / 2), 1)))
      return rc;
  }
  s.L = q.g.dx * (double)nx;
  s.ny_period = ny_period;
  return qg_slot_written(c, slot);
}
}  // namespace

int swrt_qg_snapshot(swrt_ctx* c, int slot, int which, int layer, int64_t ny_period) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  return qg_snapshot_impl(c, slot, which, layer, ny_period, false);
  GUARD_END(c)
}

int swrt_qg_snapshot_speculative(swrt_ctx* c, int slot, int64_t ny_period) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  return qg_snapshot_impl(c, slot, 0, 0, ny_period, true);
  GUARD_END(c)
}

// ---------------------------------------------------------------------------
// Owner-driver hand-off: one rank steps the PDE, the others build their
// snapshots from the top layer's spectral PV it sends (qg2layersw_raytrace.m
// :186-188 reads layer 1 only)
// ---------------------------------------------------------------------------
namespace {
// order `from`'s work so far before `to`'s later work (no-op on one stream)
int stream_order(swrt_ctx* c, hipStream_t from, hipStream_t to, int ev) {
  if (from == to) return SWRT_OK;
  if (!c->xev[ev]) HIPCHK(c, hipEventCreateWithFlags(&c->xev[ev], hipEventDisableTiming));
  HIPCHK(c, hipEventRecord(c->xev[ev], from));
  HIPCHK(c, hipStreamWaitEvent(to, c->xev[ev], 0));
  return SWRT_OK;
}
}  // namespace

int swrt_qg_export(swrt_ctx* c, int which, int layer, double* dst, int dst_mode, void* stream, double tail) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN_KEEP_CHAIN
  OnQGStream on_qg(c);
  QGState& q = c->qg;
  if (!q.init) return fail(c, SWRT_ERR_STATE, "swrt_qg_init not called");
  // (a pending speculative step writes the spare buffers only: the committed
  // qk and prev_qk stay as they are until swrt_qg_resolve)
  if (!dst) return fail(c, SWRT_ERR_ARG, "dst is NULL");
  if (which != 0 && which != 1) return fail(c, SWRT_ERR_ARG, "which must be 0 (current) or 1 (previous)");
  if (which == 1 && !q.has_prev) return fail(c, SWRT_ERR_STATE, "no previous qk before the first step");
  if (layer < 0 || layer >= q.g.nl) return fail(c, SWRT_ERR_ARG, "layer out of range");
  HIPCHK(c, hipSetDevice(c->device));
  const double2* src = (which == 0 ? q.qk : q.qk_prev) + layer * q.nhalf;
  const size_t bytes = sizeof(double2) * q.nhalf;
  if (dst_mode != 0 && dst_mode != 1 && dst_mode != 2) return fail(c, SWRT_ERR_ARG, "dst_mode must be 0, 1 or 2");
  if (dst_mode) {
    const hipStream_t ext = stream ? (hipStream_t)stream : on_qg.saved;
    if (dst_mode == 1) HIPCHK_RC(stream_order(c, ext, c->stream, 0));  // the caller's last read of dst
    hipLaunchKernelGGL(export_half_kernel, dim3(nblocks(q.nhalf + 1, 256)), dim3(256), 0, c->stream, src, dst,
                       q.nhalf, tail);
    HIPCHK(c, hipGetLastError());
    HIPCHK_RC(stream_order(c, c->stream, ext, 1));  // the caller's next use of dst
  } else {
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dst[2 * q.nhalf] = tail;
  }
  return SWRT_OK;
  GUARD_END(c)
}

int swrt_snapshot_qk(swrt_ctx* c, int slot, const double* qk, int src_on_device, void* stream, int64_t nx,
                     double L, double K_d2, double shear, double k_scale, int64_t ny_period) {
  int rc = check_slot_args(c, slot, nx);
  if (rc) return rc;
  GUARD_BEGIN_KEEP_CHAIN
  if (!qk) return fail(c, SWRT_ERR_ARG, "qk is NULL");
  if (!is_pow2(nx)) return fail(c, SWRT_ERR_ARG, "nx must be a power of two for the GPU FFT");
  if (!(L > 0)) return fail(c, SWRT_ERR_ARG, "L must be > 0");
  if (ny_period == 0) ny_period = nx;
  if (ny_period % nx) return fail(c, SWRT_ERR_ARG, "ny_period must be a multiple of nx");
  if (c->qg.init && c->qg.g.n != nx) return fail(c, SWRT_ERR_ARG, "nx differs from the QG state's");
  HIPCHK(c, hipSetDevice(c->device));
  const hipStream_t pk = c->stream;  // the packet stream
  if (!c->xq_init && !c->qg.init && c->qg_sep) {
    // from here on packet launches mark their slot use; everything queued on
    // the packet stream so far is marked by one record per slot (as swrt_qg_init)
    for (Slot& sl : c->slot)
      if (sl.nodes && hipEventRecord(sl.uev, pk) == hipSuccess) {
        sl.uref = sl.uev;
        sl.upend = true;
      }
  }
  c->xq_init = true;
  OnQGStream on_qg(c);
  const int n = (int)nx, kmax = n / 2 - 1;
  const int64_t nn = nx * nx, nhalf = (int64_t)(2 * kmax + 1) * (kmax + 1);
  if (c->xq_nx != nx) {
    HIPCHK(c, hipStreamSynchronize(c->stream));  // a queued snapshot may still use them
    for (double2** p : {&c->xq_Z, &c->xq_T, &c->xq_fk}) {
      if (*p) (void)hipFree(*p);
      *p = nullptr;
    }
    c->xq_nx = 0;
    HIPCHK(c, hipMalloc(&c->xq_Z, sizeof(double2) * 3 * nn));
    HIPCHK(c, hipMalloc(&c->xq_T, sizeof(double2) * 3 * nn));
    HIPCHK(c, hipMalloc(&c->xq_fk, sizeof(double2) * nhalf));
    c->xq_nx = nx;
  }
  if ((rc = ensure_twiddles(c, n))) return rc;
  if ((rc = qg_slot_acquire(c, slot))) return rc;
  if ((rc = ensure_slot(c, slot, nx))) return rc;
  const hipStream_t ext = stream ? (hipStream_t)stream : pk;
  const double2* fk = (const double2*)qk;
  if (src_on_device) {
    HIPCHK_RC(stream_order(c, ext, c->stream, 0));  // the caller's fill of qk (e.g. a broadcast)
  } else {
    HIPCHK(c, hipMemcpyAsync(c->xq_fk, qk, sizeof(double2) * nhalf, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // the caller's host buffer is free on return
    fk = c->xq_fk;
  }
  // grid_U of the half plane in the QG state's order (ky fastest): the
  // unfused path of swrt_qg_snapshot, bit for bit
  if ((rc = fields_from_halfplane(c, slot, fk, n, 1, K_d2, k_scale, shear, 0, c->xq_Z, c->xq_T, n / 2, 1)))
    return rc;
  if (src_on_device) HIPCHK_RC(stream_order(c, c->stream, ext, 1));  // qk read: the caller may refill it
  Slot& s = c->slot[slot];
  s.L = L;
  s.ny_period = ny_period;
  return qg_slot_written(c, slot);
  GUARD_END(c)
}

int swrt_swap_slots(swrt_ctx* c, int a, int b) {
  if (!c) return SWRT_ERR_ARG;
  if (a < 0 || a >= SWRT_MAX_SLOTS || b < 0 || b >= SWRT_MAX_SLOTS) return fail(c, SWRT_ERR_ARG, "slot out of range");
  std::swap(c->slot[a], c->slot[b]);
  return SWRT_OK;
}

// ---------------------------------------------------------------------------
// ode23 device stages (swrt_ode23.hpp)
// ---------------------------------------------------------------------------
namespace {
int ode23_prepare(swrt_ctx* c, int nslots, Ode23Args& a, double tmax, double f, double Cg, double thr,
                  double bump) {
  if (c->n <= 0 || !c->dx) return fail(c, SWRT_ERR_STATE, "no packets (swrt_packets_set)");
  if (nslots != 1 && nslots != 2) return fail(c, SWRT_ERR_ARG, "nslots must be 1 or 2");
  if (!c->slot[0].set || (nslots == 2 && !c->slot[1].set)) return fail(c, SWRT_ERR_STATE, "field slot not set");
  if (nslots == 2 && c->slot[1].nx != c->slot[0].nx) return fail(c, SWRT_ERR_ARG, "slots differ in nx");
  if (c->o_cap < c->cap) {
    for (double*& p : c->oF) { if (p) (void)hipFree(p); p = nullptr; }
    for (double** p : {&c->o_ynx, &c->o_ynk, &c->o_spx, &c->o_spk, &c->o_spF}) {
      if (*p) (void)hipFree(*p);
      *p = nullptr;
    }
    c->o_cap = 0;
    for (double*& p : c->oF) HIPCHK(c, hipMalloc(&p, sizeof(double) * 4 * c->cap));
    HIPCHK(c, hipMalloc(&c->o_ynx, sizeof(double) * 2 * c->cap));
    HIPCHK(c, hipMalloc(&c->o_ynk, sizeof(double) * 2 * c->cap));
    HIPCHK(c, hipMalloc(&c->o_spx, sizeof(double) * 2 * c->cap));
    HIPCHK(c, hipMalloc(&c->o_spk, sizeof(double) * 2 * c->cap));
    HIPCHK(c, hipMalloc(&c->o_spF, sizeof(double) * 4 * c->cap));
    c->o_cap = c->cap;
  }
  if (!c->o_dmax) {  // 3 max slots per part (part 1: split attempts)
    HIPCHK(c, hipMalloc(&c->o_dmax, 6 * sizeof(unsigned long long)));
    HIPCHK(c, hipMemsetAsync(c->o_dmax, 0, 6 * sizeof(unsigned long long), c->stream));
    c->o_dmax_cur = 0;
  }
  if (!c->o_hmax) HIPCHK(c, hipHostMalloc(&c->o_hmax, 3 * sizeof(unsigned long long)));
  if (!c->o_hpart) {
    // coherent (fine-grained): the attempt kernels' stores reach host memory
    // without the system-scope release of a separate event marker
    HIPCHK(c, hipHostMalloc((void**)&c->o_hpart, 6 * kMaxBins * sizeof(unsigned long long),
                            hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(c, hipHostGetDevicePointer((void**)&c->o_hpart_d, c->o_hpart, 0));
    std::fill(c->o_hpart, c->o_hpart + 6 * kMaxBins, kHpartEmpty);
  }
  if (!c->o_shown) {
    HIPCHK(c, hipMalloc((void**)&c->o_coef, 8 * sizeof(double)));
    HIPCHK(c, hipHostMalloc((void**)&c->o_shown, 13 * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(c, hipHostGetDevicePointer((void**)&c->o_shown_d, c->o_shown, 0));
    std::memset(c->o_shown, 0, 13 * sizeof(double));  // (ticket 0: never a launch's)
  }
  for (hipEvent_t& e : c->o_ev)
    if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (hipEvent_t& e : c->o_evb)
    if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  a.f0 = view_of(c->slot[0]);
  a.f1 = nslots == 2 ? view_of(c->slot[1]) : a.f0;
  a.nslots = nslots;
  a.n = c->n;
  a.yx = c->dx;
  a.yk = c->dk;
  for (int s = 0; s < 4; ++s) a.F[s] = c->oF[s];
  a.ynx = c->o_ynx;
  a.ynk = c->o_ynk;
  a.tmax = tmax;
  a.inv_tmax = 0.0;
  a.f2 = f * f;
  a.Cg = Cg;
  a.Cg2 = Cg * Cg;
  a.fastdisp = dispersion_fast(a.f2);
  a.thr = thr;
  a.bump = bump;
  a.dmax = c->o_dmax + c->o_dmax_cur;
  a.dmax_clear = c->o_dmax + (c->o_dmax_cur + 1) % 3;
  a.gate = nullptr;
  a.gate_scale = 0.0;
  a.gate_limit = 0.0;
  a.order = nullptr;
  a.hpart = nullptr;
  a.sh = TileShare{};
  a.coef = nullptr;
  return SWRT_OK;
}

// an attempt's stage times and coefficients (swrt_ode23.hpp o23_coeffs)
void attempt_coeffs(Ode23Args& a, double t, double h, double tnew) {
  double cf[8];
  o23_coeffs(t, h, tnew, cf);
  a.ts = cf[0];
  a.c[0] = cf[1];
  a.ts3 = cf[2];
  a.c3 = cf[3];
  a.ts4 = cf[4];
  a.c4[0] = cf[5];
  a.c4[1] = cf[6];
  a.c4[2] = cf[7];
}

// the max of the launch just queued (slot o_dmax_cur), then the next slot
int read_max(swrt_ctx* c, double* out) {
  const int slot = c->o_dmax_cur;
  c->o_dmax_cur = (slot + 1) % 3;
  if (!out) return SWRT_OK;
  HIPCHK(c, hipMemcpyAsync(c->o_hmax + slot, c->o_dmax + slot, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           c->stream));
  // (spinning on an event instead measured within noise: 2.55-2.59 vs 2.60-2.62 ms)
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::memcpy(out, c->o_hmax + slot, sizeof(double));
  return dev_err_check(c);
}
}  // namespace

}  // extern "C"
namespace {
// one ode23 stage over all packets: the LDS-tiled kernel when the packets are
// binned by the tile kernel's 16x16-cell tiles, else one lane per packet
template <int STAGE, bool TWO, bool V5>
void ode23_tile_launch(swrt_ctx* c, const Ode23Args& a, unsigned grid, const int* starts, int ntx, hipStream_t st,
                       hipEvent_t stop) {
  if constexpr (STAGE == 0) {
    if (a.coef) {  // coefficients from device memory (swrt_ode23_run's first attempt)
      hipExtLaunchKernelGGL((tile_ode23_kernel<0, TWO, kTile, kMargin, kTileThreads, V5, true>), dim3(grid),
                            dim3(kTileThreads), 0, st, nullptr, stop, 0, a, starts, ntx);
      return;
    }
  }
  hipExtLaunchKernelGGL((tile_ode23_kernel<STAGE, TWO, kTile, kMargin, kTileThreads, V5>), dim3(grid),
                        dim3(kTileThreads), 0, st, nullptr, stop, 0, a, starts, ntx);
}

// swrt_ode23_run may split each attempt into two part launches (the even and
// the odd band positions of every XCD band, swrt_share.hpp), part 1 on the
// extra packet stream: consecutive attempts then overlap one part's tail with
// the other's next launch.  Parts touch disjoint packets of one binning, so
// stream order alone orders each part's attempts; the packets must already be
// in the tiles' cell order (no order kernel between the parts).
bool ode23_split_ok(swrt_ctx* c) {
  const int ntx = (int)((c->slot[0].nx + kTile - 1) / kTile);
  return use_tile_kernel(c) && c->bin_valid && !c->src_pending && c->nbins == ntx * ntx && c->o_sorted &&
         (ntx * ntx) % 16 == 0 && c->n >= kMultiStreamFrom && c->packet_streams == 2 && c->stream == c->stream0 &&
         c->sx[0] != nullptr;
}

// part -1: one launch over every tile on the packet stream; 0 / 1: that part
// of a split attempt (part 1 on sx[0]).  *wg_out: the workgroups of the tile
// launch (each stores its max to a.hpart, whose host copy is first marked
// empty), 0 for the per-packet kernels.  `stop`: an event the tile launch
// itself completes (*stop_done = true) — no marker between consecutive
// attempts (a separate event record cost ~7 us of idle stream per launch,
// profiles/r06_ode23); the per-packet kernels leave it to the caller.
template <int STAGE>
int ode23_launch(swrt_ctx* c, const Ode23Args& a0, int part = -1, unsigned* wg_out = nullptr,
                 hipEvent_t stop = nullptr, bool* stop_done = nullptr) {
  if (wg_out) *wg_out = 0;
  if (stop_done) *stop_done = false;
  const int ntx = (int)((c->slot[0].nx + kTile - 1) / kTile);
  if (part >= 0 && !ode23_split_ok(c)) return fail(c, SWRT_ERR_STATE, "ode23 split attempt without a split binning");
  if (use_tile_kernel(c) && c->bin_valid && !c->src_pending && c->nbins == ntx * ntx) {
    const int* starts = c->bins + 2 * kMaxBins;
    const unsigned ntiles = (unsigned)(ntx * ntx);
    Ode23Args a = a0;
    a.sh = TileShare{(int)ntiles, part, part < 0 ? 1 : 2, kShareEven};
    const unsigned grid = (unsigned)share_grid(a.sh);
    const hipStream_t st = part == 1 ? c->sx[0] : c->stream;
    if (wg_out) *wg_out = grid;
    // in-tile cell order of this binning, once (swrt_ode23.hpp): the packets'
    // own order after swrt_ode23_f1's sort, else an order array
    if (c->o_sorted) {
      a.order = nullptr;
    } else if (!c->o_order_valid) {
      if (c->o_order_cap < c->cap) {
        if (c->o_order) (void)hipFree(c->o_order);
        c->o_order = nullptr;
        HIPCHK(c, hipMalloc(&c->o_order, sizeof(int) * c->cap));
        c->o_order_cap = c->cap;
      }
      const FieldView v = view_of(c->slot[0]);
      hipLaunchKernelGGL((tile_cell_order_kernel<kTile, kTileThreads>), dim3(grid), dim3(kTileThreads), 0,
                         c->stream, c->dx, c->n, starts, ntx, v.inv_dx, v.nx, c->o_order);
      HIPCHK(c, hipGetLastError());
      c->o_order_valid = true;
      a.order = c->o_order;
    } else {
      a.order = c->o_order;
    }
    if (a.hpart) {
      unsigned long long* hh = c->o_hpart + (a.hpart - c->o_hpart_d);
      std::fill(hh, hh + grid, kHpartEmpty);
    }
    const bool v5 = c->slot[0].div_free && (a.nslots == 1 || c->slot[1].div_free);
    if (a.nslots == 2) {
      if (v5) ode23_tile_launch<STAGE, true, true>(c, a, grid, starts, ntx, st, stop);
      else ode23_tile_launch<STAGE, true, false>(c, a, grid, starts, ntx, st, stop);
    } else {
      if (v5) ode23_tile_launch<STAGE, false, true>(c, a, grid, starts, ntx, st, stop);
      else ode23_tile_launch<STAGE, false, false>(c, a, grid, starts, ntx, st, stop);
    }
    if (stop_done) *stop_done = stop != nullptr;
  } else if constexpr (STAGE == 0) {  // one lane per packet: the three stage launches
    const dim3 grid(nblocks(c->n, 256)), block(256);
    Ode23Args b = a0;
    hipLaunchKernelGGL(ode23_stage_kernel<2>, grid, block, 0, c->stream, b);
    b.ts = a0.ts3;
    b.c[0] = a0.c3;
    hipLaunchKernelGGL(ode23_stage_kernel<3>, grid, block, 0, c->stream, b);
    b.ts = a0.ts4;
    for (int i = 0; i < 3; ++i) b.c[i] = a0.c4[i];
    hipLaunchKernelGGL(ode23_stage_kernel<4>, grid, block, 0, c->stream, b);
  } else {
    hipLaunchKernelGGL(ode23_stage_kernel<STAGE>, dim3(nblocks(c->n, 256)), dim3(256), 0, c->stream, a0);
  }
  HIPCHK(c, hipGetLastError());
  return SWRT_OK;
}
}  // namespace
extern "C" {

namespace {
// swrt_ode23_f1 without the read: re-binning, in-tile sort and the stage-1
// launch queued (its max in slot o_dmax_cur, not yet advanced)
int ode23_f1_queue(swrt_ctx* c, double t, double tmax, double f, double Cg, int nslots, double thr, double bump) {
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  // a spatial re-binning per kOde23RebinEvery ode23 calls (the packet order
  // is free: the error norm is a max over all components; a packet that has
  // left its tile's window since takes the global gather, so a skipped
  // re-binning changes speed only)
  const int ntx0 = (int)((c->slot[0].nx + kTile - 1) / kTile);
  const bool binned = use_tile_kernel(c) && c->bin_valid && !c->src_pending && c->nbins == ntx0 * ntx0 &&
                      c->bin_tile == kTile && c->o_sorted;
  const bool due = !binned || ++c->o_since_bin >= kOde23RebinEvery;
  if (c->rebin_every > 0 && c->slot[0].set && due) {
    c->o_since_bin = 0;
    if ((rc = rebin(c, false, use_tile_kernel(c) ? kTile : 0))) return rc;  // the ode23 tile kernel's 16x16 tiles
    const int ntx = (int)((c->slot[0].nx + kTile - 1) / kTile);
    if (use_tile_kernel(c) && c->bin_valid && !c->src_pending && c->nbins == ntx * ntx) {
      // the in-tile cell order applied to the packets (swrt_ode23.hpp tile_cell_sort_kernel)
      const FieldView v = view_of(c->slot[0]);
      hipLaunchKernelGGL((tile_cell_sort_kernel<kTile, kTileThreads>), dim3((unsigned)(ntx * ntx)),
                         dim3(kTileThreads), 0, c->stream, (const double*)c->dx, (const double*)c->dk,
                         (const int*)c->perm, c->n, (const int*)(c->bins + 2 * kMaxBins), ntx, v.inv_dx,
                         (int)v.nx, c->dx2, c->dk2, c->perm2);
      HIPCHK(c, hipGetLastError());
      std::swap(c->dx, c->dx2);
      std::swap(c->dk, c->dk2);
      std::swap(c->perm, c->perm2);
      c->o_sorted = true;
    }
  }
  Ode23Args a;
  if ((rc = ode23_prepare(c, nslots, a, tmax, f, Cg, thr, bump))) return rc;
  a.ts = t;
  return ode23_launch<1>(c, a);
}
}  // namespace

int swrt_ode23_f1(swrt_ctx* c, double t, double tmax, double f, double Cg, int nslots, double thr, double bump,
                  double* rh_raw_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  HIPCHK_RC(lost_check(c));
  SlotUse slot_use(c, false, kSlots01);
  int rc;
  if ((rc = ode23_f1_queue(c, t, tmax, f, Cg, nslots, thr, bump))) return rc;
  return read_max(c, rh_raw_out);
  GUARD_END(c)
}

int swrt_ode23_attempt(swrt_ctx* c, double t, double h, double tnew, double tmax, double f, double Cg,
                       int nslots, double thr, double bump, double* err_raw_out) {
  if (!c) return SWRT_ERR_ARG;
  GUARD_BEGIN
  HIPCHK_RC(lost_check(c));
  SlotUse slot_use(c, false, kSlots01);
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  Ode23Args a;
  if ((rc = ode23_prepare(c, nslots, a, tmax, f, Cg, thr, bump))) return rc;
  // ode23: f(:,2) at t + h*A(1), y + f*hB(:,1); f(:,3) at t + h*A(2), y + f*hB(:,2);
  // h = tnew - t; ynew = y + f*hB(:,3); f(:,4) at tnew — one launch (stage 0:
  // the tile kernel runs the three stages per packet, registers between them)
  attempt_coeffs(a, t, h, tnew);
  if ((rc = ode23_launch<0>(c, a))) return rc;
  return read_max(c, err_raw_out);
  GUARD_END(c)
}

int swrt_ode23_accept(swrt_ctx* c) {
  if (!c) return SWRT_ERR_ARG;
  c->s0_dirty = true;  // (conservative: settings and syncs may precede packet-stream work)
  if (c->in_hook) return fail(c, SWRT_ERR_STATE, "this call may touch the packets: not allowed inside an ode23 hook");
  HIPCHK_RC(lost_check(c));
  HIPCHK_RC(chain_drop(c));
  if (!c->o_ynx) return fail(c, SWRT_ERR_STATE, "no ode23 step attempted");
  std::swap(c->dx, c->o_ynx);
  std::swap(c->dk, c->o_ynk);
  std::swap(c->oF[0], c->oF[3]);
  c->keys_fresh = false;
  c->cells_sorted = false;
  return SWRT_OK;
}

namespace {
double o23_alpha(double t, double tmax) { return tmax != 0.0 ? t / tmax : 0.0; }  // the kernels' alpha_of

bool same_bits(double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; }

// The chain (swrt_ode23_chain_next): at the end of an ode23 call, the next
// call's stage 1 — re-binning when due, in-tile sort, f at t = 0 — queued on
// the accepted packets with the armed slots as slots 0 / 1, so the device runs
// it while the host returns and prepares that call.  The next call takes it
// only if it would compute exactly that (ode23_chain_take).  Behind stage 1
// go the next call's first step size and its first attempt, as that call
// would queue them (ode23_chain_first), taken only if the call's t0, tfinal,
// tmax and RelTol are the ones assumed (never in a sharded run: its first
// step size comes from every rank's stage 1).  (Round 5 chained an unsplit first attempt,
// 186 us against 123 us split, and measured no faster: profiles/r05_chain.)
int ode23_chain_first(swrt_ctx* c, int sl_f1, double tmax, double f, double Cg, double thr, double bump,
                      double rtol);
int ode23_chain_queue(swrt_ctx* c, double tmax, double f, double Cg, int nslots, double thr, double bump,
                      double rtol, bool with_first) {
  swrt_ctx::O23Chain& ch = c->o_chain;
  const bool want = ch.want;
  ch.want = false;
  ch.queued = false;
  ch.first_q = false;
  if (!want || nslots != 2 || ch.sa < 0 || ch.sb < 0 || ch.sa == ch.sb || c->packets_lost) return SWRT_OK;
  if (!c->slot[ch.sa].set || !c->slot[ch.sb].set || c->slot[ch.sa].nx != c->slot[ch.sb].nx) return SWRT_OK;
  slot_writes_wait(c);  // e.g. the hook's snapshot into slot sb on the QG stream
  Slot saved[SWRT_MAX_SLOTS];
  for (int i = 0; i < SWRT_MAX_SLOTS; ++i) saved[i] = c->slot[i];
  c->slot[0] = saved[ch.sa];
  c->slot[1] = saved[ch.sb];
  int rc = ode23_f1_queue(c, 0.0, tmax, f, Cg, 2, thr, bump);
  const int sl_f1 = c->o_dmax_cur;
  if (!rc) {
    c->o_dmax_cur = (sl_f1 + 1) % 3;
    if (with_first) rc = ode23_chain_first(c, sl_f1, tmax, f, Cg, thr, bump, rtol);
  }
  for (int i = 0; i < SWRT_MAX_SLOTS; ++i) c->slot[i] = saved[i];
  if (rc) return rc;
  ch.dmax_slot = sl_f1;
  for (int i = 0; i < 2; ++i) {
    const Slot& s = c->slot[i == 0 ? ch.sa : ch.sb];
    ch.nodes[i] = s.nodes;
    ch.wgen[i] = s.wgen;
  }
  ch.alpha = o23_alpha(0.0, tmax);
  ch.f = f;
  ch.Cg = Cg;
  ch.thr = thr;
  ch.bump = bump;
  ch.queued = true;
  return SWRT_OK;
}

// The queued chain is this call's stage 1: nothing touched the packets since
// (GUARD_BEGIN drops the chain), slots 0 / 1 hold the same, unrewritten nodes,
// and stage 1's inputs are the same bits.
bool ode23_chain_take(swrt_ctx* c, double t0, double tmax, double f, double Cg, int nslots, double thr,
                      double bump) {
  swrt_ctx::O23Chain& ch = c->o_chain;
  const bool q = ch.queued;
  ch.queued = false;
  if (!q || nslots != 2) return false;
  for (int i = 0; i < 2; ++i)
    if (!c->slot[i].set || c->slot[i].nodes != ch.nodes[i] || c->slot[i].wgen != ch.wgen[i]) return false;
  return same_bits(o23_alpha(t0, tmax), ch.alpha) && same_bits(f, ch.f) && same_bits(Cg, ch.Cg) &&
         same_bits(thr, ch.thr) && same_bits(bump, ch.bump);
}
}  // namespace

int swrt_ode23_chain_next(swrt_ctx* c, int slot_a, int slot_b) {
  if (!c) return SWRT_ERR_ARG;
  if (slot_a < 0 || slot_a >= SWRT_MAX_SLOTS || slot_b < 0 || slot_b >= SWRT_MAX_SLOTS || slot_a == slot_b)
    return fail(c, SWRT_ERR_ARG, "chain slots out of range or equal");
  c->o_chain.want = true;
  c->o_chain.sa = slot_a;
  c->o_chain.sb = slot_b;
  return SWRT_OK;
}

int swrt_ode23_run(swrt_ctx* c, double t0, double tfinal, double tmax, double f, double Cg, int nslots,
                   double rtol, double atol, double bump, double* ts_out, int64_t ts_cap, int64_t* nts_out,
                   int64_t* stats3_out) {
  return swrt_ode23_run_hooked(c, t0, tfinal, tmax, f, Cg, nslots, rtol, atol, bump, ts_out, ts_cap, nts_out,
                               stats3_out, nullptr, nullptr);
}

namespace {
// The first-step kernel (the first attempt's step size on the device) on the
// packet stream, stage 1's max slot event o_ev[sl_f1] attached to it: the
// first attempt's part 0 follows it with no marker between them, part 1 waits
// for that event, and the host reads the step size once the launch's ticket
// has reached shown[12] (DeviceExec::stage1).  SWRT_ODE23_MARKERS=1: a marker
// after it instead (~7-12 us of idle GPU before the first attempt,
// profiles/r06_ode23).
int ode23_first_step_queue(swrt_ctx* c, int sl_f1, double c0, double hmax, double htspan, double t0, double tfinal,
                           bool split, uint64_t* ticket) {
  const double tdir = std::copysign(1.0, tfinal - t0);
  const uint64_t tk = ++c->o_ticket;
  const hipEvent_t stop = c->o23_markers ? nullptr : c->o_ev[sl_f1];
  // (part 1's slots start at zero, cleared here; each launch then clears its next one)
  hipExtLaunchKernelGGL(ode23_first_step_kernel, dim3(1), dim3(64), 0, c->stream, nullptr, stop, 0,
                        c->o_dmax + sl_f1, c0, hmax, htspan, 16 * o23_spacing(t0), tdir, t0, tfinal, c->o_coef,
                        c->o_shown_d, c->o_dmax + 3, split ? 3 : 0, (unsigned long long)tk);
  HIPCHK(c, hipGetLastError());
  if (c->o23_markers) HIPCHK(c, hipEventRecord(c->o_ev[sl_f1], c->stream));
  *ticket = tk;
  return SWRT_OK;
}

// swrt_ode23_run's stages for the controller (ode23_control, swrt_ode23_ctl.cpp):
// each attempt one tile launch — two part launches when the binning allows
// (ode23_split_ok), part 1 on the extra packet stream, part p keeping max
// slots o_dmax[3p + sl] and its own events — its maxima read from host-mapped
// memory after the launch's event; three state sets (x, k, F1/F4): an attempt
// reads set `from` and writes ynew and F4 into set `to`.
class DeviceExec final : public O23Exec {
 public:
  DeviceExec(swrt_ctx* c_, const Ode23Args& base_, bool split_, bool dev_first_, int sl_f1_, void (*hook_)(void*),
             void* hook_user_, int (*reduce_)(double*, void*) = nullptr, void* reduce_user_ = nullptr)
      : c(c_), base(base_), split(split_), P(split_ ? 2 : 1), dev_first(dev_first_), sl_f1(sl_f1_), hook(hook_),
        hook_user(hook_user_), reduce(reduce_), reduce_user(reduce_user_),
        S{{c_->dx, c_->dk, c_->oF[0]}, {c_->o_ynx, c_->o_ynk, c_->oF[3]}, {c_->o_spx, c_->o_spk, c_->o_spF}} {}

  // queue an attempt (coef: its coefficients from device memory, the first attempt)
  int launch(int from, int to, double ta, double ha, double tnewa, int gate_slot, double gscale, double glimit,
             int* slot, const double* coef) {
    Ode23Args a = base;
    a.coef = coef;
    a.yx = S[from].x;
    a.yk = S[from].k;
    a.F[0] = S[from].F;
    a.F[3] = S[to].F;
    a.ynx = S[to].x;
    a.ynk = S[to].k;
    attempt_coeffs(a, ta, ha, tnewa);
    const int sl = c->o_dmax_cur;
    // The host polls a slot's maxima without waiting for the launch's event
    // (wait_max), so a launch whose maxima were never read (a guess its
    // gate discarded; in a sharded run one that ran on this rank's part of
    // the max) must have finished before its slot's host copy is re-marked
    // empty for this launch.  Its events still hold that launch.
    if (unread[sl]) {
      HIPCHK(c, hipEventSynchronize(c->o_ev[sl]));
      if (P == 2) HIPCHK(c, hipEventSynchronize(c->o_evb[sl]));
    }
    unread[sl] = true;
    a.gate_scale = gscale;
    a.gate_limit = glimit;
    for (int p = 0; p < P; ++p) {
      a.dmax = c->o_dmax + 3 * p + sl;
      a.dmax_clear = c->o_dmax + 3 * p + (sl + 1) % 3;
      // a part's guess is gated on its own part of the previous max: when the
      // whole max passes, so does every part (err = absh * max is monotone)
      a.gate = gate_slot >= 0 ? c->o_dmax + 3 * p + gate_slot : nullptr;
      a.hpart = c->o_hpart_d + (size_t)(3 * p + sl) * kMaxBins;
      const hipStream_t st = p == 0 ? c->stream : c->sx[0];
      const hipEvent_t ev = p == 0 ? c->o_ev[sl] : c->o_evb[sl];
      bool attached = false;
      HIPCHK_RC((ode23_launch<0>(c, a, split ? p : -1, &wg[p][sl], ev, &attached)));
      if (!attached) {
        if (wg[p][sl] == 0)  // the per-packet stage kernels (never split): copy the max
          HIPCHK(c, hipMemcpyAsync(c->o_hmax + sl, c->o_dmax + sl, sizeof(unsigned long long),
                                   hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipEventRecord(ev, st));
      }
    }
    c->o_dmax_cur = (sl + 1) % 3;
    if (P == 2) b_last = sl;  // the extra stream's last work
    *slot = sl;
    return SWRT_OK;
  }
  // the device's first attempt, from its own step size (before the hook)
  int queue_first() { return launch(0, 1, 0.0, 0.0, 0.0, -1, 0.0, 0.0, &first_slot, c->o_coef); }
  int first() const { return first_slot; }
  unsigned workgroups(int p, int sl) const { return wg[p][sl]; }
  // the first attempt the previous call queued (ode23_chain_first): its slot
  // and workgroups; the hook then waits for the first wait_max, so the
  // controller queues its next guess before the hook's host work
  void adopt_first(int sl, const unsigned wg_[2]) {
    first_slot = sl;
    unread[sl] = true;
    if (P == 2) b_last = sl;
    wg[0][sl] = wg_[0];
    wg[1][sl] = wg_[1];
    defer_hook = true;
  }

  int run_hook() {
    // the hook may call the library (e.g. the next QG step on the QG stream);
    // it must not touch the packets (c->in_hook refuses those calls).  Its
    // calls must not join the extra stream's attempt parts into the packet
    // stream (they run on), so the split is hidden from them and re-marked after.
    hook_due = false;
    c->b_pending = 0;
    c->in_hook = true;
    hook(hook_user);
    c->in_hook = false;
    if (split) c->b_pending = 1;
    return SWRT_OK;
  }

  int stage1(double* raw) override {
    if (hook) {
      hook_due = true;
      if (!defer_hook) HIPCHK_RC(run_hook());
    }
    // (the first-step kernel's values: read once its ticket is in, no event wait)
    if (!dev_first || c->o23_markers) HIPCHK(c, hipEventSynchronize(c->o_ev[sl_f1]));
    if (dev_first) {
      HIPCHK_RC(await_shown());
      std::memcpy(raw, &c->o_shown[0], sizeof(double));
    } else
      std::memcpy(raw, c->o_hmax + sl_f1, sizeof(double));
    HIPCHK_RC(dev_err_check(c));
    return global_max(raw);
  }
  // a sharded run: this rank's max -> the max over every rank (the caller's
  // collective, e.g. an RCCL all_reduce), in place
  int global_max(double* v) {
    if (reduce && reduce(v, reduce_user) != 0) return fail(c, SWRT_ERR_STATE, "ode23: the reduce callback failed");
    return SWRT_OK;
  }
  bool first_attempt(double absh, double h, double tnew, const double cf[8], int* slot) override {
    if (!dev_first) return false;
    // the host's computation against the kernel's mapped copy
    bool same = absh == c->o_shown[1] && h == c->o_shown[2] && tnew == c->o_shown[3];
    for (int i = 0; i < 8; ++i) same = same && cf[i] == c->o_shown[4 + i];
    *slot = first_slot;
    return same;  // else left to be overwritten by the attempt queued from the host's values
  }
  int queue(int from, int to, double t, double h, double tnew, int gate_slot, double gate_scale, double gate_limit,
            int* slot) override {
    return launch(from, to, t, h, tnew, gate_slot, gate_scale, gate_limit, slot, nullptr);
  }
  // the raw error max of the attempt in slot sl: the bit-pattern max (= the
  // value max of these non-negative doubles, as the device's atomicMax)
  int wait_max(int sl, double* out) override {
    if (hook_due) HIPCHK_RC(run_hook());
    unread[sl] = false;
    unsigned long long m = 0;
    for (int p = 0; p < P; ++p) {
      const unsigned g = wg[p][sl];
      // The tile launches' maxima are polled in host memory, every workgroup
      // storing its own at its end: no wait for the launch's event, whose
      // host wake-up trailed the kernel by ~10-20 us (the end of an interval
      // waits for it, profiles/r06_ode23).  The per-packet kernels' copied
      // max is read after its event.
      // (polling hipEventQuery instead: 1.802 / 1.831 vs 1.849 / 1.805 ms, noise; profiles/r05_ode23)
      if (g == 0 || c->o23_markers) HIPCHK(c, hipEventSynchronize(p == 0 ? c->o_ev[sl] : c->o_evb[sl]));
      if (g == 0) {
        m = std::max(m, c->o_hmax[sl]);
      } else {
        // (after an event too: the launch's own completion event carries no
        // system-scope release, so a store may land a moment after it)
        const volatile unsigned long long* hp = c->o_hpart + (size_t)(3 * p + sl) * kMaxBins;
        for (unsigned i = 0; i < g; ++i) {
          unsigned long long v = hp[i];
          if (v == kHpartEmpty) HIPCHK_RC(await_hpart(hp + i, p, &v));
          m = std::max(m, v);
        }
      }
    }
    if (c->hz.on) {  // debug: the host-mapped maxima against the device's atomicMax slots
      unsigned long long d = 0;
      for (int p = 0; p < P; ++p) {
        unsigned long long v = 0;
        HIPCHK(c, hipMemcpy(&v, c->o_dmax + 3 * p + sl, sizeof(v), hipMemcpyDeviceToHost));
        d = std::max(d, v);
      }
      if (d != m) return fail(c, SWRT_ERR_STATE, "ode23: host-mapped error max differs from the device's");
    }
    std::memcpy(out, &m, sizeof(double));
    return global_max(out);
  }
  // the first-step launch's values, once its ticket is in shown[12] (its
  // event has completed; the values may land a moment after it)
  void expect_ticket(uint64_t t) { ticket = t; }
  int await_shown() {
    const volatile unsigned long long* tk = reinterpret_cast<const volatile unsigned long long*>(c->o_shown + 12);
    const auto t0 = std::chrono::steady_clock::now();
    while (*tk != ticket) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (*tk != ticket) return fail(c, SWRT_ERR_STATE, "ode23: the first step size never reached host memory");
        break;
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return SWRT_OK;
  }
  int await_hpart(const volatile unsigned long long* e, int p, unsigned long long* out) {
    const auto t0 = std::chrono::steady_clock::now();
    while ((*out = *e) == kHpartEmpty) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) {
        HIPCHK(c, hipStreamSynchronize(p == 0 ? c->stream : c->sx[0]));
        if ((*out = *e) == kHpartEmpty)
          return fail(c, SWRT_ERR_STATE, "ode23: a workgroup's error max never reached host memory");
        break;
      }
    }
    return SWRT_OK;
  }
  // The extra stream's part launches ordered before the packet stream's next
  // work; set `cur` becomes the packets (and F1), the others the spares.
  int finish(int cur, bool failed) override {
    if (split) {
      if (!failed && b_last >= 0 && !c->o23_markers) {
        // the join is the extra stream's last launch's own event (a marker
        // recorded there would put ~7 us between the last attempt and the
        // next work); none once it has completed
        const hipEvent_t ev = c->o_evb[b_last];
        const hipError_t q = hipEventQuery(ev);
        if (q == hipErrorNotReady)
          HIPCHK(c, hipStreamWaitEvent(c->stream0, ev, 0));
        else
          HIPCHK(c, q);
        c->b_pending = 0;
        if (c->hz.on) {
          c->hz.record(ev, 1);
          c->hz.wait(0, ev);
        }
      } else {
        c->b_pending = 1;
        HIPCHK_RC(join_b(c));
      }
    }
    if (failed) HIPCHK(c, hipStreamSynchronize(c->stream));  // a queued guess may still be running
    const int o1 = (cur + 1) % 3, o2 = (cur + 2) % 3;
    c->dx = S[cur].x;
    c->dk = S[cur].k;
    c->oF[0] = S[cur].F;
    c->o_ynx = S[o1].x;
    c->o_ynk = S[o1].k;
    c->oF[3] = S[o1].F;
    c->o_spx = S[o2].x;
    c->o_spk = S[o2].k;
    c->o_spF = S[o2].F;
    c->keys_fresh = false;
    c->cells_sorted = false;
    return SWRT_OK;
  }

 private:
  swrt_ctx* c;
  Ode23Args base;
  bool split;
  int P;
  bool dev_first;
  int sl_f1;
  int first_slot = -1;
  void (*hook)(void*);
  void* hook_user;
  int (*reduce)(double*, void*);
  void* reduce_user;
  bool defer_hook = false, hook_due = false;
  uint64_t ticket = 0;
  int b_last = -1;  // the max slot of the last part-1 launch (its event: the extra stream's last work)
  bool unread[3] = {false, false, false};  // a launch in this slot whose maxima wait_max has not read
  struct Set {
    double *x, *k, *F;
  } S[3];
  unsigned wg[2][3] = {};  // workgroups of each part's launch in each slot (0: the max was copied)
};

// The next call's first step size and first attempt, queued behind the stage
// 1 the chain just queued (slots arranged as that call's 0 / 1): what
// swrt_ode23_run_hooked queues for t0 = 0, tfinal = tmax and `rtol`, on the
// tile path only.  Part 1 of a split attempt stays unjoined (c->chain_b); the
// slots' use mark of this call covers it (c->tail_ev, after sx[0] has waited
// for the packet stream's tail).
int ode23_chain_first(swrt_ctx* c, int sl_f1, double tmax, double f, double Cg, double thr, double bump,
                      double rtol) {
  swrt_ctx::O23Chain& ch = c->o_chain;
  ch.first_q = false;
  const int ntx_ = (int)((c->slot[0].nx + kTile - 1) / kTile);
  if (!c->chain_first || !(use_tile_kernel(c) && c->bin_valid && !c->src_pending && c->nbins == ntx_ * ntx_))
    return SWRT_OK;
  const bool split = ode23_split_ok(c);
  const double t0 = 0.0, tfinal = tmax;
  const double rtol_c = std::max(rtol, 100 * 2.220446049250313e-16);
  const double htspan = std::fabs(tfinal - t0);
  const double hmax = 0.1 * htspan;
  const double c0 = 0.8 * std::pow(rtol_c, 1.0 / 3.0);
  uint64_t ticket = 0;
  HIPCHK_RC(ode23_first_step_queue(c, sl_f1, c0, hmax, htspan, t0, tfinal, split, &ticket));
  if (split) {
    HIPCHK(c, hipStreamWaitEvent(c->sx[0], c->o_ev[sl_f1], 0));
    if (c->hz.on) {
      c->hz.record(c->o_ev[sl_f1], 0);
      c->hz.wait(1, c->o_ev[sl_f1]);
    }
  }
  Ode23Args base;
  int rc;
  if ((rc = ode23_prepare(c, 2, base, tmax, f, Cg, thr, bump))) return rc;
  DeviceExec ex(c, base, split, true, sl_f1, nullptr, nullptr);
  if ((rc = ex.queue_first())) return rc;
  ch.first_ticket = ticket;
  ch.first_slot = ex.first();
  for (int p = 0; p < 2; ++p) ch.first_wg[p] = ex.workgroups(p, ch.first_slot);
  if (split) {
    // one event after both parts: sx[0] waits for part 0's own (attached)
    // event, so no marker lands on the packet stream between the attempt and
    // the next call's next one
    hipEvent_t p0 = c->chain_ev[0];
    if (ch.first_wg[0] != 0 && !c->o23_markers)
      p0 = c->o_ev[ch.first_slot];
    else
      HIPCHK(c, hipEventRecord(p0, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->sx[0], p0, 0));
    HIPCHK(c, hipEventRecord(c->chain_ev[1], c->sx[0]));
    if (c->hz.on) {
      c->hz.record(p0, 0);
      c->hz.wait(1, p0);
    }
    c->tail_ev = c->chain_ev[1];
    c->chain_b = true;
  }
  ch.first_q = true;
  ch.split = split;
  ch.rtol = rtol;
  ch.tfinal = tfinal;
  ch.tmax = tmax;  // (the attempt's alpha = t / tmax; stage 1's alpha(0) does not see it)
  return SWRT_OK;
}
}  // namespace

int swrt_ode23_run_hooked(swrt_ctx* c, double t0, double tfinal, double tmax, double f, double Cg, int nslots,
                          double rtol, double atol, double bump, double* ts_out, int64_t ts_cap, int64_t* nts_out,
                          int64_t* stats3_out, void (*hook)(void*), void* hook_user) {
  return swrt_ode23_run_sharded(c, t0, tfinal, tmax, f, Cg, nslots, rtol, atol, bump, ts_out, ts_cap, nts_out,
                                stats3_out, hook, hook_user, nullptr, nullptr);
}

int swrt_ode23_run_sharded(swrt_ctx* c, double t0, double tfinal, double tmax, double f, double Cg, int nslots,
                           double rtol, double atol, double bump, double* ts_out, int64_t ts_cap, int64_t* nts_out,
                           int64_t* stats3_out, void (*hook)(void*), void* hook_user,
                           int (*reduce)(double*, void*), void* reduce_user) {
  if (!c) return SWRT_ERR_ARG;
  if (!ts_out || ts_cap < 1 || !nts_out) return fail(c, SWRT_ERR_ARG, "ts_out / ts_cap / nts_out");
  if (c->in_hook) return fail(c, SWRT_ERR_STATE, "an ode23 hook may not start another ode23 call");
  GUARD_BEGIN_KEEP_CHAIN
  HIPCHK_RC(lost_check(c));
  SlotUse slot_use(c, false, kSlots01);
  const double rtol_c = std::max(rtol, 100 * 2.220446049250313e-16);
  const double thr = atol / rtol_c;
  const double htspan = std::fabs(tfinal - t0);
  const double hmax = 0.1 * htspan;
  const double c0 = 0.8 * std::pow(rtol_c, 1.0 / 3.0);
  int rc;
  // stage 1 (with this call's re-binning and in-tile sort), its max in slot
  // sl_f1: queued by the previous call when it was chained to this one
  int sl_f1;
  // the chained first attempt is a candidate if this call asks for the first
  // attempt it assumed; anything else joins its part 1 before touching the packets
  swrt_ctx::O23Chain& ch = c->o_chain;
  const bool first_cand = ch.first_q && same_bits(t0, 0.0) && same_bits(tfinal, ch.tfinal) &&
                          same_bits(tmax, ch.tmax) && same_bits(rtol, ch.rtol);
  ch.first_q = false;
  const bool taken = ode23_chain_take(c, t0, tmax, f, Cg, nslots, thr, bump);
  if (!(taken && first_cand)) HIPCHK_RC(chain_join(c));
  if (taken) {
    sl_f1 = ch.dmax_slot;
    ++ch.taken;
  } else {
    if ((rc = ode23_f1_queue(c, t0, tmax, f, Cg, nslots, thr, bump))) return rc;
    sl_f1 = c->o_dmax_cur;
    c->o_dmax_cur = (sl_f1 + 1) % 3;
  }
  Ode23Args base;
  if ((rc = ode23_prepare(c, nslots, base, tmax, f, Cg, thr, bump))) return rc;
  // The first attempt's step size on the device (ode23_first_step_kernel,
  // the host's own operations), so the attempt is queued behind stage 1
  // without a host round trip; the controller then computes the same and
  // checks it against the kernel's mapped copy (the tile path only: its
  // attempt kernel reads device coefficients).
  // (not in a sharded run: the device would take the first step size from
  // this rank's stage-1 max, the controller takes it from every rank's)
  const int ntx_ = (int)((c->slot[0].nx + kTile - 1) / kTile);
  const bool dev_first =
      !reduce && use_tile_kernel(c) && c->bin_valid && !c->src_pending && c->nbins == ntx_ * ntx_;
  // Two part launches per attempt when the binning allows.
  const bool split = ode23_split_ok(c);
  const bool first_chained = taken && first_cand && dev_first && split == ch.split;
  uint64_t ticket = 0;  // the first-step launch's (dev_first)
  if (first_chained) {
    ticket = ch.first_ticket;
    // queued by the previous call: stage 1, the first step (and stage 1's
    // event after it), the fork and the first attempt, whose part 1 is now
    // this call's pending split
    c->chain_b = false;
    if (split) c->b_pending = 1;
    ++ch.first_taken;
  } else {
    HIPCHK_RC(chain_join(c));
    if (dev_first) {
      HIPCHK_RC(ode23_first_step_queue(c, sl_f1, c0, hmax, htspan, t0, tfinal, split, &ticket));
    } else {
      HIPCHK(c, hipMemcpyAsync(c->o_hmax + sl_f1, c->o_dmax + sl_f1, sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipEventRecord(c->o_ev[sl_f1], c->stream));
    }
    if (split) {
      // the fork is stage 1's own event (one marker in front of the first attempt, not two)
      HIPCHK(c, hipStreamWaitEvent(c->sx[0], c->o_ev[sl_f1], 0));
      if (c->hz.on) {
        c->hz.record(c->o_ev[sl_f1], 0);
        c->hz.wait(1, c->o_ev[sl_f1]);
      }
      c->b_pending = 1;  // joined into the packet stream before anything else reads the packets (join_b)
    }
  }
  DeviceExec ex(c, base, split, dev_first, sl_f1, hook, hook_user, reduce, reduce_user);
  ex.expect_ticket(ticket);
  // the first attempt from the device's coefficients, queued now (or by the
  // previous call); the caller's hook then runs (host work that overlaps
  // stage 1 and this attempt)
  if (first_chained)
    ex.adopt_first(ch.first_slot, ch.first_wg);
  else if (dev_first && (rc = ex.queue_first()))
    return rc;
  O23Stats st;
  int64_t nts = 0;
  rc = ode23_control(ex, t0, tfinal, rtol, atol, ts_out, ts_cap, &nts, &st);
  if (rc == kO23BelowHmin) return fail(c, SWRT_ERR_STATE, "ode23: step size below hmin");
  if (rc) return rc;
  if ((rc = ode23_chain_queue(c, tmax, f, Cg, nslots, thr, bump, rtol, reduce == nullptr))) return rc;
  *nts_out = nts;
  if (stats3_out) {
    stats3_out[0] = st.steps;
    stats3_out[1] = st.failed;
    stats3_out[2] = st.attempts;
  }
  c->o23_last = st;
  c->o23_first_taken += st.first_taken;
  c->o23_guesses_taken += st.guesses_taken[0] + st.guesses_taken[1] + st.guesses_taken[2];
  c->o23_split_runs += split ? 1 : 0;
  return SWRT_OK;
  GUARD_END(c)
}

#ifdef SWRT_PHASE_TIMING
// diagnostic build only (not in include/swrt.h): copy out / clear the tile
// kernel's per-workgroup phase stamps (8 u64 per tile).
int swrt_debug_phases(unsigned long long* out, int ntiles, int clear) {
  if (hipDeviceSynchronize() != hipSuccess) return SWRT_ERR_HIP;
  const size_t bytes = (size_t)ntiles * 8 * sizeof(unsigned long long);
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(swrt::swrt_phase_dbg), bytes, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return SWRT_ERR_HIP;
  if (clear) {
    static unsigned long long zeros[16384 * 8];
    if (hipMemcpyToSymbol(HIP_SYMBOL(swrt::swrt_phase_dbg), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice) != hipSuccess)
      return SWRT_ERR_HIP;
  }
  return SWRT_OK;
}
#endif

}  // extern "C"
