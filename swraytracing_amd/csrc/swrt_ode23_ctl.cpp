// swrt_ode23_ctl.cpp — MATLAB ode23's step-size controller (swrt_ode23_ctl.hpp),
// a host-only translation unit: no HIP header, no device.  swrt_api.hip runs it
// over the device stages (swrt_ode23_run_hooked); swrt_ode23_replay runs it over
// a scripted sequence of raw error maxima, so the CPU tests drive this exact
// code and swraytracing_amd/integrate.py's controller with the same sequence
// (tests/test_ode23_controller.py).
//
// The controller is the restatement of integrate.py ode23_packets operation
// for operation (std::pow is the C pow() Python's float ** calls; min / max
// keep Python's tie order, o23_min / o23_max), plus one device-side economy:
// while the host waits for an attempt's error, the attempt the controller
// will ask for next — if this one is accepted at a first try — is already
// queued, gated on the device (it runs only if err = absh * raw < a limit
// under which the controller's answer is certain without its pow; margins far
// above pow's last bit).  With temp = 1.25 * (err/rtol)^(1/3) the controller
// takes absh/temp when temp > 0.2, else 5*absh, then clamps to MaxStep, so
//   absh == MaxStep:      MaxStep    when err < 0.5119*rtol                   (temp < 1)
//   5*absh >= MaxStep:    MaxStep    when err < 0.999*rtol*(absh/(1.25*MaxStep))^3
//   else:                 5*absh     when err < 0.999*0.004096*rtol           (temp < 0.2)
// (then the clamp to tfinal).  A guess is used only if it is exactly the
// attempt the controller asks for (same state set, t, h, tnew); a wrong one
// costs one empty launch instead of a host round trip per attempt.
#include "swrt_ode23_ctl.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/swrt.h"

namespace swrt {

double o23_spacing(double t) {  // numpy.spacing
  const double a = std::fabs(t);
  const double d = std::nextafter(a, INFINITY) - a;
  return std::signbit(t) ? -d : d;
}

int ode23_control(O23Exec& ex, double t0, double tfinal, double rtol, double atol, double* ts_out, int64_t ts_cap,
                  int64_t* nts_out, O23Stats* st_out) {
  (void)atol;  // enters the stages only (thr = atol/rtol)
  O23Stats st;
  const double tdir = std::copysign(1.0, tfinal - t0);
  const double pw = 1.0 / 3.0;
  rtol = std::max(rtol, 100 * 2.220446049250313e-16);
  const double htspan = std::fabs(tfinal - t0);
  const double hmax = 0.1 * htspan;
  const double c0 = 0.8 * std::pow(rtol, pw);
  double t = t0;
  double raw = 0.0;
  int rc;
  if ((rc = ex.stage1(&raw))) return rc;
  double absh = o23_initial_absh(raw, c0, hmax, htspan, 16 * o23_spacing(t));
  struct Spec {  // an attempt already queued: the device's first one, or a guess
    bool on, ran;
    int slot, from, to, gate;  // gate: -1 the first attempt, else the guess rule (O23Stats::guesses_taken)
    double t, h, tnew;
  } spec{false, false, 0, 0, 0, -1, 0.0, 0.0, 0.0};
  {
    // the device's first attempt stands if it took exactly the controller's
    // first step (always, by construction: the same operations)
    double ab = absh, h1, tn1, cf[8];
    (void)o23_step_head(ab, hmax, 16 * o23_spacing(t), tdir, t, tfinal, h1, tn1);
    o23_coeffs(t, h1, tn1, cf);
    int slot = 0;
    if (ex.first_attempt(ab, h1, tn1, cf, &slot)) spec = {true, true, slot, 0, 1, -1, t, h1, tn1};
  }
  int cur = 0;
  int64_t nts = 0;
  if (ts_cap > 0) ts_out[0] = t;
  ++nts;
  bool done = false;
  while (!done) {
    const double hmin = 16 * o23_spacing(t);
    double h, tnew_head;
    done = o23_step_head(absh, hmax, hmin, tdir, t, tfinal, h, tnew_head);
    bool nofailed = true;
    double tnew, err;
    int to;
    while (true) {
      tnew = t + h * 1.0;
      if (done) tnew = tfinal;
      ++st.attempts;
      int slot;
      if (spec.on && spec.ran && spec.from == cur && spec.t == t && spec.h == h && spec.tnew == tnew) {
        slot = spec.slot;
        to = spec.to;
        if (spec.gate < 0)
          ++st.first_taken;
        else
          ++st.guesses_taken[spec.gate];
      } else {
        to = (cur + 1) % 3;
        if ((rc = ex.queue(cur, to, t, h, tnew, -1, 0.0, 0.0, &slot))) return rc;
      }
      spec.on = false;
      double gate_limit = 0.0;
      if (!done && nofailed) {
        double guess;
        int gate;
        if (absh == hmax) {
          guess = hmax;
          gate_limit = 0.5119 * rtol;
          gate = 0;
        } else if (5.0 * absh >= hmax) {
          guess = hmax;
          const double r = absh / (1.25 * hmax);
          gate_limit = 0.999 * rtol * (r * r * r);
          gate = 1;
        } else {
          guess = 5.0 * absh;
          gate_limit = 0.999 * 0.004096 * rtol;
          gate = 2;
        }
        const double t2 = tnew;
        double absh2 = guess, h2, tnew2;
        (void)o23_step_head(absh2, hmax, 16 * o23_spacing(t2), tdir, t2, tfinal, h2, tnew2);
        const int sto = 3 - cur - to;
        int sl2;
        if ((rc = ex.queue(to, sto, t2, h2, tnew2, slot, absh, gate_limit, &sl2))) return rc;
        ++st.guesses;
        spec = {true, false, sl2, to, sto, gate, t2, h2, tnew2};
      }
      if ((rc = ex.wait_max(slot, &raw))) return rc;
      err = absh * raw;
      spec.ran = spec.on && err < gate_limit;  // the device's gate, the same operation
      h = tnew - t;
      if (err > rtol) {
        ++st.failed;
        if (absh <= hmin) {
          if ((rc = ex.finish(cur, true))) return rc;
          st.steps = nts - 1;
          if (st_out) *st_out = st;
          if (nts_out) *nts_out = nts;
          return kO23BelowHmin;
        }
        if (nofailed) {
          nofailed = false;
          absh = std::max(hmin, absh * std::max(0.5, 0.8 * std::pow(rtol / err, pw)));
        } else {
          absh = std::max(hmin, 0.5 * absh);
        }
        h = tdir * absh;
        done = false;
      } else {
        break;
      }
    }
    cur = to;  // accept: y = ynew, F1 = F4
    t = tnew;
    // ts_cap bounds the times recorded, never the integration: the interval
    // always completes and *nts_out counts every accepted time
    if (nts < ts_cap) ts_out[nts] = t;
    ++nts;
    if (done) break;
    if (nofailed) {
      const double temp = 1.25 * std::pow(err / rtol, pw);
      absh = temp > 0.2 ? absh / temp : 5.0 * absh;
    }
  }
  // everything queued has finished: the last attempt (done) queues no guess,
  // and every earlier guess precedes it on its stream
  if ((rc = ex.finish(cur, false))) return rc;
  st.steps = nts - 1;
  if (st_out) *st_out = st;
  if (nts_out) *nts_out = nts;
  return 0;
}

namespace {
// The stages replaced by a script: raw[0] is stage 1's max, raw[1..] the
// maxima of the attempts in the order the controller consumes them.  A guess
// the controller consumes must be one the device would have run (its gate
// passes on the raw max of the attempt it is gated on); `gate_violations`
// counts any that would not.
class ScriptExec final : public O23Exec {
 public:
  ScriptExec(const double* raw, int64_t nraw, bool dev_first, double t0, double tfinal, double rtol, double* log,
             int64_t log_cap)
      : raw_(raw), nraw_(nraw), dev_first_(dev_first), t0_(t0), tfinal_(tfinal), rtol_(rtol), log_(log),
        log_cap_(log_cap) {}
  int stage1(double* raw) override {
    if (nraw_ < 1) return SWRT_ERR_ARG;
    *raw = raw_[0];
    return 0;
  }
  bool first_attempt(double absh, double h, double tnew, const double cf[8], int* slot) override {
    if (!dev_first_) return false;
    // what ode23_first_step_kernel computes from stage 1's max
    const double rtol = std::max(rtol_, 100 * 2.220446049250313e-16);
    const double htspan = std::fabs(tfinal_ - t0_), hmax = 0.1 * htspan;
    double ab = o23_initial_absh(raw_[0], 0.8 * std::pow(rtol, 1.0 / 3.0), hmax, htspan, 16 * o23_spacing(t0_));
    double h1, tn1, c[8];
    (void)o23_step_head(ab, hmax, 16 * o23_spacing(t0_), std::copysign(1.0, tfinal_ - t0_), t0_, tfinal_, h1, tn1);
    o23_coeffs(t0_, h1, tn1, c);
    q_.push_back({t0_, h1, tn1, -1, 0.0, 0.0, 0.0, false});
    *slot = (int)q_.size() - 1;
    bool same = ab == absh && h1 == h && tn1 == tnew;
    for (int i = 0; i < 8; ++i) same = same && c[i] == cf[i];
    return same;
  }
  int queue(int from, int to, double t, double h, double tnew, int gate_slot, double gate_scale, double gate_limit,
            int* slot) override {
    (void)from;
    (void)to;
    q_.push_back({t, h, tnew, gate_slot, gate_scale, gate_limit, 0.0, false});
    *slot = (int)q_.size() - 1;
    return 0;
  }
  int wait_max(int slot, double* raw) override {
    if (slot < 0 || slot >= (int)q_.size()) return SWRT_ERR_STATE;
    Q& a = q_[slot];
    if (a.gate_slot >= 0) {
      const Q& g = q_[a.gate_slot];
      if (!g.done || !(a.gate_scale * g.raw < a.gate_limit)) ++gate_violations;
    }
    if (next_ >= nraw_) return SWRT_ERR_ARG;  // the script ran out
    a.raw = raw_[next_++];
    a.done = true;
    if (nlog < log_cap_) {
      log_[4 * nlog] = a.t;
      log_[4 * nlog + 1] = a.h;
      log_[4 * nlog + 2] = a.tnew;
      log_[4 * nlog + 3] = a.raw;
    }
    ++nlog;
    *raw = a.raw;
    return 0;
  }
  int finish(int, bool) override { return 0; }
  int64_t nlog = 0, gate_violations = 0;

 private:
  struct Q {
    double t, h, tnew;
    int gate_slot;
    double gate_scale, gate_limit, raw;
    bool done;
  };
  const double* raw_;
  int64_t nraw_, next_ = 1;
  bool dev_first_;
  double t0_, tfinal_, rtol_;
  double* log_;
  int64_t log_cap_;
  std::vector<Q> q_;
};
}  // namespace

}  // namespace swrt

extern "C" int swrt_ode23_replay(double t0, double tfinal, double rtol, double atol, int dev_first,
                                 const double* raw, int64_t nraw, double* log_out, int64_t log_cap,
                                 int64_t* nlog_out, double* ts_out, int64_t ts_cap, int64_t* nts_out,
                                 int64_t* stats9_out) {
  if (!raw || nraw < 1 || (log_cap > 0 && !log_out) || (ts_cap > 0 && !ts_out) || !nlog_out || !nts_out)
    return SWRT_ERR_ARG;
  try {
    swrt::ScriptExec ex(raw, nraw, dev_first != 0, t0, tfinal, rtol, log_out, log_cap);
    swrt::O23Stats st;
    *nts_out = 0;
    const int rc = swrt::ode23_control(ex, t0, tfinal, rtol, atol, ts_out, ts_cap, nts_out, &st);
    *nlog_out = ex.nlog;
    if (stats9_out) {
      const int64_t v[9] = {st.steps,         st.failed,           st.attempts,         st.first_taken,
                            st.guesses,       st.guesses_taken[0], st.guesses_taken[1], st.guesses_taken[2],
                            ex.gate_violations};
      std::memcpy(stats9_out, v, sizeof(v));
    }
    return rc == swrt::kO23BelowHmin ? SWRT_ERR_STATE : rc;
  } catch (...) {
    return SWRT_ERR_ALLOC;
  }
}
