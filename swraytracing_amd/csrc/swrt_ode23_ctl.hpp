// swrt_ode23_ctl.hpp — MATLAB ode23's step-size controller (qgsw_raytrace.m:149,
// qg2layersw_raytrace.m:195: RelTol 1e-3, AbsTol 1e-6, MaxStep 0.1*|tspan|,
// max-norm error, initial-step heuristic, step update), GPU-free.
//
// Two parts:
//  * the step-size arithmetic shared by the host controller and the device's
//    first-step kernel (ode23_first_step_kernel, swrt_ode23.hpp): the same
//    source, the same IEEE operations on both sides;
//  * ode23_control (swrt_ode23_ctl.cpp, a plain C++ translation unit): the
//    controller loop of swraytracing_amd/integrate.py ode23_packets, operation
//    for operation, driving an O23Exec — the device stages (swrt_api.hip's
//    DeviceExec) or a scripted error sequence (swrt_ode23_replay, which the
//    CPU tests compare with the Python controller fed the same sequence).
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIP__)
#define SWRT_HD __host__ __device__
#else
#define SWRT_HD
#endif

namespace swrt {

// std::min(a, b) = b < a ? b : a, std::max(a, b) = a < b ? b : a, spelled out
// so host and device pick the same operand (Python's min/max tie order too)
SWRT_HD inline double o23_min(double a, double b) { return b < a ? b : a; }
SWRT_HD inline double o23_max(double a, double b) { return a < b ? b : a; }
// the initial step from stage 1's raw max (c0 = 0.8 * rtol^(1/3))
SWRT_HD inline double o23_initial_absh(double raw, double c0, double hmax, double htspan, double hmin0) {
  const double rh = raw / c0;
  double absh = o23_min(hmax, htspan);
  if (absh * rh > 1) absh = 1.0 / rh;
  return o23_max(absh, hmin0);
}
// the loop head: clamp absh, h, and the final-step rule; returns done
SWRT_HD inline bool o23_step_head(double& absh, double hmax, double hmin, double tdir, double t, double tfinal,
                                  double& h, double& tnew) {
  absh = o23_min(hmax, o23_max(hmin, absh));
  h = tdir * absh;
  bool done = false;
  if (1.1 * absh >= fabs(tfinal - t)) {
    h = tfinal - t;
    absh = fabs(h);
    done = true;
  }
  tnew = t + h * 1.0;
  if (done) tnew = tfinal;
  return done;
}
// an attempt's stage times and coefficients {ts, c0, ts3, c3, ts4, c4[0..2]}:
// f(:,2) at t + h*A(1), y + f*hB(:,1); f(:,3) at t + h*A(2), y + f*hB(:,2);
// h4 = tnew - t; ynew = y + f*hB(:,3); f(:,4) at tnew
SWRT_HD inline void o23_coeffs(double t, double h, double tnew, double out[8]) {
  out[0] = t + h * 0.5;
  out[1] = h * 0.5;
  out[2] = t + h * 0.75;
  out[3] = h * 0.75;
  const double h4 = tnew - t;
  out[4] = tnew;
  out[5] = h4 * (2.0 / 9.0);
  out[6] = h4 * (1.0 / 3.0);
  out[7] = h4 * (4.0 / 9.0);
}

// numpy.spacing(t): the controller's hmin = 16 * spacing(t)
double o23_spacing(double t);

// What the controller asks of whoever runs the stages.  State sets: an
// attempt reads set `from` (y, F1) and writes ynew and F4 into set `to`; the
// accepted set becomes the current one.  Three sets, so a guessed next
// attempt can be queued while the current one runs.
class O23Exec {
 public:
  virtual ~O23Exec() = default;
  // stage 1's raw max (max |F1| / max(|y|, thr)), once it is known
  virtual int stage1(double* raw) = 0;
  // The first attempt queued before stage 1's max reached the host (the
  // device's own step size, ode23_first_step_kernel), from set 0 into set 1:
  // true (and its max slot) if it exists and took exactly this step.
  virtual bool first_attempt(double absh, double h, double tnew, const double cf[8], int* slot) = 0;
  // Queue an attempt at (t, h, tnew).  gate_slot >= 0: a guess, run only if
  // gate_scale * (the raw max of gate_slot's attempt) < gate_limit (the device
  // evaluates it; every workgroup returns at once otherwise).  *slot: where
  // its max lands.
  virtual int queue(int from, int to, double t, double h, double tnew, int gate_slot, double gate_scale,
                    double gate_limit, int* slot) = 0;
  // the raw error max of the attempt in `slot`, once it has run
  virtual int wait_max(int slot, double* raw) = 0;
  // the controller is done (failed: below hmin): set `cur` holds the packets
  virtual int finish(int cur, bool failed) = 0;
};

struct O23Stats {
  int64_t steps = 0, failed = 0, attempts = 0;
  int64_t first_taken = 0;      // the device's first attempt was the controller's first
  int64_t guesses = 0;          // guessed next attempts queued
  int64_t guesses_taken[3] = {0, 0, 0};  // ... and consumed, by gate: MaxStep at MaxStep, MaxStep from 5*absh, 5*absh
};

constexpr int kO23BelowHmin = -1;  // ode23_control's code for MATLAB's "unable to meet integration tolerances"

// [~, y] = ode23(odefun, [t0 tfinal], y0)'s controller over `ex`.  Writes the
// accepted times (t0 first) to ts_out[0 .. min(nts, ts_cap)); *nts_out counts
// every one.  Returns 0, an executor's nonzero code, or kO23BelowHmin.
int ode23_control(O23Exec& ex, double t0, double tfinal, double rtol, double atol, double* ts_out, int64_t ts_cap,
                  int64_t* nts_out, O23Stats* st);

}  // namespace swrt
