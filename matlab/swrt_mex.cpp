// swrt_mex.cpp — MATLAB MEX gateway over the swrt C ABI (include/swrt.h).
//
// The reference-side binding a maintainer adds to ndefilippis/SWRaytracing so
// that SpectralScheme / ode_symplectic / interpolate_U / ode23 callers run on
// the MI355X.  Deliberately thin: argument marshalling only, every error is
// raised with mexErrMsgIdAndTxt AFTER the C call has returned (never from HIP
// code).
//
// Contexts are handles: h = swrt_mex('create', device) opens one library
// context (its own field slots, packets and streams) and every other command
// takes h as its second argument, so independent objects — two
// SpectralSchemeGPU instances, a scheme and a QG run — never share fields
// (each SpectralScheme owns its fields, SpectralScheme.m:28-35).
// Build (MATLAB R2018a+, interleaved complex):
//   mex -R2018a -I../include swrt_mex.cpp -L../swraytracing_amd -lswrt
// Usage (see SpectralSchemeGPU.m, ode_symplectic_gpu.m, ode23_packets_gpu.m):
//   h = swrt_mex('create', device);   swrt_mex('destroy', h)    % through SwrtContext (a handle class)
//   n = swrt_mex('live')                                        % open contexts
//   swrt_mex('set_field_psi', h, slot, psi_grid, L)           % SpectralScheme ctor
//   swrt_mex('set_field_qk', h, slot, qk, L, K_d2, shear, kscale, ny_period)   % grid_U
//   swrt_mex('set_field_grid', h, slot, u, v, ux, uy, vx, vy, L, ny_period)
//   swrt_mex('set_field_q', h, slot, q_grid, L, K_d2, shear, kscale, ny_period)   % grid_U(g2k(q)), read_field frame
//   swrt_mex('advance_intervals', h, dts, nsub, f, gH, alpha0, dalpha, bump)       % slots 0..numel(dts)
//   swrt_mex('set_locality', h, rebin_every, tile)
//   F6  = swrt_mex('get_fields', h, slot, nx)                 % nx x nx x 6: u v u_x u_y v_x v_y
//   psi = swrt_mex('get_psi', h, slot, nx)                    % k2g(g2k(psi)) of set_field_psi
//   out = swrt_mex('eval', h, x, y, nslots, alpha, bump)      % n x 6 (U, grad U per column)
//   FI  = swrt_mex('interpolate', h, x, y, F, dx, dy, bump)   % interpolate.m
//   [x, k, hx, hk] = swrt_mex('leapfrog', h, x0, k0, dt, nsteps, f, gH, nslots, alpha0, dalpha, bump, save_every)
//   fk = swrt_mex('g2k', h, fg);  fg = swrt_mex('k2g', h, fk);
//   swrt_mex('packets_set', h, x, k);  [x, k] = swrt_mex('packets_get', h);
//   swrt_mex('advance', h, dt, nsteps, f, gH, nslots, alpha0, dalpha, bump)
//   rh  = swrt_mex('ode23_f1', h, t, tmax, f, Cg, nslots, thr, bump)       % ode23_packets_gpu.m
//   err = swrt_mex('ode23_attempt', h, t, hstep, tnew, tmax, f, Cg, nslots, thr, bump)
//   swrt_mex('ode23_accept', h)
//   swrt_mex('qg_init', h, params_struct, qk)   % qk (2kmax+1) x (kmax+1) [x 2], complex
//   swrt_mex('qg_step', h, dt, nsteps);  U0 = swrt_mex('qg_max_speed', h);
//   [qk, t, steps] = swrt_mex('qg_get', h, nx, nlayers);  q = swrt_mex('qg_get_q', h, nx, nlayers);
//   swrt_mex('qg_snapshot', h, slot, which, layer, ny_period);  swrt_mex('swap_slots', h, a, b)
//   tf = swrt_mex('field_div_free', h, slot)   % v_y == -u_x exactly (five-sum kernels)
#include <cstring>
#include <string>
#include <vector>

#include "mex.h"
#include "swrt.h"

static std::vector<swrt_ctx*> g_ctx;  // handle h = index + 1; closed handles hold nullptr

static void cleanup() {
  for (swrt_ctx*& c : g_ctx)
    if (c) {
      swrt_destroy(c);
      c = nullptr;
    }
  g_ctx.clear();
}

static size_t live_contexts() {
  size_t n = 0;
  for (swrt_ctx* c : g_ctx) n += c != nullptr;
  return n;
}

static double scalar(const mxArray* a) { return mxGetScalar(a); }

static swrt_ctx* handle(int nrhs, const mxArray* prhs[]) {
  if (nrhs < 2 || mxGetNumberOfElements(prhs[1]) != 1)
    mexErrMsgIdAndTxt("swrt:arg", "second argument: the context handle from swrt_mex('create', device)");
  const double h = scalar(prhs[1]);
  const size_t i = (size_t)h;
  if (h < 1 || (double)i != h || i > g_ctx.size() || g_ctx[i - 1] == nullptr)
    mexErrMsgIdAndTxt("swrt:state", "invalid or closed context handle %g", h);
  return g_ctx[i - 1];
}

static void check(swrt_ctx* c, int rc, const char* what) {
  if (rc != SWRT_OK) {
    const std::string msg = std::string(what) + ": " + swrt_last_error(c);
    mexErrMsgIdAndTxt("swrt:call", "%s (code %d)", msg.c_str(), rc);
  }
}

static const double* reals(const mxArray* a, const char* name) {
  if (!mxIsDouble(a) || mxIsComplex(a)) mexErrMsgIdAndTxt("swrt:arg", "%s must be real double", name);
  return mxGetDoubles(a);
}

static const double* complexes(const mxArray* a, const char* name) {
  if (!mxIsDouble(a) || !mxIsComplex(a)) mexErrMsgIdAndTxt("swrt:arg", "%s must be complex double", name);
  return (const double*)mxGetComplexDoubles(a);  // interleaved re, im (R2018a API)
}

static void need(int nrhs, int n, const char* cmd) {
  if (nrhs < n) mexErrMsgIdAndTxt("swrt:arg", "%s: expected %d arguments after the command", cmd, n - 1);
}

// The library's own grid sizes size every output (a caller's nx that does not
// match is an error, never a buffer size).
static int64_t slot_grid(swrt_ctx* c, int slot, int64_t nx_arg) {
  const int64_t nx = swrt_field_grid(c, slot);
  if (nx < 0) mexErrMsgIdAndTxt("swrt:state", "field slot %d is not set", slot);
  if (nx_arg != nx) mexErrMsgIdAndTxt("swrt:arg", "slot %d holds a %lld^2 grid, not %lld^2", slot, (long long)nx,
                                      (long long)nx_arg);
  return nx;
}

static int64_t qg_grid(swrt_ctx* c, int64_t nx_arg, int nl_arg, int* nl) {
  const int64_t nx = swrt_qg_grid(c, nl);
  if (nx < 0) mexErrMsgIdAndTxt("swrt:state", "swrt_qg_init not called");
  if (nx_arg != nx || nl_arg != *nl)
    mexErrMsgIdAndTxt("swrt:arg", "the QG state is %lld x %lld x %d, not %lld x %lld x %d", (long long)nx,
                      (long long)nx, *nl, (long long)nx_arg, (long long)nx_arg, nl_arg);
  return nx;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs < 1 || !mxIsChar(prhs[0])) mexErrMsgIdAndTxt("swrt:arg", "first argument: command");
  char cmd[64];
  mxGetString(prhs[0], cmd, sizeof(cmd));

  if (!strcmp(cmd, "create")) {  // (device) -> h
    const int dev = nrhs > 1 ? (int)scalar(prhs[1]) : 0;
    swrt_ctx* c = nullptr;
    const int rc = swrt_create(dev, &c);
    if (rc != SWRT_OK) mexErrMsgIdAndTxt("swrt:create", "swrt_create failed (code %d)", rc);
    if (g_ctx.empty()) mexAtExit(cleanup);
    if (live_contexts() == 0) mexLock();  // stay loaded while a context is open
    g_ctx.push_back(c);  // handles are never reused: a stale copy of a closed one fails, never aliases
    plhs[0] = mxCreateDoubleScalar((double)g_ctx.size());
    return;
  }
  if (!strcmp(cmd, "live")) {  // () -> number of open contexts (SwrtContext lifetime tests)
    plhs[0] = mxCreateDoubleScalar((double)live_contexts());
    return;
  }
  swrt_ctx* c = handle(nrhs, prhs);
  const mxArray** a = prhs + 1;  // a[1] = first argument after the handle
  const int na = nrhs - 1;

  if (!strcmp(cmd, "destroy")) {  // SwrtContext.delete: the last reference to a context is gone
    swrt_destroy(c);
    g_ctx[(size_t)scalar(prhs[1]) - 1] = nullptr;
    if (live_contexts() == 0) mexUnlock();  // `clear mex` may unload the gateway again
    return;
  }
  if (!strcmp(cmd, "set_field_psi")) {  // (slot, psi, L)
    need(na, 4, cmd);
    const int64_t nx = (int64_t)mxGetM(a[2]);
    check(c, swrt_set_field_psi(c, (int)scalar(a[1]), reals(a[2], "psi"), nx, scalar(a[3])), "swrt_set_field_psi");
    return;
  }
  if (!strcmp(cmd, "set_field_qk")) {  // (slot, qk, L, K_d2, shear, kscale, ny_period)
    need(na, 8, cmd);
    const int64_t nx = (int64_t)mxGetM(a[2]) + 1;
    check(c, swrt_set_field_qk(c, (int)scalar(a[1]), complexes(a[2], "qk"), nx, scalar(a[3]), scalar(a[4]),
                               scalar(a[5]), scalar(a[6]), (int64_t)scalar(a[7])),
          "swrt_set_field_qk");
    return;
  }
  if (!strcmp(cmd, "set_field_q")) {  // (slot, q nx x nx, L, K_d2, shear, kscale, ny_period)
    need(na, 8, cmd);
    const int64_t nx = (int64_t)mxGetM(a[2]);
    if ((int64_t)mxGetN(a[2]) != nx) mexErrMsgIdAndTxt("swrt:arg", "q must be an nx x nx frame");
    check(c, swrt_set_field_q(c, (int)scalar(a[1]), reals(a[2], "q"), nx, scalar(a[3]), scalar(a[4]), scalar(a[5]),
                              scalar(a[6]), (int64_t)scalar(a[7])),
          "swrt_set_field_q");
    return;
  }
  if (!strcmp(cmd, "set_field_grid")) {  // (slot, u, v, ux, uy, vx, vy, L, ny_period)
    need(na, 10, cmd);
    const int64_t nx = (int64_t)mxGetM(a[2]);
    const size_t plane = (size_t)(nx * nx);
    for (int f = 0; f < 6; ++f)
      if (mxGetNumberOfElements(a[2 + f]) != plane) mexErrMsgIdAndTxt("swrt:arg", "fields must all be nx x nx");
    mxArray* tmp = mxCreateDoubleMatrix(plane, 6, mxREAL);  // 6 planes, MATLAB-owned scratch
    double* d = mxGetDoubles(tmp);
    for (int f = 0; f < 6; ++f) memcpy(d + f * plane, reals(a[2 + f], "field"), plane * sizeof(double));
    const int rc = swrt_set_field_grid(c, (int)scalar(a[1]), d, nx, scalar(a[8]), (int64_t)scalar(a[9]));
    mxDestroyArray(tmp);
    check(c, rc, "swrt_set_field_grid");
    return;
  }
  if (!strcmp(cmd, "get_fields")) {  // (slot, nx) -> nx x nx x 6
    need(na, 3, cmd);
    const int64_t nx = slot_grid(c, (int)scalar(a[1]), (int64_t)scalar(a[2]));
    const mwSize dims[3] = {(mwSize)nx, (mwSize)nx, 6};
    plhs[0] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
    check(c, swrt_get_field_grid(c, (int)scalar(a[1]), mxGetDoubles(plhs[0])), "swrt_get_field_grid");
    return;
  }
  if (!strcmp(cmd, "get_psi")) {  // (slot, nx) -> nx x nx
    need(na, 3, cmd);
    const int64_t nx = slot_grid(c, (int)scalar(a[1]), (int64_t)scalar(a[2]));
    plhs[0] = mxCreateDoubleMatrix((mwSize)nx, (mwSize)nx, mxREAL);
    check(c, swrt_get_psi_grid(c, (int)scalar(a[1]), mxGetDoubles(plhs[0])), "swrt_get_psi_grid");
    return;
  }
  if (!strcmp(cmd, "eval")) {  // (x, y, nslots, alpha, bump) -> n x 6
    need(na, 6, cmd);
    const size_t n = mxGetNumberOfElements(a[1]);
    if (mxGetNumberOfElements(a[2]) != n) mexErrMsgIdAndTxt("swrt:arg", "x and y must have the same size");
    plhs[0] = mxCreateDoubleMatrix(n, 6, mxREAL);  // 6 x n row blocks == n x 6 column-major
    check(c, swrt_eval(c, reals(a[1], "x"), reals(a[2], "y"), (int64_t)n, (int)scalar(a[3]), scalar(a[4]),
                       scalar(a[5]), mxGetDoubles(plhs[0])),
          "swrt_eval");
    return;
  }
  if (!strcmp(cmd, "interpolate")) {  // (x, y, F, dx, dy, bump)
    need(na, 7, cmd);
    const mxArray* F = a[3];
    const int64_t nx = (int64_t)mxGetM(F);
    const int64_t nyF = (int64_t)(mxGetNumberOfElements(F) / mxGetM(F));
    const size_t n = mxGetNumberOfElements(a[1]);
    plhs[0] = mxCreateNumericArray(mxGetNumberOfDimensions(a[1]), mxGetDimensions(a[1]), mxDOUBLE_CLASS, mxREAL);
    check(c, swrt_interpolate(c, reals(F, "F"), nx, nyF, scalar(a[4]), scalar(a[5]), scalar(a[6]),
                              reals(a[1], "x"), reals(a[2], "y"), (int64_t)n, mxGetDoubles(plhs[0])),
          "swrt_interpolate");
    return;
  }
  if (!strcmp(cmd, "leapfrog")) {
    // (x0 Nx2, k0 Nx2, dt, nsteps, f, gH, nslots, alpha0, dalpha, bump, save_every)
    need(na, 11, cmd);
    const int64_t n = (int64_t)mxGetM(a[1]);
    if (mxGetN(a[1]) != 2 || mxGetM(a[2]) != (size_t)n || mxGetN(a[2]) != 2)
      mexErrMsgIdAndTxt("swrt:arg", "x0 and k0 must be N x 2");
    const int64_t nsteps = (int64_t)scalar(a[4]);
    const int64_t save_every = na > 11 ? (int64_t)scalar(a[11]) : 0;
    plhs[0] = mxDuplicateArray(a[1]);
    plhs[1] = mxDuplicateArray(a[2]);
    double *hx = nullptr, *hk = nullptr;
    if (nlhs > 2 && save_every > 0) {
      const mwSize dims[3] = {(mwSize)n, 2, (mwSize)(nsteps / save_every)};  // frames of N x 2
      plhs[2] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
      plhs[3] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
      hx = mxGetDoubles(plhs[2]);
      hk = mxGetDoubles(plhs[3]);
    }
    check(c, swrt_leapfrog(c, mxGetDoubles(plhs[0]), mxGetDoubles(plhs[1]), n, scalar(a[3]), nsteps, scalar(a[5]),
                           scalar(a[6]), (int)scalar(a[7]), scalar(a[8]), scalar(a[9]), scalar(a[10]),
                           hx ? save_every : 0, hx, hk),
          "swrt_leapfrog");
    return;
  }
  if (!strcmp(cmd, "g2k")) {
    need(na, 2, cmd);
    const int64_t nx = (int64_t)mxGetM(a[1]);
    const int64_t kmax = nx / 2 - 1;
    plhs[0] = mxCreateDoubleMatrix(2 * kmax + 1, kmax + 1, mxCOMPLEX);
    check(c, swrt_g2k(c, reals(a[1], "fg"), nx, (double*)mxGetComplexDoubles(plhs[0])), "swrt_g2k");
    return;
  }
  if (!strcmp(cmd, "k2g")) {
    need(na, 2, cmd);
    const int64_t nx = (int64_t)mxGetM(a[1]) + 1;
    const double* fk = complexes(a[1], "fk");
    plhs[0] = mxCreateDoubleMatrix(nx, nx, mxREAL);
    check(c, swrt_k2g(c, fk, nx, mxGetDoubles(plhs[0])), "swrt_k2g");
    return;
  }
  if (!strcmp(cmd, "packets_set")) {  // (x Nx2, k Nx2)
    need(na, 3, cmd);
    check(c, swrt_packets_set(c, reals(a[1], "x"), reals(a[2], "k"), (int64_t)mxGetM(a[1])), "swrt_packets_set");
    return;
  }
  if (!strcmp(cmd, "packets_get")) {
    const int64_t n = swrt_packets_count(c);
    plhs[0] = mxCreateDoubleMatrix((mwSize)n, 2, mxREAL);
    plhs[1] = mxCreateDoubleMatrix((mwSize)n, 2, mxREAL);
    check(c, swrt_packets_get(c, mxGetDoubles(plhs[0]), mxGetDoubles(plhs[1])), "swrt_packets_get");
    return;
  }
  if (!strcmp(cmd, "advance")) {  // (dt, nsteps, f, gH, nslots, alpha0, dalpha, bump)
    need(na, 9, cmd);
    check(c, swrt_advance(c, scalar(a[1]), (int64_t)scalar(a[2]), scalar(a[3]), scalar(a[4]), (int)scalar(a[5]),
                          scalar(a[6]), scalar(a[7]), scalar(a[8]), 0),
          "swrt_advance");
    return;
  }
  if (!strcmp(cmd, "advance_intervals")) {  // (dts, nsub, f, gH, alpha0, dalpha, bump)
    need(na, 8, cmd);
    const int nint = (int)mxGetNumberOfElements(a[1]);
    check(c, swrt_advance_intervals(c, nint, reals(a[1], "dts"), (int64_t)scalar(a[2]), scalar(a[3]), scalar(a[4]),
                                    scalar(a[5]), scalar(a[6]), scalar(a[7]), 0),
          "swrt_advance_intervals");
    return;
  }
  if (!strcmp(cmd, "set_locality")) {  // (rebin_every, tile)
    need(na, 3, cmd);
    check(c, swrt_set_locality(c, (int64_t)scalar(a[1]), (int64_t)scalar(a[2])), "swrt_set_locality");
    return;
  }
  if (!strcmp(cmd, "ode23_f1")) {  // (t, tmax, f, Cg, nslots, thr, bump) -> rh_raw
    need(na, 8, cmd);
    double r = 0.0;
    check(c, swrt_ode23_f1(c, scalar(a[1]), scalar(a[2]), scalar(a[3]), scalar(a[4]), (int)scalar(a[5]),
                           scalar(a[6]), scalar(a[7]), &r),
          "swrt_ode23_f1");
    plhs[0] = mxCreateDoubleScalar(r);
    return;
  }
  if (!strcmp(cmd, "ode23_attempt")) {  // (t, h, tnew, tmax, f, Cg, nslots, thr, bump) -> err_raw
    need(na, 10, cmd);
    double r = 0.0;
    check(c, swrt_ode23_attempt(c, scalar(a[1]), scalar(a[2]), scalar(a[3]), scalar(a[4]), scalar(a[5]),
                                scalar(a[6]), (int)scalar(a[7]), scalar(a[8]), scalar(a[9]), &r),
          "swrt_ode23_attempt");
    plhs[0] = mxCreateDoubleScalar(r);
    return;
  }
  if (!strcmp(cmd, "ode23_accept")) {
    check(c, swrt_ode23_accept(c), "swrt_ode23_accept");
    return;
  }
  if (!strcmp(cmd, "qg_init")) {  // (params struct, qk complex (2kmax+1) x (kmax+1) [x nlayers])
    need(na, 3, cmd);
    const mxArray* s = a[1];
    auto fld = [&](const char* name, double dflt) {
      const mxArray* v = mxGetField(s, 0, name);
      return v ? mxGetScalar(v) : dflt;
    };
    swrt_qg_params p;
    p.nlayers = (int)fld("nlayers", 1);
    p.filter = (int)fld("filter", 1);
    p.L = fld("L", 6.283185307179586);
    p.K_d2 = fld("K_d2", 1.0);
    p.beta = fld("beta", 0.0);
    p.r_drag = fld("r_drag", 0.0);
    p.force_strength = fld("force_strength", 0.0);
    p.f = fld("f", 1.0);
    p.Cg = fld("Cg", 1.0);
    p.shear = fld("shear", 0.0);
    p.nu = fld("nu", 0.0);
    p.hyper_order = fld("hyper_order", 4.0);
    p.r = fld("r", 0.0);
    const int64_t nx = (int64_t)mxGetM(a[2]) + 1;
    check(c, swrt_qg_init(c, &p, nx, complexes(a[2], "qk")), "swrt_qg_init");
    return;
  }
  if (!strcmp(cmd, "qg_step")) {  // (dt, nsteps)
    need(na, 2, cmd);
    check(c, swrt_qg_step(c, scalar(a[1]), na > 2 ? (int64_t)scalar(a[2]) : 1), "swrt_qg_step");
    return;
  }
  if (!strcmp(cmd, "qg_max_speed")) {
    double u = 0.0;
    check(c, swrt_qg_max_speed(c, &u), "swrt_qg_max_speed");
    plhs[0] = mxCreateDoubleScalar(u);
    return;
  }
  if (!strcmp(cmd, "qg_get")) {  // (nx, nlayers) -> qk, t, steps
    need(na, 3, cmd);
    double t = 0.0;
    int64_t steps = 0;
    int nl = 0;
    const int64_t nx = qg_grid(c, (int64_t)scalar(a[1]), (int)scalar(a[2]), &nl);
    const mwSize dims[3] = {(mwSize)(nx - 1), (mwSize)(nx / 2), (mwSize)nl};
    plhs[0] = mxCreateNumericArray(nl > 1 ? 3 : 2, dims, mxDOUBLE_CLASS, mxCOMPLEX);
    check(c, swrt_qg_get(c, (double*)mxGetComplexDoubles(plhs[0]), &t, &steps), "swrt_qg_get");
    if (nlhs > 1) plhs[1] = mxCreateDoubleScalar(t);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar((double)steps);
    return;
  }
  if (!strcmp(cmd, "qg_get_q")) {  // (nx, nlayers) -> q nx x nx [x nlayers]
    need(na, 3, cmd);
    int nl = 0;
    const int64_t nx = qg_grid(c, (int64_t)scalar(a[1]), (int)scalar(a[2]), &nl);
    const mwSize dims[3] = {(mwSize)nx, (mwSize)nx, (mwSize)nl};
    plhs[0] = mxCreateNumericArray(nl > 1 ? 3 : 2, dims, mxDOUBLE_CLASS, mxREAL);
    check(c, swrt_qg_get_q(c, mxGetDoubles(plhs[0])), "swrt_qg_get_q");
    return;
  }
  if (!strcmp(cmd, "qg_snapshot")) {  // (slot, which, layer, ny_period)
    need(na, 5, cmd);
    check(c, swrt_qg_snapshot(c, (int)scalar(a[1]), (int)scalar(a[2]), (int)scalar(a[3]), (int64_t)scalar(a[4])),
          "swrt_qg_snapshot");
    return;
  }
  if (!strcmp(cmd, "swap_slots")) {
    need(na, 3, cmd);
    check(c, swrt_swap_slots(c, (int)scalar(a[1]), (int)scalar(a[2])), "swrt_swap_slots");
    return;
  }
  if (!strcmp(cmd, "field_div_free")) {
    need(na, 2, cmd);
    const int rc = swrt_field_div_free(c, (int)scalar(a[1]));
    if (rc < 0) check(c, rc, "swrt_field_div_free");
    plhs[0] = mxCreateDoubleScalar(rc == 1 ? 1.0 : 0.0);
    return;
  }
  mexErrMsgIdAndTxt("swrt:arg", "unknown command '%s'", cmd);
}
