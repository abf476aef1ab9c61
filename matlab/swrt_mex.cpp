// swrt_mex.cpp — MATLAB MEX gateway over the swrt C ABI (include/swrt.h).
//
// The reference-side binding a maintainer adds to ndefilippis/SWRaytracing so
// that SpectralScheme / ode_symplectic / interpolate_U callers run on the
// MI355X.  Deliberately thin: argument marshalling only, every error is raised
// with mexErrMsgIdAndTxt AFTER the C call has returned (never from HIP code).
// Build (MATLAB R2018a+, interleaved complex):
//   mex -R2018a -I../include swrt_mex.cpp -L../swraytracing_amd -lswrt
// Usage (see SpectralSchemeGPU.m, ode_symplectic_gpu.m):
//   swrt_mex('create', device)
//   swrt_mex('set_field_psi', slot, psi_grid, L)             % SpectralScheme ctor
//   swrt_mex('set_field_qk', slot, qk, L, K_d2, shear, kscale, ny_period)   % grid_U
//   swrt_mex('set_field_grid', slot, u, v, ux, uy, vx, vy, L, ny_period)
//   out6 = swrt_mex('eval', x, y, nslots, alpha, bump)       % 6 x n
//   FI   = swrt_mex('interpolate', x, y, F, dx, dy, bump)    % interpolate.m
//   [x, k, hx, hk] = swrt_mex('leapfrog', x0, k0, dt, nsteps, f, gH, nslots, alpha0, dalpha, bump, save_every)
//   fk = swrt_mex('g2k', fg);  fg = swrt_mex('k2g', fk);
//   swrt_mex('packets_set', x, k);  [x, k] = swrt_mex('packets_get');
//   swrt_mex('advance', dt, nsteps, f, gH, nslots, alpha0, dalpha, bump)
//   rh  = swrt_mex('ode23_f1', t, tmax, f, Cg, nslots, thr, bump)          % see ode23_packets_gpu.m
//   err = swrt_mex('ode23_attempt', t, h, tnew, tmax, f, Cg, nslots, thr, bump)
//   swrt_mex('ode23_accept')
//   swrt_mex('qg_init', params_struct, qk)   % qk (2kmax+1) x (kmax+1) [x 2], complex
//   swrt_mex('qg_step', dt, nsteps);  U0 = swrt_mex('qg_max_speed');
//   [qk, t, steps] = swrt_mex('qg_get');  q = swrt_mex('qg_get_q');
//   swrt_mex('qg_snapshot', slot, which, layer, ny_period);  swrt_mex('swap_slots', a, b)
//   tf = swrt_mex('field_div_free', slot)   % v_y == -u_x exactly (five-sum kernels)
//   swrt_mex('destroy')
#include <cstring>
#include <string>

#include "mex.h"
#include "swrt.h"

static swrt_ctx* g_ctx = nullptr;

static void cleanup() {
  if (g_ctx) {
    swrt_destroy(g_ctx);
    g_ctx = nullptr;
  }
}

static void check(int rc, const char* what) {
  if (rc != SWRT_OK) {
    std::string msg = std::string(what) + ": " + (g_ctx ? swrt_last_error(g_ctx) : "no context");
    mexErrMsgIdAndTxt("swrt:call", "%s (code %d)", msg.c_str(), rc);
  }
}

static double scalar(const mxArray* a) { return mxGetScalar(a); }

static const double* reals(const mxArray* a, const char* name) {
  if (!mxIsDouble(a) || mxIsComplex(a)) mexErrMsgIdAndTxt("swrt:arg", "%s must be real double", name);
  return mxGetDoubles(a);
}

static swrt_ctx* ctx() {
  if (!g_ctx) mexErrMsgIdAndTxt("swrt:state", "call swrt_mex('create', device) first");
  return g_ctx;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs < 1 || !mxIsChar(prhs[0])) mexErrMsgIdAndTxt("swrt:arg", "first argument: command");
  char cmd[64];
  mxGetString(prhs[0], cmd, sizeof(cmd));

  if (!strcmp(cmd, "create")) {
    if (!g_ctx) {
      const int dev = nrhs > 1 ? (int)scalar(prhs[1]) : 0;
      const int rc = swrt_create(dev, &g_ctx);
      if (rc != SWRT_OK) mexErrMsgIdAndTxt("swrt:create", "swrt_create failed (code %d)", rc);
      mexAtExit(cleanup);
      mexLock();
    }
    return;
  }
  if (!strcmp(cmd, "destroy")) {
    cleanup();
    if (mexIsLocked()) mexUnlock();
    return;
  }
  if (!strcmp(cmd, "set_field_psi")) {  // (slot, psi, L)
    const mxArray* psi = prhs[2];
    const int64_t nx = (int64_t)mxGetM(psi);
    check(swrt_set_field_psi(ctx(), (int)scalar(prhs[1]), reals(psi, "psi"), nx, scalar(prhs[3])),
          "swrt_set_field_psi");
    return;
  }
  if (!strcmp(cmd, "set_field_qk")) {  // (slot, qk, L, K_d2, shear, kscale, ny_period)
    const mxArray* qk = prhs[2];
    if (!mxIsComplex(qk)) mexErrMsgIdAndTxt("swrt:arg", "qk must be complex");
    const int64_t nx = (int64_t)mxGetM(qk) + 1;
    check(swrt_set_field_qk(ctx(), (int)scalar(prhs[1]), (const double*)mxGetComplexDoubles(qk), nx,
                            scalar(prhs[3]), scalar(prhs[4]), scalar(prhs[5]), scalar(prhs[6]),
                            (int64_t)scalar(prhs[7])),
          "swrt_set_field_qk");
    return;
  }
  if (!strcmp(cmd, "set_field_grid")) {  // (slot, u, v, ux, uy, vx, vy, L, ny_period)
    const int64_t nx = (int64_t)mxGetM(prhs[2]);
    const size_t plane = (size_t)(nx * nx);
    mxArray* tmp = mxCreateDoubleMatrix(plane, 6, mxREAL);  // 6 planes, MATLAB-owned scratch
    double* d = mxGetDoubles(tmp);
    for (int f = 0; f < 6; ++f) memcpy(d + f * plane, reals(prhs[2 + f], "field"), plane * sizeof(double));
    const int rc = swrt_set_field_grid(ctx(), (int)scalar(prhs[1]), d, nx, scalar(prhs[8]),
                                       (int64_t)scalar(prhs[9]));
    mxDestroyArray(tmp);
    check(rc, "swrt_set_field_grid");
    return;
  }
  if (!strcmp(cmd, "eval")) {  // (x, y, nslots, alpha, bump) -> 6 x n
    const size_t n = mxGetNumberOfElements(prhs[1]);
    plhs[0] = mxCreateDoubleMatrix(n, 6, mxREAL);  // column f = field f (6 x n row-major == n x 6 col-major)
    check(swrt_eval(ctx(), reals(prhs[1], "x"), reals(prhs[2], "y"), (int64_t)n, (int)scalar(prhs[3]),
                    scalar(prhs[4]), scalar(prhs[5]), mxGetDoubles(plhs[0])),
          "swrt_eval");
    return;
  }
  if (!strcmp(cmd, "interpolate")) {  // (x, y, F, dx, dy, bump)
    const mxArray* F = prhs[3];
    const int64_t nx = (int64_t)mxGetM(F);
    const int64_t nyF = (int64_t)(mxGetNumberOfElements(F) / mxGetM(F));
    const size_t n = mxGetNumberOfElements(prhs[1]);
    plhs[0] = mxCreateNumericArray(mxGetNumberOfDimensions(prhs[1]), mxGetDimensions(prhs[1]),
                                   mxDOUBLE_CLASS, mxREAL);
    check(swrt_interpolate(ctx(), reals(F, "F"), nx, nyF, scalar(prhs[4]), scalar(prhs[5]), scalar(prhs[6]),
                           reals(prhs[1], "x"), reals(prhs[2], "y"), (int64_t)n, mxGetDoubles(plhs[0])),
          "swrt_interpolate");
    return;
  }
  if (!strcmp(cmd, "leapfrog")) {
    // (x0 Nx2, k0 Nx2, dt, nsteps, f, gH, nslots, alpha0, dalpha, bump, save_every)
    const int64_t n = (int64_t)mxGetM(prhs[1]);
    const int64_t nsteps = (int64_t)scalar(prhs[4]);
    const int64_t save_every = nrhs > 11 ? (int64_t)scalar(prhs[11]) : 0;
    plhs[0] = mxDuplicateArray(prhs[1]);
    plhs[1] = mxDuplicateArray(prhs[2]);
    double *hx = nullptr, *hk = nullptr;
    if (nlhs > 2 && save_every > 0) {
      const mwSize dims[3] = {(mwSize)n, 2, (mwSize)(nsteps / save_every)};  // frames of N x 2
      plhs[2] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
      plhs[3] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
      hx = mxGetDoubles(plhs[2]);
      hk = mxGetDoubles(plhs[3]);
    }
    check(swrt_leapfrog(ctx(), mxGetDoubles(plhs[0]), mxGetDoubles(plhs[1]), n, scalar(prhs[3]), nsteps,
                        scalar(prhs[5]), scalar(prhs[6]), (int)scalar(prhs[7]), scalar(prhs[8]),
                        scalar(prhs[9]), scalar(prhs[10]), hx ? save_every : 0, hx, hk),
          "swrt_leapfrog");
    return;
  }
  if (!strcmp(cmd, "g2k")) {
    const int64_t nx = (int64_t)mxGetM(prhs[1]);
    const int64_t kmax = nx / 2 - 1;
    plhs[0] = mxCreateDoubleMatrix(2 * kmax + 1, kmax + 1, mxCOMPLEX);
    check(swrt_g2k(ctx(), reals(prhs[1], "fg"), nx, (double*)mxGetComplexDoubles(plhs[0])), "swrt_g2k");
    return;
  }
  if (!strcmp(cmd, "k2g")) {
    if (!mxIsComplex(prhs[1])) mexErrMsgIdAndTxt("swrt:arg", "fk must be complex");
    const int64_t nx = (int64_t)mxGetM(prhs[1]) + 1;
    plhs[0] = mxCreateDoubleMatrix(nx, nx, mxREAL);
    check(swrt_k2g(ctx(), (const double*)mxGetComplexDoubles(prhs[1]), nx, mxGetDoubles(plhs[0])),
          "swrt_k2g");
    return;
  }
  if (!strcmp(cmd, "packets_set")) {  // (x Nx2, k Nx2)
    check(swrt_packets_set(ctx(), reals(prhs[1], "x"), reals(prhs[2], "k"), (int64_t)mxGetM(prhs[1])),
          "swrt_packets_set");
    return;
  }
  if (!strcmp(cmd, "packets_get")) {
    const int64_t n = swrt_packets_count(ctx());
    plhs[0] = mxCreateDoubleMatrix((mwSize)n, 2, mxREAL);
    plhs[1] = mxCreateDoubleMatrix((mwSize)n, 2, mxREAL);
    check(swrt_packets_get(ctx(), mxGetDoubles(plhs[0]), mxGetDoubles(plhs[1])), "swrt_packets_get");
    return;
  }
  if (!strcmp(cmd, "advance")) {  // (dt, nsteps, f, gH, nslots, alpha0, dalpha, bump)
    check(swrt_advance(ctx(), scalar(prhs[1]), (int64_t)scalar(prhs[2]), scalar(prhs[3]), scalar(prhs[4]),
                       (int)scalar(prhs[5]), scalar(prhs[6]), scalar(prhs[7]), scalar(prhs[8]), 0),
          "swrt_advance");
    return;
  }
  if (!strcmp(cmd, "ode23_f1")) {  // (t, tmax, f, Cg, nslots, thr, bump) -> rh_raw
    double r = 0.0;
    check(swrt_ode23_f1(ctx(), scalar(prhs[1]), scalar(prhs[2]), scalar(prhs[3]), scalar(prhs[4]),
                        (int)scalar(prhs[5]), scalar(prhs[6]), scalar(prhs[7]), &r),
          "swrt_ode23_f1");
    plhs[0] = mxCreateDoubleScalar(r);
    return;
  }
  if (!strcmp(cmd, "ode23_attempt")) {  // (t, h, tnew, tmax, f, Cg, nslots, thr, bump) -> err_raw
    double r = 0.0;
    check(swrt_ode23_attempt(ctx(), scalar(prhs[1]), scalar(prhs[2]), scalar(prhs[3]), scalar(prhs[4]),
                             scalar(prhs[5]), scalar(prhs[6]), (int)scalar(prhs[7]), scalar(prhs[8]),
                             scalar(prhs[9]), &r),
          "swrt_ode23_attempt");
    plhs[0] = mxCreateDoubleScalar(r);
    return;
  }
  if (!strcmp(cmd, "ode23_accept")) {
    check(swrt_ode23_accept(ctx()), "swrt_ode23_accept");
    return;
  }
  if (!strcmp(cmd, "qg_init")) {  // (params struct, qk complex (2kmax+1) x (kmax+1) [x nlayers])
    const mxArray* s = prhs[1];
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
    if (!mxIsComplex(prhs[2])) mexErrMsgIdAndTxt("swrt:arg", "qk must be complex");
    const int64_t nx = (int64_t)mxGetM(prhs[2]) + 1;
    check(swrt_qg_init(ctx(), &p, nx, (const double*)mxGetComplexDoubles(prhs[2])), "swrt_qg_init");
    return;
  }
  if (!strcmp(cmd, "qg_step")) {  // (dt, nsteps)
    check(swrt_qg_step(ctx(), scalar(prhs[1]), nrhs > 2 ? (int64_t)scalar(prhs[2]) : 1), "swrt_qg_step");
    return;
  }
  if (!strcmp(cmd, "qg_max_speed")) {
    double u = 0.0;
    check(swrt_qg_max_speed(ctx(), &u), "swrt_qg_max_speed");
    plhs[0] = mxCreateDoubleScalar(u);
    return;
  }
  if (!strcmp(cmd, "qg_get")) {  // -> qk, t, steps (dims as given to qg_init)
    double t = 0.0;
    int64_t steps = 0;
    if (nrhs < 3) mexErrMsgIdAndTxt("swrt:arg", "qg_get needs (nx, nlayers)");
    const int64_t nx = (int64_t)scalar(prhs[1]);
    const int nl = (int)scalar(prhs[2]);
    const mwSize dims[3] = {(mwSize)(nx - 1), (mwSize)(nx / 2), (mwSize)nl};
    plhs[0] = mxCreateNumericArray(nl > 1 ? 3 : 2, dims, mxDOUBLE_CLASS, mxCOMPLEX);
    check(swrt_qg_get(ctx(), (double*)mxGetComplexDoubles(plhs[0]), &t, &steps), "swrt_qg_get");
    if (nlhs > 1) plhs[1] = mxCreateDoubleScalar(t);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar((double)steps);
    return;
  }
  if (!strcmp(cmd, "qg_get_q")) {  // (nx, nlayers) -> q nx x nx [x nlayers]
    const int64_t nx = (int64_t)scalar(prhs[1]);
    const int nl = (int)scalar(prhs[2]);
    const mwSize dims[3] = {(mwSize)nx, (mwSize)nx, (mwSize)nl};
    plhs[0] = mxCreateNumericArray(nl > 1 ? 3 : 2, dims, mxDOUBLE_CLASS, mxREAL);
    check(swrt_qg_get_q(ctx(), mxGetDoubles(plhs[0])), "swrt_qg_get_q");
    return;
  }
  if (!strcmp(cmd, "qg_snapshot")) {  // (slot, which, layer, ny_period)
    check(swrt_qg_snapshot(ctx(), (int)scalar(prhs[1]), (int)scalar(prhs[2]), (int)scalar(prhs[3]),
                           (int64_t)scalar(prhs[4])),
          "swrt_qg_snapshot");
    return;
  }
  if (!strcmp(cmd, "swap_slots")) {
    check(swrt_swap_slots(ctx(), (int)scalar(prhs[1]), (int)scalar(prhs[2])), "swrt_swap_slots");
    return;
  }
  if (!strcmp(cmd, "field_div_free")) {
    const int rc = swrt_field_div_free(ctx(), (int)scalar(prhs[1]));
    if (rc < 0) check(rc, "swrt_field_div_free");
    plhs[0] = mxCreateDoubleScalar(rc == 1 ? 1.0 : 0.0);
    return;
  }
  mexErrMsgIdAndTxt("swrt:arg", "unknown command '%s'", cmd);
}
