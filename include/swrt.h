/*
 * swrt.h — C ABI of the MI355X-native wave-packet ray-tracing hot path
 * (ndefilippis/SWRaytracing, qg_flow_ray_trace hot loop).
 *
 * The reference is MATLAB and has no native interface; each entry point below
 * names the MATLAB function (file:line, paths relative to the reference root)
 * whose behaviour it replaces.  A MEX gateway (matlab/swrt_mex.cpp) and the
 * Python ctypes front-end (swraytracing_amd/) bind exactly these symbols.
 *
 * Conventions
 *  - Every function returns an int status: SWRT_OK (0) or a SWRT_ERR_* code;
 *    swrt_last_error(ctx) returns a message for the last failure on ctx.
 *    No C++ exception or longjmp crosses this ABI.
 *  - Host buffers are caller-owned, fp64, MATLAB column-major, and are never
 *    retained after a call returns.  The context owns all device memory.
 *  - Packet arrays are N x 2 column-major: x(:,1) (all x) then x(:,2) (all y),
 *    the layout of packet_x / packet_k in qgsw_raytrace.m:54-55 and of one
 *    frame of packet_x.bin (write_field.m:38).
 *  - Gridded fields are nx x nx column-major, first index = x: F(ig, jg) at
 *    x = (ig-1)*dx, y = (jg-1)*dx (k2g.m / interpolate.m conventions).
 *  - One context per host thread; calls are synchronous with respect to the
 *    host (stream-ordered internally); not re-entrant on the same context.
 */
#ifndef SWRT_H
#define SWRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWRT_OK 0
#define SWRT_ERR_ARG 1   /* invalid argument (shape, slot, null pointer) */
#define SWRT_ERR_HIP 2   /* HIP runtime error */
#define SWRT_ERR_STATE 3 /* call out of order (e.g. field not set) */
#define SWRT_ERR_ALLOC 4 /* allocation failure */

#define SWRT_MAX_SLOTS 5 /* snapshot slots: 0 = flow1 / steady, 1 = flow2; 2..4 the later
                            snapshots of swrt_advance_intervals */

typedef struct swrt_ctx swrt_ctx;

/* ABI version (major*10000 + minor*100 + patch). */
int swrt_version(void);

/* Create a context bound to HIP device `device` (one process per GPU). */
int swrt_create(int device, swrt_ctx** out);
void swrt_destroy(swrt_ctx* ctx);
const char* swrt_last_error(const swrt_ctx* ctx);

/* ---------------------------------------------------------------------------
 * Background flow (L1/L2: field preparation, once per snapshot)
 * ------------------------------------------------------------------------ */

/* Six gridded fields (u, v, u_x, u_y, v_x, v_y), each nx*nx column-major,
 * concatenated.  Replaces holding SpectralScheme.U_field / GradU_field
 * (SpectralScheme.m:29-35) or a grid_U output struct (grid_U.m:11-17).
 * ny_period: the y-period of interpolate.m's mod (interpolate.m:15,22): nx for
 * a single layer, nlayers*nx for the 2-layer call (qg2layersw_raytrace.m:187-188)
 * where F is nx x nx x 2 and only layer 1 is read.  0 means nx.
 * If v_y == -u_x bit for bit at every node (a streamfunction flow stored that
 * way) the slot is marked divergence-free and the packet kernels carry five
 * stencil sums instead of six (v_y's is the exact negation of u_x's), with
 * unchanged results. */
int swrt_set_field_grid(swrt_ctx* ctx, int slot, const double* fields6, int64_t nx, double L,
                        int64_t ny_period);

/* 1 if slot's v_y is exactly -u_x at every node (always so for fields the
 * library derives from psi / qk: it stores v_y as -u_x, see
 * swrt_set_field_psi), 0 if not, < 0 on error. */
int swrt_field_div_free(swrt_ctx* ctx, int slot);

/* SpectralScheme(L, nx, psi_field) constructor (SpectralScheme.m:6-36):
 * psik = g2k(psi); u = k2g(-i ky psik), v = k2g(i kx psik), gradients by
 * i kx / i ky; integer wavenumbers regardless of L.  FFTs run on the GPU.
 * The filtered psi grid k2g(g2k(psi)) is kept for swrt_get_psi_grid.
 * v_y is stored as -u_x (bit-exact negation): SpectralScheme.m / grid_U.m
 * transform i ky vk separately, which equals -(i kx uk) up to the FFT's
 * roundoff (the identity u_x + v_y = 0 of a streamfunction flow); the same
 * holds for swrt_set_field_qk and swrt_qg_snapshot. */
int swrt_set_field_psi(swrt_ctx* ctx, int slot, const double* psi_grid, int64_t nx, double L);

/* grid_U(qk, K_d2, K2, kx_, ky_, shear_strength) (grid_U.m:1-18) for one
 * layer: psik = -qk./(K_d2+K2), six derivative spectra, k2g on the GPU,
 * u += shear.  qk: (2kmax+1) x (kmax+1) complex, column-major, interleaved
 * (re, im) (MATLAB -R2018a interleaved complex).  k_scale multiplies the
 * integer wavenumbers (1 for qgsw_raytrace.m:19, 2*pi/L for
 * qg2layersw_raytrace.m:20-21).  ny_period as in swrt_set_field_grid. */
int swrt_set_field_qk(swrt_ctx* ctx, int slot, const double* qk_interleaved, int64_t nx, double L,
                      double K_d2, double shear, double k_scale, int64_t ny_period);

/* grid_U(g2k(q)) into `slot` from a gridded PV frame q (nx x nx fp64,
 * column-major): the stored-field consumer's read_field -> g2k -> grid_U
 * (symplectic_full_fourier.m:18-20, read_field.m:37-98, g2k.m:8-9,
 * grid_U.m:1-18) with both transforms on the device — the same result as
 * swrt_g2k followed by swrt_set_field_qk, without the spectrum's round
 * trip through host memory.  Arguments as swrt_set_field_qk. */
int swrt_set_field_q(swrt_ctx* ctx, int slot, const double* q_grid, int64_t nx, double L, double K_d2,
                     double shear, double k_scale, int64_t ny_period);

/* g2k(fg) (g2k.m:5-9): nx x nx real grid (column-major) -> the
 * (2kmax+1) x (kmax+1) half-plane spectrum fftshift(fft2(fg))/nx^2 cropped,
 * interleaved complex, column-major.  GPU FFT. */
int swrt_g2k(swrt_ctx* ctx, const double* fg, int64_t nx, double* fk_interleaved_out);
/* k2g(fk) (k2g.m:5-6 + fulspec.m): half-plane spectrum -> nx x nx real grid
 * nx^2*ifft2(ifftshift(fulspec(fk))) (real part), column-major.  GPU FFT. */
int swrt_k2g(swrt_ctx* ctx, const double* fk_interleaved, int64_t nx, double* fg_out);

/* Download slot's six fields (nx*nx column-major each) — for checks/plots. */
int swrt_get_field_grid(swrt_ctx* ctx, int slot, double* fields6_out);
/* Download the filtered psi grid of the last swrt_set_field_psi (nx*nx). */
int swrt_get_psi_grid(swrt_ctx* ctx, int slot, double* psi_out);

/* nx of the grid held by field slot `slot` (the size swrt_get_field_grid /
 * swrt_get_psi_grid write: 6 / 1 planes of nx x nx); -1 when the slot is
 * unset or the index is out of range.  Front-ends size their outputs from
 * this, never from a caller's argument. */
int64_t swrt_field_grid(const swrt_ctx* ctx, int slot);

/* ---------------------------------------------------------------------------
 * Point evaluation (L2 boundary API)
 * ------------------------------------------------------------------------ */

/* interpolate(x, y, F, dx, dy) (interpolate.m:1-50) of an arbitrary nx x nyF
 * grid field F (only the first nx columns are read when nyF > nx, as MATLAB's
 * 2-subscript F(ig,jg) does), with the given bump (1e-10:
 * qg_flow_ray_trace/interpolate.m:13; 1e-13: ray_trace_sw/interpolate.m:13). */
int swrt_interpolate(swrt_ctx* ctx, const double* F, int64_t nx, int64_t nyF, double dx, double dy,
                     double bump, const double* x, const double* y, int64_t n, double* out);

/* U and grad U at n points from the slot fields: out is 6 x n row-major
 * (u, v, u_x, u_y, v_x, v_y).  nslots = 1: slot 0 only (SpectralScheme.U /
 * grad_U, SpectralScheme.m:45-68).  nslots = 2: interpolate_U's blend
 * (1-alpha)*slot0 + alpha*slot1 (interpolate_U.m:5-23). */
int swrt_eval(swrt_ctx* ctx, const double* x, const double* y, int64_t n, int nslots, double alpha,
              double bump, double* out6);

/* ---------------------------------------------------------------------------
 * Packets and the fused symplectic integrator (L3)
 * ------------------------------------------------------------------------ */

/* Upload / download packet state (N x 2 column-major x and k). */
int swrt_packets_set(swrt_ctx* ctx, const double* x, const double* k, int64_t n);
int swrt_packets_get(swrt_ctx* ctx, double* x, double* k);
/* The same state in the original packet order into DEVICE buffers of this
 * context's GPU: x_dev[i + j*ld], k_dev[i + j*ld] (N x 2 column-major with
 * leading dimension ld >= N), enqueued on the packet stream (swrt_get_stream)
 * without a host synchronisation — the input of a device-side gather of
 * sharded trajectories (RCCL all_gather, swraytracing_amd/dist.py). */
int swrt_packets_get_device(swrt_ctx* ctx, double* x_dev, double* k_dev, int64_t ld);
int64_t swrt_packets_count(const swrt_ctx* ctx);

/* Locality tuning: the packets are kept counting-sorted by spatial tile
 * (tile x tile cells of slot 0's grid) and re-binned every `rebin_every`
 * steps (0 disables binning; tile 0 picks a size automatically).  Binning
 * changes only the device-side order: results, downloads and history frames
 * are identical and in the original packet order. */
int swrt_set_locality(swrt_ctx* ctx, int64_t rebin_every, int64_t tile);

/* Packet-kernel variant (same results, bit for bit): 0 = automatic (the
 * LDS-tiled kernel whenever binning is on and nx >= 32), 1 = one lane per
 * packet gathering from the global node array, 2 = LDS-tiled kernel (16x16-
 * cell tiles, field window staged in LDS, in-tile cell sort). */
int swrt_set_kernel(swrt_ctx* ctx, int variant);

/* Opt-in stencil arithmetic of the LDS-tiled packet kernel for fields with
 * v_y == -u_x (every field the library derives from psi / qk): 1 = each
 * tap's wij*F added by one fused multiply-add (and the snapshot blend as
 * (1-alpha)*I1 + alpha*I2 with one FMA), which drops ~350 of the ~1,100 VALU
 * instructions of a packet-step; the sums keep interpolate.m:43-49's order
 * but round once per tap instead of twice, so results agree with the
 * reference to tolerance (per step ~1e-15 relative), not bit for bit.
 * 0 (default) = mul then add, bit-identical to the reference's arithmetic.
 * Other kernels (host-given six-field windows, the per-packet kernel, ode23,
 * xka) always use mul then add. */
int swrt_set_gather_mode(swrt_ctx* ctx, int mode);

/* Launch shape of the LDS-tiled two-snapshot launches (fields with v_y ==
 * -u_x) when tiles hold few packets: 256-thread workgroups with a 256-VGPR
 * budget whose stencil gather issues each tap's LDS reads three taps ahead
 * (instead of 512 threads, 128 VGPRs, one tap ahead), so the one busy wave a
 * SIMD has at ~120 packets per tile waits less on the LDS.  0 (default) =
 * below SWRT_SPARSE_BELOW packets per 16x16 tile on average (build default
 * 192: the 8-GPU shard of the 1e6 bench, whose driver step it shortens by
 * 2.5 % beside the PDE), 1 = never, 2 = always.  Same arithmetic in the same
 * order: bit-identical for any setting. */
int swrt_set_sparse_tiles(swrt_ctx* ctx, int mode);

/* Packet streams of the LDS-tiled leapfrog: 2 (default) or 1.  With 2 every
 * launch runs as two part launches — the even and the odd band positions of
 * each XCD band's tiles (the mapping: swraytracing_amd/csrc/swrt_share.hpp)
 * — on the context's packet stream and a second stream.
 * Between re-binnings the parts advance disjoint packet ranges, so one
 * stream's launch k overlaps the other's launch k+1: one part's tail runs
 * under the other's body instead of leaving CUs idle at every launch
 * boundary.  The launch after a re-binning's sort launch (which gathers its
 * input from any slot) and any call that reads the packets (or re-bins them)
 * first order the second stream's work before their own; swrt_synchronize
 * waits for both.  Results are bit-identical for either setting.  Ensembles
 * under 65,536 packets always use one stream (the split costs more than it
 * returns there). */
int swrt_set_packet_streams(swrt_ctx* ctx, int streams);

/* Advance the device-resident packets by nsteps leapfrog steps
 * (ode_symplectic.m:13-37: drift dt/2 with gH*k/omega, kick dt with U(x1)
 * and (grad U(x1))^T k1 (RaytracingScheme.m:9-16), drift dt/2).  The kick of
 * step s uses alpha = alpha0 + s*dalpha when nslots == 2.  bump: Lagrange
 * bump.  If save_every > 0 a frame (N x 2 x, then N x 2 k) is recorded on the
 * device after every save_every steps (frames appended to the history
 * buffer, see swrt_history_*). */
int swrt_advance(swrt_ctx* ctx, double dt, int64_t nsteps, double f, double gH, int nslots,
                 double alpha0, double dalpha, double bump, int64_t save_every);

/* nintervals consecutive PDE intervals in one call: interval i advances the
 * packets nsub leapfrog steps of size dts[i], blending slots i and i+1 with
 * alpha = alpha0 + s*dalpha (s = step within the interval) — exactly
 * nintervals swrt_advance(dts[i], nsub, ..., nslots 2) calls with slots
 * (i, i+1) moved to (0, 1) in turn, bit for bit.  Slots 0..nintervals must
 * be set on one grid; nintervals <= SWRT_MAX_SLOTS - 1; save_every (0 = no
 * history) divides nsub.  With the LDS-tiled kernel and re-binning every
 * multiple of nsub steps, up to 4 intervals run in ONE launch (each
 * workgroup re-stages its window between them), so the launch's tail and the
 * in-tile sort are paid once per 4 intervals instead of once per interval.
 * (The drivers' packet branch over several PDE steps: qgsw_raytrace.m:140-151,
 * qg2layersw_raytrace.m:185-197 with the snapshots of the PDE run ahead.) */
int swrt_advance_intervals(swrt_ctx* ctx, int nintervals, const double* dts, int64_t nsub, double f, double gH,
                           double alpha0, double dalpha, double bump, int64_t save_every);

/* History frames recorded by swrt_advance since the last swrt_history_reset. */
int64_t swrt_history_frames(const swrt_ctx* ctx);
int swrt_history_get(swrt_ctx* ctx, int64_t first, int64_t count, double* hist_x, double* hist_k);
int swrt_history_reset(swrt_ctx* ctx);

/* Host convenience = packets_set + advance + packets_get (+ history): the
 * drop-in for ode_symplectic(x0,k0,dt,T,f,gH,scheme) (ode_symplectic.m:1-31).
 * hist_x / hist_k may be NULL; otherwise they receive nsteps/save_every frames
 * of N x 2 each. */
int swrt_leapfrog(swrt_ctx* ctx, double* x, double* k, int64_t n, double dt, int64_t nsteps,
                  double f, double gH, int nslots, double alpha0, double dalpha, double bump,
                  int64_t save_every, double* hist_x, double* hist_k);

/* ---------------------------------------------------------------------------
 * Wave-action packets over an RSW background (ray_trace_sw/step_packet_xka.m)
 * ------------------------------------------------------------------------ */

/* Background of step_packet_xka(P, U, GradU, H, C0, f, dx, dy, dt)
 * (step_packet_xka.m:1): seven nx x nx column-major planes concatenated in the
 * order U.u, U.v, GradU.u_x, GradU.u_y, GradU.v_x, GradU.v_y, H. */
int swrt_xka_set_fields(swrt_ctx* ctx, const double* fields7, int64_t nx, double dx, double dy);

/* The same background built on the GPU from an RSW state, as
 * ray_trace_sw/raytrace_sw.m:16-52 does: state3 = S(:,:,1:3) = [u v eta]
 * (nx x nx x 3 column-major, :12), g2k of each (:26-28), the geostrophic
 * projection etagk = (f*etak - zetak).*f./(f^2 + gH0*K2) with gH0 = Cg^2
 * (:22-31), ug/vg and their i*k gradients (:34-41), seven k2g and
 * H = 1 + etag (:44-52).  Integer wavenumbers (L = 2*pi, :84); L sets
 * dx = dy = L/nx.  nx a power of two. */
int swrt_xka_set_rsw(swrt_ctx* ctx, const double* state3, int64_t nx, double f, double Cg, double L);

/* Download the current xka background as the seven planes of
 * swrt_xka_set_fields (U.u, U.v, GradU.u_x, u_y, v_x, v_y, H); nx x nx each
 * with nx = swrt_xka_grid(ctx). */
int swrt_xka_get_fields(swrt_ctx* ctx, double* fields7_out);
int64_t swrt_xka_grid(const swrt_ctx* ctx);

/* nsteps of Pout = step_packet_xka(P, ...) for n packets (step_packet_xka.m:
 * 38-91 with cg_sw.m:15-32 evaluated per stencil tap; interpolate of
 * ray_trace_sw, bump 1e-13).  state5 (in/out): n x 5 column-major
 * [P.x P.y P.k P.l P.a].  hist5 (may be NULL): nsteps/save_every frames of
 * n x 5 after every save_every steps. */
int swrt_xka_step(swrt_ctx* ctx, double* state5, int64_t n, double C0, double f, double dt,
                  int64_t nsteps, int64_t save_every, double* hist5);

/* ---------------------------------------------------------------------------
 * Exact spectral evaluator (scratch/fourier_interpolate_test.m:92-136)
 * ------------------------------------------------------------------------ */

/* psi(x,y) = sum_{i,j} Re(C[i,j] exp(1i*(kx_i x + ky_j y))), kx_i = (kx0+i)*s,
 * ky_j = (ky0+j)*s; C nkx x nky column-major interleaved complex.  The
 * half-plane spectrum of g2k maps to C = 2*psik (ky = 0, kx < 0 zeroed, DC
 * real, kx0 = -kmax, ky0 = 0); the scratch test's amp/phase field to
 * C = amp.*exp(1i*phase) (kx0 = ky0 = -n, s = 1). */
int swrt_spectral_set_modes(swrt_ctx* ctx, const double* C_interleaved, int64_t nkx, int64_t nky,
                            double kx0, double ky0, double s);
/* Exact U and grad U (6 x n, as swrt_eval) by the direct mode sum;
 * precision 64 (fp64) or 32 (fp32 sums, the config-5 tolerance study). */
int swrt_spectral_eval(swrt_ctx* ctx, const double* x, const double* y, int64_t n, int precision,
                       double* out6);
/* Leapfrog (ode_symplectic.m:13-37) with the exact spectral kick
 * (fourier_interpolate_test.m:73-114); x, k N x 2 column-major, in/out. */
int swrt_spectral_leapfrog(swrt_ctx* ctx, double* x, double* k, int64_t n, double dt, int64_t nsteps,
                           double f, double gH, int precision);

/* ---------------------------------------------------------------------------
 * Diagnostics (analysis/load_data.m)
 * ------------------------------------------------------------------------ */

/* Energy-vs-omega input of load_data.m:33-52 for the device-resident packets:
 * omega = sqrt(f^2 + Cg^2*|k|^2) per packet, histcounts over `edges`
 * (nbins + 1 increasing values; last bin closed) ADDED to counts_inout (so a
 * window of frames accumulates), and the ensemble mean omega of this frame
 * (load_data.m:63; deterministic block-ordered sum). */
int swrt_omega_histogram(swrt_ctx* ctx, double f, double Cg, const double* edges, int64_t nbins,
                         int64_t* counts_inout, double* mean_omega_out);

/* ---------------------------------------------------------------------------
 * ode23 packet integrator (the drivers' integrator)
 * ------------------------------------------------------------------------ */

/* Device stages of MATLAB's ode23 (Bogacki-Shampine 3(2), FSAL) over the
 * device-resident packets as ONE 4N-vector ODE (qgsw_raytrace.m:143-150 with
 * odefun :259-265: dx/dt = U + Cg*k/sqrt(f^2 + Cg^2|k|^2), dk/dt =
 * -(grad U)^T k, U from interpolate_U(slot 0, slot 1, t/tmax) — nslots = 1
 * reads slot 0 only).  The step-size controller (a global decision over the
 * max-norm error) runs on the host; thr = AbsTol/RelTol.
 * swrt_ode23_f1:     F1 = odefun(t, y);  *rh_raw = max |F1| ./ max(|y|, thr)
 * swrt_ode23_attempt: stages 2-4 of one trial step of size h ending at tnew
 *                    (ynew uses h4 = tnew - t); *err_raw = max over all
 *                    components of |F*E| ./ max(max(|y|, |ynew|), thr)
 * swrt_ode23_accept: y = ynew, F1 = F4 (FSAL). */
int swrt_ode23_f1(swrt_ctx* ctx, double t, double tmax, double f, double Cg, int nslots, double thr, double bump,
                  double* rh_raw_out);
int swrt_ode23_attempt(swrt_ctx* ctx, double t, double h, double tnew, double tmax, double f, double Cg,
                       int nslots, double thr, double bump, double* err_raw_out);
int swrt_ode23_accept(swrt_ctx* ctx);
/* [~, y] = ode23(odefun, [t0 tfinal], y) for the device-resident packets with
 * MATLAB's controller (RelTol rtol, AbsTol atol, MaxStep 0.1*|tfinal - t0|,
 * max-norm error, initial-step heuristic, step update) in the library: the
 * f1 / attempt / accept sequence above without a host interpreter between
 * attempts.  Writes the accepted times (t0 first) to ts_out[0 .. min(*nts_out,
 * ts_cap)): ts_cap bounds only the times recorded, the interval always
 * completes and *nts_out counts every accepted time.  {steps, failed,
 * attempts} go to stats3_out (may be NULL).  If the step size falls below
 * hmin (MATLAB's "unable to meet integration tolerances") the packets are
 * left at the last accepted time and SWRT_ERR_STATE is returned.  Single rank: a sharded ensemble needs the error norm's
 * max over the ranks (swrt_ode23_run_sharded). */
int swrt_ode23_run(swrt_ctx* ctx, double t0, double tfinal, double tmax, double f, double Cg, int nslots,
                   double rtol, double atol, double bump, double* ts_out, int64_t ts_cap, int64_t* nts_out,
                   int64_t* stats3_out);
/* swrt_ode23_run with a host hook: hook(hook_user) is called once, after
 * stage 1 and the first attempt are queued and before the host first waits
 * on the device — host work placed there (the drivers queue the next QG step,
 * qg2layersw_raytrace.m:166-181, through swrt_qg_step_speculative) overlaps
 * the interval's first launches instead of the gap between intervals.  The
 * hook may call the library's QG entry points; it must not touch the packets
 * or the field slots this call reads.  hook NULL: swrt_ode23_run. */
int swrt_ode23_run_hooked(swrt_ctx* ctx, double t0, double tfinal, double tmax, double f, double Cg, int nslots,
                          double rtol, double atol, double bump, double* ts_out, int64_t ts_cap, int64_t* nts_out,
                          int64_t* stats3_out, void (*hook)(void*), void* hook_user);
/* swrt_ode23_run_hooked for packets sharded over ranks: the
 * error norm is a max over every packet of every rank, so each max this
 * rank's stages produce — stage 1's, then every attempt's the controller
 * consumes — goes through reduce(&value, reduce_user), which replaces it in
 * place with the max over the ranks (the caller's collective, e.g. an RCCL
 * all_reduce) and returns 0 (else SWRT_ERR_STATE).  Every rank then takes the
 * same steps: one reduce per stage 1 and per consumed attempt, in the same
 * order on every rank (the order swraytracing_amd.integrate's controller
 * reduces in, so a rank without packets can run that one).  The first step
 * size comes from the reduced stage-1 max, so it is not guessed on the
 * device; a device-gated guess runs only if this rank's max passes its gate,
 * which the global max passing implies.  reduce NULL: swrt_ode23_run_hooked. */
int swrt_ode23_run_sharded(swrt_ctx* ctx, double t0, double tfinal, double tmax, double f, double Cg, int nslots,
                           double rtol, double atol, double bump, double* ts_out, int64_t ts_cap, int64_t* nts_out,
                           int64_t* stats3_out, void (*hook)(void*), void* hook_user,
                           int (*reduce)(double* value, void* reduce_user), void* reduce_user);
/* Chain the next swrt_ode23_run(_hooked) to the one running (or the next to
 * run): when it ends, it queues the next call's stage 1 (re-binning when due,
 * in-tile sort, f at t = 0) on the accepted packets with slot_a / slot_b as
 * slots 0 / 1, so the device runs it while the host returns and prepares that
 * call (the drivers arm it from the hook: their next interval reads this
 * interval's end snapshot and the one the hook queued).  The next call takes
 * it only if it would compute exactly that — its slots 0 / 1 hold the same
 * nodes, not rewritten since, the same f, Cg, AbsTol/RelTol, bump and
 * alpha(t0) = 0, and no call that may touch the packets ran in between — else
 * it computes its own.  Same bits either way; one call's arming is consumed
 * by that call. */
int swrt_ode23_chain_next(swrt_ctx* ctx, int slot_a, int slot_b);
/* swrt_ode23_run's controller (MATLAB ode23's step-size logic, the library's
 * own code: swrt_ode23_ctl.cpp) replayed against a scripted error sequence
 * instead of the device stages — host only, no context, no GPU.  raw[0] is
 * stage 1's max (max |F1| ./ max(|y|, thr)), raw[1..nraw) the attempts' raw
 * error maxima in the order the controller consumes them; dev_first: a first
 * attempt is queued from the device's own step size, as on the tile path.
 * log_out: per consumed attempt {t, h, tnew, raw} (4 doubles; *nlog_out
 * counts all of them); ts_out / ts_cap / nts_out as in swrt_ode23_run;
 * stats9_out: {steps, failed, attempts, first attempts taken, guesses queued,
 * guesses taken by rule (MaxStep at MaxStep, MaxStep from 5*absh, 5*absh),
 * consumed guesses whose device gate would have skipped them (always 0)}.
 * Returns SWRT_ERR_STATE below hmin (as swrt_ode23_run), SWRT_ERR_ARG if the
 * script runs out.  Replaces nothing in the reference: it pins the library's
 * controller to swraytracing_amd/integrate.py's (qgsw_raytrace.m:149). */
int swrt_ode23_replay(double t0, double tfinal, double rtol, double atol, int dev_first, const double* raw,
                      int64_t nraw, double* log_out, int64_t log_cap, int64_t* nlog_out, double* ts_out,
                      int64_t ts_cap, int64_t* nts_out, int64_t* stats9_out);

/* ---------------------------------------------------------------------------
 * QG PDE stepper: the snapshots' producer, device-resident
 * ------------------------------------------------------------------------ */

/* Parameters of the two drivers' PDEs.  nlayers = 1: qgsw_raytrace.m
 * (L = 2*pi, integer wavenumbers; update :270-286 with beta, r_drag and the
 * inertial_ring forcing :216-220; filter :222-230 when filter = 1).
 * nlayers = 2: qg2layersw_raytrace.m (wavenumbers scaled by 2*pi/L; B
 * inversion, factor_L with shear, nu*K2^hyper_order + r diffusion and beta
 * :129-144). */
typedef struct swrt_qg_params {
  int nlayers;
  int filter;
  double L;
  double K_d2;
  double beta;
  double r_drag;
  double force_strength;
  double f;
  double Cg;
  double shear;
  double nu;
  double hyper_order;
  double r;
} swrt_qg_params;

/* Load the initial spectral PV qk (nlayers blocks of the (2kmax+1) x (kmax+1)
 * g2k half plane, interleaved complex, column-major) and reset the AB3
 * history (qgsw_raytrace.m:111-112, qg2layersw_raytrace.m:120-121). */
int swrt_qg_init(swrt_ctx* ctx, const swrt_qg_params* params, int64_t nx, const double* qk_interleaved);
/* nsteps PDE steps of size dt: AB3 (forward Euler, AB2 for the first two
 * steps), 1 layer: qgsw_raytrace.m:121-137; 2 layers: qg2layersw_raytrace.m
 * :167-181 with expLdt/expL2dt recomputed on the device whenever dt changes.
 * Before each step the previous qk is kept (prev_qk, :122 / :167). */
int swrt_qg_step(swrt_ctx* ctx, double dt, int64_t nsteps);
/* Speculative PDE step (qg2layersw_raytrace.m:152-181 with the CFL rule of
 * :156-165 decided late): queue the next step with `dt` — the step size the
 * rule will keep unless U0 of the current qk says otherwise — together with
 * its post-step transforms and its CFL read-back, before the host has read
 * the current U0 (swrt_qg_max_speed_result pops read-backs oldest first).
 * The step is computed into spare buffers; the committed state (qk, history,
 * t, steps — what swrt_qg_get reports) is untouched until swrt_qg_resolve:
 * accept (1) makes it the current step, reject (0) drops it and its read-back,
 * after which the caller steps with the rule's new dt.  An accepted step is
 * the same computation as swrt_qg_step(dt): bit-identical.  Needs the fused
 * post-step transforms and, for two layers, dt equal to the dt of the last
 * step (the exponential propagators are not recomputed).  While one is
 * pending, swrt_qg_step / _snapshot / _max_speed(_async) fail with
 * SWRT_ERR_STATE. */
int swrt_qg_step_speculative(swrt_ctx* ctx, double dt);
int swrt_qg_resolve(swrt_ctx* ctx, int accept);
/* 1 (default): the swrt_qg_* calls run on a second HIP stream of the
 * context, so the next PDE step, its CFL speed and snapshot overlap the
 * packet launch that reads the previous snapshots.  Slot reads and writes
 * are ordered across the two streams with events; a swrt_qg_snapshot into a
 * slot whose buffer a queued packet launch still reads writes a spare buffer
 * instead (renaming), so it never waits for that launch.  0: one stream.
 * Results are identical; swrt_synchronize waits for both streams. */
int swrt_qg_set_stream(swrt_ctx* ctx, int separate);
/* 1 (default): the transforms every consumer of a new qk needs — the next
 * step's Jacobian, the CFL speed (swrt_qg_max_speed*) and layer 0's grid_U
 * for swrt_qg_snapshot(which 0, layer 0) — come from ONE batched inverse
 * 2-D FFT of the current qk, computed once on first use.  0: each call runs
 * its own transforms.  The same spectra and per-vector FFTs either way:
 * results are bit-identical. */
int swrt_qg_set_fused(swrt_ctx* ctx, int on);
/* U0 = sqrt(max((u + shear)^2 + v^2)) over every layer of grid_U(qk)
 * (qg2layersw_raytrace.m:156-158; qgsw_raytrace.m:63-65 with shear 0). */
int swrt_qg_max_speed(swrt_ctx* ctx, double* U0_out);
/* The same, split: _async enqueues the speed of the CURRENT qk (read back into
 * pinned memory behind an event) and returns at once, so the caller can queue
 * the packet work of this step before _result waits for U0 — the driver's
 * CFL decision for the next step no longer stalls the GPU. */
int swrt_qg_max_speed_async(swrt_ctx* ctx);
int swrt_qg_max_speed_result(swrt_ctx* ctx, double* U0_out);
/* Copy out qk (same layout as swrt_qg_init), the model time and step count. */
int swrt_qg_get(swrt_ctx* ctx, double* qk_out, double* t_out, int64_t* steps_out);
/* q = k2g(qk) per layer: nx x nx x nlayers column-major (pv.bin frames,
 * qgsw_raytrace.m:167-170). */
int swrt_qg_get_q(swrt_ctx* ctx, double* q_out);

/* nx of the QG state and (if nlayers_out) its layer count; -1 before
 * swrt_qg_init.  swrt_qg_get writes (nx-1) x nx/2 x nlayers complex values,
 * swrt_qg_get_q nx x nx x nlayers reals. */
int64_t swrt_qg_grid(const swrt_ctx* ctx, int* nlayers_out);
/* grid_U of the current (which = 0) or previous (which = 1) qk of one layer
 * straight into packet field slot `slot` (qgsw_raytrace.m:141-142,
 * qg2layersw_raytrace.m:187-188: layer 1, u += shear_strength), no host copy.
 * ny_period as in swrt_set_field_grid (0 = nx). */
int swrt_qg_snapshot(swrt_ctx* ctx, int slot, int which, int layer, int64_t ny_period);
/* swrt_qg_snapshot(slot, which = 0, layer = 0, ny_period) of the pending
 * speculative step's qk (swrt_qg_step_speculative; fused two-layer mode):
 * the snapshot that the same call would write after swrt_qg_resolve(ctx, 1),
 * bit for bit, queued before the CFL rule has decided — a driver queues it
 * with the speculative step and discards it if the step is rejected.
 * SWRT_ERR_STATE without a pending fused speculative step. */
int swrt_qg_snapshot_speculative(swrt_ctx* ctx, int slot, int64_t ny_period);
/* Owner-driver hand-off (qg2layersw_raytrace.m:186-188: the packets read the
 * top layer only).  In a sharded run one rank steps the PDE and the others
 * build their snapshots from the top layer's spectral PV it sends them.
 * swrt_qg_export: layer `layer` of the current (which = 0) or previous (1) qk,
 * (2kmax+1)*(kmax+1) interleaved complex in the device order (ky fastest:
 * element (kx, ky) at (kx + kmax)*(kmax + 1) + ky), to dst, followed by
 * `tail` (e.g. the step's dt, so one broadcast carries both: dst holds
 * 2*(2kmax+1)*(kmax+1) + 1 doubles).  dst_mode = 1: a device buffer; the
 * copy runs on the QG stream behind the step that made qk, after `stream`'s
 * work queued so far (its last read of dst) and before `stream`'s later work
 * (stream: a hipStream_t of the caller, e.g. the one a broadcast is queued
 * on; NULL = the context's packet stream).  2: the same without the first
 * ordering — the caller guarantees dst is no longer read (a wait of the QG
 * stream on another stream's event measured ~0.1 ms per step on ROCm while
 * packet launches hold the GPU).  0: host memory, returns once copied.  The committed state is exported: a pending
 * speculative step (swrt_qg_step_speculative) is neither waited for nor
 * included. */
int swrt_qg_export(swrt_ctx* ctx, int which, int layer, double* dst, int dst_mode, void* stream, double tail);
/* grid_U (grid_U.m:1-18: psi = -q/(K_d2 + K^2), u += shear) of a half plane in
 * swrt_qg_export's order into packet slot `slot`: bit for bit the
 * swrt_qg_snapshot(slot, which, layer, ny_period) of the context that exported
 * it, given that context's K_d2, shear and k_scale (2*pi/L for two layers, 1
 * for one).  src_on_device = 1: read after `stream`'s work queued so far (the
 * broadcast that filled it) and before `stream`'s later work (its next fill);
 * 0: host memory.  Runs on the QG stream with swrt_qg_snapshot's renaming: it
 * never waits for a packet launch that still reads the slot. */
int swrt_snapshot_qk(swrt_ctx* ctx, int slot, const double* qk, int src_on_device, void* stream, int64_t nx,
                     double L, double K_d2, double shear, double k_scale, int64_t ny_period);
/* Exchange two packet field slots (the previous step's "current" snapshot
 * becomes the next step's "previous" one without recomputing it). */
int swrt_swap_slots(swrt_ctx* ctx, int a, int b);

/* ---------------------------------------------------------------------------
 * Runtime helpers
 * ------------------------------------------------------------------------ */
/* Hardware conformance check of the hot loop's short IEEE sequences
 * (swrt_kernels.hpp sqrt_rn_normal, rcp_rn_normal, drift_inc's fast path —
 * the half-step drift of ode_symplectic.m:10-16): 16*n random operands over
 * their documented ranges, compared bit for bit with the compiler's IEEE
 * sqrt and division on the device.  mismatches3 = {sqrt, 1/w, drift}; all
 * zero on a conforming device.  Diagnostic; no reference counterpart. */
int swrt_check_arith(swrt_ctx* ctx, int64_t n, uint64_t seed, int64_t* mismatches3);
int swrt_synchronize(swrt_ctx* ctx);
/* The hipStream_t all of ctx's work is ordered on (for external event timing). */
int swrt_get_stream(swrt_ctx* ctx, void** stream_out);
/* Bracket every `every`-th packet-kernel launch with HIP events (default 1;
 * 0 disables).  A timestamped event between two launches costs a few µs of
 * GPU idle, so sampled timing keeps the measurement inside the timed region
 * without perturbing it. */
int swrt_set_timing(swrt_ctx* ctx, int every);
/* Sum of HIP-event-measured durations of the packet kernel launches since the
 * last reset (synchronizes). */
int swrt_kernel_time(swrt_ctx* ctx, int reset, double* total_ms, int64_t* launches);
/* Observed shader clock over a region of the packet stream: swrt_clock_stamp
 * (ctx, 0) before it and (ctx, 1) after it each enqueue (after every queued
 * packet launch) 1024 one-wave workgroups that record the shader-cycle
 * counter (s_memtime), the 100 MHz real-time counter (s_memrealtime) and the
 * CU they ran on; swrt_clock_ghz synchronises and returns the median over
 * the CUs stamped at both ends of cycles / seconds (a CU's own counter: the
 * counters of different CUs are not aligned), and (spread_out, may be NULL)
 * the per-CU clocks' (p90 - p10) / median.  Normalises a throughput measured
 * on one box to the clock it actually ran at (the chip lowers its clock
 * under load). */
int swrt_clock_stamp(swrt_ctx* ctx, int which);
int swrt_clock_ghz(swrt_ctx* ctx, double* ghz_out, double* spread_out);
/* swrt_clock_ghz's arithmetic on given stamps (host only, no context): stamps
 * = `waves` start waves then `waves` end waves, each {shader cycles, realtime
 * ticks, CU id}; realtime_hz the realtime counter's rate (100e6 on gfx950).
 * SWRT_ERR_STATE when no CU holds both a start and an end wave. */
int swrt_clock_ghz_stamps(const uint64_t* stamps, int64_t waves, double realtime_hz, double* ghz_out,
                          double* spread_out);

/* Debug knobs (test infrastructure; no reference counterpart).
 * SWRT_DEBUG_HAZARD_CHECK 0/1: a host-side happens-before checker of the
 *   packet buffers across the packet streams (swrt_set_packet_streams): every
 *   re-binning, part launch, join and synchronisation is mirrored with one
 *   vector clock per stream, each part launch's accesses covering the tiles
 *   its workgroups actually take (the device's own mapping); a launch whose
 *   reads or writes of a packet buffer are not ordered after a conflicting
 *   access on another stream is refused before it is queued (SWRT_ERR_STATE,
 *   swrt_last_error names both accesses).  Also on when the environment has SWRT_HAZARD_CHECK=1 at
 *   swrt_create.  Turning it on synchronises the context.
 * SWRT_DEBUG_SPIN_US n: each extra packet stream runs a ~n us sleep kernel
 *   before every part launch of its own, so a call's extra-stream parts
 *   overlap the next call's packet-stream part (adversarial schedule).
 * SWRT_DEBUG_LEGACY_PARK 0/1: test-only; 1 restores the ordering before the
 *   third packet buffers (the launch after a source-gather sort launch
 *   overwrites the buffer that launch gathers from) — a known race the
 *   checker must report.
 * SWRT_DEBUG_HAZARD_CHECKS (get only): accesses the checker has compared.
 * SWRT_DEBUG_QG_JFUSE 0/1 (default 1): two-layer fused mode runs the inverse
 *   column pass fused with the Jacobian, the CFL max and J's first forward
 *   pass (one kernel); 0 = the separate column pass + Jacobian-rows kernel —
 *   the same values, kept so tests can compare them bit for bit.  Applies
 *   when no packets share the context (beside packet launches the separate
 *   passes' smaller workgroups run faster).
 * SWRT_DEBUG_QG_UPDATE_COLS 0/1 (default 1): fused mode runs the last pass of
 *   J's forward transform inside the AB3 update (one kernel; the spectrum
 *   never goes to memory); 0 = the separate column pass + update — the same
 *   values, kept so tests can compare them bit for bit.  Applies, like
 *   SWRT_DEBUG_QG_JFUSE, unless packet launches share the context beside a
 *   separate QG stream.
 * SWRT_DEBUG_SHARE_SKEW 0/1: test-only; 1 makes the launch that ends each
 *   re-binning cycle split its tiles unevenly between the two packet streams
 *   (2/3 : 1/3) — a tile-to-stream mapping that differs from the previous
 *   launch's, the race of round 4.  Accepted only while the hazard checker is
 *   on, which models the tiles each part launch takes and refuses such a
 *   launch (SWRT_ERR_STATE) before it is queued.
 * SWRT_DEBUG_CORRUPT_COUNT d: test-only; the next re-binning adds d to one
 *   tile's count before its scan.  The scan's own check (counts >= 0, summing
 *   to the packets) then leaves an empty binning — no kernel runs over a bad
 *   range — and the next host synchronisation (swrt_synchronize,
 *   swrt_packets_get, ...) returns SWRT_ERR_STATE; the packet state is lost
 *   until swrt_packets_set.
 * SWRT_DEBUG_ODE23_CHAINED (get only): ode23 calls that took the stage 1 the
 *   previous call queued (swrt_ode23_chain_next).
 * SWRT_DEBUG_ODE23_FIRST_TAKEN, SWRT_DEBUG_ODE23_GUESSES_TAKEN (get only):
 *   swrt_ode23_run calls whose first attempt was the one the device queued
 *   from its own step size, and attempts taken from a gated guess (queued
 *   before the previous attempt's error was known), summed over the calls.
 * SWRT_DEBUG_ODE23_SPLIT_RUNS (get only): swrt_ode23_run calls whose attempts
 *   ran as two part launches on the two packet streams.
 * SWRT_DEBUG_ODE23_FIRST_CHAINED (get only): ode23 calls that took the first
 *   step size and first attempt the previous call queued behind their chained
 *   stage 1 (t0 = 0, tfinal = tmax and RelTol as that call assumed). */
#define SWRT_DEBUG_HAZARD_CHECK 1
#define SWRT_DEBUG_SPIN_US 2
#define SWRT_DEBUG_LEGACY_PARK 3
#define SWRT_DEBUG_HAZARD_CHECKS 4
#define SWRT_DEBUG_QG_JFUSE 5
#define SWRT_DEBUG_QG_UPDATE_COLS 7
#define SWRT_DEBUG_SHARE_SKEW 8
#define SWRT_DEBUG_CORRUPT_COUNT 9
#define SWRT_DEBUG_ODE23_CHAINED 10
#define SWRT_DEBUG_ODE23_FIRST_TAKEN 11
#define SWRT_DEBUG_ODE23_GUESSES_TAKEN 12
#define SWRT_DEBUG_ODE23_SPLIT_RUNS 13
#define SWRT_DEBUG_ODE23_FIRST_CHAINED 14
int swrt_debug_set(swrt_ctx* ctx, int key, int64_t value);
int swrt_debug_get(swrt_ctx* ctx, int key, int64_t* value_out);

#ifdef __cplusplus
}
#endif
#endif /* SWRT_H */
