/*
 * swrt_oracle.c — CPU restatement of the qg_flow_ray_trace packet hot loop.
 * TEST INFRASTRUCTURE ONLY: compiled into oracle/build/libswrt_oracle.so and
 * used by tests/ (checker) and bench.py's cpu_baseline leg.  Never linked
 * into the product library.
 *
 * Same algorithm and same IEEE-754 operation order as the numpy restatement
 * (oracle/swrt_oracle.py), which follows the MATLAB reference:
 *   interpolate.m:12-50        6x6 periodic Lagrange stencil
 *   interpolate_U.m:19-23      two-snapshot blend
 *   ode_symplectic.m:10-37     Strang drift/kick/drift
 *   RaytracingScheme.m:9-16    (grad U)^T k
 * Build with -ffp-contract=off (no FMA contraction) so it is bit-identical to
 * the numpy restatement.  OpenMP over packets (independent given the field).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#define NTAP 6

/* MATLAB mod(a,m) = a - floor(a/m)*m  (m > 0) */
static inline double mmod(double a, double m) { return a - floor(a / m) * m; }

/* interpolate.m:21-41 : cell index (0-based, may equal period) and weights */
static inline int64_t cell_weights(double x, double d, double period, double bump, double w[NTAP]) {
    double xl = mmod(x / d, period);
    double fl = floor(xl);
    double i0 = 1.0 + fl;
    double a = (1.0 + xl) - i0;
    for (int i = -2; i <= 3; ++i) {
        double wi = 1.0;
        for (int j = -2; j <= 3; ++j) {
            if (i != j) wi = wi * ((a - (double)j) + bump) / (double)(j - i);
        }
        w[i + 2] = wi;
    }
    return (int64_t)fl;
}

/* fields: 6 planes (u,v,ux,uy,vx,vy), each nx*nx column-major (F[ig + nx*jg]) */
static void interp6(const double* fields, int64_t nx, double nyF, double dx, double bump,
                    double x, double y, double out[6]) {
    double wx[NTAP], wy[NTAP];
    int64_t ic = cell_weights(x, dx, (double)nx, bump, wx);
    int64_t jc = cell_weights(y, dx, nyF, bump, wy);
    int64_t ig[NTAP], jg[NTAP];
    for (int t = 0; t < NTAP; ++t) {
        int64_t a = (ic + t - 2) % nx; if (a < 0) a += nx; ig[t] = a;
        int64_t b = (jc + t - 2) % nx; if (b < 0) b += nx; jg[t] = b;
    }
    const int64_t plane = nx * nx;
    for (int f = 0; f < 6; ++f) {
        const double* F = fields + f * plane;
        double FI = 0.0;
        for (int i = 0; i < NTAP; ++i)
            for (int j = 0; j < NTAP; ++j)
                FI = FI + wx[i] * wy[j] * F[ig[i] + nx * jg[j]];
        out[f] = FI;
    }
}

/* Evaluate U, grad U (6 values per point) at n points: out is 6 x n (row per field). */
void oracle_eval(const double* fields0, const double* fields1, double alpha, int64_t nx,
                 double nyF, double dx, double bump, const double* x, const double* y, int64_t n,
                 double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < n; ++p) {
        double a[6], b[6];
        interp6(fields0, nx, nyF, dx, bump, x[p], y[p], a);
        if (fields1) {
            interp6(fields1, nx, nyF, dx, bump, x[p], y[p], b);
            for (int f = 0; f < 6; ++f) a[f] = (1 - alpha) * a[f] + alpha * b[f];
        }
        for (int f = 0; f < 6; ++f) out[f * n + p] = a[f];
    }
}

/*
 * Leapfrog over nsteps.  State x,k are N x 2 column-major (x(:,1) then x(:,2)).
 * hist (optional): frames of N x 2 after every save_every steps.
 */
void oracle_leapfrog(const double* fields0, const double* fields1, double alpha0, double dalpha,
                     int64_t nx, double nyF, double dx, double bump, double* x, double* k,
                     int64_t n, double dt, int64_t nsteps, double f, double gH,
                     int64_t save_every, double* hist_x, double* hist_k) {
    const double half = dt / 2;
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < n; ++p) {
        double x0 = x[p], y0 = x[n + p], k0 = k[p], l0 = k[n + p];
        int64_t frame = 0;
        for (int64_t s = 0; s < nsteps; ++s) {
            double w = sqrt(f * f + gH * (k0 * k0 + l0 * l0));
            double x1 = x0 + half * (gH * k0 / w);
            double y1 = y0 + half * (gH * l0 / w);
            double I[6];
            if (fields1) {
                double a[6], b[6];
                double alpha = alpha0 + (double)s * dalpha;
                interp6(fields0, nx, nyF, dx, bump, x1, y1, a);
                interp6(fields1, nx, nyF, dx, bump, x1, y1, b);
                for (int q = 0; q < 6; ++q) I[q] = (1 - alpha) * a[q] + alpha * b[q];
            } else {
                interp6(fields0, nx, nyF, dx, bump, x1, y1, I);
            }
            double x2 = x1 + dt * I[0];
            double y2 = y1 + dt * I[1];
            double k2 = k0 - dt * (I[2] * k0 + I[4] * l0);
            double l2 = l0 - dt * (I[3] * k0 + I[5] * l0);
            w = sqrt(f * f + gH * (k2 * k2 + l2 * l2));
            x0 = x2 + half * (gH * k2 / w);
            y0 = y2 + half * (gH * l2 / w);
            k0 = k2;
            l0 = l2;
            if (save_every > 0 && (s + 1) % save_every == 0 && hist_x) {
                double* hx = hist_x + frame * 2 * n;
                double* hk = hist_k + frame * 2 * n;
                hx[p] = x0; hx[n + p] = y0; hk[p] = k0; hk[n + p] = l0;
                ++frame;
            }
        }
        x[p] = x0; x[n + p] = y0; k[p] = k0; k[n + p] = l0;
    }
}

/*
 * The same leapfrog (same IEEE operations in the same order, so the same
 * bits) arranged for a CPU: used as bench.py's cpu_baseline, not as the
 * checker.  Differences from oracle_leapfrog are ones of layout and reuse only:
 *  - the six fields of a snapshot are interleaved per node in a halo-padded
 *    (nx+5)^2 array (2 ghost nodes below, 3 above), so one stencil row is 36
 *    contiguous doubles and no tap wraps;
 *  - cell and weights are computed once per point for both snapshots and all
 *    six fields (interpolate.m recomputes identical values per call);
 *  - the drift increment half*gH*k/omega(k) is computed once per step: the
 *    closing drift of a step and the opening drift of the next use the same k.
 * Each field's sum keeps interpolate.m:43-49's order (i outer, j inner,
 * FI = FI + (wx_i*wy_j)*F from FI = 0).
 */
static double* pad_nodes(const double* fields, int64_t nx) {
    const int64_t np = nx + 5, plane = nx * nx;
    double* nodes = (double*)malloc(sizeof(double) * 6 * np * np);
    for (int64_t ip = 0; ip < np; ++ip)
        for (int64_t jp = 0; jp < np; ++jp) {
            int64_t ig = ((ip - 2) % nx + nx) % nx, jg = ((jp - 2) % nx + nx) % nx;
            for (int f = 0; f < 6; ++f) nodes[(ip * np + jp) * 6 + f] = fields[f * plane + ig + nx * jg];
        }
    return nodes;
}

static inline void gather_nodes(const double* nodes, int64_t np, int64_t ic, int64_t jc, const double wx[NTAP],
                                const double wy[NTAP], double out[6]) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0, s5 = 0.0;
    for (int i = 0; i < NTAP; ++i) {
        const double* row = nodes + ((ic + i) * np + jc) * 6;
        for (int j = 0; j < NTAP; ++j) {
            const double wij = wx[i] * wy[j];
            const double* r = row + 6 * j;
            s0 = s0 + wij * r[0]; s1 = s1 + wij * r[1]; s2 = s2 + wij * r[2];
            s3 = s3 + wij * r[3]; s4 = s4 + wij * r[4]; s5 = s5 + wij * r[5];
        }
    }
    out[0] = s0; out[1] = s1; out[2] = s2; out[3] = s3; out[4] = s4; out[5] = s5;
}

void oracle_leapfrog_fast(const double* fields0, const double* fields1, double alpha0, double dalpha,
                          int64_t nx, double nyF, double dx, double bump, double* x, double* k,
                          int64_t n, double dt, int64_t nsteps, double f, double gH) {
    const double half = dt / 2;
    const int64_t np = nx + 5;
    double* n0 = pad_nodes(fields0, nx);
    double* n1 = fields1 ? pad_nodes(fields1, nx) : NULL;
#pragma omp parallel for schedule(static)
    for (int64_t p = 0; p < n; ++p) {
        double x0 = x[p], y0 = x[n + p], k0 = k[p], l0 = k[n + p];
        double w = sqrt(f * f + gH * (k0 * k0 + l0 * l0));
        double hcx = half * (gH * k0 / w), hcy = half * (gH * l0 / w);
        for (int64_t s = 0; s < nsteps; ++s) {
            const double x1 = x0 + hcx, y1 = y0 + hcy;
            double wx[NTAP], wy[NTAP], I[6];
            int64_t ic = cell_weights(x1, dx, (double)nx, bump, wx) % nx;
            int64_t jc = cell_weights(y1, dx, nyF, bump, wy) % nx;
            if (ic < 0 || ic >= nx) ic = 0;  /* NaN position: any in-range cell (the result is NaN) */
            if (jc < 0 || jc >= nx) jc = 0;
            gather_nodes(n0, np, ic, jc, wx, wy, I);
            if (n1) {
                double b[6];
                const double alpha = alpha0 + (double)s * dalpha;
                gather_nodes(n1, np, ic, jc, wx, wy, b);
                for (int q = 0; q < 6; ++q) I[q] = (1 - alpha) * I[q] + alpha * b[q];
            }
            const double x2 = x1 + dt * I[0];
            const double y2 = y1 + dt * I[1];
            const double k2 = k0 - dt * (I[2] * k0 + I[4] * l0);
            const double l2 = l0 - dt * (I[3] * k0 + I[5] * l0);
            w = sqrt(f * f + gH * (k2 * k2 + l2 * l2));
            hcx = half * (gH * k2 / w);
            hcy = half * (gH * l2 / w);
            x0 = x2 + hcx;
            y0 = y2 + hcy;
            k0 = k2;
            l0 = l2;
        }
        x[p] = x0; x[n + p] = y0; k[p] = k0; k[n + p] = l0;
    }
    free(n0);
    free(n1);
}

/* Thread count of the next oracle calls (n <= 0: all processors). */
void oracle_set_threads(int n) {
#ifdef _OPENMP
    extern void omp_set_num_threads(int);
    extern int omp_get_num_procs(void);
    omp_set_num_threads(n > 0 ? n : omp_get_num_procs());
#else
    (void)n;
#endif
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    extern int omp_get_max_threads(void);
    return omp_get_max_threads();
#else
    return 1;
#endif
}
