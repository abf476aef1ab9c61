// swrt_cli — the packet hot loop driven through the C ABI alone (no Python,
// no torch): the third front-end of SURVEY §7 next to the MEX gateway and
// the ctypes mirror, and what a C/C++ host (or a MATLAB engine app) links.
//
// Workload = bench.py's (BASELINE.json configs[3]): 2-layer QG background,
// layer 1 (L = 20, k scaled by 2*pi/L, shear 0.5, y-period 2*nx), two
// snapshots blended (interpolate_U), packets on the omega0 = 4f ring
// (f = 3, Cg = 1), one call per PDE interval dt = 0.25*dx/U0 advanced by
// --substeps (5) leapfrog steps of 0.05*dx/U0, re-binning every --rebin (20)
// steps.  Synthetic random-phase ring spectrum 10 < |k| <= 30
// normalised to max|U| = 0.2 (std::mt19937_64, not bench.py's numpy stream).
//
//   swrt_cli [--nx 512] [--packets 1000000] [--steps 50] [--warmup 5]
//            [--device 0] [--substeps 5] [--rebin 20]
// Prints one JSON line: packet-steps/s (wall clock over the timed steps,
// synchronised) and the sampled kernel time per launch.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "swrt.h"

namespace {

int check(swrt_ctx* c, int rc, const char* what) {
  if (rc != SWRT_OK) {
    std::fprintf(stderr, "swrt_cli: %s failed (%d): %s\n", what, rc, c ? swrt_last_error(c) : "");
    std::exit(1);
  }
  return rc;
}

// half-plane qk, (2kmax+1) x (kmax+1) column-major interleaved complex:
// unit-amplitude random phases on kmin < |k| <= kring, then a phase jitter
// of `jitter` radians (the second snapshot)
std::vector<double> ring_spectrum(int nx, int kmin, int kring, std::mt19937_64& rng, double jitter,
                                  double scale) {
  const int kmax = nx / 2 - 1, nkx = 2 * kmax + 1;
  std::vector<double> qk(2 * (size_t)nkx * (kmax + 1), 0.0);
  std::uniform_real_distribution<double> ph(0.0, 2 * M_PI);
  std::normal_distribution<double> jit(0.0, 1.0);
  for (int ky = 0; ky <= kmax; ++ky)
    for (int kx = -kmax; kx <= kmax; ++kx) {
      const double p = ph(rng) + jitter * jit(rng);
      const int r2 = kx * kx + ky * ky;
      if (r2 > kmin * kmin && r2 <= kring * kring) {
        const size_t i = (size_t)(kx + kmax) + (size_t)nkx * ky;
        qk[2 * i] = scale * std::cos(p);
        qk[2 * i + 1] = scale * std::sin(p);
      }
    }
  return qk;
}

double max_speed(swrt_ctx* c, int slot, int nx, double shear) {
  std::vector<double> f((size_t)6 * nx * nx);
  check(c, swrt_get_field_grid(c, slot, f.data()), "swrt_get_field_grid");
  double m = 0.0;
  const size_t plane = (size_t)nx * nx;
  for (size_t i = 0; i < plane; ++i) {
    const double u = f[i] - shear, v = f[plane + i];
    m = std::fmax(m, u * u + v * v);
  }
  return std::sqrt(m);
}

}  // namespace

int main(int argc, char** argv) {
  int nx = 512, device = 0, steps = 50, warmup = 5, substeps = 5, rebin = 20;
  long long npk = 1000000;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) { std::fprintf(stderr, "swrt_cli: %s needs a value\n", a.c_str()); std::exit(2); }
      return argv[++i];
    };
    if (a == "--nx") nx = std::atoi(next());
    else if (a == "--packets") npk = std::atoll(next());
    else if (a == "--steps") steps = std::atoi(next());
    else if (a == "--warmup") warmup = std::atoi(next());
    else if (a == "--device") device = std::atoi(next());
    else if (a == "--substeps") substeps = std::atoi(next());
    else if (a == "--rebin") rebin = std::atoi(next());
    else if (a == "--help" || a == "-h") {
      std::printf("usage: swrt_cli [--nx N] [--packets P] [--steps K] [--warmup W] [--device D] [--substeps S] "
                  "[--rebin R]\n");
      return 0;
    } else {
      std::fprintf(stderr, "swrt_cli: unknown option %s\n", a.c_str());
      return 2;
    }
  }
  if (nx < 32 || (nx & (nx - 1)) != 0 || npk <= 0 || steps <= 0 || substeps <= 0 || rebin < 0) {
    std::fprintf(stderr, "swrt_cli: nx must be a power of two >= 32; packets, steps, substeps > 0; rebin >= 0\n");
    return 2;
  }
  const double L = 20.0, f = 3.0, Cg = 1.0, Ug = 0.2, shear = 0.5, K_d2 = f / Cg;
  const double ks = 2 * M_PI / L, bump = 1e-10;  // qg_flow_ray_trace/interpolate.m:13
  swrt_ctx* c = nullptr;
  check(nullptr, swrt_create(device, &c), "swrt_create");

  std::mt19937_64 rng(146);
  auto q1 = ring_spectrum(nx, 10, 30, rng, 0.0, 1.0);
  std::mt19937_64 rng2(147);
  auto q2 = q1;  // slot 1: the same spectrum with jittered phases
  {
    std::normal_distribution<double> jit(0.0, 0.05);
    for (size_t i = 0; i + 1 < q2.size(); i += 2) {
      const double p = jit(rng2), cr = std::cos(p), sr = std::sin(p);
      const double re = q2[i], im = q2[i + 1];
      q2[i] = re * cr - im * sr;
      q2[i + 1] = re * sr + im * cr;
    }
  }
  // normalise to max|U| = Ug (initial_q, qg2layersw_raytrace.m:279-280)
  check(c, swrt_set_field_qk(c, 0, q1.data(), nx, L, K_d2, 0.0, ks, 2 * nx), "swrt_set_field_qk");
  const double s = Ug / max_speed(c, 0, nx, 0.0);
  for (auto& v : q1) v *= s;
  for (auto& v : q2) v *= s;
  check(c, swrt_set_field_qk(c, 0, q1.data(), nx, L, K_d2, shear, ks, 2 * nx), "swrt_set_field_qk");
  check(c, swrt_set_field_qk(c, 1, q2.data(), nx, L, K_d2, shear, ks, 2 * nx), "swrt_set_field_qk");
  const double U0 = max_speed(c, 0, nx, 0.0);  // with the shear, as the drivers' CFL sees it
  const double dt = 0.25 * (L / nx) / U0;      // qg2layersw_raytrace.m:31,78

  // packets: uniform in [-L/2, L/2)^2, k on the omega0 = 4f ring (qgsw_raytrace.m:56-60)
  std::vector<double> x(2 * (size_t)npk), k(2 * (size_t)npk);
  std::uniform_real_distribution<double> u01(0.0, 1.0);
  const double wf = std::sqrt((16.0 - 1.0) * f * f / (Cg * Cg));
  for (long long i = 0; i < npk; ++i) {
    x[i] = L * u01(rng) - L / 2;
    x[npk + i] = L * u01(rng) - L / 2;
    const double th = 2 * M_PI * (double)(i + 1) / (double)npk;
    k[i] = wf * std::cos(th);
    k[npk + i] = wf * std::sin(th);
  }
  check(c, swrt_packets_set(c, x.data(), k.data(), npk), "swrt_packets_set");
  check(c, swrt_set_locality(c, rebin, 0), "swrt_set_locality");

  const double h = dt / substeps;
  auto step = [&]() {
    check(c, swrt_advance(c, h, substeps, f, Cg * Cg, 2, 0.5 / substeps, 1.0 / substeps, bump, 0),
          "swrt_advance");
  };
  for (int i = 0; i < warmup; ++i) step();
  check(c, swrt_synchronize(c), "swrt_synchronize");
  check(c, swrt_set_timing(c, 5), "swrt_set_timing");
  double kms = 0.0;
  int64_t launches = 0;
  check(c, swrt_kernel_time(c, 1, &kms, &launches), "swrt_kernel_time");
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < steps; ++i) step();
  check(c, swrt_synchronize(c), "swrt_synchronize");
  const auto t1 = std::chrono::steady_clock::now();
  check(c, swrt_kernel_time(c, 1, &kms, &launches), "swrt_kernel_time");
  const double el = std::chrono::duration<double>(t1 - t0).count();
  check(c, swrt_packets_get(c, x.data(), k.data()), "swrt_packets_get");
  bool finite = true;
  for (size_t i = 0; i < x.size(); ++i) finite = finite && std::isfinite(x[i]) && std::isfinite(k[i]);
  std::printf("{\"metric\": \"packet-steps/sec @ %d^2 field, %lld packets (C ABI driver)\", \"value\": %.6g, "
              "\"unit\": \"packet-steps/s\", \"steps\": %d, \"substeps\": %d, \"ms_per_step\": %.6g, "
              "\"avg_launch_ms\": %.6g, \"timed_launches\": %lld, \"dtype\": \"f64\", \"finite\": %s}\n",
              nx, npk, (double)npk * substeps * steps / el, steps, substeps, el / steps * 1e3,
              launches > 0 ? kms / launches : 0.0, (long long)launches, finite ? "true" : "false");
  swrt_destroy(c);
  return finite ? 0 : 3;
}
