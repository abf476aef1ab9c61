"""Host submission cost per swrt_advance call vs GPU time (diagnostic)."""
import time, sys, os
import numpy as np
import torch  # noqa: F401  (one HIP runtime)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import swraytracing_amd as sw
from bench import ring_spectrum
ctx = sw.Context(0)
nx, L = 512, 20.0
rng = np.random.default_rng(1)
qk = ring_spectrum(nx, 10, 30, rng) * 0.01
ctx.set_field_qk(0, qk, nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
ctx.set_field_qk(1, qk, nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
for n in (1000, 1_000_000):
    x = L * rng.random((n, 2)) - L / 2
    k = rng.normal(size=(n, 2)) * 10
    ctx.packets_set(x, k)
    ctx.set_timing(0)
    ctx.advance(0.001, 8, 3.0, 1.0, nslots=2); ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        ctx.advance(0.001, 1, 3.0, 1.0, nslots=2)
    t1 = time.perf_counter()
    ctx.synchronize()
    t2 = time.perf_counter()
    ctx.advance(0.001, 200, 3.0, 1.0, nslots=2)
    t3 = time.perf_counter()
    ctx.synchronize()
    t4 = time.perf_counter()
    print(f"n={n}: 200x advance(1): submit {1e6*(t1-t0)/200:.1f} us/call, total {1e6*(t2-t0)/200:.1f} us/step; "
          f"advance(200): submit {1e6*(t3-t2)/200:.1f} us/step, total {1e6*(t4-t2)/200:.1f} us/step")
