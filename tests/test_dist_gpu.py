"""The sharded multi-GPU path on one GPU: two processes (torch.distributed.run,
gloo backend so both ranks may share GPU 0 — RCCL refuses two ranks on one
device), each running the HIP packet path on its contiguous shard with the
field replicated, then the device-side gather (swraytracing_amd.dist.
gather_packets: swrt_packets_get_device into a torch buffer, one all_gather).
The gathered trajectories must equal a single-process run bit for bit (the
packet kernels are bit-exact whatever the ensemble's size, order or binning)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["SWRT_ROOT"])
import swraytracing_amd as sw
from swraytracing_amd.dist import gather_packets, shard_range
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
w = np.load(sys.argv[1])
nx, N = int(w["nx"]), w["x"].shape[0]
ctx = sw.Context(0)
ctx.set_locality(4, 0)
ctx.set_field_grid(0, w["p0"], nx, float(w["L"]), 2 * nx)
ctx.set_field_grid(1, w["p1"], nx, float(w["L"]), 2 * nx)
lo, hi = shard_range(N, world, rank)
ctx.packets_set(w["x"][lo:hi], w["k"][lo:hi])
for s in range(int(w["calls"])):
    ctx.advance(float(w["dt"]), int(w["nsub"]), 3.0, 1.0, nslots=2, alpha0=0.1, dalpha=0.15, bump=sw.BUMP_QG)
out = gather_packets(ctx, N, world, rank)
if rank == 0:
    np.savez(sys.argv[2], x=out[0], k=out[1])
ctx.close()
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_sharded_hip_path_gathers_bit_identical(ctx, tmp_path):
    from oracle import swrt_oracle as orc
    nx, L, N = 128, 20.0, 30_001  # odd: the shards differ by one packet
    rng = np.random.default_rng(2)
    kmax = nx // 2 - 1
    qk = np.zeros((2 * kmax + 1, kmax + 1), complex)
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(kmax + 1)[None, :]
    ring = (kx * kx + ky * ky > 9) & (kx * kx + ky * ky <= 100)
    qk[ring] = 0.01 * np.exp(2j * np.pi * rng.random(ring.sum()))
    ctx.set_field_qk(0, qk, nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
    ctx.set_field_qk(1, qk * np.exp(0.1j), nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
    p0, p1 = ctx.get_field_grid(0, nx), ctx.get_field_grid(1, nx)
    x, k = orc.initial_packets(N, L, 4.0, 3.0, 1.0, rng)
    w = dict(nx=nx, L=L, p0=p0, p1=p1, x=x, k=k, dt=0.02, nsub=5, calls=6)
    np.savez(tmp_path / "in.npz", **w)
    # single process, same calls
    ctx.set_locality(4, 0)
    ctx.set_field_grid(0, p0, nx, L, 2 * nx)
    ctx.set_field_grid(1, p1, nx, L, 2 * nx)
    ctx.packets_set(x, k)
    for _ in range(w["calls"]):
        ctx.advance(w["dt"], w["nsub"], 3.0, 1.0, nslots=2, alpha0=0.1, dalpha=0.15, bump=orc.BUMP_QG)
    xr, kr = ctx.packets_get()
    (tmp_path / "worker.py").write_text(WORKER)
    env = dict(os.environ, SWRT_ROOT=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(tmp_path / "worker.py"),
           str(tmp_path / "in.npz"), str(tmp_path / "out.npz")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(tmp_path / "out.npz")
    assert got["x"].shape == (N, 2)
    np.testing.assert_array_equal(got["x"], xr)
    np.testing.assert_array_equal(got["k"], kr)


DRIVER = r"""
import os, sys
import torch
import torch.distributed as dist
sys.path.insert(0, os.environ["SWRT_ROOT"])
import swraytracing_amd as sw
torch.cuda.set_device(0)
dist.init_process_group("gloo")
ctx = sw.Context(0)
drv, integrator, pde, w0, lb = sys.argv[2], sys.argv[3], sys.argv[4], float(sys.argv[5]), sys.argv[6]
if drv == "qg2":
    sw.qg2layersw_raytrace(64, 5001, 4.0, 10.0, 0.0, 0.2, 3.0, 1.0, out_dir=sys.argv[1], nsub=2, max_steps=30,
                           seed=5, integrator=integrator, ctx=ctx, pde=pde, owner_weight=w0, link_buffers=lb)
else:
    sw.qgsw_raytrace(64, 4001, 4.0, 20.0, 0.0, 0.2, 3.0, 1.0, out_dir=sys.argv[1], nsub=2, max_steps=24,
                     integrator=integrator, r_drag=0.0, ctx=ctx, pde=pde, owner_weight=w0, link_buffers=lb)
ctx.close()
dist.destroy_process_group()
"""

_REF = {}


def _single(ctx, tmp_path, drv, integrator):
    """The single-process run's files (cached per driver and integrator)."""
    import swraytracing_amd as sw
    key = (drv, integrator)
    if key not in _REF:
        ref = tmp_path / "single"
        if drv == "qg2":
            sw.qg2layersw_raytrace(64, 5001, 4.0, 10.0, 0.0, 0.2, 3.0, 1.0, out_dir=str(ref), nsub=2, max_steps=30,
                                   seed=5, integrator=integrator, ctx=ctx)
        else:
            sw.qgsw_raytrace(64, 4001, 4.0, 20.0, 0.0, 0.2, 3.0, 1.0, out_dir=str(ref), nsub=2, max_steps=24,
                             integrator=integrator, r_drag=0.0, ctx=ctx)
        _REF[key] = {n: (ref / n).read_bytes() for n in ("packet_x.bin", "packet_k.bin", "packet_time.bin", "pv.bin")}
    return _REF[key]


def _rank_report(stderr, tail=40):
    """The last lines of each rank's own output ([rankN]: prefixes) and of the
    launcher, so a failing rank's traceback is never cut off by another's."""
    by = {}
    for ln in stderr.splitlines():
        key = ln.split("]:", 1)[0] + "]" if ln.startswith("[rank") else "launcher"
        by.setdefault(key, []).append(ln)
    return "\n".join(f"--- {k} ---\n" + "\n".join(v[-tail:]) for k, v in sorted(by.items()))


@pytest.mark.parametrize("drv,world,pde,w0,integrator,lb", [
    ("qg2", 2, "replicated", 1.0, "leapfrog", "auto"),
    ("qg2", 2, "replicated", 1.0, "ode23", "auto"),
    ("qg2", 2, "owner", 0.5, "leapfrog", "host"),
    ("qg2", 2, "owner", 0.5, "ode23", "host"),
    ("qg2", 4, "owner", 0.5, "leapfrog", "host"),
    ("qg2", 4, "owner", 0.5, "ode23", "host"),
    ("qg2", 2, "owner", 0.0, "ode23", "host"),  # the owner holds no packets: it only joins the collectives
    ("qg1", 2, "owner", 0.5, "leapfrog", "host"),
    # the nccl form of the link (device buffers, the export and the
    # receivers' snapshots fenced on the host, dt on a gloo side group) over
    # gloo's CUDA-tensor broadcast: RCCL itself needs one GPU per rank
    ("qg2", 2, "owner", 0.5, "leapfrog", "device"),
    ("qg2", 4, "owner", 0.25, "leapfrog", "device"),
    ("qg2", 2, "owner", 0.5, "ode23", "device"),
    ("qg1", 2, "owner", 0.5, "leapfrog", "device"),
])
def test_sharded_driver_files_equal_single_process(ctx, tmp_path, drv, world, pde, w0, integrator, lb):
    """The drivers sharded over `world` ranks sharing GPU 0 (gloo), frames
    gathered on the device and written by rank 0, ode23's error norm
    max-reduced over the ranks: with the replicated PDE (every rank steps it,
    packets split evenly) and in the PDE-owner form (rank 0 steps the PDE and
    broadcasts each step's top-layer qk and dt, qg2layersw_raytrace.m:186-188;
    the others build their snapshots from it, swrt_snapshot_qk), the run
    writes the same packet_x/k/time.bin and pv.bin as one process, byte for
    byte."""
    ref = _single(ctx, tmp_path, drv, integrator)
    (tmp_path / "driver.py").write_text(DRIVER)
    out = tmp_path / "sharded"
    env = dict(os.environ, SWRT_ROOT=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(tmp_path / "driver.py"), str(out),
           drv, integrator, pde, str(w0), lb]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, _rank_report(r.stderr)
    for name, a in ref.items():
        b = (out / name).read_bytes()
        assert len(a) > 0 and a == b, name


@pytest.mark.parametrize("driver", ["none", "owner"])
def test_bench_gpus_2_strong_scaling_line(tmp_path, driver):
    """`bench.py --gpus 2` with no torch.distributed environment launches two
    ranks as a child torch.distributed.run (gloo: both share GPU 0) and relays
    rank 0's line: n_gpus 2, the metric's 1e6 packets split 5e5 per GPU; with
    `--driver-pde owner` also the driver step in the PDE-owner form."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    extra = ["--driver-steps", "0"] if driver == "none" else ["--driver-steps", "5", "--driver-warmup", "4",
                                                              "--driver-pde", "owner", "--owner-weight", "0.25",
                                                              "--no-forecast"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "3", "--warmup", "1", "--ode23-steps", "0", "--no-cpu-baseline", "--gather"] + extra,
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    # every rank's own last lines (a failing rank's traceback sits mid-stream, before the launcher's report)
    assert r.returncode == 0, _rank_report(r.stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["config"]["packets_total"] == 1_000_000 and out["config"]["packets_per_gpu"] == 500_000
    assert out["value"] > 0 and out["finite"] and out["gathered_finite"]
    if driver == "owner":
        d = out["driver_step"]
        assert d["pde"].startswith("owner form") and d["ms_per_pde_step"] > 0
