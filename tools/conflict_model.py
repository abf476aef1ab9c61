"""Diagnostic (CPU, test infrastructure only): ds_read_b128 bank-conflict
model of the tile kernel's LDS gather over one re-binning cycle.

Rebuilds the bench field (bench.py build_workload, numpy oracle grid_U),
advances the packets of a block of tiles with the C oracle, and for each
launch of the 4-step cycle counts, per 16-lane ds_read_b128 group, the LDS
cycles max_q #distinct nodes on 16-B slot q (node n -> slot n mod 16, row
stride WS).  Every tap shifts all of a group's nodes by the same offset, so
one count per group and launch stands for all 180 reads.  Compares in-tile
sort keys (performance only: any order gives the same results)."""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cbind, swrt_oracle as orc  # noqa: E402

T, M, WS = 16, 3, 28  # tile cells, margin, window row stride (--tile 32: 32, 3, 44)


def zorder(dx, dy):
    k = np.zeros_like(dx)
    for b in range(5):
        k |= ((dy >> b) & 1) << (2 * b) | ((dx >> b) & 1) << (2 * b + 1)
    return k


def lane_rank_groups():
    """rank (0..63) of each lane, and the b128 group of each lane"""
    rank = np.zeros(64, int)
    for lane in range(64):
        h, t = lane & 32, lane & 31
        if t < 4: k = t
        elif t < 12: k = 16 + (t - 4)
        elif t < 16: k = 4 + (t - 12)
        elif t < 20: k = 24 + (t - 16)
        elif t < 28: k = 8 + (t - 20)
        else: k = t
        rank[lane] = h + k
    grp = np.zeros(64, int)
    for lane in range(64):
        t = lane & 31
        g = 0 if (t < 4 or 12 <= t < 16 or 20 <= t < 28) else 1
        grp[lane] = g + (2 if lane >= 32 else 0)
    return rank, grp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=512)
    ap.add_argument("--tiles", type=int, default=6, help="side of the block of tiles simulated")
    ap.add_argument("--cfl", type=float, default=0.05, help="leapfrog dt in units of dx/U0 (bench: 0.05)")
    ap.add_argument("--cycle", type=int, default=20, help="steps between re-binnings (bench: 20)")
    ap.add_argument("--launch", type=int, default=5, help="steps per launch (bench: 5)")
    ap.add_argument("--packets", type=int, default=1_000_000, help="ensemble size (a strong-scaling shard: 125000)")
    ap.add_argument("--tile", type=int, default=16, help="tile cells (16, or 32 with row stride 44)")
    ap.add_argument("--only-deal", action="store_true", help="only the Z-order baseline and the class deal")
    args = ap.parse_args()
    global T, WS
    if args.tile == 32:
        T, WS = 32, 44
    nx, L, f, Cg, Ug = args.nx, 20.0, 3.0, 1.0, 0.2
    rng = np.random.default_rng(146)
    import bench
    qk1 = bench.ring_spectrum(nx, 10, 30, rng)
    qk2 = qk1 * np.exp(1j * np.random.default_rng(147).normal(0, 0.05, qk1.shape))
    kx_, ky_, K2 = orc.wavenumber_grids(nx, L, scale=True)
    fl = orc.grid_U(qk1, f / Cg, K2, kx_, ky_, 0.0)
    s = Ug / math.sqrt(float((np.asarray(fl["u"]) ** 2 + np.asarray(fl["v"]) ** 2).max()))
    fl1 = orc.grid_U(qk1 * s, f / Cg, K2, kx_, ky_, 0.5)
    fl2 = orc.grid_U(qk2 * s, f / Cg, K2, kx_, ky_, 0.5)
    p0, p1 = cbind.planes_of(fl1), cbind.planes_of(fl2)
    U0 = math.sqrt(float((np.asarray(fl1["u"]) ** 2 + np.asarray(fl1["v"]) ** 2).max()))
    dx = L / nx
    dt = args.cfl * dx / U0
    N = args.packets
    x = L * rng.random((N, 2)) - L / 2
    i = np.arange(1, N + 1)
    wf = math.sqrt(15 * f * f)
    k = np.stack([wf * np.cos(2 * np.pi * i / N), wf * np.sin(2 * np.pi * i / N)], axis=1)
    # packets of a block of tiles (by the binning cell of x0)
    cell = np.floor(x / dx).astype(int) % nx
    nt = args.tiles
    sel = (cell[:, 0] // T < nt) & (cell[:, 1] // T < nt)
    x, k = x[sel], k[sel]
    n = x.shape[0]
    R = args.cycle
    _, _, hx, hk = cbind.leapfrog(p0, p1, 0.5, 0.0, nx, 2 * nx, dx, orc.BUMP_QG, x, k, dt, R, f, 1.0, save_every=1)
    X = [x] + [hx[j].T for j in range(R - 1)]  # state at the start of steps 0..R-1
    K = [k] + [hk[j].T for j in range(R - 1)]
    half = 0.5 * dt

    def x1(j):
        w = np.sqrt(f * f + (K[j] ** 2).sum(1))
        return X[j] + half * K[j] / w[:, None]

    def cells(p):
        return np.floor(p / dx).astype(int) % nx

    tile0 = cells(X[0]) // T
    rank, grp = lane_rank_groups()
    w0 = np.sqrt(f * f + (K[0] ** 2).sum(1))
    cg0 = K[0] / w0[:, None]
    x1_0 = x1(0)
    U = cbind.eval6(p0, p1, 0.5, nx, 2 * nx, dx, orc.BUMP_QG, x1_0[:, 0], x1_0[:, 1])[:2].T
    policies = {"x0 (no lead)": X[0]}
    for frac in (0.25, 0.4, 0.5, 0.6):
        policies[f"x0 + {frac:g} R dt cg"] = X[0] + frac * R * dt * cg0
    policies[f"x1 + 0.5 R dt (cg + U(x1))"] = x1_0 + 0.5 * R * dt * (cg0 + U)
    policies["exact x1 each step (sort every step)"] = None
    # the tile order of the 0.5 lead, then every launch (args.launch steps)
    # each wave's 64 packets re-ordered among its lanes by the Z-order of
    # their cell led half a launch (the wave keeps its packets)
    lead = X[0] + 0.5 * R * dt * cg0
    policies["0.5 lead + in-wave re-sort per launch"] = ("wave", lead)
    policies["class deal per step (quad of x1, over the tile)"] = "deal"
    if args.only_deal:
        policies = {k: v for k, v in policies.items() if k.startswith("x0 + 0.5") or isinstance(v, str)}
    for name, keypos in policies.items():
        if isinstance(keypos, str):  # per step: deal the tile's packets to 16-lane groups by LDS slot class
            tot = np.zeros(R)
            base = np.zeros(R)
            for tx in range(nt):
                for ty in range(nt):
                    m = np.where((tile0[:, 0] == tx) & (tile0[:, 1] == ty))[0]
                    if len(m) == 0:
                        continue
                    for j in range(R):
                        cj = cells(x1(j)[m])
                        node = (cj[:, 0] - tx * T + M) * WS + (cj[:, 1] - ty * T + M)
                        q = node % 16
                        o = np.argsort(q, kind="stable")
                        G = -(-len(m) // 16)
                        grp_of = np.empty(len(m), int)
                        grp_of[o] = np.arange(len(m)) % G
                        for g in range(G):
                            nd = np.unique(node[grp_of == g])
                            if len(nd) == 0:
                                continue
                            tot[j] += np.bincount(nd % 16, minlength=16).max()
                            base[j] += 1
            per = tot / base
            print(f"{name:42s} LDS cycles / conflict-free: first {per[0]:.3f} mid {per[R // 2]:.3f} last {per[-1]:.3f}"
                  f"   mean {tot.sum() / base.sum():.3f}")
            continue
        wave_mode = isinstance(keypos, tuple)
        if wave_mode:
            keypos = keypos[1]
        tot = np.zeros(R)
        base = np.zeros(R)
        for tx in range(nt):
            for ty in range(nt):
                m = np.where((tile0[:, 0] == tx) & (tile0[:, 1] == ty))[0]
                for j in range(R):
                    kp = keypos if keypos is not None else x1(j)
                    c = cells(kp[m])
                    key = zorder(np.clip(c[:, 0] - tx * T, 0, T - 1), np.clip(c[:, 1] - ty * T, 0, T - 1))
                    order = m[np.argsort(key, kind="stable")]
                    if wave_mode:
                        j0 = (j // args.launch) * args.launch
                        wk = X[j0] + 0.5 * args.launch * dt * (K[j0] / np.sqrt(f * f + (K[j0] ** 2).sum(1))[:, None])
                        order = order.copy()
                        for w0_ in range(0, len(order), 64):
                            blk = order[w0_:w0_ + 64]
                            cw = cells(wk[blk])
                            kk = zorder(np.clip(cw[:, 0] - tx * T, 0, T - 1), np.clip(cw[:, 1] - ty * T, 0, T - 1))
                            order[w0_:w0_ + 64] = blk[np.argsort(kk, kind="stable")]
                    cj = cells(x1(j)[order])
                    node = (cj[:, 0] - tx * T + M) * WS + (cj[:, 1] - ty * T + M)
                    for w0_ in range(0, len(order), 64):
                        nodes = node[w0_:w0_ + 64]
                        for g in range(4):
                            lanes = [l for l in range(64) if grp[l] == g and rank[l] < len(nodes)]
                            if not lanes:
                                continue
                            nd = np.unique(nodes[rank[lanes]])
                            cnt = np.bincount(nd % 16, minlength=16)
                            tot[j] += cnt.max()
                            base[j] += 1
        per = tot / base
        print(f"{name:42s} LDS cycles / conflict-free: first {per[0]:.3f} mid {per[R // 2]:.3f} last {per[-1]:.3f}"
              f"   mean {tot.sum() / base.sum():.3f}")


if __name__ == "__main__":
    main()
