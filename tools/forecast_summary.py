"""Summarise a bench.py line's scaling forecasts: the packets-only strong
scaling, the replicated-PDE driver step and the PDE-owner driver step (every
leg measured).  usage: python tools/forecast_summary.py <bench.json>"""
import json
import sys


def main(path):
    lines = [ln for ln in open(path).read().splitlines() if ln.startswith("{")]
    d = json.loads(lines[-1])
    print(f"value {d['value']:.4g}  clock {d['roofline'].get('clock_ghz_observed')}")
    ds = d.get("driver_step", {})
    print(f"driver step (1 GPU, all packets) {ds.get('ms_per_pde_step', float('nan')):.4f} ms")
    ss = d.get("strong_scaling_forecast", {})
    if ss:
        print("packets alone:", {G: round(v["efficiency"], 3) for G, v in ss.items()})
    fc = d.get("driver_step_forecast")
    if not fc:
        return
    print(f"pde_alone {fc['pde_alone_ms']:.4f} ms; replicated:",
          {G: (round(fc[G]["ms_per_pde_step"], 4), round(fc[G]["efficiency"], 3)) for G in "248" if G in fc})
    o = fc.get("owner")
    if not o:
        return
    for G in "248":
        b = o[G]
        print(f"owner G={G}: w={b['owner_weight']} n0={b['packets_owner']} nr={b['packets_per_receiver']} "
              f"owner {b['owner_ms']:.4f} recv {b['receiver_ms']:.4f} step {b['step_ms']:.4f} "
              f"eff {b['efficiency']:.3f}")
        for leg in b["legs"]:
            print(f"     w={leg['owner_weight']:<5} n0={leg['packets_owner']:<7} nr={leg['packets_per_receiver']:<8} "
                  f"owner {leg['owner_ms']:.4f} recv {leg['receiver_ms']:.4f}")


if __name__ == "__main__":
    main(sys.argv[1])
