"""Print the numbers of a bench.py JSON line that a session log needs: the
headline, the roofline fractions, the strong-scaling forecasts (one interval
and multi-interval calls), the driver-step forecast.
usage: python tools/summarize_bench.py <file with the bench line>"""
import json
import sys


def main():
    line = [t for t in open(sys.argv[1]) if t.startswith("{")][-1]
    d = json.loads(line)
    r = d.get("roofline", {})
    print("value %.4e  ms/step %.4f  frac %s  alg_frac %.3f" % (d["value"], d["ms_per_step"], r.get("frac"),
                                                              r.get("algorithmic_frac") or 0.0))
    for key in ("strong_scaling_forecast", "strong_scaling_forecast_intervals"):
        fc = d.get(key)
        if not fc:
            continue
        row = ["%s:%.3e/%.2f" % (G, v["value_1gpu"], v["efficiency"]) for G, v in fc.items() if isinstance(v, dict)]
        print(key, " ".join(row))
    ds = d.get("driver_step")
    if ds:
        print("driver_step %.4f ms" % ds["ms_per_pde_step"])
    fc = d.get("driver_step_forecast")
    if fc:
        row = ["%s:%.4fms/%.2f/%s" % (G, v["ms_per_pde_step"], v["efficiency"], v.get("bound"))
               for G, v in fc.items() if isinstance(v, dict)]
        print("driver_forecast pde_alone %.4f ms " % fc["pde_alone_ms"] + " ".join(row))
    o = d.get("driver_step_ode23")
    if o:
        print("driver_step_ode23 %.4f ms" % o["ms_per_pde_step"])


if __name__ == "__main__":
    main()
