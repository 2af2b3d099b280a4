"""One line per bench JSON (dev tool): value, ms/step, kernel times, roofline frac, steady state, e2e."""
import json
import sys

for path in sys.argv[1:]:
    lines = [ln for ln in open(path).read().strip().splitlines() if ln.startswith("{")]
    d = json.loads(lines[-1])
    e2e = d.get("e2e") or {}
    print(path, f"value {d['value'] / 1e6:.2f}M", f"ms/step {d['ms_per_step']:.4f}",
          "kernels", {k: v for k, v in (d.get("kernel_ms") or {}).items() if k != "samples_timed"},
          f"frac {d['roofline'].get('frac')}", "steady", (d.get("steady_state") or {}).get("ms_per_step"),
          "e2e_go", (e2e.get("gram_only") or {}).get("ms"), "e2e_full", (e2e.get("full") or {}).get("ms"),
          "cpu", (d.get("cpu_baseline") or {}).get("value"))
