"""One line per bench JSON file: value, ms/step, roofline frac, BDPT value, per-kernel ms per frame.
usage: python tools/bench_summary.py a.json [b.json ...]"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:   # noqa: BLE001
        print(f, "unreadable:", e)
        continue
    r = d.get("roofline", {})
    print(f, d["value"], d["ms_per_step"], "frac", r.get("frac"), "BDPT", d.get("bdpt", {}).get("value"),
          "parity_ref", d.get("parity_vs_reference", {}).get("pixels_bit_exact"),
          {k: round(v["ms_per_frame"], 4) for k, v in d.get("kernels", {}).items()},
          "bdpt", {k: round(v["ms_per_frame"], 4) for k, v in d.get("bdpt", {}).get("kernels", {}).items()})
