"""Full-frame run of the compact walk's tie premise (tests/test_tie_premise_cpu.py): the bench
camera at 1920 x 1080, camera and bounce-1 extension rays of frame 0, on the San-Miguel proxy and on
the same scene moved 1000 units from the origin.  Writes a JSON summary (default
profiles/r06/tie_premise.json).  CPU only (the oracle, oracle/mcrt_oracle.c orc_tie_premise)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "monte-carlo-raytracer_amd"), ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

from helpers import path_rays  # noqa: E402
from mcrt import scenes  # noqa: E402
from mcrt.camera import scene_camera_at  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

ALPHA = 2.0 ** -18


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r06", "tie_premise.json")
    W, H = (int(v) for v in (sys.argv[2:4] if len(sys.argv) > 3 else (1920, 1080)))
    threads = os.cpu_count() or 8
    base = scenes.san_miguel_proxy()
    res = {"what": "order-dependent hit pairs of the reference's closest-hit walk (orc_tie_premise), per ray: "
                   "X hit at t_X with leaf box entry e_X > t_Y > t_X for another acceptable hit Y; beyond the "
                   "near-tie margin when (t_Y - t_X) / t_Y > 2^-18",
           "scene": f"san_miguel_proxy ({base.num_triangles} tris)", "resolution": [W, H], "frame": 0, "cases": {}}
    for off in (0.0, 1000.0):
        sc = base if off == 0.0 else scenes.translated(base, (off,) * 3)
        cam = scene_camera_at("san_miguel_proxy", W, H, (off,) * 3, jitter=True)
        o = po.OracleScene(sc)
        o.build()
        t0 = time.time()
        case = {}
        for b, rays in enumerate(path_rays(o, cam, threads=threads)):
            p = o.tie_premise(rays, ALPHA, threads=threads)
            hit = np.isfinite(p[:, 0])
            bad = p[:, 1] > ALPHA
            case["camera" if b == 0 else "extension"] = {
                "rays": int(len(rays)), "hit": int(hit.sum()),
                "rays_with_irregular_hit": int((p[:, 4] > 0).sum()),
                "rays_with_hit_irregular_beyond_margin": int((p[:, 2] > ALPHA).sum()),
                "rays_order_dependent_beyond_margin": int(bad.sum()),
                "worst_gap": float(p[:, 1].max()), "incomplete": int(p[:, 5].sum()),
                "examples_t": [float(v) for v in p[bad, 0][:8]]}
        case["seconds"] = round(time.time() - t0, 1)
        res["cases"]["origin" if off == 0.0 else f"moved_{off:g}"] = case
        print(json.dumps(case), flush=True)
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
