"""GPU box: the reference pipeline's per-bounce buffers (clref_read) on a sample of rows of the
headline frame, for stage-by-stage comparison with the oracle on the CPU (tools/oracle_divergence.py
finds WHICH pixels differ; this dump shows at WHICH stage the float values start to differ).

usage: python tools/oracle_stage_dump.py OUT.npz [frame] [row_step]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from mcrt.camera import scene_camera
    from oracle import pyoracle as po
    from clref_job import scale_scene
    out_path = sys.argv[1]
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    step = int(sys.argv[3]) if len(sys.argv) > 3 else 27
    W, H = 1920, 1080
    rows = np.arange(0, H, step)
    sc = scale_scene("san_miguel_proxy")
    cam = scene_camera("san_miguel_proxy", W, H, frame=frame, jitter=True)
    cs = po.CLRefScene(sc, "ieee")
    out = {"rows": rows}

    def take(which, sz):
        return cs.read(which, W, H).reshape(H, W, sz)[rows]
    for D in (1, 2):
        out[f"radiance_d{D}"] = cs.render(cam, frame=frame, max_depth=D)[rows]
        out[f"temp_d{D}"] = take("temp", 16)
        out[f"rays_d{D}"] = take("rays", 48)
        out[f"isect_d{D}"] = take("isect", 32)
        out[f"shadow_rays_d{D}"] = take("shadow_rays", 48)
        out[f"occlusion_d{D}"] = take("occlusion", 4)
        out[f"throughput_d{D}"] = take("throughput", 32)
    np.savez_compressed(out_path, **out)
    print("rows", len(rows), "bytes", sum(v.nbytes for v in out.values()))


if __name__ == "__main__":
    main()
