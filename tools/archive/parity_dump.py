"""Renders the clref parity CASES (tests/clref_job.py) with the product and saves the raw
radiance frames, for offline bit-level comparison with the reference's OpenCL outputs.
usage: python tools/parity_dump.py OUT.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from clref_job import CASES, build_scene  # noqa: E402
from mcrt import lib  # noqa: E402
from mcrt import types as T  # noqa: E402
from mcrt.camera import scene_camera  # noqa: E402


def main():
    ctx = lib.Context(0)
    res = {}
    for name, W, H, frames, D in CASES:
        ds = lib.DeviceScene(ctx, build_scene(name))
        fb = lib.FrameBuffer(ctx, W, H)
        cam = scene_camera("dragon_proxy" if name == "dragon_small" else name, W, H)
        for f in frames:
            fb.render(ds, cam, frame=f, max_depth=D, sampler=T.SAMPLER_RANDOM)
            res[f"{name}_{W}x{H}_d{D}_f{f}"] = fb.read(0)
        fb.close()
        ds.close()
    np.savez_compressed(sys.argv[1], **res)


if __name__ == "__main__":
    main()
