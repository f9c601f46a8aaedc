"""Times the REFERENCE's OpenCL pipeline (oracle/_ref, GPU box) on a bench workload, for a
per-kernel comparison under rocprofv3.

usage: python tools/clref_bench.py [--variant fast|ieee] [--frames K] [--integrator pt|bdpt]
                                   [--scene san_miguel_proxy|dragon_proxy|sponza_proxy|instanced_proxy]
                                   [--width W --height H] [--two-level]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="fast")
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--integrator", default="pt", choices=["pt", "bdpt"])
    ap.add_argument("--scene", default="san_miguel_proxy")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-depth", type=int, default=2)
    ap.add_argument("--two-level", action="store_true",
                    help="RadeonRays IntersectorTwoLevel kernels over the reference's two-level build (instanced scenes)")
    a = ap.parse_args()
    from mcrt import scenes
    from mcrt.camera import scene_camera
    from oracle import pyoracle as po
    sc = getattr(scenes, a.scene)()
    cs = po.CLRefScene(sc, a.variant, two_level=a.two_level)
    W, H = a.width, a.height
    cam = scene_camera(a.scene, W, H)
    render = cs.render_bdpt if a.integrator == "bdpt" else cs.render
    render(cam, frame=0, max_depth=a.max_depth)
    t0 = time.perf_counter()
    for f in range(a.frames):
        render(cam, frame=f, max_depth=a.max_depth)
    dt = (time.perf_counter() - t0) / a.frames
    print(f"reference OpenCL {a.integrator} ({a.variant}{', two-level' if a.two_level else ''}) {a.scene} {W}x{H} D={a.max_depth}: "
          f"{dt * 1e3:.3f} ms/frame, {W * H / dt / 1e6:.1f} Mpaths/s")


if __name__ == "__main__":
    main()
