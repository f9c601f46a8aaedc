"""Times the REFERENCE's OpenCL pipeline (oracle/_ref, GPU box) on the bench workload, for a
per-kernel comparison under rocprofv3.  usage: python tools/clref_bench.py [variant] [frames] [pt|bdpt]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)


def main():
    from mcrt import scenes
    from mcrt.camera import scene_camera
    from oracle import pyoracle as po
    variant = sys.argv[1] if len(sys.argv) > 1 else "fast"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    integ = sys.argv[3] if len(sys.argv) > 3 else "pt"
    sc = scenes.san_miguel_proxy()
    cs = po.CLRefScene(sc, variant)
    cam = scene_camera("san_miguel_proxy", 1920, 1080)
    render = cs.render_bdpt if integ == "bdpt" else cs.render
    render(cam, frame=0, max_depth=2)
    t0 = time.perf_counter()
    for f in range(frames):
        render(cam, frame=f, max_depth=2)
    dt = (time.perf_counter() - t0) / frames
    print(f"reference OpenCL {integ} ({variant}) {dt * 1e3:.3f} ms/frame, {1920 * 1080 / dt / 1e6:.1f} Mpaths/s")


if __name__ == "__main__":
    main()
