"""Times the device SAH build (mcrt_accel_opts.device_build = 2) of a scene; run under rocprofv3
--kernel-trace --stats for the per-kernel split.  usage: python tools/prof_build.py [tris] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))


def main():
    from mcrt import lib, scenes
    tris = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    sc = scenes.san_miguel_proxy(tris=tris)
    ctx = lib.Context(0)
    ds = lib.DeviceScene(ctx, sc, build=False)
    for mode in (2,) * reps + (3,):
        t0 = time.perf_counter()
        ds.build(device_build=mode)
        ctx.sync()
        print(f"builder {ds.builder()} ({'device SAH' if mode == 2 else 'host'}): {(time.perf_counter() - t0) * 1e3:.1f} ms "
              f"(build_ms {ds.info()['build_ms']:.1f}), depth {ds.layout()['depth']}", flush=True)
    ds.close()
    ctx.close()


if __name__ == "__main__":
    main()
