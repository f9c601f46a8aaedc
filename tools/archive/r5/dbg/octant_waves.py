"""Share of the extension waves (64 consecutive queue entries) whose rays share a direction octant,
for the headline call shape (SM proxy 1080p, D = 2, 20 frames): the compact walk's octant-specialised
slab test only runs for those (mcrt_traverse.h traverseQ)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)
import torch
torch.cuda.init()
from mcrt import lib, scenes
from mcrt.camera import scene_camera
sc = scenes.san_miguel_proxy()
ctx = lib.Context(0)
ds = lib.DeviceScene(ctx, sc)
W, H = 1920, 1080
fb = lib.FrameBuffer(ctx, W, H)
cams = [scene_camera("san_miguel_proxy", W, H, frame=k, jitter=True) for k in range(20)]
fb.set_frames_in_flight(1)
fb.render_frames(ds, cams, frame=0, max_depth=2)
ctx.sync()
a, b, c = fb.read_queue(1)
d = b[:, :3]
oct_ = (d[:, 0] < 0).astype(int) | ((d[:, 1] < 0).astype(int) << 1) | ((d[:, 2] < 0).astype(int) << 2)
n = len(oct_) // 64 * 64
w = oct_[:n].reshape(-1, 64)
uni = (w == w[:, :1]).all(1)
ax = np.argmax(np.abs(d[:n]), 1).reshape(-1, 64)
print({"rays": int(len(oct_)), "waves": int(len(w)), "octant_uniform_waves": round(float(uni.mean()), 4),
       "distinct_octants_per_wave_mean": round(float(np.mean([len(set(r)) for r in w[:20000]])), 3)})
