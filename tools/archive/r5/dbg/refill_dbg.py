"""Debug: radiance of one batched call (sm proxy 1M tris, 256x144, D) with the library in MCRT_LIB_PATH,
saved to argv[1] (compare runs of two libraries)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)
import torch
torch.cuda.init()
from mcrt import lib, scenes
from mcrt.camera import scene_camera
D = int(sys.argv[2])
sc = scenes.san_miguel_proxy(tris=1_000_000)
ctx = lib.Context(0)
ds = lib.DeviceScene(ctx, sc)
fb = lib.FrameBuffer(ctx, 256, 144)
cams = [scene_camera("san_miguel_proxy", 256, 144, frame=k, jitter=True) for k in range(4)]
fb.render_frames(ds, cams, frame=0, max_depth=D)
ctx.sync()
np.save(sys.argv[1], np.stack([fb.read_frame(k) for k in range(4)]))
