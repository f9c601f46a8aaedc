"""Attainable HBM bandwidth of the in-repo stream copy (mcrt_ctx_stream_copy) at several sizes.
usage: python tools/stream_copy_probe.py (GPU box)"""
import sys; sys.path.insert(0,'monte-carlo-raytracer_amd')
from mcrt import lib
ctx = lib.Context(0)
for gb in (1, 2, 4, 8):
    print(gb, "GiB", [round(ctx.stream_copy_gbps(gb << 30, 5), 1) for _ in range(2)])
