"""The measurement entry points the bench's roofline uses (mcrt_ctx_stream_copy,
mcrt_ctx_gather_chase): they run, give plausible rates, and order as the memory hierarchy
does (a dependent gather over an L2-resident array beats one over an HBM-sized array)."""
import pytest

from mcrt import lib

pytestmark = pytest.mark.gpu


def test_stream_copy_rate(hip_ctx):
    g = hip_ctx.stream_copy_gbps(1 << 30, 2)
    assert 500.0 < g < 8000.0, g   # HBM3E: 8 TB/s peak


def test_gather_chase_hierarchy(hip_ctx):
    l2 = hip_ctx.gather_chase_gsteps(32768, 64, 2)
    hbm = hip_ctx.gather_chase_gsteps(20_000_000, 64, 2)
    assert l2 > hbm > 1.0, (l2, hbm)
    with pytest.raises(lib.MCRTError):
        hip_ctx.gather_chase_gsteps(8, 64, 1)   # fewer records than a wave's chains need
