"""bench.py's world-size handling, without a GPU: --gpus N is the job's rank count.  A plain
`python bench.py --gpus N` starts torch.distributed.run with N ranks itself (a child process);
under a launcher WORLD_SIZE must equal --gpus; nccl ranks need one GPU each."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env)
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=240, env=e)


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 4" in r.stderr


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0 and "--gpus must be >= 1" in r.stderr


def test_plain_command_launches_ranks():
    # no GPU here: the 2 launched nccl ranks each refuse to run on fewer GPUs than ranks, and the
    # launcher's failure is bench.py's exit status
    # (no GPU visible to the ranks even on a GPU box, where 2 visible GPUs would run a real bench)
    r = _run(["--gpus", "2", "--steps", "1"], HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    if "2 ranks over nccl need 2 GPUs" not in r.stderr:
        import torch
        if torch.cuda.device_count() >= 2:   # the empty device lists did not hide this box's GPUs
            pytest.skip("2 GPUs visible to the ranks: a real 2-rank bench, not the refusal")
    assert "launching 2 ranks" in r.stderr and "torch.distributed.run" in r.stderr
    assert r.returncode != 0
    assert "2 ranks over nccl need 2 GPUs" in r.stderr, r.stderr[-3000:]
