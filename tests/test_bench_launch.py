"""bench.py --gpus N without a launcher starts its own N ranks (torch.distributed.run as a child process) before
any GPU call; each rank gets RANK / LOCAL_RANK / WORLD_SIZE and a 127.0.0.1 rendezvous, and a rank whose
LOCAL_RANK has no GPU stops with a clear message.  CPU-only (the ranks stop before touching a device)."""

import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(n, extra_env):
    env = dict(os.environ, **extra_env)
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "1", "--warmup", "0"], env=env,
                          capture_output=True, text=True, timeout=300, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_its_ranks(n):
    r = _run(n, {"RSLRL_BENCH_RANK_ENV_ONLY": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == n, r.stdout
    assert sorted(int(d["RANK"]) for d in lines) == list(range(n))
    assert sorted(int(d["LOCAL_RANK"]) for d in lines) == list(range(n))
    for d in lines:
        assert d["WORLD_SIZE"] == str(n) and d["LOCAL_WORLD_SIZE"] == str(n)
        assert d["MASTER_ADDR"] == "127.0.0.1"
    assert len({d["MASTER_PORT"] for d in lines}) == 1


def test_bench_ranks_without_gpus_fail_clearly():
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has the GPUs")
    r = _run(2, {})
    assert r.returncode != 0
    assert "needs 2 GPUs on this node" in r.stderr, r.stderr[-3000:]
