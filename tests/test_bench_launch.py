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


def _bare_runner(device):
    from rsl_rl_amd.runners import OnPolicyRunner

    r = OnPolicyRunner.__new__(OnPolicyRunner)  # only _configure_multi_gpu's inputs
    r.device = device
    return r


@pytest.mark.parametrize("env, device, message", [
    ({"WORLD_SIZE": "2", "LOCAL_RANK": "1", "RANK": "1"}, "cuda:0",
     "Device 'cuda:0' does not match expected device for local rank '1'."),
    ({"WORLD_SIZE": "2", "LOCAL_RANK": "2", "RANK": "0"}, "cuda:2",
     "Local rank '2' is greater than or equal to world size '2'."),
    ({"WORLD_SIZE": "2", "LOCAL_RANK": "1", "RANK": "2"}, "cuda:1",
     "Global rank '2' is greater than or equal to world size '2'."),
])
def test_configure_multi_gpu_validation_matches_reference(monkeypatch, env, device, message):
    """The world > 1 checks of on_policy_runner.py:377-390 (reference), same order and messages, raised before any
    process group is created (CPU)."""
    monkeypatch.delenv("RSLRL_TEST_ONE_DEVICE", raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with pytest.raises(ValueError) as e:
        _bare_runner(device)._configure_multi_gpu()
    assert str(e.value) == message


def test_configure_multi_gpu_world1(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    r = _bare_runner("cpu")
    r._configure_multi_gpu()
    assert (r.is_distributed, r.gpu_local_rank, r.gpu_global_rank, r.multi_gpu_cfg) == (False, 0, 0, None)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_end_to_end(cuda_device):
    """`python3 bench.py --gpus 2` end to end on one GPU: spawn_ranks -> torch.distributed.run -> two ranks, each with
    its 16384-env shard of a 32768-env total (strong partition), the runner's world-2 path (_configure_multi_gpu,
    broadcast_parameters, one all-reduce of gradients + KL per mini-batch), the barriers, the MAX all-reduce of the
    elapsed time, the N > 1 config label and the teardown.  RSLRL_TEST_ONE_DEVICE=1 puts both ranks on cuda:0 over
    gloo (RCCL refuses two ranks on one device); everything else is the code the 8-GPU run executes."""
    env = dict(os.environ, RSLRL_TEST_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--global-num-envs", "32768", "--steps", "2",
                        "--warmup", "1", "--no-extra", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                       timeout=540, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]  # rank 0 is the only printer of the result line
    # nothing else of ours on stdout: the runner's and the policy's prints go to stderr (the other text is gloo's
    # C++ rendezvous notices, "[Gloo] Rank ...", whose lines two ranks may interleave on the shared pipe)
    extra = [ln for ln in r.stdout.splitlines() if ln.strip() and ln != lines[0]]
    ours = ("Actor MLP", "Critic MLP", "MLP(", "Synchronizing", "Learning iteration", "Computation", "Mean ", "Total ")
    assert not [ln for ln in extra if any(k in ln for k in ours)], extra
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["global_num_envs"] == 32768 and d["config"]["num_envs_per_gpu"] == 16384
    assert d["config"]["parallelism"].startswith("dp2")
    assert d["value"] > 0 and d["value"] == d["value"] and d["value"] != float("inf")
    # value = T x total envs x K / the max-over-ranks elapsed time
    assert abs(d["value"] - 24 * 32768 * 2 / (d["ms_per_step"] * 2e-3)) <= 1e-3 * d["value"]
    assert d["cpu_baseline"] is None and "extra_configs" not in d
