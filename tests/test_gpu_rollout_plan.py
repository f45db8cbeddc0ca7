"""The fused rollout step through the storage's cached argument struct (kernels.RolloutRecordPlan) against the general
rollout_record call it short-cuts: bit-identical storages (records, rewards, dones, values, log-probs) and parameters
over whole training iterations, and one plan built per storage (not one per step)."""

import contextlib
import io

import pytest
import torch

from rsl_rl_amd import kernels
from rsl_rl_amd.env import SyntheticVecEnv
from rsl_rl_amd.runners import OnPolicyRunner
from rsl_rl_amd.storage import rollout_storage

pytestmark = pytest.mark.gpu


def _cfg():
    return {"num_steps_per_env": 8, "save_interval": 10**9, "obs_groups": {"policy": ["policy"], "critic": ["policy"]},
            "policy": {"class_name": "ActorCritic", "activation": "elu", "actor_hidden_dims": [64, 64],
                       "critic_hidden_dims": [64, 64], "init_noise_std": 1.0},
            "algorithm": {"class_name": "PPO", "num_learning_epochs": 2, "num_mini_batches": 2}}


def _run(plan: bool, monkeypatch, dev, iters=3):
    built = []
    real = kernels.RolloutRecordPlan.__init__

    def counting(self, *a, **k):
        built.append(1)
        real(self, *a, **k)

    monkeypatch.setattr(kernels.RolloutRecordPlan, "__init__", counting)
    if not plan:
        monkeypatch.setattr(rollout_storage.RolloutStorage, "_record_plan", lambda self, *a: None)
    torch.manual_seed(5)
    env = SyntheticVecEnv(3000, 48, 12, device=dev, seed=2, timeout_prob=0.2)
    with contextlib.redirect_stdout(io.StringIO()):
        runner = OnPolicyRunner(env, _cfg(), log_dir=None, device=dev)
        snaps = []
        for _ in range(iters):
            runner.learn(1)
            st = runner.alg.storage
            assert st.records is not None, "the record layout is the GPU default"
            snaps.append({"records": st.records.clone(), "rewards": st.rewards.clone(), "dones": st.dones.clone(),
                          "values": st.values.clone(), "logp": st.actions_log_prob.clone()})
    params = [p.detach().clone() for p in runner.alg.policy.parameters()]
    monkeypatch.undo()
    return snaps, params, len(built)


def test_rollout_plan_matches_general_call(cuda_device, monkeypatch):
    general, p_general, _ = _run(False, monkeypatch, cuda_device)
    planned, p_planned, n_built = _run(True, monkeypatch, cuda_device)
    assert n_built == 1, n_built
    for a, b in zip(general, planned):
        for k in a:
            assert torch.equal(a[k], b[k]), k
    for a, b in zip(p_general, p_planned):
        assert torch.equal(a, b)


def test_rollout_and_gather_launches_bound_to_events(cuda_device):
    """rslrl_launch_timing_* tags (ABI 14): while armed, every rollout-record launch of an iteration (8 env steps) and
    the update's record gather carry their own event pair, read back per kernel with positive durations."""
    torch.manual_seed(5)
    env = SyntheticVecEnv(3000, 48, 12, device=cuda_device, seed=2)
    with contextlib.redirect_stdout(io.StringIO()):
        runner = OnPolicyRunner(env, _cfg(), log_dir=None, device=cuda_device)
        runner.learn(1)
        torch.cuda.synchronize()
        kernels.timer.arm_launch_events(256)
        try:
            runner.learn(1)
            torch.cuda.synchronize()
        finally:
            kernels.timer.disarm_launch_events()
    ms_r, n_r = kernels.timer.launch_events("rollout_record")
    ms_g, n_g = kernels.timer.launch_events("gather_rows")
    ms_l, n_l = kernels.timer.launch_events("ppo_loss")
    assert n_r == 8 and ms_r > 0.0
    assert n_g == 1 and ms_g > 0.0
    assert n_l == 4 and ms_l > 0.0  # 2 epochs x 2 mini-batches: the 2x64 actor is not the fused head's shape
