"""Single-rank PPO.update() variants against the reference's update (fixtures: make_golden.make_update_rnd /
make_update_std), on the GPU path:

* RND (config C5's predictor/target 48->48->1 at the 3x256 policy, and a state-normalised 16->32->3 RND at C1's
  shape): the predictor is trained every mini-batch -- MSE of predictor against the detached target
  (ppo.py:352-363), its own backward (:369-372) and an unclipped Adam step (:383-384) -- and "rnd" joins the loss
  statistics (:391-392);
* the std parameterisations the manual (autograd-free) update chains by hand (ActorCritic.train_backward):
  state-dependent std with scalar and with log std (actor_critic.py:63-86, :119-128) and a log_std parameter.
  Each runs once on the manual path and once with it disabled (the autograd path), both against the reference,
  and the two against each other.

Tolerances as tests/update_fixtures.check_update: learning-rate trace exact, loss means rtol 1e-4, first-mini-batch
gradients 1e-5 of each tensor's max, parameters atol 2e-5 (C1 width) or within twice the reference's own one-ulp
sensitivity (3x256), the RND predictor within 1e-3 of how far it moved.
"""

import numpy as np
import pytest
import torch

from conftest import golden_path

pytestmark = pytest.mark.gpu


def _run(meta, z, dev):
    from update_fixtures import build_update, run_recorded_update

    alg, pol = build_update(z, "r0/", meta, meta["ranks"][0], dev)
    grads, rnd_grads = [None], [None]
    loss, lr_trace = run_recorded_update(alg, grads, rnd_grads if alg.rnd else None)
    out = {"loss": loss, "lr_trace": lr_trace, "lr": alg.learning_rate,
           "final": {k: v.detach().cpu() for k, v in pol.state_dict().items()}, "grad_mb0": grads[0]}
    if alg.rnd:
        out["rnd_final"] = {k: v.detach().cpu() for k, v in alg.rnd.predictor.state_dict().items()}
        out["rnd_grad_mb0"] = rnd_grads[0]
    return out


@pytest.mark.parametrize("case", ["rnd_c5_w1", "rnd_statenorm_w1"])
def test_rnd_update_matches_reference(case, golden_meta, cuda_device):
    from update_fixtures import check_update

    meta = golden_meta["update_rnd"][case]
    z = np.load(golden_path(f"update_{case}.npz"))
    out = _run(meta, z, cuda_device)
    errs, rnd_errs = check_update(out, z, meta, 0)
    print(case, "policy", {k: f"{a:.1e}/{m:.1e}" for k, (a, m) in errs.items()})
    print(case, "rnd", {k: f"{a:.1e}/{m:.1e}" for k, (a, m) in rnd_errs.items()})


@pytest.mark.parametrize("case", ["sdstd_scalar", "sdstd_log", "logstd"])
def test_std_parameterisations_match_reference(case, golden_meta, cuda_device, monkeypatch):
    from rsl_rl_amd.modules import ActorCritic
    from update_fixtures import check_update

    meta = golden_meta["update_std"][case]
    z = np.load(golden_path(f"update_{case}.npz"))
    taken = []
    orig = ActorCritic.manual_update_ok

    def spy(self, obs):
        ok = orig(self, obs)
        taken.append(ok)
        return ok

    monkeypatch.setattr(ActorCritic, "manual_update_ok", spy)
    manual = _run(meta, z, cuda_device)
    assert taken and all(taken), "the fixture's shape must take the manual update path"
    check_update(manual, z, meta, 0, mode="manual")
    monkeypatch.setattr(ActorCritic, "manual_update_ok", lambda self, obs: False)
    autograd = _run(meta, z, cuda_device)
    check_update(autograd, z, meta, 0, mode="autograd")
    # the hand-chained backward and autograd through the same fused forward: the same arithmetic up to the
    # order of a few fp32 operations
    torch.testing.assert_close(manual["grad_mb0"], autograd["grad_mb0"], rtol=1e-5, atol=1e-6)
    for k, v in manual["final"].items():
        torch.testing.assert_close(v, autograd["final"][k], rtol=0, atol=1e-5, msg=k)


def _two_group_rnd_update(dev, fused):
    """update() of a PPO whose RND state is two observation groups (rnd.py get_rnd_state: a fresh torch.cat per
    mini-batch), over 2 epochs x 4 mini-batches; fused=False forces the autograd RND step."""
    from rsl_rl_amd.algorithms import PPO
    from rsl_rl_amd.modules import ActorCritic

    T, N, A = 8, 512, 4
    dims = {"policy": 16, "extra": 8}
    groups = {"policy": ["policy"], "critic": ["policy"], "rnd_state": ["policy", "extra"]}
    torch.manual_seed(3)
    obs0 = {k: torch.zeros(N, d) for k, d in dims.items()}
    pol = ActorCritic(obs0, groups, A, actor_hidden_dims=[32, 32], critic_hidden_dims=[32, 32])
    rnd_cfg = {"weight": 1.0, "num_outputs": 3, "predictor_hidden_dims": [32], "target_hidden_dims": [32],
               "learning_rate": 1e-3, "state_normalization": False, "reward_normalization": False,
               "num_states": 24, "obs_groups": groups}
    alg = PPO(pol, num_learning_epochs=2, num_mini_batches=4, device=dev, rnd_cfg=rnd_cfg)
    alg.init_storage("rl", N, T, {k: torch.zeros(N, d) for k, d in dims.items()}, [A])
    g = torch.Generator().manual_seed(11)
    st = alg.storage
    for k, d in dims.items():
        st.observations[k].copy_(torch.randn(T, N, d, generator=g))
    st.rewards.copy_(torch.randn(T, N, 1, generator=g))
    st.dones.copy_((torch.rand(T, N, 1, generator=g) < 0.05).to(torch.uint8))
    mu = 0.3 * torch.randn(T, N, A, generator=g)
    st.mu.copy_(mu)
    st.sigma.fill_(1.0)
    st.actions.copy_(mu + torch.randn(T, N, A, generator=g))
    st.values.copy_(torch.randn(T, N, 1, generator=g))
    st.actions_log_prob.copy_(-4 + 0.1 * torch.randn(T, N, 1, generator=g))
    st.step = T
    with torch.inference_mode():
        alg.compute_returns({k: torch.randn(N, d, generator=g).to(dev) for k, d in dims.items()})
    torch.manual_seed(5)
    planned = []
    orig = PPO._rnd_update_plan

    def plan(self, *a):
        ok = orig(self, *a) if fused else False
        planned.append(ok)
        return ok

    PPO._rnd_update_plan = plan
    try:
        loss = alg.update()
    finally:
        PPO._rnd_update_plan = orig
    assert planned == [fused]
    return loss, {k: v.detach().cpu() for k, v in alg.rnd.predictor.state_dict().items()}


def test_rnd_update_two_state_groups(cuda_device):
    """the fused RND step's per-update target cache must not confuse mini-batches whose (concatenated)
    state tensors reuse one address; the fused step against the autograd one over 8 mini-batches."""
    loss_f, pred_f = _two_group_rnd_update(cuda_device, fused=True)
    loss_a, pred_a = _two_group_rnd_update(cuda_device, fused=False)
    assert abs(loss_f["rnd"] - loss_a["rnd"]) <= 1e-5 * abs(loss_a["rnd"]), (loss_f["rnd"], loss_a["rnd"])
    for k in ("value_function", "surrogate", "entropy"):
        assert abs(loss_f[k] - loss_a[k]) <= 1e-4 * abs(loss_a[k]) + 1e-6, (k, loss_f[k], loss_a[k])
    for k, v in pred_f.items():
        torch.testing.assert_close(v, pred_a[k], rtol=0, atol=2e-6, msg=k)
