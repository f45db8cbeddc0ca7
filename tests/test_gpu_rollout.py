"""Rollout-side record (csrc/rollout.hip, §8f row 1) vs the reference's captured rollout.

The fixtures (tests/golden/rollout_*.npz, make_golden.py::make_rollout) hold, per env step, the inputs the
reference saw (obs, next obs, rewards, dones, time-outs), the transition its act() produced and, after
T steps, its storage.  Here our PPO runs the same steps on the GPU with the reference's policy / RND
weights; the transition fields that depend on sampling or on the policy GEMMs (actions, values, mu,
sigma) are replaced by the captured ones before process_env_step, so the fused record kernel sees the
reference's exact inputs.  Tolerances: copies, dones bit-exact; reward bit-exact without RND; log-prob
2e-6 (the reference's sum over actions has an unspecified order); RND intrinsic reward 1e-5 relative to
its max (two fp32 MLPs and a difference of similar embeddings).
"""

import numpy as np
import pytest
import torch

from conftest import golden_path
from rsl_rl_amd import kernels
from rsl_rl_amd.algorithms import PPO
from rsl_rl_amd.modules import ActorCritic

pytestmark = pytest.mark.gpu


def _build(m, z, dev):
    N, O, A = m["N"], m["O"], m["A"]
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"], "rnd_state": ["policy"]}
    pol = ActorCritic(obs0, groups, A, actor_hidden_dims=m["actor_hidden"], critic_hidden_dims=m["actor_hidden"])
    pol.load_state_dict({k[5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("init/")})
    cfg = None if m["rnd_cfg"] is None else dict(m["rnd_cfg"], num_states=O, obs_groups=groups)
    alg = PPO(pol, device=dev, rnd_cfg=cfg)
    if alg.rnd is not None:
        alg.rnd.load_state_dict({k[9:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("rnd_init/")})
    alg.init_storage("rl", N, m["T"], {"policy": torch.zeros(N, O, device=dev)}, [A])
    return alg


@pytest.mark.parametrize("layout", ["records", "fields"])
@pytest.mark.parametrize("case", ["rnd_c5like", "rnd_statenorm_q3", "plain_timeouts", "rnd_linear_sched"])
def test_rollout_record_matches_reference(case, layout, golden_meta, cuda_device, monkeypatch):
    """Both storage layouts: transition records (the default here: every width a multiple of 4) and one
    buffer per field (RSLRL_RECORD_LAYOUT=0)."""
    monkeypatch.setenv("RSLRL_RECORD_LAYOUT", "1" if layout == "records" else "0")
    m = golden_meta["rollout"][case]
    z = np.load(golden_path(f"rollout_{case}.npz"))
    dev = cuda_device
    alg = _build(m, z, dev)
    assert (alg.storage.records is not None) == (layout == "records")
    g = lambda k: torch.from_numpy(z[k]).to(dev)  # noqa: E731
    ddtype = {"int64": torch.int64, "bool": torch.bool, "float": torch.float32}[m["dones_dtype"]]
    for t in range(m["T"]):
        with torch.inference_mode():
            alg.act({"policy": g(f"step{t}/obs")})
            assert alg.transition.actions_log_prob is None  # computed by the fused record
            # our own policy forward agrees with the reference's (x6 MFMA GEMMs)
            torch.testing.assert_close(alg.transition.action_mean, g(f"step{t}/action_mean"), rtol=1e-4, atol=1e-5)
            torch.testing.assert_close(alg.transition.values, g(f"step{t}/values"), rtol=1e-4, atol=1e-5)
            tr = alg.transition
            tr.actions = g(f"step{t}/actions")
            tr.values = g(f"step{t}/values")
            tr.action_mean = g(f"step{t}/action_mean")
            sig = g(f"step{t}/action_sigma")
            tr.action_sigma = sig[0].expand_as(sig) if (sig == sig[0]).all() else sig
            dones = g(f"step{t}/dones").to(ddtype)
            alg.process_env_step({"policy": g(f"step{t}/next_obs")}, g(f"step{t}/rewards"), dones,
                                 {"time_outs": g(f"step{t}/time_outs")})
            if alg.rnd is not None:
                ref = g(f"step{t}/intrinsic")
                err = (alg.intrinsic_rewards - ref).abs().max().item()
                assert err <= 1e-5 * ref.abs().max().item() + 1e-7, (t, err)
                assert alg.rnd.weight == float(z[f"step{t}/rnd_weight"])  # the host schedule, bit-exact
    st = alg.storage
    for k in ("actions", "mu", "sigma", "values"):
        assert torch.equal(getattr(st, k).cpu(), torch.from_numpy(z[f"storage/{k}"])), k
    assert torch.equal(st.observations["policy"].cpu(), torch.from_numpy(z["storage/obs_policy"]))
    assert torch.equal(st.dones.cpu(), torch.from_numpy(z["storage/dones"]))
    torch.testing.assert_close(st.actions_log_prob.cpu(), torch.from_numpy(z["storage/actions_log_prob"]),
                               rtol=2e-6, atol=2e-6)
    ref_r = torch.from_numpy(z["storage/rewards"])
    if m["rnd_cfg"] is None:
        assert torch.equal(st.rewards.cpu(), ref_r)
    else:
        assert (st.rewards.cpu() - ref_r).abs().max().item() <= 1e-5 * ref_r.abs().max().item()


def test_rollout_record_kernel_direct(cuda_device):
    """The C-ABI call on its own: shared vs per-row sigma, A not a multiple of 4, extra reward, no
    time-outs, several observation groups -- against the oracle restatement."""
    from oracle import ppo_oracle as po
    torch.manual_seed(5)
    dev = cuda_device
    for A, per_row, with_to in ((3, False, False), (12, True, True), (5, True, True)):
        N, O1, O2 = 1000, 8, 20
        obs1, obs2 = torch.randn(N, O1, device=dev), torch.randn(N, O2, device=dev)
        actions, mu = torch.randn(N, A, device=dev), torch.randn(N, A, device=dev)
        sigma = (0.5 + torch.rand(N, A, device=dev)) if per_row else (0.5 + torch.rand(A, device=dev))
        values, rewards = torch.randn(N, 1, device=dev), torch.randn(N, device=dev)
        extra = torch.randn(N, device=dev)
        dones = torch.rand(N, device=dev) < 0.3
        to = (torch.rand(N, device=dev) < 0.4).float() if with_to else None
        outs = {k: torch.full((N, A), -1.0, device=dev) for k in ("actions", "mu", "sigma")}
        o1, o2 = torch.empty_like(obs1), torch.empty_like(obs2)
        r, v, lp = torch.empty(N, 1, device=dev), torch.empty(N, 1, device=dev), torch.empty(N, 1, device=dev)
        d = torch.empty(N, 1, dtype=torch.uint8, device=dev)
        kernels.rollout_record(0, obs_pairs=[(obs1, o1), (obs2, o2)], actions=actions, mu=mu, sigma=sigma,
                               values=values, rewards=rewards, dones=dones, time_outs=to, gamma=0.97,
                               out_actions=outs["actions"], out_rewards=r, out_dones=d, out_values=v, out_logp=lp,
                               out_mu=outs["mu"], out_sigma=outs["sigma"], extra_reward=extra)
        assert torch.equal(o1, obs1) and torch.equal(o2, obs2)
        assert torch.equal(outs["actions"], actions) and torch.equal(outs["mu"], mu)
        assert torch.equal(outs["sigma"], sigma.expand(N, A))
        assert torch.equal(v, values) and torch.equal(d[:, 0], dones.to(torch.uint8))
        c = lambda x: x.cpu().numpy()  # noqa: E731
        np.testing.assert_allclose(c(lp[:, 0]), po.normal_log_prob_sum(c(actions), c(mu), c(sigma)), rtol=2e-6, atol=2e-6)
        ref_r = po.step_reward(c(rewards), c(values), c(to) if to is not None else None, 0.97, c(extra))
        np.testing.assert_array_equal(c(r[:, 0]), ref_r)


def test_act_sampling_equals_torch_normal(cuda_device):
    """ActorCritic.act draws normal_(0, 1) * scale + loc itself (skipping torch.normal's host-synchronising
    std >= 0 check); the values are those of Normal(loc, scale).sample() for the same generator state."""
    torch.manual_seed(0)
    pol = ActorCritic({"policy": torch.zeros(8, 16)}, {"policy": ["policy"], "critic": ["policy"]}, 4,
                      actor_hidden_dims=[32], critic_hidden_dims=[32]).to(cuda_device)
    obs = {"policy": torch.randn(5000, 16, device=cuda_device)}
    state = torch.cuda.get_rng_state()
    ours = pol.act(obs)
    torch.cuda.set_rng_state(state)
    ref = pol.distribution.sample()
    assert torch.equal(ours, ref)


@pytest.mark.parametrize("per_row", [False, True])
def test_rollout_record_kernel_record_mode(per_row, cuda_device):
    """Record mode: obs groups, actions, mu and sigma land in their record fields (row stride R), the rest of
    each record is zero-filled (whole records: no partial-line writes); the scalar outputs as in the plain mode."""
    torch.manual_seed(6)
    dev = cuda_device
    N, O1, O2, A, R = 777, 8, 20, 12, 96
    rec = torch.full((N, R), 7.0, device=dev)
    offs = {"o1": 0, "o2": 8, "actions": 28, "mu": 40, "sigma": 52}
    obs1, obs2 = torch.randn(N, O1, device=dev), torch.randn(N, O2, device=dev)
    actions, mu = torch.randn(N, A, device=dev), torch.randn(N, A, device=dev)
    sigma = (0.5 + torch.rand(N, A, device=dev)) if per_row else (0.5 + torch.rand(A, device=dev))
    values, rewards = torch.randn(N, 1, device=dev), torch.randn(N, device=dev)
    dones = torch.rand(N, device=dev) < 0.3
    r, v, lp = torch.empty(N, 1, device=dev), torch.empty(N, 1, device=dev), torch.empty(N, 1, device=dev)
    d = torch.empty(N, 1, dtype=torch.uint8, device=dev)
    f = lambda k, w: rec[:, offs[k]:offs[k] + w]  # noqa: E731
    kernels.rollout_record(0, obs_pairs=[(obs1, f("o1", O1)), (obs2, f("o2", O2))], actions=actions, mu=mu,
                           sigma=sigma, values=values, rewards=rewards, dones=dones, time_outs=None, gamma=0.97,
                           out_actions=f("actions", A), out_rewards=r, out_dones=d, out_values=v, out_logp=lp,
                           out_mu=f("mu", A), out_sigma=f("sigma", A), out_records=rec)
    torch.cuda.synchronize()
    assert torch.equal(f("o1", O1), obs1) and torch.equal(f("o2", O2), obs2)
    assert torch.equal(f("actions", A), actions) and torch.equal(f("mu", A), mu)
    assert torch.equal(f("sigma", A), sigma.expand(N, A))
    assert (rec[:, 64:] == 0).all()  # past the fields: the record is written whole
    assert torch.equal(v, values) and torch.equal(d[:, 0], dones.to(torch.uint8))
    # the copy blocks' log-prob (terms on a row's four lanes, summed in action order through quad broadcasts; the
    # last block partial: 777 = 12 x 64 + 9) is the per-env form's bit for bit, and the oracle's within fp32
    lp2 = torch.empty_like(lp)
    scratch = {k: torch.empty(N, A, device=dev) for k in ("actions", "mu", "sigma")}
    kernels.rollout_record(0, obs_pairs=[(obs1, torch.empty_like(obs1)), (obs2, torch.empty_like(obs2))],
                           actions=actions, mu=mu, sigma=sigma, values=values, rewards=rewards, dones=dones,
                           time_outs=None, gamma=0.97, out_actions=scratch["actions"], out_rewards=torch.empty_like(r),
                           out_dones=torch.empty_like(d), out_values=torch.empty_like(v), out_logp=lp2,
                           out_mu=scratch["mu"], out_sigma=scratch["sigma"])
    torch.cuda.synchronize()
    assert torch.equal(lp, lp2)
    from oracle import ppo_oracle as po

    c = lambda x: x.cpu().numpy()  # noqa: E731
    np.testing.assert_allclose(c(lp[:, 0]), po.normal_log_prob_sum(c(actions), c(mu), c(sigma)), rtol=2e-6, atol=2e-6)
