"""Pins the CPU oracle (oracle/) to the golden vectors captured from the reference.

Bit-exact: GAE returns and un-normalised advantages, randperm (and the generator state it leaves),
mini-batch gathers.  Tolerance: normalised advantages (fp64 statistics vs torch's fp32 reduction),
loss scalars / KL / gradients (rtol 1e-5; the oracle uses numpy's exp/log instead of torch's).
"""

import hashlib

import numpy as np
import pytest
import torch

from conftest import golden_path
from oracle import ppo_oracle as O


def _gae_cases(meta):
    return sorted(meta["gae"].items())


def test_gae_bit_exact(golden_meta):
    z = np.load(golden_path("gae.npz"))
    for name, m in _gae_cases(golden_meta):
        g = lambda k: z[f"{name}/{k}"]  # noqa: E731
        ret, adv = O.gae(g("values"), g("rewards"), g("dones"), g("last_values"), m["gamma"], m["lam"])
        assert np.array_equal(ret, g("returns")), name
        assert np.array_equal(adv, g("advantages_raw")), name


def test_gae_normalized(golden_meta):
    z = np.load(golden_path("gae.npz"))
    for name, m in _gae_cases(golden_meta):
        g = lambda k: z[f"{name}/{k}"]  # noqa: E731
        _, adv = O.compute_returns(g("values"), g("rewards"), g("dones"), g("last_values"), m["gamma"], m["lam"])
        ref = g("advantages_norm")
        if m["T"] * m["N"] == 1:
            assert np.isnan(adv).all() and np.isnan(ref).all()
            continue
        np.testing.assert_allclose(adv, ref, rtol=1e-5, atol=1e-6, err_msg=name)


def test_randperm_bit_exact_and_state(golden_meta):
    z = np.load(golden_path("perm.npz"))
    for name, m in golden_meta["perm"].items():
        if f"{name}/state" not in z:
            continue
        perm, st = O.randperm(z[f"{name}/state"], m["n"])
        assert np.array_equal(perm, z[f"{name}/perm"]), name
        assert np.array_equal(st, z[f"{name}/state_after"]), name


@pytest.mark.parametrize("name", ["n393216", "n1572864"])
def test_randperm_large_hash(golden_meta, name):
    m = golden_meta["perm"][name]
    g = torch.Generator().manual_seed(m["seed"])
    perm, _ = O.randperm(g.get_state().numpy(), m["n"])
    assert perm[:32].tolist() == m["head"] and perm[-32:].tolist() == m["tail"]
    assert hashlib.sha256(perm.tobytes()).hexdigest() == m["sha256_int64"]


def test_minibatch_generator(golden_meta):
    m = golden_meta["minibatch"]
    z = np.load(golden_path("minibatch.npz"))
    fields = {k[3:]: z[k] for k in z.files if k.startswith("in/") and k != "in/gen_state"}
    perm, mb, _ = O.minibatch_indices(m["N"], m["T"], m["M"], z["in/gen_state"])
    order = {"obs_policy": "obs_policy", "obs_extra": "obs_extra", "actions": "actions", "target_values": "values",
             "advantages": "advantages", "returns": "returns", "old_logp": "actions_log_prob", "old_mu": "mu",
             "old_sigma": "sigma"}
    batches = list(O.minibatches(fields, perm, mb, m["M"], m["E"]))
    assert len(batches) == m["num_batches"]
    for j, b in enumerate(batches):
        for out_name, in_name in order.items():
            assert np.array_equal(b[in_name], z[f"mb{j}/{out_name}"]), (j, out_name)


def _loss_kwargs(m):
    kw = m["ppo_kw"]
    return dict(clip_param=kw.get("clip_param", 0.2), value_loss_coef=kw.get("value_loss_coef", 1.0),
                entropy_coef=kw.get("entropy_coef", 0.01), use_clipped_value_loss=kw.get("use_clipped_value_loss", True),
                compute_kl=m["adaptive"],
                normalize_advantage_per_mini_batch=kw.get("normalize_advantage_per_mini_batch", False))


def _rel_err(a, ref):
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(a - ref)) / (np.max(np.abs(ref)) + 1e-30))


def test_loss_and_gradients(golden_meta):
    for name, m in sorted(golden_meta["loss"].items()):
        z = np.load(golden_path(f"loss_{name}.npz"))
        for j in range(m["num_batches"]):
            g = lambda k: z[f"mb{j}/{k}"]  # noqa: E731
            o = O.ppo_loss(g("mu"), g("sigma"), g("V"), g("actions"), g("old_logp"), g("advantages"),
                           g("target_values"), g("returns"), g("old_mu"), g("old_sigma"), **_loss_kwargs(m))
            assert _rel_err(o["dmu"], g("dmu")) < 1e-5, (name, j)
            assert _rel_err(o["dsigma"], g("dsigma")) < 1e-5, (name, j)
            assert _rel_err(o["dV"], g("dV").reshape(-1)) < 1e-5, (name, j)
            if m["adaptive"]:
                assert abs(o["kl_mean"] - float(g("kl_mean"))) <= 1e-5 * abs(float(g("kl_mean"))) + 1e-9
            if m["num_batches"] == 1:
                for k in ("surrogate", "value_function", "entropy"):
                    assert abs(o[k] - m["loss_dict"][k]) <= 1e-5 * abs(m["loss_dict"][k]) + 1e-7, (name, k)


# ---------------------------------------------------------------------------------------------------
# rollout side (ppo.py:129-169, rnd.py:113-135) -- oracle vs the reference's captured rollout
# ---------------------------------------------------------------------------------------------------
def _rnd_layers(z, prefix, net):
    keys = sorted({k.rsplit(".", 1)[0] for k in z.files if k.startswith(f"{prefix}{net}.")},
                  key=lambda k: int(k.rsplit(".", 1)[1]))
    return [(z[k + ".weight"], z[k + ".bias"]) for k in keys]


@pytest.mark.parametrize("case", ["rnd_c5like", "rnd_statenorm_q3", "plain_timeouts", "rnd_linear_sched"])
def test_oracle_rollout_record(case, golden_meta):
    from oracle import ppo_oracle as po
    m = golden_meta["rollout"][case]
    z = np.load(golden_path(f"rollout_{case}.npz"))
    T = m["T"]
    for t in range(T):
        lp = po.normal_log_prob_sum(z[f"step{t}/actions"], z[f"step{t}/action_mean"], z[f"step{t}/action_sigma"])
        np.testing.assert_allclose(lp, z[f"step{t}/actions_log_prob"], rtol=2e-6, atol=2e-6)
        intr = None
        if m["rnd_cfg"] is not None:
            if not m["rnd_cfg"].get("state_normalization"):  # (normaliser statistics evolve: GPU test)
                ours = po.rnd_intrinsic(z[f"step{t}/next_obs"], _rnd_layers(z, "rnd_init/", "target"),
                                        _rnd_layers(z, "rnd_init/", "predictor"), z[f"step{t}/rnd_weight"])
                np.testing.assert_allclose(ours, z[f"step{t}/intrinsic"], rtol=1e-5, atol=1e-6)
            intr = z[f"step{t}/intrinsic"]  # the reward composition itself is checked bit-exactly
        r = po.step_reward(z[f"step{t}/rewards"], z[f"step{t}/values"], z[f"step{t}/time_outs"], m["gamma"], intr)
        np.testing.assert_array_equal(r, z["storage/rewards"][t, :, 0])
        np.testing.assert_array_equal(z["storage/dones"][t, :, 0], z[f"step{t}/dones"])


def test_oracle_normalizer(golden_meta):
    """EmpiricalNormalization / EmpiricalDiscountedVariationNormalization (normalization.py:44-99) vs the
    reference's captured sequence (fp64 moments here vs torch's fp32 reductions: rtol 1e-5)."""
    from oracle import ppo_oracle as po
    z = np.load(golden_path("normalizer.npz"))
    m = golden_meta["normalizer"]
    mean, var, count = np.zeros(7, np.float32), np.ones(7, np.float32), 0
    for k in range(m["obs_updates"]):
        mean, var, std, count = po.normalizer_update(z[f"obs/x{k}"], mean, var, count, until=m["until"])
        assert count == int(z[f"obs/count{k}"])
        np.testing.assert_allclose(mean, z[f"obs/mean{k}"][0], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(var, z[f"obs/var{k}"][0], rtol=1e-5)
        np.testing.assert_allclose(std, z[f"obs/std{k}"][0], rtol=1e-5)
        np.testing.assert_allclose(po.normalizer_apply(z[f"obs/x{k}"], z[f"obs/mean{k}"][0], z[f"obs/std{k}"][0]),
                                   z[f"obs/y{k}"], rtol=0, atol=0)  # the forward itself is bit-exact
    mean, var, count, avg = np.zeros(1, np.float32), np.ones(1, np.float32), 0, None
    for k in range(m["reward_steps"]):
        r = z[f"rew/r{k}"]
        avg = r.copy() if avg is None else (avg * np.float32(m["gamma"]) + r).astype(np.float32)
        np.testing.assert_array_equal(avg, z[f"rew/avg{k}"])
        mean, var, std, count = po.normalizer_update(avg[:, None], mean, var, count)
        np.testing.assert_allclose(std, z[f"rew/std{k}"], rtol=1e-5)
        np.testing.assert_allclose((r / z[f"rew/std{k}"]).astype(np.float32), z[f"rew/out{k}"], rtol=0, atol=0)
