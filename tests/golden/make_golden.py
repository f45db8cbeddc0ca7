"""Generate the golden fixtures under tests/golden/ by running the REFERENCE (rsl_rl 3.1.0) on CPU.

Test infrastructure only: this script runs in the build container (where /root/reference exists) and
writes small .npz/.json fixtures that the CPU oracle and the HIP path are checked against.  Nothing from
the reference travels with the repo or to the GPU box; only the captured input/output vectors do.

The reference imports two packages that this image lacks:
  * ``git`` (GitPython) -- used only by ``store_code_state`` which is never reached with log_dir=None,
    so an empty module object stands in;
  * ``tensordict`` -- the reference uses ``TensorDict`` purely as a keyed container with row indexing
    (``rollout_storage.py:48-52,83,168,188``); it performs no arithmetic on this path.  A container with
    exactly that behaviour (``_RowDict`` below) is registered under that name.
All arithmetic that the fixtures pin (GAE, normalisation, randperm, gathers, PPO loss/KL/gradients,
Adam update) is executed by the reference's own code and by torch 2.10.0 CPU kernels.

Usage:  python tests/golden/make_golden.py [--reference /root/reference]
"""

from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------------------------------
# import shims (see module docstring)
# --------------------------------------------------------------------------------------------------
class _RowDict:
    """Keyed container of tensors sharing leading batch dims (the subset of TensorDict rsl_rl uses)."""

    def __init__(self, source, batch_size=None, device=None):
        self._d = dict(source)
        if batch_size is None:
            first = next(iter(self._d.values()))
            batch_size = [first.shape[0]]
        self.batch_size = torch.Size(batch_size)
        self.device = device

    def __getitem__(self, key):
        if isinstance(key, str):
            return self._d[key]
        out = {k: v[key] for k, v in self._d.items()}
        first = next(iter(out.values()))
        nb = max(len(self.batch_size) - (1 if isinstance(key, int) else 0), 1)
        return _RowDict(out, batch_size=list(first.shape[:nb]), device=self.device)

    def __contains__(self, key):
        return key in self._d

    def keys(self):
        return self._d.keys()

    def items(self):
        return self._d.items()

    def values(self):
        return self._d.values()

    def copy_(self, other):
        for k, v in self._d.items():
            v.copy_(other[k])
        return self

    def flatten(self, a, b):
        out = {k: v.flatten(a, b) for k, v in self._d.items()}
        bs = list(self.batch_size)
        nbs = bs[:a] + [int(np.prod(bs[a : b + 1]))] + bs[b + 1 :]
        return _RowDict(out, batch_size=nbs, device=self.device)

    def to(self, device):
        return _RowDict({k: v.to(device) for k, v in self._d.items()}, self.batch_size, device)

    @property
    def shape(self):
        return self.batch_size


def import_reference(path):
    sys.dont_write_bytecode = True
    sys.modules.setdefault("git", types.ModuleType("git"))
    td = types.ModuleType("tensordict")
    td.TensorDict = _RowDict
    sys.modules["tensordict"] = td
    sys.path.insert(0, path)
    import rsl_rl  # noqa: F401
    from rsl_rl.algorithms import PPO
    from rsl_rl.modules import ActorCritic
    from rsl_rl.storage import RolloutStorage

    return PPO, ActorCritic, RolloutStorage


def f32(x):
    return np.ascontiguousarray(x.detach().cpu().numpy().astype(np.float32))


# --------------------------------------------------------------------------------------------------
# GAE  (rollout_storage.py:127-149)
# --------------------------------------------------------------------------------------------------
GAE_CASES = [
    # name, T, N, p_done, gamma, lam, seed, done_pattern
    ("t16_n512", 16, 512, 0.02, 0.99, 0.95, 0, "bernoulli"),
    ("t24_n4096", 24, 4096, 0.02, 0.99, 0.95, 1, "bernoulli"),
    ("t1_n70", 1, 70, 0.02, 0.99, 0.95, 2, "bernoulli"),
    ("t5_n1000_alldone", 5, 1000, 1.0, 0.99, 0.95, 3, "all"),
    ("t7_n130_nodone", 7, 130, 0.0, 0.99, 0.95, 4, "none"),
    ("t8_n64_lastdone", 8, 64, 0.0, 0.99, 0.95, 5, "last"),
    ("t24_n333_g1l1", 24, 333, 0.05, 1.0, 1.0, 6, "bernoulli"),
    ("t3_n1", 3, 1, 0.5, 0.97, 0.9, 7, "bernoulli"),
    ("t32_n257_heavy", 32, 257, 0.3, 0.995, 0.98, 8, "bernoulli"),
]


def make_gae(RolloutStorage):
    out = {}
    for name, T, N, p, gamma, lam, seed, pat in GAE_CASES:
        g = torch.Generator().manual_seed(1000 + seed)
        values = torch.randn(T, N, 1, generator=g)
        rewards = torch.randn(T, N, 1, generator=g)
        last_values = torch.randn(N, 1, generator=g)
        if pat == "bernoulli":
            dones = (torch.rand(T, N, 1, generator=g) < p).to(torch.uint8)
        elif pat == "all":
            dones = torch.ones(T, N, 1, dtype=torch.uint8)
        elif pat == "none":
            dones = torch.zeros(T, N, 1, dtype=torch.uint8)
        else:
            dones = torch.zeros(T, N, 1, dtype=torch.uint8)
            dones[T - 1] = 1
        res = {}
        for norm in (False, True):
            st = RolloutStorage("rl", N, T, {"policy": torch.zeros(N, 1)}, [1], "cpu")
            st.values.copy_(values)
            st.rewards.copy_(rewards)
            st.dones.copy_(dones)
            st.compute_returns(last_values.clone(), gamma, lam, normalize_advantage=norm)
            res[norm] = (f32(st.returns), f32(st.advantages))
        assert np.array_equal(res[False][0], res[True][0])
        out[name] = dict(
            T=T, N=N, gamma=gamma, lam=lam,
            values=f32(values).reshape(T, N), rewards=f32(rewards).reshape(T, N),
            dones=dones.numpy().reshape(T, N).astype(np.uint8), last_values=f32(last_values).reshape(N),
            returns=res[False][0].reshape(T, N), advantages_raw=res[False][1].reshape(T, N),
            advantages_norm=res[True][1].reshape(T, N),
        )
    arrays = {}
    meta = {}
    for name, d in out.items():
        meta[name] = {k: d[k] for k in ("T", "N", "gamma", "lam")}
        for k in ("values", "rewards", "dones", "last_values", "returns", "advantages_raw", "advantages_norm"):
            arrays[f"{name}/{k}"] = d[k]
    np.savez_compressed(os.path.join(HERE, "gae.npz"), **arrays)
    return meta


# --------------------------------------------------------------------------------------------------
# randperm  (rollout_storage.py:165 -> torch CPU randperm)
# --------------------------------------------------------------------------------------------------
PERM_CASES = [
    # name, n, seed, pre_draw (consume generator before randperm to exercise a mid-stream state)
    ("n1", 1, 0, 0),
    ("n2", 2, 1, 0),
    ("n3", 3, 2, 0),
    ("n10", 10, 3, 0),
    ("n1000", 1000, 4, 0),
    ("n8192", 8192, 5, 0),
    ("n98304", 98304, 6, 0),
    ("n4097_mid", 4097, 7, 1234),
    ("n777_mid_odd", 777, 8, 623),
    ("n5000_mid_long", 5000, 9, 5000),
]
BIG_PERM = [("n1572864", 1572864, 0), ("n393216", 393216, 11)]


def make_perm():
    arrays, meta = {}, {}
    for name, n, seed, pre in PERM_CASES:
        g = torch.Generator().manual_seed(seed)
        if pre:
            torch.randint(0, 2**31 - 1, (pre,), generator=g)  # consumes `pre` mt19937 words
        state = g.get_state().numpy().copy()
        perm = torch.randperm(n, generator=g).numpy().astype(np.int64)
        state_after = g.get_state().numpy().copy()
        arrays[f"{name}/state"] = state
        arrays[f"{name}/perm"] = perm
        arrays[f"{name}/state_after"] = state_after
        meta[name] = {"n": n, "seed": seed, "pre_draw": pre}
    for name, n, seed in BIG_PERM:
        g = torch.Generator().manual_seed(seed)
        perm = torch.randperm(n, generator=g).numpy().astype(np.int64)
        meta[name] = {
            "n": n, "seed": seed, "pre_draw": 0,
            "sha256_int64": hashlib.sha256(perm.tobytes()).hexdigest(),
            "head": perm[:32].tolist(), "tail": perm[-32:].tolist(),
        }
    np.savez_compressed(os.path.join(HERE, "perm.npz"), **arrays)
    return meta


# --------------------------------------------------------------------------------------------------
# mini-batch generator  (rollout_storage.py:160-203)
# --------------------------------------------------------------------------------------------------
def make_minibatch(RolloutStorage):
    T, N, A, M, E = 4, 6, 2, 3, 2
    g = torch.Generator().manual_seed(77)
    obs0 = {"policy": torch.zeros(N, 3), "extra": torch.zeros(N, 2)}
    st = RolloutStorage("rl", N, T, obs0, [A], "cpu")
    fields = {}
    fields["obs_policy"] = torch.randn(T, N, 3, generator=g)
    fields["obs_extra"] = torch.randn(T, N, 2, generator=g)
    st.observations["policy"].copy_(fields["obs_policy"])
    st.observations["extra"].copy_(fields["obs_extra"])
    for k, shape in (("actions", (T, N, A)), ("values", (T, N, 1)), ("returns", (T, N, 1)),
                     ("actions_log_prob", (T, N, 1)), ("advantages", (T, N, 1)), ("mu", (T, N, A)),
                     ("sigma", (T, N, A))):
        fields[k] = torch.randn(*shape, generator=g)
        getattr(st, k).copy_(fields[k])
    torch.manual_seed(4242)
    state = torch.default_generator.get_state().numpy().copy()
    batches = list(st.mini_batch_generator(M, E))
    arrays = {f"in/{k}": f32(v) for k, v in fields.items()}
    arrays["in/gen_state"] = state
    names = ["actions", "target_values", "advantages", "returns", "old_logp", "old_mu", "old_sigma"]
    for j, b in enumerate(batches):
        arrays[f"mb{j}/obs_policy"] = f32(b[0]["policy"])
        arrays[f"mb{j}/obs_extra"] = f32(b[0]["extra"])
        for nm, t in zip(names, b[1:8]):
            arrays[f"mb{j}/{nm}"] = f32(t)
        assert b[8] == (None, None) and b[9] is None
    np.savez_compressed(os.path.join(HERE, "minibatch.npz"), **arrays)
    return {"T": T, "N": N, "A": A, "M": M, "E": E, "num_batches": len(batches), "torch_seed": 4242}


# --------------------------------------------------------------------------------------------------
# PPO loss / KL / gradients (ppo.py:221-315, 367) and one full update (ppo.py:178-422)
# --------------------------------------------------------------------------------------------------
def _fill_storage(st, T, N, A, O, g, policy=None):
    """Rollout-like storage contents.

    policy=None: obs~N(0,1); mu~N(0,.25); sigma~U(.5,1.5) per action; actions sampled around mu; old
    log-prob perturbed by N(0,.3^2) (large KL -> exercises the lr-decrease branch).
    policy given: mu/sigma/values/log-prob are what the policy itself produces for the stored obs, as in
    a real rollout (ppo.py:129-140), so the first mini-batch's KL is ~0 (lr-increase branch).
    """
    obs = torch.randn(T, N, O, generator=g)
    st.observations["policy"].copy_(obs)
    st.rewards.copy_(torch.randn(T, N, 1, generator=g))
    st.dones.copy_((torch.rand(T, N, 1, generator=g) < 0.05).to(torch.uint8))
    if policy is None:
        st.values.copy_(torch.randn(T, N, 1, generator=g))
        mu = torch.randn(T, N, A, generator=g) * 0.5
        sigma = 0.5 + torch.rand(1, 1, A, generator=g).expand(T, N, A)
        actions = mu + sigma * torch.randn(T, N, A, generator=g)
        logp = torch.distributions.Normal(mu, sigma).log_prob(actions).sum(-1, keepdim=True)
        logp = logp + 0.3 * torch.randn(T, N, 1, generator=g)
    else:
        with torch.inference_mode():
            o = {"policy": obs.reshape(T * N, O)}
            policy.update_distribution(policy.actor_obs_normalizer(policy.get_actor_obs(o)))
            mu = policy.action_mean.reshape(T, N, A).clone()
            sigma = policy.action_std.reshape(T, N, A).clone()
            actions = mu + sigma * torch.randn(T, N, A, generator=g)
            logp = policy.distribution.log_prob(actions.reshape(T * N, A)).sum(-1).reshape(T, N, 1).clone()
            st.values.copy_(policy.evaluate(o).reshape(T, N, 1))
    st.mu.copy_(mu)
    st.sigma.copy_(sigma)
    st.actions.copy_(actions)
    st.actions_log_prob.copy_(logp)
    st.step = T


def _record_update(PPO, ActorCritic, RolloutStorage, *, T, N, O, A, M, E, hidden, policy_kw, ppo_kw, seed,
                   normalize_in_storage, consistent=False):
    """Run ONE reference PPO.update() and capture every per-mini-batch loss input/output.

    Captures via (a) a recording ActorCritic subclass (retain_grad on the distribution loc/scale and on
    the value head output), (b) the multi-GPU hooks: with multi_gpu_cfg world_size=1 the reference calls
    torch.distributed.all_reduce(kl_mean) and all_reduce(flat_grads) (ppo.py:273, :453); we intercept
    those calls (identity over one rank) to read kl_mean and the pre-clip flat gradient exactly as the
    reference computed them.
    """
    torch.manual_seed(seed)

    class RecAC(ActorCritic):
        def update_distribution(self, obs):
            super().update_distribution(obs)
            if torch.is_grad_enabled():
                self.distribution.loc.retain_grad()
                self.distribution.scale.retain_grad()

        def evaluate(self, obs, **kw):
            v = super().evaluate(obs, **kw)
            if torch.is_grad_enabled() and v.requires_grad:
                v.retain_grad()
                self._last_v = v
            return v

    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    pol = RecAC(obs0, groups, A, actor_hidden_dims=hidden, critic_hidden_dims=hidden, **policy_kw)
    alg = PPO(pol, num_learning_epochs=E, num_mini_batches=M, device="cpu",
              multi_gpu_cfg={"global_rank": 0, "local_rank": 0, "world_size": 1}, **ppo_kw)
    alg.init_storage("rl", N, T, obs0, [A])
    g = torch.Generator().manual_seed(seed + 1)
    _fill_storage(alg.storage, T, N, A, O, g, policy=pol if consistent else None)
    last_obs = torch.randn(N, O, generator=g)
    with torch.inference_mode():
        alg.compute_returns({"policy": last_obs})

    init_state = {k: f32(v) for k, v in pol.state_dict().items()}
    st = alg.storage
    storage_in = {k: f32(getattr(st, k)) for k in ("rewards", "values", "returns", "advantages",
                                                   "actions_log_prob", "mu", "sigma", "actions")}
    storage_in["dones"] = st.dones.numpy().copy()
    storage_in["obs_policy"] = f32(st.observations["policy"])

    records = []
    reduce_calls = []
    orig_ar, orig_bc = torch.distributed.all_reduce, torch.distributed.broadcast

    def fake_all_reduce(t, op=None, **kw):
        reduce_calls.append(t.detach().clone())

    torch.distributed.all_reduce = fake_all_reduce
    torch.distributed.broadcast = lambda t, src=0, **kw: None

    orig_gen = st.mini_batch_generator

    def rec_gen(m, e):
        for b in orig_gen(m, e):
            records.append({"batch": b})
            yield b

    st.mini_batch_generator = rec_gen
    orig_clip = torch.nn.utils.clip_grad_norm_

    def rec_clip(params, max_norm, *a, **kw):
        rec = records[-1]
        d = pol.distribution
        rec["mu"] = f32(d.loc)
        rec["sigma"] = f32(d.scale)
        rec["dmu"] = f32(d.loc.grad)
        rec["dsigma"] = f32(d.scale.grad)
        rec["V"] = f32(pol._last_v)
        rec["dV"] = f32(pol._last_v.grad)
        rec["param_grads"] = {n: f32(p.grad) for n, p in pol.named_parameters()}
        return orig_clip(params, max_norm, *a, **kw)

    torch.nn.utils.clip_grad_norm_ = rec_clip
    gen_state = torch.default_generator.get_state().numpy().copy()
    lr_trace = []
    orig_step = alg.optimizer.step

    def rec_step(*a, **kw):
        lr_trace.append(alg.optimizer.param_groups[0]["lr"])
        return orig_step(*a, **kw)

    alg.optimizer.step = rec_step
    try:
        loss_dict = alg.update()
    finally:
        torch.distributed.all_reduce, torch.distributed.broadcast = orig_ar, orig_bc
        torch.nn.utils.clip_grad_norm_ = orig_clip
    kl_calls = [c for c in reduce_calls if c.dim() == 0]
    grad_calls = [c for c in reduce_calls if c.dim() == 1]
    adaptive = ppo_kw.get("schedule", "adaptive") == "adaptive" and ppo_kw.get("desired_kl", 0.01) is not None
    arrays = {}
    for j, rec in enumerate(records):
        b = rec["batch"]
        names = ["actions", "target_values", "advantages", "returns", "old_logp", "old_mu", "old_sigma"]
        arrays[f"mb{j}/obs"] = f32(b[0]["policy"])
        for nm, t in zip(names, b[1:8]):
            arrays[f"mb{j}/{nm}"] = f32(t)
        for k in ("mu", "sigma", "dmu", "dsigma", "V", "dV"):
            arrays[f"mb{j}/{k}"] = rec[k]
        for n_, gr in rec["param_grads"].items():
            arrays[f"mb{j}/grad/{n_}"] = gr
        arrays[f"mb{j}/flat_grad"] = f32(grad_calls[j])
        if adaptive:
            arrays[f"mb{j}/kl_mean"] = np.float32(kl_calls[j].item())
    for k, v in init_state.items():
        arrays[f"init/{k}"] = v
    for k, v in storage_in.items():
        arrays[f"storage/{k}"] = v
    arrays["storage/last_obs"] = f32(last_obs)
    arrays["gen_state"] = gen_state
    for k, v in pol.state_dict().items():
        arrays[f"final/{k}"] = f32(v)
    meta = dict(T=T, N=N, O=O, A=A, M=M, E=E, hidden=hidden, policy_kw=policy_kw, ppo_kw=ppo_kw,
                consistent=consistent, multi_gpu_cfg_world_size=1,
                normalize_in_storage=normalize_in_storage, loss_dict=loss_dict, lr_trace=lr_trace,
                final_lr=alg.learning_rate, num_batches=len(records), adaptive=adaptive,
                param_order=[n for n, _ in pol.named_parameters()])
    return arrays, meta


LOSS_CASES = [
    # name, T, N, O, A, M, E, hidden, policy_kw, ppo_kw[, consistent]
    ("default_b111", 3, 37, 5, 3, 1, 1, [8], {}, {}),
    ("tail_drop_m2", 3, 37, 5, 3, 2, 1, [8], {}, {}),
    ("consistent_m4e2", 8, 64, 6, 4, 4, 2, [16], {}, {}, True),
    ("consistent_state_dep", 8, 64, 6, 4, 2, 2, [16], {"state_dependent_std": True}, {}, True),
    ("default_m2e2", 8, 128, 6, 4, 2, 2, [16], {}, {}),
    ("noclip_value", 4, 50, 5, 3, 1, 1, [8], {}, {"use_clipped_value_loss": False}),
    ("log_std", 4, 50, 5, 3, 1, 1, [8], {"noise_std_type": "log"}, {}),
    ("state_dep_scalar", 4, 50, 5, 3, 1, 1, [8], {"state_dependent_std": True}, {}),
    ("state_dep_log", 4, 50, 5, 3, 1, 1, [8], {"state_dependent_std": True, "noise_std_type": "log"}, {}),
    ("mb_adv_norm", 4, 64, 5, 3, 2, 1, [8], {}, {"normalize_advantage_per_mini_batch": True}),
    ("fixed_schedule", 4, 50, 5, 3, 1, 1, [8], {}, {"schedule": "fixed"}),
    ("a12_b1536", 6, 256, 48, 12, 1, 1, [32], {}, {}),
    ("hicoef", 4, 50, 5, 3, 1, 1, [8], {}, {"clip_param": 0.1, "value_loss_coef": 0.5,
                                          "entropy_coef": 0.05}),
]


def make_loss(PPO, ActorCritic, RolloutStorage):
    meta = {}
    for i, case in enumerate(LOSS_CASES):
        name, T, N, O, A, M, E, hidden, pkw, akw = case[:10]
        consistent = len(case) > 10 and case[10]
        arrays, m = _record_update(PPO, ActorCritic, RolloutStorage, T=T, N=N, O=O, A=A, M=M, E=E,
                                   hidden=hidden, policy_kw=pkw, ppo_kw=akw, seed=100 + i,
                                   normalize_in_storage=not akw.get("normalize_advantage_per_mini_batch", False),
                                   consistent=consistent)
        np.savez_compressed(os.path.join(HERE, f"loss_{name}.npz"), **arrays)
        meta[name] = m
    return meta


def make_update_c1(PPO, ActorCritic, RolloutStorage):
    """Config C1 (N512 T16 O16 A4, 2x64 ELU, E5 M4): one full update from a rollout-like storage."""
    arrays, m = _record_update(PPO, ActorCritic, RolloutStorage, T=16, N=512, O=16, A=4, M=4, E=5,
                               hidden=[64, 64], policy_kw={}, ppo_kw={}, seed=31337,
                               normalize_in_storage=True, consistent=True)
    keep = {k: v for k, v in arrays.items() if not k.startswith("mb") or k.endswith("kl_mean")}
    np.savez_compressed(os.path.join(HERE, "update_c1.npz"), **keep)
    return m


# --------------------------------------------------------------------------------------------------
# full updates whose storage is regenerated from numpy seeds on the test side (the fixture stores only what
# the reference's policy produced): multi-rank W = 2 / 4 over gloo (ppo.py:271-294, :428-469) and one update
# at the real network width (config C2's shape: O48 A12 3x256)
# --------------------------------------------------------------------------------------------------
def storage_noise(seed, T, N, O, A):
    """The policy-independent storage inputs, drawn with numpy's PCG64 (bit-reproducible across machines for
    a given numpy; tests/test_*update*.py regenerate them): obs, rewards, dones, action noise, last obs."""
    rng = np.random.default_rng(seed)
    return {
        "obs": rng.standard_normal((T, N, O), dtype=np.float32),
        "rewards": rng.standard_normal((T, N, 1), dtype=np.float32),
        "dones": (rng.random((T, N, 1)) < 0.05).astype(np.uint8),
        "noise": rng.standard_normal((T, N, A), dtype=np.float32),
        "last_obs": rng.standard_normal((N, O), dtype=np.float32),
    }


def _fill_storage_from_noise(st, policy, nz, mu_fp16):
    """Rollout-consistent storage (as ppo.py:129-140 would record it): mu / sigma / values from the policy for the
    stored obs, actions = mu + sigma * noise (fp32 mul then add), log-prob of those actions under N(mu, sigma).
    mu_fp16: the stored mean is rounded to fp16 first (a compact fixture; the first mini-batch's KL then is the
    small non-zero KL of that rounding).  Returns the arrays the fixture must store."""
    T, N, O = nz["obs"].shape
    A = nz["noise"].shape[-1]
    obs = torch.from_numpy(nz["obs"])
    st.observations["policy"].copy_(obs)
    st.rewards.copy_(torch.from_numpy(nz["rewards"]))
    st.dones.copy_(torch.from_numpy(nz["dones"]))
    with torch.inference_mode():
        o = {"policy": obs.reshape(T * N, O)}
        policy.update_distribution(policy.actor_obs_normalizer(policy.get_actor_obs(o)))
        mu = policy.action_mean.reshape(T, N, A).clone()
        sigma = policy.action_std.reshape(T, N, A).clone()
        if mu_fp16:
            mu = mu.half().float()
        actions = mu + sigma * torch.from_numpy(nz["noise"])
        logp = torch.distributions.Normal(mu, sigma).log_prob(actions).sum(-1, keepdim=True)
        values = policy.evaluate(o).reshape(T, N, 1).clone()
    st.values.copy_(values)
    st.mu.copy_(mu)
    st.sigma.copy_(sigma)
    st.actions.copy_(actions)
    st.actions_log_prob.copy_(logp)
    st.step = T
    assert torch.equal(sigma, sigma[:1, :1].expand_as(sigma))
    return {"mu": mu.half().numpy() if mu_fp16 else f32(mu), "sigma": f32(sigma[0, 0]), "values": f32(values),
            "actions_log_prob": f32(logp)}


def _run_recorded_update(alg, grad_batches=0):
    """update() recording the lr of every optimizer step and the pre-clip policy gradient (concatenated in
    parameters() order) of the first `grad_batches` mini-batches (with RND: also the RND predictor's gradient,
    after reduce_parameters, as rnd_optimizer.step sees it)."""
    lr_trace, grads, rnd_grads = [], [], []
    orig_step = alg.optimizer.step
    orig_clip = torch.nn.utils.clip_grad_norm_

    def rec_clip(params, *a, **kw):
        if len(grads) < grad_batches:
            grads.append(torch.cat([p.grad.reshape(-1) for p in alg.policy.parameters()]).clone())
        return orig_clip(params, *a, **kw)

    def rec_step(*a, **kw):
        lr_trace.append(alg.optimizer.param_groups[0]["lr"])
        return orig_step(*a, **kw)

    alg.optimizer.step = rec_step
    if alg.rnd_optimizer is not None:
        orig_rnd_step = alg.rnd_optimizer.step

        def rec_rnd_step(*a, **kw):
            if len(rnd_grads) < grad_batches:
                rnd_grads.append(torch.cat([p.grad.reshape(-1) for p in alg.rnd.predictor.parameters()]).clone())
            return orig_rnd_step(*a, **kw)

        alg.rnd_optimizer.step = rec_rnd_step
    torch.nn.utils.clip_grad_norm_ = rec_clip
    try:
        loss_dict = alg.update()
    finally:
        torch.nn.utils.clip_grad_norm_ = orig_clip
    return loss_dict, lr_trace, grads, rnd_grads


def _update_case(PPO, ActorCritic, RolloutStorage, *, T, N, O, A, hidden, seed, rank, world, mu_fp16, lr=1e-3,
                 grad_batches=0, logp_ulp=False, rnd_cfg=None, policy_kw=None):
    """One reference update() on rank `rank` of `world` (world > 1: inside an initialised gloo group).
    rnd_cfg: the PPO rnd_cfg (num_states / obs_groups filled in here, rnd.py:185-209); with state_normalization the
    RND state normaliser is first fed two batches of numpy-seeded states, as the rollout's update_normalization
    would (ppo.py:145-146)."""
    torch.manual_seed(seed + 17 * rank)  # different initial weights per rank; broadcast_parameters syncs them
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    if rnd_cfg is not None:
        groups["rnd_state"] = ["policy"]
    pol = ActorCritic(obs0, groups, A, actor_hidden_dims=hidden, critic_hidden_dims=hidden, **(policy_kw or {}))
    mcfg = {"global_rank": rank, "local_rank": rank, "world_size": world} if world > 1 else None
    rcfg = None if rnd_cfg is None else dict(rnd_cfg, num_states=O, obs_groups=groups)
    alg = PPO(pol, num_learning_epochs=5, num_mini_batches=4, device="cpu", multi_gpu_cfg=mcfg, learning_rate=lr,
              rnd_cfg=rcfg)
    if world > 1:
        alg.broadcast_parameters()  # on_policy_runner.py:99-101
    init_state = {k: f32(v) for k, v in pol.state_dict().items()}
    if isinstance(logp_ulp, str) and logp_ulp.startswith("par"):  # sensitivity probe: every initial policy
        # parameter one ulp up or down at random (as a GEMM's last-bit rounding moves every forward value)
        g = torch.Generator().manual_seed(int(logp_ulp[3:]) * 1000 + 7)
        with torch.no_grad():
            for p in pol.parameters():
                up = torch.nextafter(p, torch.full_like(p, float("inf")))
                down = torch.nextafter(p, torch.full_like(p, float("-inf")))
                p.copy_(torch.where(torch.rand(p.shape, generator=g) < 0.5, up, down))
    rnd_init = {}
    if alg.rnd is not None:
        if alg.rnd.state_normalization:
            nrng = np.random.default_rng(seed * 100 + rank + 50)
            for _ in range(2):
                x = nrng.standard_normal((N, O), dtype=np.float32) * 1.5 + 0.25
                alg.rnd.update_normalization({"policy": torch.from_numpy(x)})
        rnd_init = {k: (v.numpy().copy() if v.dtype == torch.int64 else f32(v))
                    for k, v in alg.rnd.state_dict().items()}
    alg.init_storage("rl", N, T, obs0, [A])
    nz = storage_noise(seed * 100 + rank, T, N, O, A)
    stored = _fill_storage_from_noise(alg.storage, pol, nz, mu_fp16)
    if logp_ulp and not (isinstance(logp_ulp, str) and logp_ulp.startswith("par")):  # sensitivity probe: the stored log-probs one ulp off (True / "up": every one up; "down": every
        # one down; "rand<k>": up or down at random per sample, seeded by k and the rank)
        lp = alg.storage.actions_log_prob
        up = torch.nextafter(lp, torch.full_like(lp, float("inf")))
        down = torch.nextafter(lp, torch.full_like(lp, float("-inf")))
        if logp_ulp is True or logp_ulp == "up":
            lp.copy_(up)
        elif logp_ulp == "down":
            lp.copy_(down)
        else:
            g = torch.Generator().manual_seed(int(logp_ulp[4:]) * 1000 + rank)
            lp.copy_(torch.where(torch.rand(lp.shape, generator=g) < 0.5, up, down))
    with torch.inference_mode():
        alg.compute_returns({"policy": torch.from_numpy(nz["last_obs"])})
    torch.manual_seed(5000 + rank)  # the permutation's generator, per rank
    gen_state = torch.default_generator.get_state().numpy().copy()
    loss_dict, lr_trace, grads, rnd_grads = _run_recorded_update(alg, grad_batches)
    arrays = {f"init/{k}": v for k, v in init_state.items()}
    for j, g in enumerate(grads):  # pre-clip gradients of the first mini-batches (before any trajectory drift)
        arrays[f"grad_mb{j}"] = f32(g)
    for j, g in enumerate(rnd_grads):
        arrays[f"rnd_grad_mb{j}"] = f32(g)
    arrays.update({f"final/{k}": f32(v) for k, v in pol.state_dict().items()})
    if alg.rnd is not None:
        arrays.update({f"rnd_init/{k}": v for k, v in rnd_init.items()})
        arrays.update({f"rnd_final/{k}": f32(v) for k, v in alg.rnd.predictor.state_dict().items()})
    arrays.update({f"storage/{k}": v for k, v in stored.items()})
    arrays["storage/returns_head"] = f32(alg.storage.returns[:2])  # after compute_returns (un-cleared buffer)
    arrays["gen_state"] = gen_state
    arrays["obs_sha256"] = np.frombuffer(hashlib.sha256(nz["obs"].tobytes()).digest(), dtype=np.uint8)
    meta = {"loss_dict": loss_dict, "lr_trace": lr_trace, "final_lr": alg.learning_rate,
            "noise_seed": seed * 100 + rank}
    return arrays, meta


C5_RND = dict(weight=1.0 * 0.02, num_outputs=1, predictor_hidden_dims=[-1], target_hidden_dims=[-1],
              learning_rate=1e-3)  # config C5: weight 1.0 x step_dt 0.02, 48->48->1
MULTIRANK_CASES = [  # name, world, T, N per rank, O, A, hidden, seed, learning rate[, options]
    ("w2", 2, 16, 256, 16, 4, [64, 64], 71, 1e-3),
    ("w4", 4, 16, 128, 16, 4, [64, 64], 73, 6e-3),  # large steps: the lr-decrease branch is taken as well
    # round 3: eight ranks at C1's shape, and two ranks at C4's per-rank network (3x256, O48, A12)
    ("w8", 8, 16, 64, 16, 4, [64, 64], 79, 1e-3, {"sensitivity": True}),
    ("w2_c4net", 2, 24, 1024, 48, 12, [256, 256, 256], 83, 1e-3,
     {"mu_fp16": True, "sensitivity": True, "shared_params": True, "grad_batches": 1}),
]
# PPO.update() with RND (ppo.py:352-372, :383-384, :447-450): the predictor trained every mini-batch
RND_UPDATE_CASES = [
    ("rnd_c5_w1", 1, 24, 1024, 48, 12, [256, 256, 256], 89, 1e-3,
     {"mu_fp16": True, "sensitivity": True, "grad_batches": 1, "rnd": C5_RND}),
    ("rnd_c5_w2", 2, 24, 512, 48, 12, [256, 256, 256], 97, 1e-3,
     {"mu_fp16": True, "sensitivity": True, "shared_params": True, "grad_batches": 1, "rnd": C5_RND}),
    ("rnd_statenorm_w1", 1, 16, 256, 16, 4, [64, 64], 101, 1e-3,
     {"sensitivity": True, "grad_batches": 1,
      "rnd": dict(weight=0.5, num_outputs=3, predictor_hidden_dims=[32], target_hidden_dims=[32],
                  state_normalization=True, learning_rate=2e-3)}),
]


# the std parameterisations through a whole update at a shape the fused MLP path takes (O a multiple of 4):
# state-dependent std (actor_critic.py:63-86, :119-128) with scalar and log std, and a log_std parameter
STD_UPDATE_CASES = [
    ("sdstd_scalar", 1, 8, 256, 16, 4, [64, 64], 103, 1e-3,
     {"grad_batches": 1, "policy_kw": {"state_dependent_std": True}}),
    ("sdstd_log", 1, 8, 256, 16, 4, [64, 64], 107, 1e-3,
     {"grad_batches": 1, "policy_kw": {"state_dependent_std": True, "noise_std_type": "log"}}),
    ("logstd", 1, 8, 256, 16, 4, [64, 64], 109, 1e-3, {"grad_batches": 1, "policy_kw": {"noise_std_type": "log"}}),
]


def _case_kw(case, logp_ulp=False):
    name, world, T, N, O, A, hidden, seed, lr = case[:9]
    opt = case[9] if len(case) > 9 else {}
    return dict(T=T, N=N, O=O, A=A, hidden=hidden, seed=seed, world=world, mu_fp16=opt.get("mu_fp16", False),
                lr=lr, grad_batches=opt.get("grad_batches", 0), logp_ulp=logp_ulp,
                rnd_cfg=dict(opt["rnd"]) if opt.get("rnd") else None, policy_kw=opt.get("policy_kw"))


def _multirank_worker(rank, world, port, ref_path, case, out_dir, logp_ulp):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    PPO, ActorCritic, RolloutStorage = import_reference(ref_path)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arrays, meta = _update_case(PPO, ActorCritic, RolloutStorage, rank=rank, **_case_kw(case, logp_ulp))
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), **arrays)
        with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
            json.dump(meta, f)
    finally:
        torch.distributed.destroy_process_group()


def _run_update_case(ref_path, case, logp_ulp=False):
    """All ranks of one case: ({f"r{rank}/...": array}, [per-rank meta])."""
    import socket
    import tempfile

    import torch.multiprocessing as mp

    world = case[1]
    if world == 1:
        PPO, ActorCritic, RolloutStorage = import_reference(ref_path)
        a, m = _update_case(PPO, ActorCritic, RolloutStorage, rank=0, **_case_kw(case, logp_ulp))
        return {f"r0/{k}": v for k, v in a.items()}, [m]
    with tempfile.TemporaryDirectory() as d:
        sock = socket.socket()
        sock.bind(("127.0.0.1", 0))
        port = sock.getsockname()[1]
        sock.close()
        mp.spawn(_multirank_worker, args=(world, port, ref_path, case, d, logp_ulp), nprocs=world, join=True)
        arrays, ranks = {}, []
        for r in range(world):
            z = np.load(os.path.join(d, f"r{r}.npz"))
            arrays.update({f"r{r}/{k}": z[k] for k in z.files})
            with open(os.path.join(d, f"r{r}.json")) as f:
                ranks.append(json.load(f))
    return arrays, ranks


def _make_update_family(ref_path, cases):
    """Reference update() captures of `cases`: tests/golden/update_<name>.npz + their golden.json entries.

    options: mu_fp16 (stored mean rounded to fp16: a compact fixture), grad_batches (pre-clip gradients of the first
    mini-batches), sensitivity (the reference's own parameter movement when every stored log-prob is one ulp up,
    per tensor relative to how far the update moved it -- the bound the tests use at widths where the surrogate's
    clip discontinuity makes last-bit log-prob differences visible, see make_update_c2), shared_params (initial and
    final parameters and the recorded (all-reduced) gradients stored for rank 0 only: every rank holds the same ones
    after broadcast_parameters / reduce_parameters; asserted here), rnd (rnd_cfg of the PPO)."""
    meta = {}
    for case in cases:
        name, world, T, N, O, A, hidden, seed, lr = case[:9]
        opt = case[9] if len(case) > 9 else {}
        arrays, ranks = _run_update_case(ref_path, case)
        if opt.get("shared_params"):
            for r in range(1, world):
                for k in [k for k in arrays if k.startswith(f"r{r}/") and (
                        k.split("/")[1] in ("init", "final", "rnd_final")
                        or k.split("/")[1].startswith(("grad_mb", "rnd_grad_mb")))]:
                    assert np.array_equal(arrays[k], arrays["r0/" + k.split("/", 1)[1]]), k
                    del arrays[k]
        m = {"world": world, "T": T, "N": N, "O": O, "A": A, "hidden": hidden, "M": 4, "E": 5, "seed": seed,
             "learning_rate": lr, "ranks": ranks, "mu_fp16": opt.get("mu_fp16", False),
             "shared_params": bool(opt.get("shared_params")), "rnd_cfg": opt.get("rnd"),
             "policy_kw": opt.get("policy_kw") or {}}
        if opt.get("sensitivity"):
            # the envelope over several one-ulp probes of the reference itself: the stored log-probs all up, all
            # down, up/down at random, and the initial policy parameters up/down at random (two patterns; as a
            # GEMM's last-bit rounding moves every forward value).  One probe may happen to flip no sample at a clip
            # bound where another last-bit pattern flips one (each flipped sample moves a mini-batch gradient by
            # ~1/sqrt(B), and Adam carries it on)
            sens = {}
            probes = ("up", "down", "rand0", "par0", "par1")
            for probe in probes:
                ulp, _ = _run_update_case(ref_path, case, logp_ulp=probe)
                for pre, init_pre in (("r0/final/", "r0/init/"), ("r0/rnd_final/", None)):
                    for k in [k for k in arrays if k.startswith(pre)]:
                        pname = k[len(pre):]
                        init = (arrays[init_pre + pname] if init_pre else
                                arrays["r0/rnd_init/predictor." + pname])
                        moved = np.linalg.norm(arrays[k].astype(np.float64) - init.astype(np.float64))
                        d = np.linalg.norm(ulp[k].astype(np.float64) - arrays[k].astype(np.float64))
                        key = ("rnd/" if init_pre is None else "") + pname
                        sens[key] = max(sens.get(key, 0.0), float(d / moved) if moved else float(d))
            m["ulp_sensitivity"] = sens
            m["ulp_probes"] = list(probes)
        np.savez_compressed(os.path.join(HERE, f"update_{name}.npz"), **arrays)
        meta[name] = m
        print("update case", name, "lr", ranks[0]["lr_trace"][:4], "...", ranks[0]["final_lr"], flush=True)
    return meta


def make_multirank(ref_path, names=None):
    return _make_update_family(ref_path, [c for c in MULTIRANK_CASES if names is None or c[0] in names])


def make_update_rnd(ref_path):
    return _make_update_family(ref_path, RND_UPDATE_CASES)


def make_update_std(ref_path):
    return _make_update_family(ref_path, STD_UPDATE_CASES)


def make_update_c2(PPO, ActorCritic, RolloutStorage):
    """One reference update at config C2's shape: N4096 T24 O48 A12, actor/critic 3x256 ELU, E5 M4 (mini-batch
    24,576 rows); storage regenerated from numpy seeds on the test side, mean stored as fp16."""
    T, N, O, A, hidden, seed = 24, 4096, 48, 12, [256, 256, 256], 91
    arrays, m = _update_case(PPO, ActorCritic, RolloutStorage, T=T, N=N, O=O, A=A, hidden=hidden, seed=seed,
                             rank=0, world=1, mu_fp16=True, grad_batches=1)
    np.savez_compressed(os.path.join(HERE, "update_c2.npz"), **arrays)
    # the reference's own sensitivity: the same update with every stored log-prob one ulp up.  The surrogate's
    # clip/max branches are discontinuous, so samples at a clip bound flip and the trajectory moves; the test
    # bounds our deviation by this (per tensor, relative to how far the update moved it)
    ulp, _ = _update_case(PPO, ActorCritic, RolloutStorage, T=T, N=N, O=O, A=A, hidden=hidden, seed=seed, rank=0,
                          world=1, mu_fp16=True, logp_ulp=True)
    sens = {}
    for k in arrays:
        if k.startswith("final/"):
            name = k[6:]
            moved = np.linalg.norm(arrays[k].astype(np.float64) - arrays["init/" + name].astype(np.float64))
            sens[name] = float(np.linalg.norm(ulp[k].astype(np.float64) - arrays[k].astype(np.float64)) / moved)
    m["ulp_sensitivity"] = sens
    m.update({"T": T, "N": N, "O": O, "A": A, "hidden": hidden, "M": 4, "E": 5, "seed": seed, "mu_fp16": True,
              "learning_rate": 1e-3})
    return m


# --------------------------------------------------------------------------------------------------
# one reference update at config C3's full size (N 65536, T 24, O 48, A 12, 3x256; 393,216-row mini-batches):
# the first mini-batch's pre-clip gradient, the loss means and the lr trace.  The whole storage is regenerated from
# one numpy seed on the test side (policy-independent: 1.57 M transitions cannot travel as a fixture), so the stored
# mean / values / log-probs are seeded draws, not the policy's outputs -- the rollout policy's std (1.0) is stored as
# sigma, as a rollout with a shared std records it.  The fixture holds the initial weights, the gradient and the
# generator state (~2.3 MB).
# --------------------------------------------------------------------------------------------------
def storage_c3(seed, T, N, O, A):
    """Every storage input of the C3 fixture from one PCG64 stream (tests/test_gpu_update_c3.py draws the same)."""
    rng = np.random.default_rng(seed)
    nz = {
        "obs": rng.standard_normal((T, N, O), dtype=np.float32),
        "rewards": rng.standard_normal((T, N, 1), dtype=np.float32),
        "dones": (rng.random((T, N, 1)) < 0.02).astype(np.uint8),
        "noise": rng.standard_normal((T, N, A), dtype=np.float32),
        "last_obs": rng.standard_normal((N, O), dtype=np.float32),
        "mu": rng.standard_normal((T, N, A), dtype=np.float32),
        "values": rng.standard_normal((T, N, 1), dtype=np.float32),
    }
    nz["mu"] *= np.float32(0.3)
    # the stored log-prob of the actions mu + 1.0 * noise under N(mu, 1): -0.5 sum_a noise_a^2 - A/2 log(2 pi), by
    # elementwise fp32 operations in action order (correctly rounded on any CPU: bit-reproducible)
    s = np.zeros((T, N), dtype=np.float32)
    for a in range(A):
        s = s + nz["noise"][..., a] * nz["noise"][..., a]
    nz["logp"] = (np.float32(-0.5) * s - np.float32(A * 0.9189385332046727))[..., None]
    return nz


def make_update_c3(PPO, ActorCritic, RolloutStorage):
    T, N, O, A, hidden, seed = 24, 65536, 48, 12, [256, 256, 256], 113
    torch.manual_seed(seed)
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    pol = ActorCritic(obs0, groups, A, actor_hidden_dims=hidden, critic_hidden_dims=hidden)
    alg = PPO(pol, num_learning_epochs=5, num_mini_batches=4, device="cpu")
    init_state = {k: f32(v) for k, v in pol.state_dict().items()}
    alg.init_storage("rl", N, T, obs0, [A])
    nz = storage_c3(seed * 100, T, N, O, A)
    st = alg.storage
    std = pol.std.detach().clone()  # noise_std_type "scalar": the distribution's std is this parameter
    st.observations["policy"].copy_(torch.from_numpy(nz["obs"]))
    st.rewards.copy_(torch.from_numpy(nz["rewards"]))
    st.dones.copy_(torch.from_numpy(nz["dones"]))
    mu = torch.from_numpy(nz["mu"])
    sig = std.reshape(1, 1, A).expand(T, N, A)
    st.mu.copy_(mu)
    st.sigma.copy_(sig)
    st.actions.copy_(mu + sig * torch.from_numpy(nz["noise"]))
    st.values.copy_(torch.from_numpy(nz["values"]))
    st.actions_log_prob.copy_(torch.from_numpy(nz["logp"]))
    st.step = T
    with torch.inference_mode():
        alg.compute_returns({"policy": torch.from_numpy(nz["last_obs"])})
    torch.manual_seed(5000)
    gen_state = torch.default_generator.get_state().numpy().copy()
    loss_dict, lr_trace, grads, _ = _run_recorded_update(alg, grad_batches=1)
    arrays = {f"init/{k}": v for k, v in init_state.items()}
    arrays["grad_mb0"] = f32(grads[0])
    arrays["std"] = f32(std)
    arrays["gen_state"] = gen_state
    arrays["returns_head"] = f32(st.returns[:2, :256])
    arrays["advantages_head"] = f32(st.advantages[:2, :256])
    arrays["obs_sha256"] = np.frombuffer(hashlib.sha256(nz["obs"].tobytes()).digest(), dtype=np.uint8)
    arrays["logp_sha256"] = np.frombuffer(hashlib.sha256(nz["logp"].tobytes()).digest(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "update_c3.npz"), **arrays)
    print("update_c3 lr", lr_trace[:4], "...", alg.learning_rate, loss_dict, flush=True)
    return {"T": T, "N": N, "O": O, "A": A, "hidden": hidden, "M": 4, "E": 5, "seed": seed, "noise_seed": seed * 100,
            "loss_dict": loss_dict, "lr_trace": lr_trace, "final_lr": alg.learning_rate}


# --------------------------------------------------------------------------------------------------
# rollout side: act + process_env_step + add_transitions + RND (ppo.py:129-169, rollout_storage.py:77-103,
# rnd.py:113-135) -- the inputs of each step, the transition act() produced, and the storage after T steps
# --------------------------------------------------------------------------------------------------
ROLLOUT_CASES = [
    # name, N, O, A, T, rnd_cfg (None: no RND), p(time_out), dones dtype, seed
    ("rnd_c5like", 300, 48, 12, 3,
     dict(weight=1.0 * 0.02, num_outputs=1, predictor_hidden_dims=[-1], target_hidden_dims=[-1]), 0.3, "int64", 7),
    ("rnd_statenorm_q3", 130, 16, 4, 3,
     dict(weight=0.5, num_outputs=3, predictor_hidden_dims=[32], target_hidden_dims=[32], state_normalization=True,
          weight_schedule={"mode": "step", "final_step": 2, "final_value": 0.25}), 0.2, "bool", 8),
    ("plain_timeouts", 257, 16, 4, 2, None, 0.5, "float", 9),
    # linear weight schedule (rnd.py:175-182): weights strictly between the end points on steps 3..5
    ("rnd_linear_sched", 64, 16, 4, 8,
     dict(weight=0.3, num_outputs=2, predictor_hidden_dims=[16], target_hidden_dims=[16],
          weight_schedule={"mode": "linear", "initial_step": 2, "final_step": 6, "final_value": 0.7}), 0.2, "int64", 10),
]


def make_rollout(PPO, ActorCritic, RolloutStorage):
    meta = {}
    for name, N, O, A, T, rnd_cfg, p_to, dt, seed in ROLLOUT_CASES:
        torch.manual_seed(seed)
        obs0 = {"policy": torch.zeros(N, O)}
        groups = {"policy": ["policy"], "critic": ["policy"], "rnd_state": ["policy"]}
        pol = ActorCritic(obs0, groups, A, actor_hidden_dims=[64, 64], critic_hidden_dims=[64, 64])
        cfg = None
        if rnd_cfg is not None:
            cfg = dict(rnd_cfg, num_states=O, obs_groups=groups)
        alg = PPO(pol, device="cpu", rnd_cfg=cfg)
        alg.init_storage("rl", N, T, obs0, [A])
        arrays = {f"init/{k}": f32(v) for k, v in pol.state_dict().items()}
        if alg.rnd is not None:
            arrays.update({f"rnd_init/{k}": f32(v) for k, v in alg.rnd.state_dict().items()})
        g = torch.Generator().manual_seed(seed + 1)
        obs = torch.randn(N, O, generator=g)
        for t in range(T):
            with torch.inference_mode():
                alg.act({"policy": obs})
                tr = alg.transition
                arrays[f"step{t}/obs"] = f32(obs)
                for k in ("actions", "values", "actions_log_prob", "action_mean", "action_sigma"):
                    arrays[f"step{t}/{k}"] = f32(getattr(tr, k))
                nobs = torch.randn(N, O, generator=g)
                rew = torch.randn(N, generator=g)
                d = torch.rand(N, generator=g) < 0.1
                dones = {"int64": d.long(), "bool": d, "float": d.float()}[dt]
                to = (torch.rand(N, generator=g) < p_to).float()
                arrays[f"step{t}/next_obs"] = f32(nobs)
                arrays[f"step{t}/rewards"] = f32(rew)
                arrays[f"step{t}/dones"] = d.numpy().astype(np.uint8)
                arrays[f"step{t}/time_outs"] = f32(to)
                alg.process_env_step({"policy": nobs}, rew, dones, {"time_outs": to})
                if alg.rnd is not None:
                    arrays[f"step{t}/intrinsic"] = f32(alg.intrinsic_rewards)
                    arrays[f"step{t}/rnd_weight"] = np.float64(alg.rnd.weight)  # the host-side Python float
                obs = nobs
        st = alg.storage
        for k in ("rewards", "values", "actions_log_prob", "mu", "sigma", "actions"):
            arrays[f"storage/{k}"] = f32(getattr(st, k))
        arrays["storage/dones"] = st.dones.numpy().copy()
        arrays["storage/obs_policy"] = f32(st.observations["policy"])
        np.savez_compressed(os.path.join(HERE, f"rollout_{name}.npz"), **arrays)
        meta[name] = {"N": N, "O": O, "A": A, "T": T, "rnd_cfg": rnd_cfg, "dones_dtype": dt, "gamma": alg.gamma,
                      "p_time_out": p_to, "actor_hidden": [64, 64]}
    return meta


# --------------------------------------------------------------------------------------------------
# normalisers (networks/normalization.py): a sequence of updates with an `until` limit, forward outputs,
# and the discounted reward normaliser over several steps
# --------------------------------------------------------------------------------------------------
def make_normalizer(ref_path):
    sys.path.insert(0, ref_path)
    from rsl_rl.networks.normalization import EmpiricalDiscountedVariationNormalization, EmpiricalNormalization

    g = torch.Generator().manual_seed(77)
    arrays = {}
    norm = EmpiricalNormalization(shape=[7], until=2500)
    norm.train()
    for k in range(4):  # 1000 rows each: the 4th update is skipped (count 3000 >= 2500)
        x = torch.randn(1000, 7, generator=g) * torch.linspace(0.5, 3.0, 7) + torch.linspace(-2.0, 5.0, 7)
        norm.update(x)
        arrays[f"obs/x{k}"] = f32(x)
        arrays[f"obs/mean{k}"], arrays[f"obs/var{k}"] = f32(norm._mean), f32(norm._var)
        arrays[f"obs/std{k}"], arrays[f"obs/count{k}"] = f32(norm._std), np.int64(norm.count.item())
        arrays[f"obs/y{k}"] = f32(norm(x))
    rn = EmpiricalDiscountedVariationNormalization(shape=[], gamma=0.99)
    rn.train()
    for k in range(5):
        r = torch.randn(300, generator=g) * 2.0 + 0.5
        out = rn(r)
        arrays[f"rew/r{k}"], arrays[f"rew/out{k}"] = f32(r), f32(out)
        arrays[f"rew/std{k}"], arrays[f"rew/avg{k}"] = f32(rn.emp_norm._std), f32(rn.disc_avg.avg)
    np.savez_compressed(os.path.join(HERE, "normalizer.npz"), **arrays)
    return {"obs_updates": 4, "until": 2500, "reward_steps": 5, "gamma": 0.99}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=os.environ.get("RSL_RL_REFERENCE", "/root/reference"))
    ap.add_argument("--only", choices=["rollout", "normalizer", "multirank", "update_c2", "update_rnd",
                                           "update_std", "update_c3"],
                    help="regenerate one fixture family, keep the rest")
    ap.add_argument("--cases", default=None, help="with --only multirank: comma-separated case names to (re)generate")
    args = ap.parse_args()
    torch.set_num_threads(4)
    PPO, ActorCritic, RolloutStorage = import_reference(args.reference)
    if args.only:
        with open(os.path.join(HERE, "golden.json")) as f:
            meta = json.load(f)
        if args.only == "rollout":
            meta["rollout"] = make_rollout(PPO, ActorCritic, RolloutStorage)
        elif args.only == "multirank":
            names = args.cases.split(",") if args.cases else None
            meta["multirank"] = dict(meta.get("multirank", {}), **make_multirank(args.reference, names))
        elif args.only == "update_rnd":
            meta["update_rnd"] = make_update_rnd(args.reference)
        elif args.only == "update_std":
            meta["update_std"] = make_update_std(args.reference)
        elif args.only == "update_c2":
            meta["update_c2"] = make_update_c2(PPO, ActorCritic, RolloutStorage)
        elif args.only == "update_c3":
            torch.set_num_threads(8)
            meta["update_c3"] = make_update_c3(PPO, ActorCritic, RolloutStorage)
        else:
            meta["normalizer"] = make_normalizer(args.reference)
        with open(os.path.join(HERE, "golden.json"), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        print("wrote", args.only, "fixtures")
        return
    meta = {
        "generator": "tests/golden/make_golden.py",
        "reference": "rsl-rl-lib 3.1.0 (kaixi287/rsl_rl snapshot 2025-10-17)",
        "torch": torch.__version__,
        "gae": make_gae(RolloutStorage),
        "perm": make_perm(),
        "minibatch": make_minibatch(RolloutStorage),
        "loss": make_loss(PPO, ActorCritic, RolloutStorage),
        "update_c1": make_update_c1(PPO, ActorCritic, RolloutStorage),
        "rollout": make_rollout(PPO, ActorCritic, RolloutStorage),
        "normalizer": make_normalizer(args.reference),
        "multirank": make_multirank(args.reference),
        "update_c2": make_update_c2(PPO, ActorCritic, RolloutStorage),
        "update_rnd": make_update_rnd(args.reference),
        "update_std": make_update_std(args.reference),
        "update_c3": make_update_c3(PPO, ActorCritic, RolloutStorage),
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
