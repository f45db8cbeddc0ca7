"""CPU PPO iteration built on the oracle -- TEST / BASELINE INFRASTRUCTURE ONLY.

A complete on-policy iteration (rollout + compute_returns + update) restated on the CPU: the policy
MLPs, sampling, Adam and grad clipping use torch on the CPU exactly like the reference does there; the
hot path uses the oracle (oracle/oracle.c GAE, mt19937 randperm and row gathers; the numpy PPO
loss/gradient restatement of ppo.py:259-315).  bench.py times it as the `cpu_baseline` ("port") on the
GPU box's host cores; tests use it as the integration-level checker.  Never imported by rsl_rl_amd.
"""

from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn as nn

from . import ppo_oracle as O


class _MLP(nn.Sequential):
    def __init__(self, i, o, hidden):
        dims = [i] + list(hidden)
        layers = []
        for a, b in zip(dims[:-1], dims[1:]):
            layers += [nn.Linear(a, b), nn.ELU()]
        layers.append(nn.Linear(dims[-1], o))
        super().__init__(*layers)


class CpuPPO:
    """Gaussian actor (shared std parameter) + critic, reference hyper-parameters (ppo.py:25-48)."""

    def __init__(self, num_envs, num_obs, num_actions, hidden=(256, 256, 256), T=24, E=5, M=4, seed=0, lr=1e-3,
                 clip=0.2, gamma=0.99, lam=0.95, value_coef=1.0, entropy_coef=0.01, max_grad_norm=1.0,
                 desired_kl=0.01):
        torch.manual_seed(seed)
        self.N, self.O, self.A, self.T, self.E, self.M = num_envs, num_obs, num_actions, T, E, M
        self.actor = _MLP(num_obs, num_actions, hidden)
        self.critic = _MLP(num_obs, 1, hidden)
        self.std = nn.Parameter(torch.ones(num_actions))
        self.params = [self.std] + list(self.actor.parameters()) + list(self.critic.parameters())
        self.opt = torch.optim.Adam(self.params, lr=lr)
        self.lr = lr
        self.hp = dict(clip=clip, gamma=gamma, lam=lam, value_coef=value_coef, entropy_coef=entropy_coef,
                       max_grad_norm=max_grad_norm, desired_kl=desired_kl)
        self.gen = torch.Generator().manual_seed(seed + 1)
        self.obs = torch.randn(num_envs, num_obs, generator=self.gen)

    def _env_step(self):
        n = self.N
        obs = torch.randn(n, self.O, generator=self.gen)
        rew = torch.randn(n, generator=self.gen)
        dones = (torch.rand(n, generator=self.gen) < 0.02).to(torch.uint8)
        return obs, rew, dones

    def rollout(self):
        T, N, A, O = self.T, self.N, self.A, self.O
        buf = {k: np.empty((T, N) + s, np.float32) for k, s in
               (("obs", (O,)), ("actions", (A,)), ("mu", (A,)), ("sigma", (A,)), ("values", ()), ("rewards", ()),
                ("logp", ()))}
        buf["dones"] = np.empty((T, N), np.uint8)
        with torch.inference_mode():
            for t in range(T):
                mean = self.actor(self.obs)
                std = self.std.expand_as(mean)
                d = torch.distributions.Normal(mean, std)
                a = d.sample()
                buf["obs"][t] = self.obs.numpy()
                buf["actions"][t] = a.numpy()
                buf["mu"][t] = mean.numpy()
                buf["sigma"][t] = std.numpy()
                buf["values"][t] = self.critic(self.obs).numpy()[:, 0]
                buf["logp"][t] = d.log_prob(a).sum(-1).numpy()
                self.obs, rew, dones = self._env_step()
                buf["rewards"][t] = rew.numpy()
                buf["dones"][t] = dones.numpy()
            last_v = self.critic(self.obs).numpy()[:, 0]
        return buf, last_v

    def update(self, buf, last_v):
        hp = self.hp
        t0 = time.perf_counter()
        ret, adv = O.compute_returns(buf["values"], buf["rewards"], buf["dones"], last_v, hp["gamma"], hp["lam"])
        fields = {"obs": buf["obs"], "actions": buf["actions"], "values": buf["values"][..., None],
                  "advantages": adv[..., None], "returns": ret[..., None], "logp": buf["logp"][..., None],
                  "mu": buf["mu"], "sigma": buf["sigma"]}
        perm, mb, new_state = O.minibatch_indices(self.N, self.T, self.M, torch.default_generator.get_state().numpy())
        torch.default_generator.set_state(torch.from_numpy(new_state))
        sums = np.zeros(3)
        # hot path (GAE, shuffle + gathers, fused loss) timed apart from the MLPs / optimizer
        hot = time.perf_counter() - t0
        batches = O.minibatches(fields, perm, mb, self.M, self.E)
        while True:
            t0 = time.perf_counter()
            b = next(batches, None)
            hot += time.perf_counter() - t0
            if b is None:
                break
            obs = torch.from_numpy(b["obs"])
            mean = self.actor(obs)
            value = self.critic(obs)
            t0 = time.perf_counter()
            out = O.ppo_loss(mean.detach().numpy(), np.broadcast_to(self.std.detach().numpy(), mean.shape),
                             value.detach().numpy(), b["actions"], b["logp"], b["advantages"], b["values"],
                             b["returns"], b["mu"], b["sigma"], clip_param=hp["clip"],
                             value_loss_coef=hp["value_coef"], entropy_coef=hp["entropy_coef"])
            hot += time.perf_counter() - t0
            kl = out["kl_mean"]
            if kl > hp["desired_kl"] * 2.0:
                self.lr = max(1e-5, self.lr / 1.5)
            elif 0.0 < kl < hp["desired_kl"] / 2.0:
                self.lr = min(1e-2, self.lr * 1.5)
            for g in self.opt.param_groups:
                g["lr"] = self.lr
            self.opt.zero_grad()
            torch.autograd.backward([mean, value, self.std],
                                    [torch.from_numpy(out["dmu"]), torch.from_numpy(out["dV"]).view(-1, 1),
                                     torch.from_numpy(out["dsigma"].sum(0))])
            nn.utils.clip_grad_norm_(self.params, hp["max_grad_norm"])
            self.opt.step()
            sums += (out["value_function"], out["surrogate"], out["entropy"])
        n = self.E * self.M
        self.hot_path_seconds = hot
        return {"value_function": sums[0] / n, "surrogate": sums[1] / n, "entropy": sums[2] / n}

    def iteration(self):
        buf, last_v = self.rollout()
        return self.update(buf, last_v)


def time_iterations(num_envs, num_obs=48, num_actions=12, T=24, iters=1, warmup=1, threads=None, detail=False):
    """env-steps/s of `iters` full CPU iterations after `warmup` ones (detail: also the hot-path-only rate,
    GAE + shuffle/gathers + loss, and the update-phase rate)."""
    if threads:
        torch.set_num_threads(threads)
    ppo = CpuPPO(num_envs, num_obs, num_actions, T=T)
    for _ in range(warmup):
        ppo.iteration()
    hot = upd = 0.0
    t0 = time.perf_counter()
    for _ in range(iters):
        buf, last_v = ppo.rollout()
        t1 = time.perf_counter()
        ppo.update(buf, last_v)
        upd += time.perf_counter() - t1
        hot += ppo.hot_path_seconds
    dt = time.perf_counter() - t0
    steps = num_envs * T * iters
    if detail:
        return steps / dt, dt, {"hot_path": steps / hot, "update": steps / upd, "hot_path_seconds": hot,
                                "update_seconds": upd}
    return steps / dt, dt
