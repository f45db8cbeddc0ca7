"""The reference's PPO iteration restated in torch-CPU ops -- BASELINE INFRASTRUCTURE ONLY.

bench.py times this as `cpu_baseline` ("port"): what rsl_rl itself does per iteration on a CPU, in the
reference's operation order, with torch's CPU kernels on every core it is given.  Never imported by
rsl_rl_amd/.  The parity checker is oracle/ppo_oracle.py + oracle.c; this file is about speed.

Per iteration (config C2/C3 shape: T steps x N envs, obs O, A actions, actor/critic 3x256 ELU, E5 M4):
  rollout        on_policy_runner.py:103-129 + ppo.py:129-169 + rollout_storage.py:77-103 (act: actor MLP,
                 Normal sample, log-prob; critic; synthetic env step; time-out bootstrap; storage copies)
  returns        ppo.py:171-176 + rollout_storage.py:127-149 (critic on the last obs, the Python loop over T,
                 advantage normalisation over all T*N)
  generator      rollout_storage.py:160-203 (randperm once, 8 gathers per mini-batch)
  update         ppo.py:246-384 (actor/critic forward, Normal log-prob / entropy, KL + adaptive lr,
                 clipped surrogate, clipped value loss, backward, clip_grad_norm_, Adam, .item() statistics)
"""

from __future__ import annotations

import time

import torch
import torch.nn as nn


def _mlp(i, o, hidden):
    dims = [i] + list(hidden)
    layers = []
    for a, b in zip(dims[:-1], dims[1:]):
        layers += [nn.Linear(a, b), nn.ELU()]
    layers.append(nn.Linear(dims[-1], o))
    return nn.Sequential(*layers)


class TorchCpuPPO:
    def __init__(self, N, O, A, T=24, hidden=(256, 256, 256), E=5, M=4, seed=0, lr=1e-3, clip=0.2, gamma=0.99,
                 lam=0.95, value_coef=1.0, entropy_coef=0.01, max_grad_norm=1.0, desired_kl=0.01):
        torch.manual_seed(seed)
        self.N, self.O, self.A, self.T, self.E, self.M = N, O, A, T, E, M
        self.actor, self.critic = _mlp(O, A, hidden), _mlp(O, 1, hidden)
        self.std = nn.Parameter(torch.ones(A))
        self.params = [self.std] + list(self.actor.parameters()) + list(self.critic.parameters())
        self.opt = torch.optim.Adam(self.params, lr=lr)
        self.lr = lr
        self.clip, self.gamma, self.lam = clip, gamma, lam
        self.value_coef, self.entropy_coef = value_coef, entropy_coef
        self.max_grad_norm, self.desired_kl = max_grad_norm, desired_kl
        self.gen = torch.Generator().manual_seed(seed + 1)
        self.obs = torch.randn(N, O, generator=self.gen)
        z = lambda *s, dt=torch.float32: torch.zeros(*s, dtype=dt)  # noqa: E731
        self.st = {"obs": z(T, N, O), "actions": z(T, N, A), "rewards": z(T, N, 1), "dones": z(T, N, 1, dt=torch.uint8),
                   "values": z(T, N, 1), "logp": z(T, N, 1), "mu": z(T, N, A), "sigma": z(T, N, A),
                   "returns": z(T, N, 1), "advantages": z(T, N, 1)}
        self.timing = {}

    # ---------------------------------------------------------------- rollout
    def _env_step(self):
        g, N = self.gen, self.N
        obs = torch.randn(N, self.O, generator=g)
        rew = torch.randn(N, generator=g)
        dones = (torch.rand(N, generator=g) < 0.02).long()
        return obs, rew, dones, {"time_outs": torch.zeros(N)}

    def rollout(self):
        st = self.st
        with torch.inference_mode():
            for t in range(self.T):
                mean = self.actor(self.obs)
                dist = torch.distributions.Normal(mean, self.std.expand_as(mean))
                actions = dist.sample()
                values = self.critic(self.obs)
                logp = dist.log_prob(actions).sum(dim=-1)
                obs_t = self.obs
                self.obs, rew, dones, extras = self._env_step()
                rewards = rew.clone()
                rewards += self.gamma * torch.squeeze(values * extras["time_outs"].unsqueeze(1), 1)
                st["obs"][t].copy_(obs_t)
                st["actions"][t].copy_(actions)
                st["rewards"][t].copy_(rewards.view(-1, 1))
                st["dones"][t].copy_(dones.view(-1, 1))
                st["values"][t].copy_(values)
                st["logp"][t].copy_(logp.view(-1, 1))
                st["mu"][t].copy_(mean)
                st["sigma"][t].copy_(dist.stddev)

    # ---------------------------------------------------------------- GAE
    def compute_returns(self):
        st = self.st
        with torch.inference_mode():
            last_values = self.critic(self.obs)
            advantage = 0
            for step in reversed(range(self.T)):
                next_values = last_values if step == self.T - 1 else st["values"][step + 1]
                next_is_not_terminal = 1.0 - st["dones"][step].float()
                delta = st["rewards"][step] + next_is_not_terminal * self.gamma * next_values - st["values"][step]
                advantage = delta + next_is_not_terminal * self.gamma * self.lam * advantage
                st["returns"][step] = advantage + st["values"][step]
            st["advantages"] = st["returns"] - st["values"]
            st["advantages"] = (st["advantages"] - st["advantages"].mean()) / (st["advantages"].std() + 1e-8)

    # ---------------------------------------------------------------- update
    def _batches(self):
        st = self.st
        n = self.N * self.T
        mb = n // self.M
        indices = torch.randperm(self.M * mb, requires_grad=False)
        flat = {k: v.flatten(0, 1) for k, v in st.items() if k != "rewards" and k != "dones"}
        for _ in range(self.E):
            for i in range(self.M):
                idx = indices[i * mb:(i + 1) * mb]
                yield {k: v[idx] for k, v in flat.items()}

    def update(self, max_mini_batches=None):
        """One update; with max_mini_batches only that many of the E*M mini-batches run (a bounded sample; the
        wall time of each, generator gather included, is in self.timing["mini_batch_seconds"])."""
        sums = [0.0, 0.0, 0.0]
        hot = 0.0
        gen = self._batches()
        mb_times = []
        while True:
            if max_mini_batches is not None and len(mb_times) >= max_mini_batches:
                break
            t_mb = time.perf_counter()
            t0 = time.perf_counter()
            b = next(gen, None)
            hot += time.perf_counter() - t0
            if b is None:
                break
            mean = self.actor(b["obs"])
            dist = torch.distributions.Normal(mean, self.std.expand_as(mean))
            t0 = time.perf_counter()
            logp = dist.log_prob(b["actions"]).sum(dim=-1)
            hot += time.perf_counter() - t0
            value = self.critic(b["obs"])
            t0 = time.perf_counter()
            mu, sigma = dist.mean, dist.stddev
            entropy = dist.entropy().sum(dim=-1)
            with torch.inference_mode():
                kl = torch.sum(torch.log(sigma / b["sigma"] + 1.0e-5)
                               + (torch.square(b["sigma"]) + torch.square(b["mu"] - mu)) / (2.0 * torch.square(sigma))
                               - 0.5, axis=-1)
                kl_mean = torch.mean(kl)
                if kl_mean > self.desired_kl * 2.0:
                    self.lr = max(1e-5, self.lr / 1.5)
                elif kl_mean < self.desired_kl / 2.0 and kl_mean > 0.0:
                    self.lr = min(1e-2, self.lr * 1.5)
                for g in self.opt.param_groups:
                    g["lr"] = self.lr
            ratio = torch.exp(logp - torch.squeeze(b["logp"]))
            adv = torch.squeeze(b["advantages"])
            surrogate_loss = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 1.0 - self.clip, 1.0 + self.clip)).mean()
            value_clipped = b["values"] + (value - b["values"]).clamp(-self.clip, self.clip)
            value_loss = torch.max((value - b["returns"]).pow(2), (value_clipped - b["returns"]).pow(2)).mean()
            loss = surrogate_loss + self.value_coef * value_loss - self.entropy_coef * entropy.mean()
            hot += time.perf_counter() - t0
            self.opt.zero_grad()
            loss.backward()
            nn.utils.clip_grad_norm_(self.params, self.max_grad_norm)
            self.opt.step()
            sums[0] += value_loss.item()
            sums[1] += surrogate_loss.item()
            sums[2] += entropy.mean().item()
            mb_times.append(time.perf_counter() - t_mb)
        n = self.E * self.M
        self.timing["hot_loss_and_batches"] = hot
        self.timing["mini_batch_seconds"] = mb_times
        return {"value_function": sums[0] / n, "surrogate": sums[1] / n, "entropy": sums[2] / n}

    def iteration(self):
        t0 = time.perf_counter()
        self.rollout()
        t1 = time.perf_counter()
        self.compute_returns()
        t2 = time.perf_counter()
        self.update()
        t3 = time.perf_counter()
        self.timing.update(rollout=t1 - t0, returns=t2 - t1, update=t3 - t2, total=t3 - t0)
        return self.timing


def time_iterations(N, O=48, A=12, T=24, iters=1, warmup=1, threads=None):
    """(env-steps/s end to end, seconds timed, phase rates) of `iters` iterations after `warmup`."""
    if threads:
        torch.set_num_threads(threads)
    ppo = TorchCpuPPO(N, O, A, T=T)
    for _ in range(warmup):
        ppo.iteration()
    agg = {"rollout": 0.0, "returns": 0.0, "update": 0.0, "total": 0.0, "hot_loss_and_batches": 0.0}
    for _ in range(iters):
        tm = ppo.iteration()
        for k in agg:
            agg[k] += tm[k]
    steps = N * T * iters
    hot = agg["returns"] + agg["hot_loss_and_batches"]
    # the full-size sample's extrapolation (time_full_size_sample: first + (E*M - 1) x mean of the next k - 1
    # mini-batches) applied to this whole iteration's own mini-batch times, against its measured update
    mbs = tm["mini_batch_seconds"]
    check = {}
    for k in (3, 5):
        if len(mbs) > k:
            est = mbs[0] + (len(mbs) - 1) * sum(mbs[1:k]) / (k - 1)
            check[f"first_{k}"] = {"update_extrapolated": round(est, 3), "update_measured": round(sum(mbs), 3),
                                   "rel_error": round(est / sum(mbs) - 1.0, 4)}
    return steps / agg["total"], agg["total"], {
        "update_env_steps_per_s": steps / (agg["returns"] + agg["update"]),
        "hot_path_env_steps_per_s": steps / hot,
        "seconds": {k: round(v, 3) for k, v in agg.items()},
        "extrapolation_check": check,
    }


def time_full_size_sample(N, O=48, A=12, T=24, mini_batches=3, threads=None):
    """A bounded sample of one iteration at the full size N (no shrinking of the workload): the whole rollout and
    compute_returns are timed, then the first `mini_batches` of the E*M mini-batches of the update (each with its
    generator gathers; the first one also draws the permutation); the update time is extrapolated as
    first + (E*M - 1) * mean(the others).  Returns (env-steps/s end to end, seconds of CPU work timed, details)."""
    if threads:
        torch.set_num_threads(threads)
    ppo = TorchCpuPPO(N, O, A, T=T)
    with torch.inference_mode():  # first-touch / thread-pool warm-up on one small forward, outside the timing
        ppo.actor(torch.randn(1024, O))
    t0 = time.perf_counter()
    ppo.rollout()
    t1 = time.perf_counter()
    ppo.compute_returns()
    t2 = time.perf_counter()
    ppo.update(max_mini_batches=mini_batches)
    t3 = time.perf_counter()
    mbs = ppo.timing["mini_batch_seconds"]
    n_mb = ppo.E * ppo.M
    rest = sum(mbs[1:]) / max(1, len(mbs) - 1) if len(mbs) > 1 else mbs[0]
    update_est = mbs[0] + (n_mb - 1) * rest
    steps = N * T
    total_est = (t1 - t0) + (t2 - t1) + update_est
    return steps / total_est, t3 - t0, {
        "update_env_steps_per_s": steps / ((t2 - t1) + update_est),
        "seconds": {"rollout": round(t1 - t0, 3), "returns": round(t2 - t1, 3),
                    "mini_batches_timed": [round(x, 3) for x in mbs], "update_extrapolated": round(update_est, 3),
                    "iteration_extrapolated": round(total_est, 3)},
    }
