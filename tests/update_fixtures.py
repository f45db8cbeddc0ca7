"""Rebuild the storage of the full-update fixtures (tests/golden/make_golden.py: make_multirank, make_update_c2)
on any device: the policy-independent inputs (obs, rewards, dones, action noise, last obs) are regenerated from
the fixture's numpy seed (PCG64, bit-reproducible), the policy-dependent ones (mean, std, values, log-prob) come
from the fixture, and actions = mean + std * noise with the reference's fp32 mul-then-add."""

import hashlib

import numpy as np
import torch


def storage_noise(seed, T, N, O, A):
    # same draw order as make_golden.storage_noise
    rng = np.random.default_rng(seed)
    return {
        "obs": rng.standard_normal((T, N, O), dtype=np.float32),
        "rewards": rng.standard_normal((T, N, 1), dtype=np.float32),
        "dones": (rng.random((T, N, 1)) < 0.05).astype(np.uint8),
        "noise": rng.standard_normal((T, N, A), dtype=np.float32),
        "last_obs": rng.standard_normal((N, O), dtype=np.float32),
    }


def build_update(z, prefix, meta, rank_meta, device, world=1, rank=0):
    """(PPO, policy, last_obs) ready for update(): initial weights, storage and generator state of the fixture;
    compute_returns has run."""
    from rsl_rl_amd.algorithms import PPO
    from rsl_rl_amd.modules import ActorCritic

    T, N, O, A = meta["T"], meta["N"], meta["O"], meta["A"]
    nz = storage_noise(rank_meta["noise_seed"], T, N, O, A)
    assert hashlib.sha256(nz["obs"].tobytes()).digest() == z[prefix + "obs_sha256"].tobytes(), "numpy stream differs"
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    pol = ActorCritic(obs0, groups, A, actor_hidden_dims=meta["hidden"], critic_hidden_dims=meta["hidden"])
    pol.load_state_dict({k[len(prefix) + 5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith(prefix + "init/")})
    mcfg = {"global_rank": rank, "local_rank": 0, "world_size": world} if world > 1 else None
    alg = PPO(pol, num_learning_epochs=meta["E"], num_mini_batches=meta["M"], device=device, multi_gpu_cfg=mcfg,
              learning_rate=meta.get("learning_rate", 1e-3))
    alg.init_storage("rl", N, T, {"policy": torch.zeros(N, O)}, [A])
    st = alg.storage
    mu = torch.from_numpy(z[prefix + "storage/mu"].astype(np.float32))
    sigma = torch.from_numpy(z[prefix + "storage/sigma"]).reshape(1, 1, A).expand(T, N, A)
    actions = mu + sigma * torch.from_numpy(nz["noise"])  # the fixture's fp32 mul then add (CPU, IEEE)
    st.observations["policy"].copy_(torch.from_numpy(nz["obs"]))
    st.rewards.copy_(torch.from_numpy(nz["rewards"]))
    st.dones.copy_(torch.from_numpy(nz["dones"]))
    st.mu.copy_(mu)
    st.sigma.copy_(sigma)
    st.actions.copy_(actions)
    st.values.copy_(torch.from_numpy(z[prefix + "storage/values"]))
    st.actions_log_prob.copy_(torch.from_numpy(z[prefix + "storage/actions_log_prob"]))
    st.step = T
    with torch.inference_mode():
        alg.compute_returns({"policy": torch.from_numpy(nz["last_obs"]).to(device)})
    torch.default_generator.set_state(torch.from_numpy(z[prefix + "gen_state"].copy()))
    return alg, pol


def run_recorded_update(alg, grads=None):
    """update() with the learning rate of every optimizer step recorded (ppo.py:374 sees param_groups' lr); when
    `grads` is a list, the pre-clip policy gradients of the first len(grads)... mini-batches are appended to it
    (concatenated in parameters() order) until it holds grad_batches entries -- pass [None] * k to get k."""
    lr_trace = []
    want = 0 if grads is None else len(grads)
    got = []
    stepper = alg._clip_adam if alg._clip_adam is not None else alg.optimizer
    step = stepper.step

    def rec(*a, **k):
        # the reference records its Python-float self.learning_rate; ours lives on the device in update()
        lr = getattr(alg, "learning_rate_device", None)
        lr_trace.append(float(lr if lr is not None else alg.optimizer.param_groups[0]["lr"]))
        if len(got) < want:
            got.append(torch.cat([p.grad.reshape(-1) for p in alg.policy.parameters()]).cpu())
        return step(*a, **k)

    stepper.step = rec
    try:
        loss = alg.update()
    finally:
        stepper.step = step
    if grads is not None:
        grads[:] = got
    return loss, lr_trace


def param_errors(final, z, prefix):
    """Per parameter: (max |ours - ref|, ||ours - ref|| / ||ref - init||) -- the second relative to how far the
    update moved the parameter."""
    out = {}
    for k in z.files:
        if k.startswith(prefix + "final/"):
            name = k[len(prefix) + 6:]
            ref = torch.from_numpy(z[k]).double()
            init = torch.from_numpy(z[prefix + "init/" + name]).double()
            ours = final[name].detach().cpu().double()
            d = (ours - ref)
            moved = (ref - init).norm().item()
            out[name] = (d.abs().max().item(), d.norm().item() / moved if moved > 0 else d.norm().item())
    return out
