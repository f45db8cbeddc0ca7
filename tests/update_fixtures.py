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
    """(PPO, policy) ready for update(): initial weights, storage and generator state of the fixture; compute_returns
    has run.  meta["shared_params"]: the initial parameters are stored under rank 0's prefix only.  meta["rnd_cfg"]:
    the PPO gets that rnd_cfg and the rank's RND state (predictor, target, state normaliser) from `rnd_init/`.
    meta["policy_kw"]: extra ActorCritic arguments (std parameterisation)."""
    from rsl_rl_amd.algorithms import PPO
    from rsl_rl_amd.modules import ActorCritic

    T, N, O, A = meta["T"], meta["N"], meta["O"], meta["A"]
    nz = storage_noise(rank_meta["noise_seed"], T, N, O, A)
    assert hashlib.sha256(nz["obs"].tobytes()).digest() == z[prefix + "obs_sha256"].tobytes(), "numpy stream differs"
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    rnd_cfg = meta.get("rnd_cfg")
    if rnd_cfg:
        groups["rnd_state"] = ["policy"]
        rnd_cfg = dict(rnd_cfg, num_states=O, obs_groups=groups)
    pol = ActorCritic(obs0, groups, A, actor_hidden_dims=meta["hidden"], critic_hidden_dims=meta["hidden"],
                      **meta.get("policy_kw", {}))
    pp = "r0/" if meta.get("shared_params") else prefix
    pol.load_state_dict({k[len(pp) + 5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pp + "init/")})
    mcfg = {"global_rank": rank, "local_rank": 0, "world_size": world} if world > 1 else None
    alg = PPO(pol, num_learning_epochs=meta["E"], num_mini_batches=meta["M"], device=device, multi_gpu_cfg=mcfg,
              learning_rate=meta.get("learning_rate", 1e-3), rnd_cfg=rnd_cfg)
    if rnd_cfg:
        pre = prefix + "rnd_init/"
        alg.rnd.load_state_dict({k[len(pre):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pre)})
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


def run_recorded_update(alg, grads=None, rnd_grads=None):
    """update() with the learning rate of every optimizer step recorded (ppo.py:374 sees param_groups' lr); when
    `grads` is a list of k entries, it is replaced by the pre-clip policy gradients (concatenated in parameters()
    order, after any all-reduce) of the first k mini-batches -- pass [None] * k; `rnd_grads` likewise for the RND
    predictor's gradients as its optimizer step sees them."""
    lr_trace = []
    want = 0 if grads is None else len(grads)
    want_rnd = 0 if rnd_grads is None else len(rnd_grads)
    got, got_rnd = [], []
    stepper = alg._clip_adam if alg._clip_adam is not None else alg.optimizer
    step = stepper.step

    def rec(*a, **k):
        if len(got) < want:  # pre-clip: the step writes the clipped gradients back
            got.append(torch.cat([p.grad.reshape(-1) for p in alg.policy.parameters()]).cpu())
        r = step(*a, **k)
        # the reference records its Python-float self.learning_rate; ours lives on the device in update(), set by
        # the per-mini-batch tail -- which runs inside the step's first launch when fused (FusedClipAdam tail=)
        lr = getattr(alg, "learning_rate_device", None)
        lr_trace.append(float(lr if lr is not None else alg.optimizer.param_groups[0]["lr"]))
        return r

    stepper.step = rec
    # the RND predictor's step: a fused clip-free Adam when the update runs it on the device, else the torch optimizer
    rnd_stepper = (getattr(alg, "_rnd_adam", None) or alg.rnd_optimizer) if want_rnd else None
    if rnd_stepper is not None:
        rnd_step = rnd_stepper.step

        def rec_rnd(*a, **k):
            if len(got_rnd) < want_rnd:
                got_rnd.append(torch.cat([p.grad.reshape(-1) for p in alg.rnd.predictor.parameters()]).cpu())
            return rnd_step(*a, **k)

        rnd_stepper.step = rec_rnd
    try:
        loss = alg.update()
    finally:
        stepper.step = step
        if rnd_stepper is not None:
            rnd_stepper.step = rnd_step
    if grads is not None:
        grads[:] = got
    if rnd_grads is not None:
        rnd_grads[:] = got_rnd
    return loss, lr_trace


def param_errors(final, z, prefix, group="final/", init_group="init/"):
    """Per parameter: (max |ours - ref|, ||ours - ref|| / ||ref - init||) -- the second relative to how far the
    update moved the parameter.  group / init_group: "rnd_final/" / "rnd_init/predictor." for the RND predictor."""
    out = {}
    for k in z.files:
        if k.startswith(prefix + group):
            name = k[len(prefix) + len(group):]
            ref = torch.from_numpy(z[k]).double()
            init = torch.from_numpy(z[prefix + init_group + name]).double()
            ours = final[name].detach().cpu().double()
            d = (ours - ref)
            moved = (ref - init).norm().item()
            out[name] = (d.abs().max().item(), d.norm().item() / moved if moved > 0 else d.norm().item())
    return out


def check_update(out, z, meta, rank, mode=""):
    """Assert one rank's update result against the reference fixture (see tests/test_multi_rank_update.py):
    learning-rate trace exact, loss means rtol 1e-4 (incl. "rnd"), first-mini-batch gradients within 1e-5 of each
    tensor's max, and parameters within the tolerance of the network width: atol 2e-5 for the C1-width networks (as
    test_update_c1), the reference's own one-ulp sensitivity bound for 3x256 (as test_update_c2_width); the RND
    predictor (smooth MSE loss, no clip discontinuity) within 1e-3 of how far it moved.  Returns the errors."""
    ref = meta["ranks"][rank]
    pre = f"r{rank}/"
    pp = "r0/" if meta.get("shared_params") else pre
    assert out["lr_trace"] == ref["lr_trace"], (mode, rank, out["lr_trace"], ref["lr_trace"])
    assert out["lr"] == ref["final_lr"], (mode, rank, out["lr"], ref["final_lr"])
    assert set(out["loss"]) == set(ref["loss_dict"]), (out["loss"].keys(), ref["loss_dict"].keys())
    for k, v in ref["loss_dict"].items():
        assert abs(out["loss"][k] - v) <= 1e-4 * abs(v) + 1e-6, (mode, rank, k, out["loss"][k], v)
    for key, ours in (("grad_mb0", out.get("grad_mb0")), ("rnd_grad_mb0", out.get("rnd_grad_mb0"))):
        if pp + key in z.files:
            r = torch.from_numpy(z[pp + key]).double()
            err = (ours.double() - r).abs().max().item() / r.abs().max().item()
            assert err <= 1e-5, (mode, rank, key, err)
    errs = param_errors(out["final"], z, pp)
    print(mode, rank, "param errors (max abs / ||d|| over ||moved||):",
          {k: f"{a:.1e}/{m:.1e}" for k, (a, m) in errs.items()})
    wide = max(meta["hidden"]) >= 256
    sens = meta.get("ulp_sensitivity", {})
    for name, (abs_err, rel_moved) in errs.items():
        if wide:
            assert rel_moved <= 2 * sens[name] + 1e-4, (mode, rank, name, rel_moved, sens[name])
        else:
            assert abs_err <= 2e-5, (mode, rank, name, abs_err)
    rnd_errs = {}
    if meta.get("rnd_cfg"):
        rnd_errs = param_errors(out["rnd_final"], z, pp, "rnd_final/", "rnd_init/predictor.")
        print(mode, rank, "rnd predictor errors:", {k: f"{a:.1e}/{m:.1e}" for k, (a, m) in rnd_errs.items()})
        assert rnd_errs
        for name, (abs_err, rel_moved) in rnd_errs.items():
            assert rel_moved <= 1e-3, (mode, rank, "rnd", name, rel_moved)
    return errs, rnd_errs
