"""Full PPO.update() on the GPU vs the reference's update captured on CPU, and an end-to-end OnPolicyRunner
smoke on the synthetic VecEnv.

C1 (N512 T16 O16 A4, 2x64 ELU, E5 M4): the fixture ran the reference with multi_gpu_cfg world_size=1 (so its
learning rate went through the fp32 broadcast, ppo.py:287-290); the test does the same over a one-rank RCCL
("nccl") group, which also exercises the one-collective-per-mini-batch path (gradient arena + KL).  Same
permutation (torch CPU randperm from the captured generator state), same storage, same initial weights; the
MLP GEMMs run on our fused MFMA kernels (x6 split-bf16 by default) instead of CPU BLAS, so parameters are
compared with a tolerance (atol 2e-5 after 20 Adam steps at lr <= 2.25e-3) while the learning-rate trace
(the adaptive-KL decisions) must match exactly.  C2's shape (3x256, O48, A12) is the second update test.
"""

import os
import tempfile

import numpy as np
import pytest
import torch

from conftest import golden_path
from rsl_rl_amd.algorithms import PPO
from rsl_rl_amd.env import SyntheticVecEnv
from rsl_rl_amd.modules import ActorCritic
from rsl_rl_amd.runners import OnPolicyRunner

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def one_rank_group(cuda_device):
    import torch.distributed as dist

    if not dist.is_initialized():
        fd, path = tempfile.mkstemp()
        os.close(fd)
        dist.init_process_group("nccl", init_method=f"file://{path}", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def test_update_c1_matches_reference(golden_meta, cuda_device, one_rank_group):
    m = golden_meta["update_c1"]
    z = np.load(golden_path("update_c1.npz"))
    T, N, O, A = m["T"], m["N"], m["O"], m["A"]
    dev = cuda_device
    obs0 = {"policy": torch.zeros(N, O)}
    groups = {"policy": ["policy"], "critic": ["policy"]}
    pol = ActorCritic(obs0, groups, A, actor_hidden_dims=m["hidden"], critic_hidden_dims=m["hidden"])
    pol.load_state_dict({k[5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("init/")})
    alg = PPO(pol, num_learning_epochs=m["E"], num_mini_batches=m["M"], device=dev,
              multi_gpu_cfg={"global_rank": 0, "local_rank": 0, "world_size": 1})
    alg.init_storage("rl", N, T, obs0, [A])
    st = alg.storage
    st.observations["policy"].copy_(torch.from_numpy(z["storage/obs_policy"]))
    for k in ("rewards", "values", "actions_log_prob", "mu", "sigma", "actions"):
        getattr(st, k).copy_(torch.from_numpy(z[f"storage/{k}"]))
    st.dones.copy_(torch.from_numpy(z["storage/dones"]))
    st.step = T
    with torch.inference_mode():
        alg.compute_returns({"policy": torch.from_numpy(z["storage/last_obs"]).to(dev)})
    torch.testing.assert_close(st.returns.cpu(), torch.from_numpy(z["storage/returns"]), rtol=2e-6, atol=2e-6)
    torch.testing.assert_close(st.advantages.cpu(), torch.from_numpy(z["storage/advantages"]), rtol=1e-5, atol=1e-5)

    lr_trace = []
    stepper = alg._clip_adam if alg._clip_adam is not None else alg.optimizer  # fused clip + Adam on a GPU
    assert alg._clip_adam is not None
    step = stepper.step
    # the lr the step uses, read after it: the per-mini-batch tail that sets it runs inside the step when fused
    stepper.step = lambda *a, **k: (step(*a, **k), lr_trace.append(float(alg.optimizer.param_groups[0]["lr"])))[0]
    torch.default_generator.set_state(torch.from_numpy(z["gen_state"].copy()))
    loss = alg.update()
    assert lr_trace == m["lr_trace"]
    assert alg.learning_rate == m["final_lr"]
    for k, v in m["loss_dict"].items():
        assert abs(loss[k] - v) <= 1e-4 * abs(v) + 1e-5, (k, loss[k], v)
    final = pol.state_dict()
    for k in z.files:
        if k.startswith("final/"):
            ref = torch.from_numpy(z[k])
            torch.testing.assert_close(final[k[6:]].cpu(), ref, rtol=0, atol=2e-5, msg=k)


def test_runner_end_to_end(cuda_device, tmp_path):
    torch.manual_seed(0)
    env = SyntheticVecEnv(512, 16, 4, device=cuda_device, seed=0, timeout_prob=0.25)
    cfg = {
        "num_steps_per_env": 16, "save_interval": 50, "obs_groups": {"policy": ["policy"]},
        "policy": {"class_name": "ActorCritic", "actor_hidden_dims": [64, 64], "critic_hidden_dims": [64, 64],
                   "activation": "elu", "init_noise_std": 1.0},
        "algorithm": {"class_name": "PPO", "num_learning_epochs": 5, "num_mini_batches": 4},
    }
    runner = OnPolicyRunner(env, cfg, log_dir=None, device=str(cuda_device))
    runner.learn(3)
    s = runner.last_iteration_stats
    assert s["total_fps"] > 0 and all(np.isfinite(v) for v in s["loss_dict"].values())
    path = str(tmp_path / "model.pt")
    runner.save(path)
    sd = {k: v.clone() for k, v in runner.alg.policy.state_dict().items()}
    runner2 = OnPolicyRunner(SyntheticVecEnv(512, 16, 4, device=cuda_device), {
        **cfg, "policy": dict(cfg["policy"], class_name="ActorCritic"),
        "algorithm": dict(cfg["algorithm"], class_name="PPO")}, log_dir=None, device=str(cuda_device))
    runner2.load(path)
    for k, v in runner2.alg.policy.state_dict().items():
        assert torch.equal(v, sd[k]), k
    assert runner2.current_learning_iteration == runner.current_learning_iteration


@pytest.mark.parametrize("reward_norm", [False, True])
def test_runner_with_normalizers_and_rnd(cuda_device, reward_norm):
    """Observation normalisers on, RND (fused into the rollout record, or -- with reward normalisation --
    evaluated in PyTorch and added by the record kernel), state-dependent std: the whole loop runs and
    the normalisers' running statistics are updated on the device."""
    torch.manual_seed(1)
    env = SyntheticVecEnv(1024, 48, 12, device=cuda_device, seed=3, timeout_prob=0.1)
    cfg = {
        "num_steps_per_env": 8, "save_interval": 10**9,
        "obs_groups": {"policy": ["policy"], "critic": ["policy"], "rnd_state": ["policy"]},
        "policy": {"class_name": "ActorCritic", "actor_hidden_dims": [256, 256], "critic_hidden_dims": [256, 256],
                   "activation": "elu", "init_noise_std": 1.0, "actor_obs_normalization": True,
                   "critic_obs_normalization": True},
        "algorithm": {"class_name": "PPO", "num_learning_epochs": 2, "num_mini_batches": 2,
                      "rnd_cfg": {"weight": 1.0, "num_outputs": 1, "predictor_hidden_dims": [-1],
                                  "target_hidden_dims": [-1], "learning_rate": 1e-3, "state_normalization": True,
                                  "reward_normalization": reward_norm}},
    }
    runner = OnPolicyRunner(env, cfg, log_dir=None, device=str(cuda_device))
    runner.learn(2)
    s = runner.last_iteration_stats
    assert all(np.isfinite(v) for v in s["loss_dict"].values())
    n = runner.alg.policy.actor_obs_normalizer
    assert n.count.item() == 2 * 8 * 1024
    assert torch.isfinite(n._mean).all() and (n._std > 0).all()
    assert runner.alg.rnd.state_normalizer.count.item() == 2 * 8 * 1024
    assert torch.isfinite(runner.alg.intrinsic_rewards).all()


def test_update_c2_width_matches_reference(golden_meta, cuda_device):
    """One full update() at config C2's shape (N4096 T24 O48 A12, actor/critic 3x256 ELU, E5 M4; mini-batch 24,576
    rows) against the reference's update on CPU (make_golden.make_update_c2), once through the default x6
    split-bf16 GEMMs (the actor's head with the loss fused: rslrl_actor_head_fwd_bwd) and once through the exact-fp32
    MFMA GEMMs (separate loss kernel).

    * first mini-batch (no drift yet): every parameter's gradient within 1e-5 of its max |g|;
    * learning-rate trace (increase, then two decreases) exact; loss means rtol 1e-4;
    * parameters after the 20 Adam steps, per tensor: ||ours - ref|| <= 2 s + 1e-4 times ||ref - init||, where s is
      the REFERENCE's own sensitivity (golden.json update_c2.ulp_sensitivity): how far its parameters move, in the
      same units, when every stored log-prob is raised by one ulp (0.7-2.3 % for the actor, 0 for the critic).
      The surrogate's clip/max is discontinuous: a sample whose ratio sits within rounding of 1 +- clip_param
      takes the other branch when its log-prob differs in the last bit (our exp/log vs torch CPU's), which moves
      the gradient by ~1/sqrt(B) and Adam carries it on.  The GEMM arithmetic is not the residual: the x6 and
      f32 runs end >100x closer to each other than to the reference (||x6 - f32|| <= 1e-3 ||ref - init||)."""
    from update_fixtures import build_update, param_errors, run_recorded_update
    from rsl_rl_amd.networks import fused_mlp

    m = golden_meta["update_c2"]
    z = np.load(golden_path("update_c2.npz"))
    finals = {}
    for mode in ("x6", "f32"):
        prev = fused_mlp.set_gemm_mode({"x6": fused_mlp.GEMM_X6, "f32": fused_mlp.GEMM_F32}[mode])
        try:
            alg, pol = build_update(z, "", m, m, cuda_device)
            head = torch.from_numpy(z["storage/returns_head"])
            torch.testing.assert_close(alg.storage.returns[:2].cpu(), head, rtol=1e-5, atol=1e-5)
            grads = [None]
            launches = fused_mlp.actor_head_launches
            loss, lr_trace = run_recorded_update(alg, grads)
            # x6: every mini-batch's actor head ran the loss and its backward fused (rslrl_actor_head_fwd_bwd)
            assert fused_mlp.actor_head_launches - launches == (20 if mode == "x6" else 0), mode
        finally:
            fused_mlp.set_gemm_mode(prev)
        ref_g = torch.from_numpy(z["grad_mb0"]).double()
        ours_g = grads[0].double()
        off = 0
        for name, p in pol.named_parameters():
            r, o = ref_g[off:off + p.numel()], ours_g[off:off + p.numel()]
            off += p.numel()
            err = (o - r).abs().max().item() / r.abs().max().item()
            assert err <= 1e-5, (mode, name, err)
        assert lr_trace == m["lr_trace"], mode
        assert alg.learning_rate == m["final_lr"]
        for k, v in m["loss_dict"].items():
            assert abs(loss[k] - v) <= 1e-4 * abs(v) + 1e-6, (mode, k, loss[k], v)
        errs = param_errors(pol.state_dict(), z, "")
        print(mode, {k: (f"{a:.2e}", f"{r:.2e}") for k, (a, r) in errs.items()})
        sens = m["ulp_sensitivity"]
        for name, (abs_err, rel_moved) in errs.items():
            assert rel_moved <= 2 * sens[name] + 1e-4, (mode, name, rel_moved, sens[name])
        finals[mode] = {k: v.detach().cpu().double() for k, v in pol.state_dict().items()}
    for k in finals["x6"]:
        ref = torch.from_numpy(z["final/" + k]).double()
        moved = (ref - torch.from_numpy(z["init/" + k]).double()).norm().item()
        d = (finals["x6"][k] - finals["f32"][k]).norm().item()
        print(k, f"||x6 - f32|| / moved = {d / moved:.2e}")
        assert d <= 1e-3 * moved, (k, d / moved)


def test_update_two_streams_bit_identical(golden_meta, cuda_device, monkeypatch):
    """The opt-in side stream for the critic's MLP launches (RSLRL_TWO_STREAMS=1, update and rollout forward)
    changes only where the launches run, not what they compute: the C2-shape update ends with bit-identical
    parameters, learning-rate trace and loss statistics either way.  (The one-stream update otherwise pairs the
    actor's and the critic's layers per launch, whose weight-gradient slices round differently: compared unpaired,
    the pairing has its own test, test_gpu_pair_train.py.)"""
    from update_fixtures import build_update, run_recorded_update
    from rsl_rl_amd.networks import fused_mlp

    monkeypatch.setattr(fused_mlp, "_PAIR_TRAIN", False)
    m = golden_meta["update_c2"]
    z = np.load(golden_path("update_c2.npz"))
    res = {}
    for two in ("0", "1"):
        monkeypatch.setenv("RSLRL_TWO_STREAMS", two)
        alg, pol = build_update(z, "", m, m, cuda_device)
        loss, lr_trace = run_recorded_update(alg)
        torch.cuda.synchronize()
        res[two] = (loss, lr_trace, {k: v.detach().cpu().clone() for k, v in pol.state_dict().items()})
    assert res["0"][0] == res["1"][0] and res["0"][1] == res["1"][1]
    for k, v in res["0"][2].items():
        assert torch.equal(v, res["1"][2][k]), k


def test_runner_resumes_non_fused_adam_checkpoint(cuda_device, tmp_path):
    """A checkpoint whose optimizer state was written by a plain (non-fused) torch Adam -- as a reference run
    saves it: param group fused=None, step tensors on the CPU -- loads through OnPolicyRunner.load and the next
    learn() iteration runs the fused clip+Adam step on it (steps moved to the device, the trajectory continued)."""
    torch.manual_seed(0)
    cfg = {
        "num_steps_per_env": 16, "save_interval": 10**9, "obs_groups": {"policy": ["policy"]},
        "policy": {"class_name": "ActorCritic", "actor_hidden_dims": [64, 64], "critic_hidden_dims": [64, 64],
                   "activation": "elu", "init_noise_std": 1.0},
        "algorithm": {"class_name": "PPO", "num_learning_epochs": 2, "num_mini_batches": 2},
    }
    runner = OnPolicyRunner(SyntheticVecEnv(512, 16, 4, device=cuda_device, seed=0), cfg, log_dir=None,
                            device=str(cuda_device))
    params = [p.detach().clone().requires_grad_(True) for p in runner.alg.policy.parameters()]
    plain = torch.optim.Adam(params, lr=1e-3, foreach=False)
    for p in params:
        p.grad = torch.randn_like(p) * 0.1
    plain.step()
    plain.step()
    sd = plain.state_dict()
    assert sd["param_groups"][0]["fused"] is None
    with torch.no_grad():
        pol_sd = {k: v.clone() for k, v in runner.alg.policy.state_dict().items()}
    torch.save({"model_state_dict": pol_sd, "optimizer_state_dict": sd, "iter": 7, "infos": None},
               str(tmp_path / "ref.pt"))
    runner.load(str(tmp_path / "ref.pt"))
    assert runner.alg._clip_adam is not None
    runner.learn(1)
    s = runner.last_iteration_stats
    assert all(np.isfinite(v) for v in s["loss_dict"].values())
    opt = runner.alg.optimizer
    assert opt.param_groups[0]["fused"] is True
    for p in runner.alg.policy.parameters():
        st = opt.state[p]
        assert st["step"].device == p.device and float(st["step"]) == 2 + 2 * 2  # + E * M fused steps
        assert torch.isfinite(p).all()
