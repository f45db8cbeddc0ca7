"""Multi-rank PPO.update() against the reference's own multi-rank update (config C4's data-parallel structure).

The fixtures (tests/golden/update_<case>.npz; make_golden.make_multirank / make_update_rnd) ran the reference's
PPO.update with world_size 2, 4 and 8 over a gloo group on CPU: every rank its own storage shard and permutation
generator, gradients averaged by reduce_parameters (ppo.py:441-469), the KL all-reduced and the learning rate
decided on rank 0 and broadcast as fp32 (ppo.py:271-294).  Here the same ranks run our update on the GPU (all on
cuda:0, a gloo group: RCCL refuses two ranks on one device), where each mini-batch issues ONE all-reduce carrying
the gradient arena and the KL.  Cases:
  * w2, w4, w8: C1's network (2x64, O16, A4) per rank;
  * w2_c4net: C4's per-rank network (3x256 ELU, O48, A12), 1024 envs x T24 per rank (6144-row mini-batches);
  * rnd_c5_w2: the same network with C5's RND (predictor/target 48->48->1): the predictor's gradients ride in the
    same all-reduce (ppo.py:447-450) and its Adam runs unclipped (ppo.py:383-384).
Per rank: learning-rate trace exact, loss means rtol 1e-4, the first mini-batch's averaged gradients within 1e-5,
parameters within the width's tolerance (tests/update_fixtures.check_update); and every rank ends with
bit-identical parameters (they must, as in the reference: the same averaged gradients and lr on every rank).

test_ranks_c4_share: 2 and 8 ranks x 16384 envs (C4's per-GPU share at N = 8; 8 ranks = C4's whole 131,072-env
workload) through a real rollout on the synthetic VecEnv and one update at 3x256: finite losses, identical
learning-rate traces, bit-identical parameters.  test_rccl_update_path_world1: the same path over RCCL.
"""

import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port, backend="gloo"):
    import sys

    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    return dist


def _worker(rank, world, port, case, meta, out_dir):
    dist = _setup(rank, world, port)
    try:
        from update_fixtures import build_update, run_recorded_update

        z = np.load(os.path.join(GOLDEN, f"update_{case}.npz"))
        alg, pol = build_update(z, f"r{rank}/", meta, meta["ranks"][rank], "cuda:0", world=world, rank=rank)
        grads, rnd_grads = [None], [None]
        loss, lr_trace = run_recorded_update(alg, grads, rnd_grads if alg.rnd else None)
        out = {"loss": loss, "lr_trace": lr_trace, "lr": alg.learning_rate,
               "final": {k: v.detach().cpu() for k, v in pol.state_dict().items()}, "grad_mb0": grads[0]}
        if alg.rnd:
            out["rnd_final"] = {k: v.detach().cpu() for k, v in alg.rnd.predictor.state_dict().items()}
            out["rnd_grad_mb0"] = rnd_grads[0]
        torch.save(out, os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _family(case, golden_meta):
    return golden_meta["update_rnd"][case] if case.startswith("rnd_") else golden_meta["multirank"][case]


@pytest.mark.parametrize("case", ["w2", "w4", "w8", "w2_c4net", "rnd_c5_w2"])
def test_multi_rank_update_matches_reference(case, golden_meta, cuda_device):
    from update_fixtures import check_update

    meta = _family(case, golden_meta)
    world = meta["world"]
    z = np.load(os.path.join(GOLDEN, f"update_{case}.npz"))
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), case, meta, d), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    for r, out in enumerate(res):
        errs, rnd_errs = check_update(out, z, meta, r)
        if r == 0:
            print(case, "policy", {k: f"{a:.1e}/{m:.1e}" for k, (a, m) in errs.items()})
            if rnd_errs:
                print(case, "rnd", {k: f"{a:.1e}/{m:.1e}" for k, (a, m) in rnd_errs.items()})
    for r in range(1, world):  # data parallel: identical parameters on every rank
        for k, v in res[0]["final"].items():
            assert torch.equal(v, res[r]["final"][k]), (r, k)
        for k, v in res[0].get("rnd_final", {}).items():
            assert torch.equal(v, res[r]["rnd_final"][k]), (r, "rnd", k)


def _share_worker(rank, world, port, n_envs, out_dir, backend="gloo"):
    dist = _setup(rank, world, port, backend)
    try:
        from rsl_rl_amd.algorithms import PPO
        from rsl_rl_amd.env import SyntheticVecEnv
        from rsl_rl_amd.modules import ActorCritic
        from update_fixtures import run_recorded_update

        dev = "cuda:0"
        T, O, A = 24, 48, 12
        env = SyntheticVecEnv(n_envs, O, A, device=dev, seed=rank, timeout_prob=0.005)
        obs = env.get_observations()
        groups = {"policy": ["policy"], "critic": ["policy"]}
        torch.manual_seed(1 + 17 * rank)  # different initial weights per rank: broadcast_parameters syncs them
        pol = ActorCritic(obs, groups, A, actor_hidden_dims=[256] * 3, critic_hidden_dims=[256] * 3)
        alg = PPO(pol, device=dev, multi_gpu_cfg={"global_rank": rank, "local_rank": 0, "world_size": world})
        alg.broadcast_parameters()
        init = {k: v.detach().cpu().clone() for k, v in pol.state_dict().items()}
        alg.init_storage("rl", n_envs, T, obs, [A])
        with torch.inference_mode():
            for _ in range(T):
                actions = alg.act(obs)
                obs, rew, dones, extras = env.step(actions)
                alg.process_env_step(obs, rew, dones, extras)
            alg.compute_returns(obs)
        torch.manual_seed(5000 + rank)
        loss, lr_trace = run_recorded_update(alg)
        torch.cuda.synchronize()
        torch.save({"loss": loss, "lr_trace": lr_trace, "init": init,
                    "final": {k: v.detach().cpu() for k, v in pol.state_dict().items()}},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _run_share(world, n, backend="gloo"):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_share_worker, args=(world, _free_port(), n, d, backend), nprocs=world, join=True,
                           start_method="spawn")
        return [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 8])
def test_ranks_c4_share(world, cuda_device):
    """C4's data-parallel path at its per-GPU size: `world` ranks x 16384 envs (the share of each of 8 GPUs; at
    world 8 this is C4's whole 131,072-env workload), T = 24, 3x256 actor/critic: one rollout through the fused
    record kernel, GAE, and an update whose 20 mini-batches of 98,304 rows each issue one all-reduce of the
    gradient arena + KL.  Size-independent properties: every loss finite, the same learning-rate trace on every
    rank (the KL is averaged before the lr rule), bit-identical parameters on every rank after the update, and the
    parameters moved."""
    n = 16384
    res = _run_share(world, n)
    for out in res:
        assert all(np.isfinite(v) for v in out["loss"].values()), out["loss"]
        assert len(out["lr_trace"]) == 20
    for r in range(1, world):
        assert res[0]["lr_trace"] == res[r]["lr_trace"], r
        for k, v in res[0]["final"].items():
            assert torch.isfinite(v).all(), k
            assert torch.equal(v, res[r]["final"][k]), (r, k)
            assert torch.equal(res[0]["init"][k], res[r]["init"][k]), (r, k)  # broadcast_parameters
    for k, v in res[0]["final"].items():
        assert not torch.equal(v, res[0]["init"][k]), k
    # the losses are per-rank means over each rank's own shard: they differ between ranks (different envs)
    assert all(res[0]["loss"] != res[r]["loss"] for r in range(1, world))


@pytest.mark.timeout(600)
def test_rccl_update_path_world1(cuda_device):
    """The multi-GPU update path on RCCL ("nccl", the backend the runner and bench.py use) on a real device: a
    world-1 group, so broadcast_parameters, the per-mini-batch arena + KL all-reduce and the fp32 lr rounding all
    run through RCCL (two ranks cannot share one device under RCCL).  A world-1 SUM and the division by 1 are
    exact, so the result must be bit-identical to the same run over gloo."""
    n = 16384
    rccl = _run_share(1, n, "nccl")[0]
    gloo = _run_share(1, n, "gloo")[0]
    assert rccl["lr_trace"] == gloo["lr_trace"]
    assert rccl["loss"] == gloo["loss"]
    for k, v in rccl["final"].items():
        assert torch.equal(v, gloo["final"][k]), k
        assert not torch.equal(v, rccl["init"][k]), k
