"""World-size-2 gloo tests (CPU) of PPO's distributed host logic (ppo.py:271-294, :428-469):
parameter broadcast, the flat-buffer gradient all-reduce (and the reference's cat/copy-back fallback),
and the KL all-reduce + adaptive learning-rate rule with the reference's fp32 lr rounding."""

import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rsl_rl_amd.algorithms import PPO
from rsl_rl_amd.algorithms.ppo import adapt_learning_rate
from rsl_rl_amd.modules import ActorCritic

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_ppo(rank, **kw):
    torch.manual_seed(100 + rank)  # deliberately different initial weights per rank
    obs = {"policy": torch.zeros(4, 6)}
    pol = ActorCritic(obs, {"policy": ["policy"], "critic": ["policy"]}, 3, actor_hidden_dims=[8],
                      critic_hidden_dims=[8])
    return PPO(pol, device="cpu", multi_gpu_cfg={"global_rank": rank, "local_rank": rank, "world_size": WORLD}, **kw)


def _worker(rank, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        res = {}
        ppo = _make_ppo(rank)
        ppo.broadcast_parameters()
        res["params"] = {k: v.clone() for k, v in ppo.policy.state_dict().items()}

        # flat-buffer path: rank-specific gradients, averaged by one all-reduce of the flat buffer
        ppo._bind_flat_grads()
        for i, p in enumerate(ppo.policy.parameters()):
            p.grad.copy_(torch.full_like(p, float(rank + 1) * (i + 1)))
        ppo.reduce_parameters()
        res["flat_grads"] = [p.grad.clone() for p in ppo.policy.parameters()]

        # reference fallback path (grads not backed by the flat buffer)
        for i, p in enumerate(ppo.policy.parameters()):
            p.grad = torch.full_like(p, float(rank + 1) * (i + 2))
        ppo.reduce_parameters()
        res["cat_grads"] = [p.grad.clone() for p in ppo.policy.parameters()]

        # KL all-reduce + lr rule (kl: rank0 0.003, rank1 0.001 -> mean 0.002 < desired/2 -> lr * 1.5)
        kl = ppo._sync_kl_and_lr(torch.tensor([0.003 if rank == 0 else 0.001]))
        res["kl"] = kl
        res["lr"] = ppo.learning_rate
        res["group_lr"] = ppo.optimizer.param_groups[0]["lr"]
        torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def results():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(_free_port(), d), nprocs=WORLD, join=True)
        yield [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]


def test_broadcast_parameters(results):
    ref = _make_ppo(0).policy.state_dict()
    for r in results:
        for k, v in r["params"].items():
            assert torch.equal(v, ref[k]), k


def test_flat_gradient_allreduce(results):
    for r in results:
        for i, g in enumerate(r["flat_grads"]):
            assert torch.all(g == (1 + 2) * (i + 1) / WORLD)
    for a, b in zip(results[0]["flat_grads"], results[1]["flat_grads"]):
        assert torch.equal(a, b)


def test_reference_cat_path(results):
    for r in results:
        for i, g in enumerate(r["cat_grads"]):
            assert torch.all(g == (1 + 2) * (i + 2) / WORLD)


def test_kl_and_learning_rate(results):
    expected_lr = torch.tensor(adapt_learning_rate(1e-3, 0.002, 0.01), dtype=torch.float32).item()
    for r in results:
        assert abs(r["kl"] - 0.002) < 1e-9
        assert r["lr"] == expected_lr == r["group_lr"]
    assert expected_lr != 1.5e-3  # the fp32 rounding of the broadcast lr (ppo.py:288-290) is reproduced


def test_adapt_learning_rate_rule():
    assert adapt_learning_rate(1e-3, 0.05, 0.01) == 1e-3 / 1.5
    assert adapt_learning_rate(1e-5, 0.05, 0.01) == 1e-5
    assert adapt_learning_rate(1e-3, 0.001, 0.01) == 1e-3 * 1.5
    assert adapt_learning_rate(1e-2, 0.001, 0.01) == 1e-2
    assert adapt_learning_rate(1e-3, 0.0, 0.01) == 1e-3  # kl == 0: unchanged (ppo.py:283)
    assert adapt_learning_rate(1e-3, 0.01, 0.01) == 1e-3


def _reference_rule(lr, kl_t, desired):
    # ppo.py:280-284 as written: a 0-d fp32 tensor compared with Python floats, lr a Python float
    if kl_t > desired * 2.0:
        return max(1e-5, lr / 1.5)
    elif kl_t < desired / 2.0 and kl_t > 0.0:
        return min(1e-2, lr * 1.5)
    return lr


def test_adapt_learning_rate_device_matches_host_rule():
    """The device-resident rule of PPO.update (fp64 lr tensor, fp32 KL) follows ppo.py:280-284 exactly,
    including the fp32 comparisons at the 2*kl* / kl*/2 thresholds and the clamps."""
    from rsl_rl_amd.algorithms.ppo import adapt_learning_rate_device
    desired = 0.01
    kls = [0.0, 1e-9, 0.004999, 0.005, 0.0050001, 0.01, 0.019999, 0.02, 0.0200001, 0.5, -1e-3]
    lrs = [1e-5, 1.2e-5, 3e-4, 1e-3, 6.7e-3, 1e-2]
    for lr in lrs:
        for kl in kls:
            kl_t = torch.tensor(kl, dtype=torch.float32)
            got = adapt_learning_rate_device(torch.tensor(lr, dtype=torch.float64), kl_t.reshape(1), desired)
            assert got.dtype == torch.float64
            assert got.item() == _reference_rule(lr, kl_t, desired), (lr, kl, got.item())
