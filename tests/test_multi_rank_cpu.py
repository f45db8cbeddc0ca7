"""World-size-2 gloo tests (CPU) of PPO's distributed host logic (ppo.py:271-294, :428-469):
parameter broadcast, the gradient-arena all-reduce that update() issues once per mini-batch (gradients and
the KL in one buffer), the reference's cat/copy-back fallback (with the KL appended), and the KL
all-reduce + adaptive learning-rate rule with the reference's fp32 lr rounding.  The full multi-rank
update() against the reference's own W=2 / W=4 runs is tests/test_multi_rank_update.py."""

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
    os.environ["RSLRL_OVERLAP_ALLREDUCE"] = "1"  # the opt-in early-prefix layout (off by default since round 6)
    try:
        res = {}
        ppo = _make_ppo(rank)
        ppo.broadcast_parameters()
        res["params"] = {k: v.clone() for k, v in ppo.policy.state_dict().items()}

        # gradient-arena path of update(): every .grad a view of one buffer whose tail holds the KL, averaged
        # by the one all-reduce update() issues per mini-batch
        arena = ppo.grad_arena()
        arena.bind()
        for i, p in enumerate(ppo.policy.parameters()):
            p.grad.copy_(torch.full_like(p, float(rank + 1) * (i + 1)))
        arena.extra[:1].fill_(0.003 if rank == 0 else 0.001)
        ppo._all_reduce_arena(arena, with_kl=True)
        res["arena_grads"] = [p.grad.clone() for p in ppo.policy.parameters()]
        res["arena_kl"] = arena.extra[0].item()
        res["arena_is_grad"] = all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(ppo.policy.parameters(),
                                                                                     arena.views))
        # reduce_parameters() on arena-backed gradients: the same single collective
        ppo.reduce_parameters()
        res["arena_grads2"] = [p.grad.clone() for p in ppo.policy.parameters()]

        # the overlapped form of update(): the early prefix (every Linear but the first of actor and critic) handed
        # to an asynchronous all-reduce during the backward, the rest (+ the KL) reduced after it
        for i, p in enumerate(ppo.policy.parameters()):
            p.grad.copy_(torch.full_like(p, float(rank + 1) * (i + 3)))
        arena.extra[:1].fill_(0.005 if rank == 0 else 0.001)
        work = dist.all_reduce(arena.flat[:arena.early_numel], op=dist.ReduceOp.SUM, async_op=True)
        ppo._all_reduce_arena(arena, with_kl=True, skip=arena.early_numel, pending=[work])
        res["split_grads"] = [p.grad.clone() for p in ppo.policy.parameters()]
        res["split_kl"] = arena.extra[0].item()
        early = {id(p) for p in ppo._early_params()}
        res["early_numel"] = arena.early_numel
        res["early_in_prefix"] = all(
            (arena.slot(p).data_ptr() - arena.flat.data_ptr()) // 4 + p.numel() <= arena.early_numel
            for p in ppo.policy.parameters() if id(p) in early)
        res["late_after_prefix"] = all(
            (arena.slot(p).data_ptr() - arena.flat.data_ptr()) // 4 >= arena.early_numel
            for p in ppo.policy.parameters() if id(p) not in early)
        res["early_count"] = len(early)

        # reference cat path (grads not backed by the arena), with the KL appended to the concatenation
        for i, p in enumerate(ppo.policy.parameters()):
            p.grad = torch.full_like(p, float(rank + 1) * (i + 2))
        kl_t = torch.tensor([0.004 if rank == 0 else 0.002])
        ppo.reduce_parameters(kl_mean=kl_t)
        res["cat_grads"] = [p.grad.clone() for p in ppo.policy.parameters()]
        res["cat_kl"] = kl_t.item()

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


def test_arena_allreduce(results):
    for r in results:
        assert r["arena_is_grad"]
        for i, g in enumerate(r["arena_grads"]):
            assert torch.all(g == (1 + 2) * (i + 1) / WORLD)
        for i, g in enumerate(r["arena_grads2"]):
            assert torch.all(g == (1 + 2) * (i + 1) / WORLD)  # identical inputs on both ranks: unchanged
        assert r["arena_kl"] == torch.tensor((0.003 + 0.001) / WORLD, dtype=torch.float32).item()
    for a, b in zip(results[0]["arena_grads"], results[1]["arena_grads"]):
        assert torch.equal(a, b)


def test_overlapped_arena_allreduce(results):
    """The early-prefix all-reduce (overlapping the first layers' backward in update()) + the rest: the same averaged
    gradients and KL as one all-reduce of the whole arena, identical on every rank; the prefix holds exactly the
    early parameters (4 per network here: the second Linear's weight and bias of actor and critic)."""
    for r in results:
        assert r["early_count"] == 4 and r["early_numel"] > 0
        assert r["early_in_prefix"] and r["late_after_prefix"]
        for i, g in enumerate(r["split_grads"]):
            assert torch.all(g == (1 + 2) * (i + 3) / WORLD)
        assert r["split_kl"] == torch.tensor((0.005 + 0.001) / WORLD, dtype=torch.float32).item()
    for a, b in zip(results[0]["split_grads"], results[1]["split_grads"]):
        assert torch.equal(a, b)


def test_reference_cat_path(results):
    for r in results:
        for i, g in enumerate(r["cat_grads"]):
            assert torch.all(g == (1 + 2) * (i + 2) / WORLD)
        kl = torch.tensor(0.004, dtype=torch.float32) + torch.tensor(0.002, dtype=torch.float32)
        assert r["cat_kl"] == (kl / WORLD).item()


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


def test_single_collective_is_the_default(monkeypatch):
    """Round 6: without RSLRL_OVERLAP_ALLREDUCE=1 the arena has no early prefix, so update() issues ONE
    all-reduce of the gradients + KL per mini-batch after the backward."""
    monkeypatch.delenv("RSLRL_OVERLAP_ALLREDUCE", raising=False)
    ppo = _make_ppo(0)
    assert ppo._early_params() == ()
    assert ppo.grad_arena().early_numel == 0
    monkeypatch.setenv("RSLRL_OVERLAP_ALLREDUCE", "1")
    assert len(ppo._early_params()) == 4
