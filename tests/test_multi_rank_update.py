"""Multi-rank PPO.update() against the reference's own multi-rank update (config C4's data-parallel structure).

The fixtures (tests/golden/update_w2.npz, update_w4.npz; make_golden.make_multirank) ran the reference's
PPO.update with world_size 2 and 4 over a gloo group on CPU: every rank its own storage shard and
permutation generator, gradients averaged by reduce_parameters (ppo.py:441-469), the KL all-reduced and the
learning rate decided on rank 0 and broadcast as fp32 (ppo.py:271-294).  Here the same ranks run our update
on the GPU (all on cuda:0, a gloo group: RCCL refuses two ranks on one device), where each mini-batch issues
ONE all-reduce carrying the gradient arena and the KL.  Per rank: learning-rate trace exact, loss means
rtol 1e-4, parameters within the tolerance of the single-rank C1 test; and every rank ends with bit-identical
parameters (they must, as in the reference: the same averaged gradients and the same lr on every rank)."""

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


def _worker(rank, world, port, case, meta, out_dir):
    import sys

    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from update_fixtures import build_update, run_recorded_update

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = np.load(os.path.join(GOLDEN, f"update_{case}.npz"))
        alg, pol = build_update(z, f"r{rank}/", meta, meta["ranks"][rank], "cuda:0", world=world, rank=rank)
        loss, lr_trace = run_recorded_update(alg)
        torch.save({"loss": loss, "lr_trace": lr_trace, "lr": alg.learning_rate,
                    "final": {k: v.detach().cpu() for k, v in pol.state_dict().items()}},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["w2", "w4"])
def test_multi_rank_update_matches_reference(case, golden_meta, cuda_device):
    from update_fixtures import param_errors

    meta = golden_meta["multirank"][case]
    world = meta["world"]
    z = np.load(os.path.join(GOLDEN, f"update_{case}.npz"))
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), case, meta, d), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    for r, out in enumerate(res):
        ref = meta["ranks"][r]
        assert out["lr_trace"] == ref["lr_trace"], (r, out["lr_trace"], ref["lr_trace"])
        assert out["lr"] == ref["final_lr"]
        for k, v in ref["loss_dict"].items():
            assert abs(out["loss"][k] - v) <= 1e-4 * abs(v) + 1e-6, (r, k, out["loss"][k], v)
        for name, (abs_err, _) in param_errors(out["final"], z, f"r{r}/").items():
            assert abs_err <= 2e-5, (r, name, abs_err)
    for r in range(1, world):  # data parallel: identical parameters on every rank
        for k, v in res[0]["final"].items():
            assert torch.equal(v, res[r]["final"][k]), (r, k)
