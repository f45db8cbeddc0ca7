"""Product host code: rslrl_randperm_mt19937 (rollout_storage.py:165 semantics) is bit-exact with the
reference's torch CPU randperm, including the generator state it leaves behind."""

import numpy as np
import pytest
import torch

from conftest import golden_path
from rsl_rl_amd import kernels


def test_golden_permutations(golden_meta):
    z = np.load(golden_path("perm.npz"))
    for name, m in golden_meta["perm"].items():
        if f"{name}/state" not in z:
            continue
        g = torch.Generator()
        g.set_state(torch.from_numpy(z[f"{name}/state"].copy()))
        perm = kernels.randperm_mt19937(m["n"], g)
        assert perm.dtype == torch.int32
        assert np.array_equal(perm.numpy().astype(np.int64), z[f"{name}/perm"]), name
        assert np.array_equal(g.get_state().numpy(), z[f"{name}/state_after"]), name


@pytest.mark.parametrize("n,seed,pre", [(0, 0, 0), (1, 1, 5), (2, 2, 0), (623, 3, 1), (624, 4, 0), (625, 5, 623),
                                        (1249, 6, 624), (20000, 7, 10), (393216, 8, 0)])
def test_matches_torch_randperm(n, seed, pre):
    g1 = torch.Generator().manual_seed(seed)
    g2 = torch.Generator().manual_seed(seed)
    if pre:
        torch.randint(0, 10, (pre,), generator=g1)
        torch.randint(0, 10, (pre,), generator=g2)
    ref = torch.randperm(n, generator=g1)
    ours = kernels.randperm_mt19937(n, g2)
    assert torch.equal(ref.to(torch.int32), ours)
    # the generators stay in lock-step afterwards
    assert torch.equal(torch.rand(7, generator=g1), torch.rand(7, generator=g2))


def test_consecutive_draws_and_default_generator():
    torch.manual_seed(123)
    a1 = torch.randperm(5000)
    a2 = torch.randperm(777)
    torch.manual_seed(123)
    b1 = kernels.randperm_mt19937(5000)
    b2 = kernels.randperm_mt19937(777)
    assert torch.equal(a1.to(torch.int32), b1) and torch.equal(a2.to(torch.int32), b2)
