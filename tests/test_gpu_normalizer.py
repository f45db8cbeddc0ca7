"""Running normalisers on the HIP kernels (csrc/normalizer.hip, §8f row 3) vs the reference's captured
sequence (tests/golden/normalizer.npz) and vs the oracle at C3 size.  Moments: fp64 on the device vs
torch's fp32 reductions in the reference -> rtol 1e-5; the forward and the reward scaling are bit-exact
given the same statistics; `until` and the count are exact."""

import numpy as np
import pytest
import torch

from conftest import golden_path
from rsl_rl_amd.networks import EmpiricalDiscountedVariationNormalization, EmpiricalNormalization

pytestmark = pytest.mark.gpu


def test_normalizer_matches_reference(golden_meta, cuda_device):
    m = golden_meta["normalizer"]
    z = np.load(golden_path("normalizer.npz"))
    norm = EmpiricalNormalization(shape=[7], until=m["until"]).to(cuda_device)
    norm.train()
    for k in range(m["obs_updates"]):
        x = torch.from_numpy(z[f"obs/x{k}"]).to(cuda_device)
        norm.update(x)
        assert norm.count.item() == int(z[f"obs/count{k}"])
        torch.testing.assert_close(norm._mean.cpu(), torch.from_numpy(z[f"obs/mean{k}"]), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(norm._var.cpu(), torch.from_numpy(z[f"obs/var{k}"]), rtol=1e-5, atol=0)
        torch.testing.assert_close(norm._std.cpu(), torch.from_numpy(z[f"obs/std{k}"]), rtol=1e-5, atol=0)
        # forward with the reference's statistics is bit-exact
        ref_norm = EmpiricalNormalization(shape=[7]).to(cuda_device)
        ref_norm._mean.copy_(torch.from_numpy(z[f"obs/mean{k}"]))
        ref_norm._std.copy_(torch.from_numpy(z[f"obs/std{k}"]))
        assert torch.equal(ref_norm(x).cpu(), torch.from_numpy(z[f"obs/y{k}"]))
    rn = EmpiricalDiscountedVariationNormalization(shape=[], gamma=m["gamma"]).to(cuda_device)
    rn.train()
    for k in range(m["reward_steps"]):
        r = torch.from_numpy(z[f"rew/r{k}"]).to(cuda_device)
        out = rn(r)
        assert torch.equal(rn.disc_avg.avg.cpu(), torch.from_numpy(z[f"rew/avg{k}"]))
        torch.testing.assert_close(rn.emp_norm._std.cpu(), torch.from_numpy(z[f"rew/std{k}"]), rtol=1e-5, atol=0)
        torch.testing.assert_close(out.cpu(), torch.from_numpy(z[f"rew/out{k}"]), rtol=2e-5, atol=0)
    rn.eval()
    r = torch.from_numpy(z["rew/r0"]).to(cuda_device)
    assert torch.equal(rn(r), r / rn.emp_norm._std)  # eval: no update


def test_normalizer_c3_size_vs_oracle(cuda_device):
    from oracle import ppo_oracle as po
    torch.manual_seed(3)
    norm = EmpiricalNormalization(shape=[48], until=None).to(cuda_device)
    mean, var, count = np.zeros(48, np.float32), np.ones(48, np.float32), 0
    base = torch.randn(48, device=cuda_device) * 3
    for _ in range(3):
        x = torch.randn(65536, 48, device=cuda_device) * 0.7 + base
        norm.update(x)
        mean, var, std, count = po.normalizer_update(x.cpu().numpy(), mean, var, count)
    np.testing.assert_allclose(norm._mean.cpu().numpy()[0], mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(norm._var.cpu().numpy()[0], var, rtol=1e-6)
    assert norm.count.item() == count
    # non-contiguous rows (a column slice of a wider observation) go through the row stride
    wide = torch.randn(5000, 64, device=cuda_device)
    n2 = EmpiricalNormalization(shape=[48]).to(cuda_device)
    n2.update(wide[:, 8:56])
    m2, v2, _, _ = po.normalizer_update(wide[:, 8:56].cpu().numpy(), np.zeros(48, np.float32),
                                        np.ones(48, np.float32), 0)
    np.testing.assert_allclose(n2._mean.cpu().numpy()[0], m2, rtol=1e-6, atol=1e-7)
    y = n2(wide[:, 8:56])
    np.testing.assert_array_equal(y.cpu().numpy(), po.normalizer_apply(wide[:, 8:56].cpu().numpy(),
                                                                       n2._mean.cpu().numpy()[0],
                                                                       n2._std.cpu().numpy()[0]))
