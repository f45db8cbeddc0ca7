"""HIP GAE (rslrl_compute_returns) vs the golden vectors and the oracle.

Bit-exact: returns and un-normalised advantages.  Normalised advantages: |diff| <= 1e-5 * (1 + |x|)
(fp64 statistics, summation order differs from torch's fp32 mean/std).
"""

import numpy as np
import pytest
import torch

from conftest import golden_path
from oracle import ppo_oracle as O
from rsl_rl_amd import kernels

pytestmark = pytest.mark.gpu


def _run(values, rewards, dones, last_values, gamma, lam, normalize, dev):
    T, N = values.shape
    v = torch.from_numpy(values).reshape(T, N, 1).to(dev)
    r = torch.from_numpy(rewards).reshape(T, N, 1).to(dev)
    d = torch.from_numpy(dones).reshape(T, N, 1).to(dev)
    lv = torch.from_numpy(last_values).reshape(N, 1).to(dev)
    ret = torch.empty(T, N, 1, device=dev)
    adv = torch.empty(T, N, 1, device=dev)
    kernels.compute_returns(v, r, d, lv, gamma, lam, normalize, ret, adv)
    torch.cuda.synchronize()
    return ret.cpu().numpy().reshape(T, N), adv.cpu().numpy().reshape(T, N)


def test_golden(golden_meta, cuda_device):
    z = np.load(golden_path("gae.npz"))
    for name, m in sorted(golden_meta["gae"].items()):
        g = lambda k: z[f"{name}/{k}"]  # noqa: E731
        args = (g("values"), g("rewards"), g("dones"), g("last_values"), m["gamma"], m["lam"])
        ret, adv = _run(*args, False, cuda_device)
        assert np.array_equal(ret, g("returns")), name
        assert np.array_equal(adv, g("advantages_raw")), name
        ret2, advn = _run(*args, True, cuda_device)
        assert np.array_equal(ret2, g("returns")), name
        ref = g("advantages_norm")
        if m["T"] * m["N"] == 1:
            assert np.isnan(advn).all()
        else:
            np.testing.assert_allclose(advn, ref, rtol=1e-5, atol=1e-5, err_msg=name)


@pytest.mark.parametrize("T,N,p", [(24, 65536, 0.02), (24, 4096, 0.02), (1, 1000, 0.5), (40, 3001, 0.1),
                                   (33, 257, 0.05), (16, 512, 0.0), (8, 100003, 1.0), (32, 70000, 0.3)])
def test_random_vs_oracle(T, N, p, cuda_device):
    rng = np.random.default_rng(T * 1000 + N)
    values = rng.standard_normal((T, N), dtype=np.float32)
    rewards = rng.standard_normal((T, N), dtype=np.float32)
    dones = (rng.random((T, N)) < p).astype(np.uint8)
    last = rng.standard_normal(N, dtype=np.float32)
    ret, adv = _run(values, rewards, dones, last, 0.99, 0.95, False, cuda_device)
    oret, oadv = O.gae(values, rewards, dones, last, 0.99, 0.95)
    assert np.array_equal(ret, oret)
    assert np.array_equal(adv, oadv)
    _, advn = _run(values, rewards, dones, last, 0.99, 0.95, True, cuda_device)
    np.testing.assert_allclose(advn, O.adv_normalize(oadv), rtol=1e-5, atol=1e-5)


def test_full_size_properties(cuda_device):
    """C3 size (T=24, N=65536): normalised advantages have mean ~0 / std ~1, and the scan is
    idempotent and deterministic run to run (fixed reduction order)."""
    T, N = 24, 65536
    g = torch.Generator(device=cuda_device).manual_seed(5)
    v = torch.randn(T, N, 1, generator=g, device=cuda_device)
    r = torch.randn(T, N, 1, generator=g, device=cuda_device)
    d = (torch.rand(T, N, 1, generator=g, device=cuda_device) < 0.02).to(torch.uint8)
    lv = torch.randn(N, 1, generator=g, device=cuda_device)
    outs = []
    for _ in range(2):
        ret = torch.empty_like(v)
        adv = torch.empty_like(v)
        kernels.compute_returns(v, r, d, lv, 0.99, 0.95, True, ret, adv)
        outs.append((ret, adv))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    a = outs[0][1].double()
    assert abs(a.mean().item()) < 1e-6
    assert abs(a.std().item() - 1.0) < 1e-5
    # returns - values is the raw advantage: re-normalising it reproduces the normalised advantages
    raw = outs[0][0] - v
    ref = (raw - raw.double().mean().float()) / (raw.double().std().float() + 1e-8)
    assert torch.allclose(outs[0][1], ref, atol=1e-5)
