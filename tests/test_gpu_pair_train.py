"""The update's actor + critic passes with their same-shape layers batched per launch (fused_mlp.train_forward_pair /
train_backward_pair) against the two separate passes (RSLRL_PAIR_TRAIN=0 path): forward outputs, output-layer
gradients and every input gradient bit-identical; hidden weight gradients (half the row slices, twice the rows per
slice) within fp32 accumulation error (1e-5 of the tensor's max, the north_star tolerance)."""

import pytest
import torch

from rsl_rl_amd.modules import ActorCritic
from rsl_rl_amd.networks import fused_mlp

pytestmark = pytest.mark.gpu


def _arena(params, dev):
    """Adjacent fp32 slots in parameter order (a Linear's weight then its bias), as the gradient arena lays them."""
    n = sum(p.numel() for p in params)
    flat = torch.zeros(n, device=dev)
    slots, off = {}, 0
    for p in params:
        slots[p] = flat[off:off + p.numel()].view_as(p)
        off += p.numel()
    return flat, slots


@pytest.mark.parametrize("B", [8192, 98304, 3000])
def test_pair_matches_separate_passes(B, cuda_device):
    torch.manual_seed(B)
    obs = {"policy": torch.randn(B, 48, device=cuda_device)}
    pol = ActorCritic(obs, {"policy": ["policy"], "critic": ["policy"]}, 12, actor_hidden_dims=[256, 256, 256],
                      critic_hidden_dims=[256, 256, 256], activation="elu").to(cuda_device)
    params = list(pol.parameters())
    g_mean = torch.randn(B, 12, device=cuda_device) * 1e-3
    g_value = torch.randn(B, 1, device=cuda_device) * 1e-3
    g_sigma = torch.randn(12, device=cuda_device)
    res = {}
    for paired in (False, True):
        fused_mlp._PAIR_TRAIN = paired
        try:
            with torch.no_grad():
                mean, sigma, value, tape = pol.train_forward(obs)
                assert tape[3] == paired
                flat, slots = _arena(params, cuda_device)
                pol.train_backward(tape, g_mean.clone(), g_sigma.clone(), g_value.clone(), sigma, slots.__getitem__)
            torch.cuda.synchronize()
            res[paired] = (mean.clone(), value.clone(), {id(p): slots[p].clone() for p in params})
        finally:
            fused_mlp._PAIR_TRAIN = True
    m0, v0, g0 = res[False]
    m1, v1, g1 = res[True]
    assert torch.equal(m0, m1) and torch.equal(v0, v1)
    lin = lambda mlp: [m for m in mlp if isinstance(m, torch.nn.Linear)]  # noqa: E731
    for mlp in (pol.actor, pol.critic):
        layers = lin(mlp)
        for l, m in enumerate(layers):
            for p in (m.weight, m.bias):
                a, b = g0[id(p)], g1[id(p)]
                if l == len(layers) - 1:  # the fused output-layer backward: one launch either way
                    assert torch.equal(a, b), l
                else:
                    err = ((a - b).abs().max() / (a.abs().max() + 1e-30)).item()
                    assert err < 1e-5, (l, err)
