"""Split-K weight-gradient Linear (rsl_rl_amd/networks/linear.py) == torch Linear autograd (fp32 tol)."""

import pytest
import torch

from rsl_rl_amd.networks import MLP
from rsl_rl_amd.networks.linear import SplitKLinearFunction

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,fin,fout", [(393216, 256, 256), (100003, 48, 256), (7000, 256, 12), (5000, 256, 1),
                                        (100, 16, 4)])
def test_grads_match_torch(B, fin, fout, cuda_device):
    torch.manual_seed(0)
    x = torch.randn(B, fin, device=cuda_device, requires_grad=True)
    w = torch.randn(fout, fin, device=cuda_device, requires_grad=True)
    b = torch.randn(fout, device=cuda_device, requires_grad=True)
    g = torch.randn(B, fout, device=cuda_device)
    SplitKLinearFunction.apply(x, w, b).backward(g)
    ours = [t.grad.clone() for t in (x, w, b)]
    for t in (x, w, b):
        t.grad = None
    torch.nn.functional.linear(x, w, b).backward(g)
    for a, r in zip(ours, (x.grad, w.grad, b.grad)):
        assert (a - r).abs().max().item() <= 1e-5 * r.abs().max().item()


def test_mlp_forward_backward_matches_sequential(cuda_device):
    torch.manual_seed(1)
    mlp = MLP(48, 12, [256, 256, 256], "elu").to(cuda_device)
    x = torch.randn(20000, 48, device=cuda_device)
    y = mlp(x)
    y.square().sum().backward()
    ours = [p.grad.clone() for p in mlp.parameters()]
    mlp.zero_grad()
    ref = x
    for layer in mlp:
        ref = layer(ref)
    assert torch.allclose(y, ref, rtol=1e-6, atol=1e-6)
    ref.square().sum().backward()
    for a, p in zip(ours, mlp.parameters()):
        assert (a - p.grad).abs().max().item() <= 1e-5 * p.grad.abs().max().item()
