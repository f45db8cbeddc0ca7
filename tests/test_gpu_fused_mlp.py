"""Fused fp32 MFMA MLP (networks/fused_mlp.py, csrc/mlp_gemm.hip) vs the same nn.Sequential evaluated
layer by layer by torch (hipBLASLt + ATen ELU).  Tolerance 1e-5 relative to each tensor's max: the MFMA
k-order differs from hipBLASLt's at fp32 epsilon."""

import pytest
import torch

from rsl_rl_amd.networks import MLP
from rsl_rl_amd.networks.fused_mlp import fusable_structure, linear_dgrad_elu, linear_fwd

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _close(a, b, tol=TOL):
    assert (a - b).abs().max().item() <= tol * b.abs().max().item() + 1e-12, (a - b).abs().max().item()


def _reference(mlp, x):
    y = x
    for layer in mlp:
        y = layer(y)
    return y


@pytest.mark.parametrize("M,K,N,elu", [(393216, 256, 256, True), (65536, 48, 256, True), (1000, 16, 64, False),
                                       (777, 48, 48, True), (129, 256, 256, True), (1, 4, 8, True)])
def test_linear_fwd(M, K, N, elu, cuda_device):
    torch.manual_seed(M)
    x = torch.randn(M, K, device=cuda_device)
    w = torch.randn(N, K, device=cuda_device) / K ** 0.5
    b = torch.randn(N, device=cuda_device)
    ref = torch.nn.functional.linear(x, w, b)
    if elu:
        ref = torch.nn.functional.elu(ref)
    _close(linear_fwd(x, w, b, elu), ref)


@pytest.mark.parametrize("M,N,K", [(393216, 256, 256), (5000, 12, 256), (1000, 64, 64), (300, 48, 48)])
def test_linear_dgrad_elu(M, N, K, cuda_device):
    torch.manual_seed(N + K)
    dz = torch.randn(M, N, device=cuda_device)
    w = torch.randn(N, K, device=cuda_device) / N ** 0.5
    h = torch.nn.functional.elu(torch.randn(M, K, device=cuda_device))
    out, db = linear_dgrad_elu(dz, w, h)
    ref = dz.mm(w)
    ref = torch.where(h > 0, ref, ref * (h + 1))
    _close(out, ref)
    _close(db, ref.double().sum(0).float(), 1e-4)


@pytest.mark.parametrize("din,dout,hidden,M", [(48, 12, [256, 256, 256], 393216), (48, 1, [256, 256, 256], 65536),
                                               (16, 4, [64, 64], 2048), (48, [2, 12], [256, 256, 256], 5000),
                                               (48, 1, [-1], 3001)])
def test_mlp_forward_backward(din, dout, hidden, M, cuda_device):
    torch.manual_seed(7)
    mlp = MLP(din, dout, hidden, "elu").to(cuda_device)
    assert mlp._fused and fusable_structure(mlp)
    x = torch.randn(M, din, device=cuda_device)
    y = mlp(x)
    g = torch.randn_like(y)
    y.backward(g)
    ours = [p.grad.clone() for p in mlp.parameters()]
    mlp.zero_grad()
    ref = _reference(mlp, x)
    _close(y, ref)
    ref.backward(g)
    for (name, p), a in zip(mlp.named_parameters(), ours):
        _close(a, p.grad, 2e-5 if "bias" in name else TOL)
    with torch.inference_mode():
        _close(mlp(x), ref.detach())


def test_input_gradient(cuda_device):
    torch.manual_seed(3)
    mlp = MLP(48, 12, [256, 256], "elu").to(cuda_device)
    x = torch.randn(4096, 48, device=cuda_device, requires_grad=True)
    mlp(x).square().sum().backward()
    gx = x.grad.clone()
    x.grad = None
    _reference(mlp, x).square().sum().backward()
    _close(gx, x.grad)


def test_unfusable_structures_fall_back_to_layers():
    assert not fusable_structure(MLP(48, 12, [256], "relu"))
    assert not fusable_structure(MLP(50, 12, [256], "elu"))  # in_features % 4
    assert not fusable_structure(MLP(48, 12, [512], "elu"))  # width > 256

