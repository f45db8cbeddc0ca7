"""Fused RND predictor step (kernels.rnd_update -> rslrl_rnd_update) against torch autograd of the reference's
expressions (rsl_rl/algorithms/ppo.py:352-363 loss, :369-372 backward; rsl_rl/modules/rnd.py networks), fp32 on
the same device.  The kernel's dot products are fp32 FMA chains and its row sums fp32 per workgroup folded in
fp64, so the tolerance is GEMM-class: gradients within 2e-5 of each tensor's max magnitude (rtol 1e-5 of the
loss value), and the target-embedding cache (the later epochs of update()) gives the same bits as computing it."""

import pytest
import torch

from rsl_rl_amd import kernels
from rsl_rl_amd.networks import MLP

pytestmark = pytest.mark.gpu


def _reference(state, pred, targ, mean=None, std=None, eps=0.0):
    s = state if mean is None else (state - mean) / (std + eps)
    p = pred(s)
    t = targ(s).detach()
    loss = torch.nn.functional.mse_loss(p, t)
    grads = torch.autograd.grad(loss, list(pred.parameters()))
    return loss.detach(), torch.cat([g.reshape(-1) for g in grads]), t.detach()


@pytest.mark.parametrize("B,n_in,H,Q,norm", [
    (393216, 48, 48, 1, False),  # config C5's mini-batch
    (5000, 48, 48, 1, True),
    (257, 16, 32, 3, True),
    (1000, 64, 64, 8, False),
    (1, 7, 5, 2, False),
    (70001, 33, 40, 4, False),
])
def test_rnd_update_matches_autograd(B, n_in, H, Q, norm, cuda_device):
    torch.manual_seed(B + n_in)
    dev = cuda_device
    pred = MLP(n_in, Q, [H], "elu").to(dev)
    targ = MLP(n_in, Q, [H], "elu").to(dev)
    # a row-strided state view (a mini-batch slice of a wider gathered buffer)
    big = torch.randn(B, n_in + 3, device=dev)
    state = big[:, :n_in]
    kw = {}
    mean = std = None
    if norm:
        mean, std = 0.3 * torch.randn(n_in, device=dev), 0.5 + torch.rand(n_in, device=dev)
        kw = dict(state_mean=mean, state_std=std, state_eps=1e-2)
    loss_ref, grad_ref, t_ref = _reference(state, pred, targ, mean, std, kw.get("state_eps", 0.0))
    P = grad_ref.numel()
    grad = torch.full((P,), float("nan"), device=dev)
    temb = torch.empty(B, Q, device=dev)
    loss_sum = torch.full((1,), 0.25, dtype=torch.float64, device=dev)
    loss = torch.empty(1, device=dev)
    pl, tl = kernels.rnd_linears(pred), kernels.rnd_linears(targ)
    kernels.rnd_update(state, pl, tl, temb, grad, loss_sum=loss_sum, loss=loss, **kw)
    torch.cuda.synchronize()
    assert torch.isfinite(grad).all()
    assert abs(loss.item() - loss_ref.item()) <= 1e-5 * abs(loss_ref.item()) + 1e-9
    assert abs(loss_sum.item() - 0.25 - loss.item()) == 0.0  # loss_sum += (double)(float)mse
    torch.testing.assert_close(temb, t_ref, rtol=0, atol=2e-5 * t_ref.abs().max().item() + 1e-7)
    off = 0
    for prm in pred.parameters():
        g, r = grad[off:off + prm.numel()], grad_ref[off:off + prm.numel()]
        off += prm.numel()
        assert (g - r).abs().max().item() <= 2e-5 * r.abs().max().item() + 1e-9, prm.shape
    # later epochs: the target embedding from the cache -> the same bits
    grad2 = torch.empty_like(grad)
    loss2 = torch.empty(1, device=dev)
    kernels.rnd_update(state, pl, None, temb, grad2, loss=loss2, **kw)
    torch.cuda.synchronize()
    assert torch.equal(grad2, grad) and torch.equal(loss2, loss)
    # deterministic run to run
    grad3 = torch.empty_like(grad)
    kernels.rnd_update(state, pl, tl, None, grad3, **kw)
    torch.cuda.synchronize()
    assert torch.equal(grad3, grad)


def test_rnd_update_rejects_bad_arguments(cuda_device):
    dev = cuda_device
    pred, targ = MLP(8, 1, [8], "elu").to(dev), MLP(8, 1, [8], "elu").to(dev)
    pl, tl = kernels.rnd_linears(pred), kernels.rnd_linears(targ)
    state = torch.randn(10, 8, device=dev)
    with pytest.raises(ValueError):
        kernels.rnd_update(state, pl, tl, None, torch.empty(5, device=dev))  # wrong gradient size
    with pytest.raises(ValueError):
        kernels.rnd_update(state, pl, None, None, torch.empty(8 * 8 + 8 + 8 + 1, device=dev))  # no target at all
    with pytest.raises(RuntimeError):
        kernels.rnd_update(state.cpu(), pl, tl, None, torch.empty(81))  # no CPU fallback
    assert kernels.rnd_linears(MLP(8, 1, [8, 8], "elu")) is None  # two hidden layers: not the fused form
    assert kernels.rnd_linears(MLP(80, 1, [8], "elu")) is None  # wider than the kernel's 64 inputs
