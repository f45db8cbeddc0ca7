"""Fused gradient clipping + Adam (csrc/optim.hip, kernels.FusedClipAdam) vs torch: clip_grad_norm_ then
torch.optim.Adam(fused=True).step() (ppo.py:373-374) on the same parameters and gradients.  Without clipping
(coefficient exactly 1) the update follows torch's fused-Adam arithmetic step by step: parameters and both
moments bit-identical; with clipping active the norm is accumulated in another order (fp64 here, per-tensor
fp32 norms in torch), so parameters agree to 1e-6 relative."""

import pytest
import torch

from rsl_rl_amd import kernels

pytestmark = pytest.mark.gpu


def _make(dev, seed):
    torch.manual_seed(seed)
    shapes = [(256, 48), (256,), (256, 256), (256,), (12, 256), (12,), (12,)]
    return [torch.nn.Parameter(torch.randn(s, device=dev) * 0.1) for s in shapes]


@pytest.mark.parametrize("max_norm,tensor_lr", [(1e9, False), (1e9, True), (0.5, True)])
def test_clip_adam_matches_torch(max_norm, tensor_lr, cuda_device):
    ours = _make(cuda_device, 0)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    lr = torch.tensor(1e-3, device=cuda_device) if tensor_lr else 1e-3
    opt_o = torch.optim.Adam(ours, lr=lr, fused=True)
    opt_r = torch.optim.Adam(ref, lr=lr.clone() if tensor_lr else lr, fused=True)
    assert kernels.FusedClipAdam.supported(opt_o)
    fused = kernels.FusedClipAdam(opt_o, max_norm)
    g = torch.Generator(device=cuda_device).manual_seed(1)
    for it in range(5):
        for po, pr in zip(ours, ref):
            gr = torch.randn(po.shape, device=cuda_device, generator=g) * (0.3 if it % 2 else 3.0)
            po.grad = gr.clone()
            pr.grad = gr.clone()
        fused.step()
        torch.nn.utils.clip_grad_norm_(ref, max_norm)
        opt_r.step()
    torch.cuda.synchronize()
    for po, pr in zip(ours, ref):
        so, sr = opt_o.state[po], opt_r.state[pr]
        assert float(so["step"]) == float(sr["step"]) == 5.0
        if max_norm > 1e6:
            assert torch.equal(po.data, pr.data)
            assert torch.equal(so["exp_avg"], sr["exp_avg"]) and torch.equal(so["exp_avg_sq"], sr["exp_avg_sq"])
        else:
            torch.testing.assert_close(po.data, pr.data, rtol=1e-6, atol=1e-7)
    # the optimizer's state_dict keeps torch's layout (checkpoints load into a plain torch Adam)
    opt_r.load_state_dict(opt_o.state_dict())


def test_unsupported_optimizers_fall_back():
    p = [torch.nn.Parameter(torch.zeros(3))]
    assert not kernels.FusedClipAdam.supported(torch.optim.SGD(p, lr=0.1))
    assert not kernels.FusedClipAdam.supported(torch.optim.Adam(p, lr=0.1, weight_decay=0.1))
