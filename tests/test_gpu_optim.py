"""Fused gradient clipping + Adam (csrc/optim.hip, kernels.FusedClipAdam) vs torch: clip_grad_norm_ then
torch.optim.Adam(fused=True).step() (ppo.py:373-374) on the same parameters and gradients.  Without clipping
(coefficient exactly 1) the update follows torch's fused-Adam arithmetic step by step: parameters and both
moments bit-identical; with clipping active the norm is accumulated in another order (fp64 here, per-tensor
fp32 norms in torch), so parameters agree to 1e-6 relative."""

import io

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


@pytest.mark.parametrize("max_norm", [1.0, 1e9])
def test_nan_gradient_poisons_every_parameter(max_norm, cuda_device):
    """clip_grad_norm_ with a NaN total norm: torch.clamp(coef, max=1) keeps the NaN, every gradient is scaled
    by it and Adam turns every parameter NaN -- the fused step must fail the same way, not only where the
    gradient was NaN."""
    ours = _make(cuda_device, 2)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    opt_o = torch.optim.Adam(ours, lr=1e-3, fused=True)
    opt_r = torch.optim.Adam(ref, lr=1e-3, fused=True)
    fused = kernels.FusedClipAdam(opt_o, max_norm)
    for po, pr in zip(ours, ref):
        gr = torch.randn(po.shape, device=cuda_device)
        po.grad, pr.grad = gr.clone(), gr.clone()
    ours[2].grad[3, 5] = float("nan")
    ref[2].grad[3, 5] = float("nan")
    fused.step()
    torch.nn.utils.clip_grad_norm_(ref, max_norm)
    opt_r.step()
    torch.cuda.synchronize()
    for po, pr in zip(ours, ref):
        assert torch.isnan(pr.data).all()
        assert torch.isnan(po.data).all()
        assert torch.isnan(po.grad).all()  # .grad holds the clipped (NaN-scaled) gradient, as after clip_grad_norm_


def test_clipped_gradient_written_back(cuda_device):
    """After the step .grad holds the clipped gradient (clip_grad_norm_ scales in place), also for a
    non-contiguous .grad (the kernel works on a contiguous copy, copied back)."""
    ours = _make(cuda_device, 3)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    opt_o = torch.optim.Adam(ours, lr=1e-3, fused=True)
    fused = kernels.FusedClipAdam(opt_o, 0.5)
    for po, pr in zip(ours, ref):
        gr = torch.randn(po.shape, device=cuda_device) * 2.0
        if gr.dim() == 2:  # a transposed (non-contiguous) view with the same values
            po.grad = gr.t().contiguous().t()
            assert not po.grad.is_contiguous()
        else:
            po.grad = gr.clone()
        pr.grad = gr.clone()
    fused.step()
    torch.nn.utils.clip_grad_norm_(ref, 0.5)
    torch.cuda.synchronize()
    for po, pr in zip(ours, ref):
        torch.testing.assert_close(po.grad, pr.grad, rtol=1e-6, atol=1e-8)


def test_resume_from_non_fused_adam_state(cuda_device):
    """A checkpoint written by a plain (non-fused) torch Adam -- what a reference run saves -- loads with
    fused=None in its param group and CPU step tensors (torch keeps non-fused steps on the host).  PPO.update()
    calls adopt_loaded_state(); the fused step must then continue the same Adam trajectory as the plain Adam
    that wrote the checkpoint (steps on the device, moments continued), without touching host memory."""
    ours = _make(cuda_device, 4)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ours]
    plain = torch.optim.Adam(ref, lr=1e-3, foreach=False)
    g = torch.Generator(device=cuda_device).manual_seed(5)
    grads = [[torch.randn(p.shape, device=cuda_device, generator=g) for p in ours] for _ in range(5)]
    for it in range(3):
        for pr, gr in zip(ref, grads[it]):
            pr.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        plain.step()
    buf = io.BytesIO()  # a checkpoint round trip (load_state_dict alone would share the moment tensors)
    torch.save(plain.state_dict(), buf)
    buf.seek(0)
    sd = torch.load(buf, weights_only=True)
    with torch.no_grad():
        for po, pr in zip(ours, ref):
            po.copy_(pr)
    opt_o = torch.optim.Adam(ours, lr=1e-3, fused=True)
    opt_o.load_state_dict(sd)
    assert opt_o.param_groups[0]["fused"] is None  # what the advisor saw: the checkpoint's flag wins
    assert opt_o.state[ours[0]]["step"].device.type == "cpu"
    fused = kernels.FusedClipAdam(opt_o, 1.0)
    fused.adopt_loaded_state()
    assert opt_o.param_groups[0]["fused"] is True
    for po in ours:
        st = opt_o.state[po]
        assert st["step"].device == po.device and st["step"].dtype == torch.float32 and float(st["step"]) == 3.0
    for it in range(3, 5):
        for po, pr, gr in zip(ours, ref, grads[it]):
            po.grad, pr.grad = gr.clone(), gr.clone()
        fused.step()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        plain.step()
    torch.cuda.synchronize()
    for po, pr in zip(ours, ref):
        assert float(opt_o.state[po]["step"]) == 5.0
        # plain (for-loop) Adam vs torch's fused arithmetic: fp32 rounding apart
        torch.testing.assert_close(po.data, pr.data, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(opt_o.state[po]["exp_avg_sq"], plain.state[pr]["exp_avg_sq"], rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("round_fp32,with_lr", [(False, True), (True, True), (False, False)])
def test_tail_inside_the_norm_launch_matches_separate_launches(round_fp32, with_lr, cuda_device):
    """FusedClipAdam.step(tail=...) (rslrl_clip_adam_step_tail: the per-mini-batch lr rule and loss sums inside the
    norm launch) against rslrl_ppo_update_tail then step(): the same lr trace, loss sums, parameters and moments, bit
    for bit, over KLs that raise, lower and keep the lr."""
    dev = cuda_device
    runs = []
    for fused in (False, True):
        ps = _make(dev, 3)
        lr32 = torch.full((), 1e-3, dtype=torch.float32, device=dev)
        lr = torch.full((), 1e-3, dtype=torch.float64, device=dev)
        opt = torch.optim.Adam(ps, lr=lr32 if with_lr else 1e-3, fused=True)
        fca = kernels.FusedClipAdam(opt, 1.0)
        sums = torch.zeros(4, dtype=torch.float64, device=dev)
        g = torch.Generator(device=dev).manual_seed(2)
        trace = []
        for it, kl in enumerate((0.05, 0.001, 0.01, 0.03, 0.0001, 0.0)):
            for p in ps:
                p.grad = torch.randn(p.shape, device=dev, generator=g)
            stats = torch.randn(8, device=dev, generator=g)
            stats[kernels.STATS_KL] = kl
            kl_src = stats[kernels.STATS_KL:kernels.STATS_KL + 1]
            tail = kernels.ppo_tail_args(stats, kl_src if with_lr else None, lr if with_lr else None,
                                         lr32 if with_lr else None, 0.01, sums, round_fp32=round_fp32)
            if fused:
                fca.step(tail=tail)
            else:
                kernels.ppo_update_tail_args(tail, dev)
                fca.step()
            trace.append((float(lr), float(lr32)))
        torch.cuda.synchronize()
        runs.append((trace, sums.clone(), [p.detach().clone() for p in ps],
                     [opt.state[p]["exp_avg_sq"].clone() for p in ps]))
    (t0, s0, p0, v0), (t1, s1, p1, v1) = runs
    assert t0 == t1 and len(set(t0)) > 1 if with_lr else t0 == t1
    assert torch.equal(s0, s1)
    assert all(torch.equal(a, b) for a, b in zip(p0, p1)) and all(torch.equal(a, b) for a, b in zip(v0, v1))
