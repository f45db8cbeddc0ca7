"""Host logic of the one-launch rollout forward (fused_mlp.rollout_mlp_pair): the shapes it declines return None before
any launch, so they run on CPU tensors here -- the GPU tests (tests/test_gpu_rollout_mlp.py) cover what it takes."""

import torch

from rsl_rl_amd.networks import fused_mlp


def _nets(k0=48, hidden=3, width=256, nouts=(12, 1)):
    ws, bs, imgs = [], [], []
    for nout in nouts:
        w = [torch.zeros(width, k0)] + [torch.zeros(width, width) for _ in range(hidden - 1)] + [torch.zeros(nout, width)]
        b = [torch.zeros(width) for _ in range(hidden)] + [torch.zeros(nout)]
        ws.append(w)
        bs.append(b)
        imgs.append(([torch.zeros(16) for _ in range(hidden)], None, torch.zeros(16)))
    return ws, bs, imgs


def _xs(M, k0):
    return [torch.zeros(M, k0), torch.zeros(M, k0)]


def test_declined_shapes_return_none_before_launching():
    ws, bs, imgs = _nets()
    assert fused_mlp.rollout_mlp_pair(_xs(1000, 48), ws, bs, imgs, 3) is None  # M not a multiple of 64
    ws40, bs40, imgs40 = _nets(k0=40)
    assert fused_mlp.rollout_mlp_pair(_xs(1024, 40), ws40, bs40, imgs40, 3) is None  # input width not 16/32/48/64
    ws1, bs1, imgs1 = _nets(hidden=1)
    assert fused_mlp.rollout_mlp_pair(_xs(1024, 48), ws1, bs1, imgs1, 1) is None  # one hidden layer
    ws5, bs5, imgs5 = _nets(hidden=5)
    assert fused_mlp.rollout_mlp_pair(_xs(1024, 48), ws5, bs5, imgs5, 5) is None  # more than 4 hidden layers
    wsn, bsn, imgsn = _nets(width=128)
    assert fused_mlp.rollout_mlp_pair(_xs(1024, 48), wsn, bsn, imgsn, 3) is None  # hidden width not 256
    ws24, bs24, imgs24 = _nets(nouts=(24, 1))
    assert fused_mlp.rollout_mlp_pair(_xs(1024, 48), ws24, bs24, imgs24, 3) is None  # 24 outputs (> 16)
    noimg = [(i[0], None, None) for i in imgs]
    assert fused_mlp.rollout_mlp_pair(_xs(1024, 48), ws, bs, noimg, 3) is None  # output layer not fused
    x = torch.zeros(1024 * 48 + 1)[1:].view(1024, 48)  # 4-byte aligned only
    assert fused_mlp.rollout_mlp_pair([x, x], ws, bs, imgs, 3) is None
    assert fused_mlp.rollout_mlp_pair([torch.zeros(1024, 48), torch.zeros(512, 48)], ws, bs, imgs, 3) is None
