"""Diagnostic: x6 input-gradient kernel vs torch on one or two full tiles; prints the error per 32 x 32 block."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd.networks.fused_mlp import bimage, linear_dgrad_elu  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
M = int(os.environ.get("DM", 256))
dz = torch.randn(M, 256, device=dev)
w = torch.randn(256, 256, device=dev) / 16
h = torch.nn.functional.elu(torch.randn(M, 256, device=dev))
out = linear_dgrad_elu(dz, w, h, bimage(w, True))[0]
ref = (dz.double() @ w.double()) * torch.where(h > 0, torch.ones_like(h), h + 1).double()
err = (out.double() - ref).abs()
blk = err.view(M // 32, 32, 8, 32).amax(dim=(1, 3))
torch.set_printoptions(precision=2, linewidth=200)
print(blk)
bad = (err > 1e-3).nonzero()
print(bad[:20])

from rsl_rl_amd import _lib  # noqa: E402
from rsl_rl_amd.networks.fused_mlp import linear_dgrad_elu_ex  # noqa: E402

for want_db in (True, False):
    o2 = linear_dgrad_elu_ex(dz, h, bimage(w, True), _lib.ARITH_X6, None, False, want_db=want_db)[0]
    e2 = (o2.double() - ref).abs()
    print("ex want_db", want_db, e2.max().item(), (e2 > 1e-3).nonzero()[:8].tolist())
