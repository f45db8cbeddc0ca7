"""One Adam step from random state: torch fused Adam vs rslrl_clip_adam_step; dumps the inputs and both outputs
of the elements that differ (gpurun_out/adam_diag.npz) so the arithmetic can be matched on the CPU."""

import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from rsl_rl_amd import kernels  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
n = 1 << 20
p0 = torch.randn(n, device=dev) * 0.1
g0 = torch.randn(n, device=dev)
m0 = torch.randn(n, device=dev) * 0.1
v0 = torch.rand(n, device=dev) * 0.01
out = {}
for name in ("ours", "torch"):
    p = torch.nn.Parameter(p0.clone())
    p.grad = g0.clone()
    opt = torch.optim.Adam([p], lr=1e-3, fused=True)
    st = opt.state[p]
    st["step"] = torch.tensor(3.0, device=dev)
    st["exp_avg"] = m0.clone()
    st["exp_avg_sq"] = v0.clone()
    if name == "ours":
        kernels.FusedClipAdam(opt, 0.0).step()
    else:
        opt.step()
    torch.cuda.synchronize()
    out[name] = (p.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(), float(st["step"]))
res = {}
for i, k in enumerate(("param", "exp_avg", "exp_avg_sq")):
    d = out["ours"][i] != out["torch"][i]
    res[k] = int(d.sum())
res["step"] = [out["ours"][3], out["torch"][3]]
bad = ((out["ours"][0] != out["torch"][0]) | (out["ours"][1] != out["torch"][1]) |
       (out["ours"][2] != out["torch"][2])).nonzero().flatten()[:4096]
bad = torch.cat([bad, torch.arange(4096, device=dev)])  # plus the first elements, equal or not
np.savez("gpurun_out/adam_diag.npz", p=p0[bad].cpu().numpy(), g=g0[bad].cpu().numpy(), m=m0[bad].cpu().numpy(),
         v=v0[bad].cpu().numpy(), **{f"{a}_{k}": out[a][i][bad].cpu().numpy() for a in ("ours", "torch")
                                     for i, k in enumerate(("p", "m", "v"))})
print(json.dumps(res))
