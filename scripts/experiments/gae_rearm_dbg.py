import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from rsl_rl_amd import kernels
dev = torch.device("cuda:0")
T, N = 24, 65536
rng = np.random.default_rng(7)
f = lambda *s: torch.from_numpy(rng.standard_normal(s, dtype=np.float32)).to(dev)
values, rewards, logp, last = f(T, N, 1), f(T, N, 1), f(T, N, 1), f(N, 1)
dones = torch.from_numpy((rng.random((T, N, 1)) < 0.05).astype(np.uint8)).to(dev)
def one():
    ret, adv = torch.empty_like(values), torch.empty_like(values)
    slots = torch.full((T, N, 4), float("nan"), device=dev)
    st = kernels.compute_returns_slots(values, rewards, dones, last, 0.99, 0.95, ret, adv, logp, slots)
    return ret, adv, slots, st
for variant in ("plain_between", "nothing_between", "slots2_between"):
    outs = []
    for i in range(4):
        outs.append(one())
        if variant == "plain_between":
            kernels.compute_returns(values, rewards, dones, last, 0.99, 0.95, True, torch.empty_like(values), torch.empty_like(values))
        elif variant == "slots2_between":
            kernels.debug_knob("gae_form", 0)
            one()
            kernels.debug_knob("gae_form", -1)
    torch.cuda.synchronize()
    for i, o in enumerate(outs[1:], 1):
        r = [torch.equal(a, b) for a, b in zip(outs[0][:3], o[:3])]
        d = (o[1] - outs[0][1]).abs()
        print(variant, i, r, "status", int(o[3].item()), "adv maxdiff", float(d.max()), "ndiff", int((d > 0).sum()),
              "ratio", float((o[1] / outs[0][1]).median()))
ws = kernels._gae_workspace(dev, T, N)
off = kernels._lib.lib().rslrl_compute_returns_status_offset() - 8
print("words", ws[off:off + 24].view(torch.int32).cpu().tolist(), "gens", [ws[off + 256 * (1 + g):off + 256 * (1 + g) + 4].view(torch.int32).item() for g in range(16)])
