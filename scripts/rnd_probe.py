"""RND predictor step (kernels.rnd_update) at config C5's mini-batch (B 393216, 48 -> 48 -> 1): event-timed launches
with the target computed (first epoch) and read from the cache (later epochs).  python scripts/rnd_probe.py [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import kernels  # noqa: E402
from rsl_rl_amd.networks import MLP  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = "cuda:0"
    torch.manual_seed(0)
    B, n_in, H, Q = 393216, 48, 48, 1
    pred, targ = MLP(n_in, Q, [H], "elu").to(dev), MLP(n_in, Q, [H], "elu").to(dev)
    pl, tl = kernels.rnd_linears(pred), kernels.rnd_linears(targ)
    state = torch.randn(B, n_in, device=dev)
    temb = torch.empty(B, Q, device=dev)
    grad = torch.empty(sum(p.numel() for p in pred.parameters()), device=dev)
    out = {}
    for name, tgt in (("with_target", tl), ("cached_target", None)):
        kernels.rnd_update(state, pl, tgt, temb, grad)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for a, b in ev:
            a.record()
            kernels.rnd_update(state, pl, tgt, temb, grad)
            b.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(sum(a.elapsed_time(b) for a, b in ev) / iters * 1e3, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
