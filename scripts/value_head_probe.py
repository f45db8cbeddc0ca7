"""The critic's fused head at C3's mini-batch (393,216 rows): median launch time in this process and, with --dump, its
values / a slice of dz / the folded [dW | db] saved for a cross-process comparison.  RSLRL_VALUE_HEAD_STREAM=1 (read
once per process) selects the streaming form; run one process per form on one box."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import _lib  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402


def main():
    iters = 20
    dump = sys.argv[1] if len(sys.argv) > 1 else None
    dev = torch.device("cuda:0")
    M = N = K = 0
    M, K, N = 393216, 256, 256
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.nn.functional.elu(torch.randn(M, K, device=dev, generator=g))
    w = torch.randn(N, K, device=dev, generator=g) / 16
    b = torch.randn(N, device=dev, generator=g) * 0.1
    wo = torch.randn(1, N, device=dev, generator=g) / 16
    bo = torch.randn(1, device=dev, generator=g) * 0.1
    tv = torch.randn(M, 1, device=dev, generator=g) * 0.3
    ret = torch.randn(M, 1, device=dev, generator=g)
    img, out_img = fused_mlp.bimages([(w, False), (wo, False, _lib.BIMAGE_LAYOUT_OUT)])
    head = fused_mlp.ValueHead(tv, ret, 0.2, 1.0, True)
    ts = []
    for it in range(iters + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        res = fused_mlp.value_head_fwd_bwd(x, b, N, img, bo, out_img, wo, head)
        e1.record()
        torch.cuda.synchronize()
        if it >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    dz, y, wpart = res
    folds = fused_mlp._FoldBatch()
    dwb = torch.empty(N + 1, device=dev)
    folds.add(wpart, wpart.shape[0], wpart.shape[1], dwb, N + 1)
    folds.run(dev)
    torch.cuda.synchronize()
    if dump:
        torch.save({"y": y.cpu(), "dz": dz[:8192].cpu(), "dz_sum": float(dz.double().sum()), "dwb": dwb.cpu(),
                    "rows": wpart.shape[0]}, dump)
    print(json.dumps({"stream": os.environ.get("RSLRL_VALUE_HEAD_STREAM", "0"), "median_us": round(ts[len(ts) // 2], 1),
                      "min_us": round(ts[0], 1), "partial_rows": int(wpart.shape[0])}))


if __name__ == "__main__":
    main()
