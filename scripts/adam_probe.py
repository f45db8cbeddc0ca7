"""grad_sq + Adam launch durations in isolation (run under rocprofv3 --kernel-trace --stats): C3's actor + critic
parameter list (16 tensors, ~290k elements) vs the same element count as one tensor, to see whether the ~14 us per
launch in the training step is per-tensor latency or inherent to the launch."""

import sys

import torch

sys.path.insert(0, ".")
from rsl_rl_amd import kernels  # noqa: E402


def shapes_c3():
    out = []
    for dims in ([48, 256, 256, 256, 12], [48, 256, 256, 256, 1]):
        for i in range(len(dims) - 1):
            out += [(dims[i + 1], dims[i]), (dims[i + 1],)]
    return out + [(12,)]


def run(shapes, iters=100):
    dev = torch.device("cuda:0")
    ps = [torch.nn.Parameter(torch.randn(*s, device=dev)) for s in shapes]
    for p in ps:
        p.grad = torch.randn_like(p) * 1e-2
    opt = torch.optim.Adam(ps, lr=1e-3)
    fa = kernels.FusedClipAdam(opt, 1.0)
    for _ in range(iters):
        fa.step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    sh = shapes_c3()
    n = sum(int(torch.tensor(s).prod()) for s in sh)
    print(len(sh), "tensors", n, "elements")
    run(sh)
    run([(n,)])
