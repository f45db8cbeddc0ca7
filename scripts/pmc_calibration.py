"""PMC calibration workload: a known-byte 16-B streaming copy next to the hot-path kernels at C3 shapes.

Run under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE` (MI355X_MICROARCH.md: the two
do not fit one pass).  The copy moves exactly COPY_BYTES each way, which calibrates FETCH_SIZE /
WRITE_SIZE (KB units; gfx950 FETCH_SIZE counts half of a wide streaming read) before they are read as
HBM traffic of the hot-path kernels (scripts/pmc_summary.py).
"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import kernels  # noqa: E402

COPY_BYTES = 512 * 1024 * 1024


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    src = torch.randn(COPY_BYTES // 4, device=dev, generator=g)
    dst = torch.empty_like(src)
    for _ in range(3):
        dst.copy_(src)
    del src, dst
    T, N, O, A, M = 24, 65536, 48, 12, 4
    B = N * T // M
    # GAE
    v = torch.randn(T, N, 1, device=dev, generator=g)
    r = torch.randn(T, N, 1, device=dev, generator=g)
    d = (torch.rand(T, N, 1, device=dev, generator=g) < 0.02).to(torch.uint8)
    lv = torch.randn(N, 1, device=dev, generator=g)
    ret, adv = torch.empty_like(v), torch.empty_like(v)
    for _ in range(3):
        kernels.compute_returns(v, r, d, lv, 0.99, 0.95, True, ret, adv)
    # loss at C3 mini-batch size, 4 distinct mini-batches (> Infinity Cache together)
    sets = []
    for _ in range(4):
        sets.append((torch.randn(B, A, device=dev, generator=g), 0.5 + torch.rand(A, device=dev, generator=g),
                     torch.randn(B, 1, device=dev, generator=g), torch.randn(B, A, device=dev, generator=g),
                     *[torch.randn(B, 1, device=dev, generator=g) for _ in range(4)],
                     torch.randn(B, A, device=dev, generator=g), 0.5 + torch.rand(B, A, device=dev, generator=g)))
    for i in range(8):
        kernels.ppo_loss_fwd_bwd(*sets[i % 4])
    del sets
    # gather of the full C3 storage
    rows = T * N
    fields = [torch.randn(rows, O, device=dev, generator=g)] + [torch.randn(rows, A, device=dev, generator=g)
                                                                 for _ in range(3)]
    fields += [torch.randn(rows, 1, device=dev, generator=g) for _ in range(4)]
    idx = torch.randperm(rows, device=dev, generator=g).to(torch.int32)
    pairs = [(f, torch.empty_like(f)) for f in fields]
    for _ in range(2):
        kernels.gather_rows(pairs, idx)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
