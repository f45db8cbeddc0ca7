"""What a plain device copy achieves at rollout_record's size (DESIGN.md §6 roofline note): the 43.3 MB per launch
of the C3 record (21.7 MB read + 21.7 MB written) and larger copies for the asymptote, through the runtime's copy
(`copy_` -> hipMemcpyAsync's blit kernel) and a torch elementwise kernel (`mul(src, 1, out=dst)`).  Run under
`rocprofv3 --kernel-trace`; the dispatches come in the order printed (size by size, `reps` each after `warm`)."""

import json

import torch


def main():
    dev = torch.device("cuda:0")
    sizes_mb = [21.66, 43.3, 173.3, 693.0]
    warm, reps = 5, 40
    plan = []
    for mb in sizes_mb:
        n = int(mb * 1e6 / 4) // 64 * 64
        src = torch.randn(n, device=dev)
        dst = torch.empty_like(src)
        for op in ("copy", "mul"):
            for _ in range(warm + reps):
                if op == "copy":
                    dst.copy_(src)
                else:
                    torch.mul(src, 1.0, out=dst)
            torch.cuda.synchronize()
            plan.append({"op": op, "bytes_read": 4 * n, "warm": warm, "reps": reps})
        del src, dst
    # the rollout's pattern: a ring of 3 sources (the env's observation buffers) into the t-th slice of a [24, ...]
    # storage (520 MB, over the Infinity Cache), so that the writes go to lines no earlier launch left in the cache
    n = int(21.66e6 / 4) // 64 * 64
    ring = [torch.randn(n, device=dev) for _ in range(3)]
    store = torch.empty(24, n, device=dev)
    for op in ("copy_rot", "mul_rot"):
        for i in range(warm + reps):
            if op == "copy_rot":
                store[i % 24].copy_(ring[i % 3])
            else:
                torch.mul(ring[i % 3], 1.0, out=store[i % 24])
        torch.cuda.synchronize()
        plan.append({"op": op, "bytes_read": 4 * n, "warm": warm, "reps": reps})
    print(json.dumps(plan))


if __name__ == "__main__":
    main()
