"""How the HBM takes strided partial-record writes: torch strided copies into [T*N, 96] fp32 records (C3's
transition records), writing w floats at the end of each 384-byte record, timed with HIP events.  Diagnostic."""
import torch

dev = torch.device("cuda:0")
n, R = 24 * 65536, 96
rec = torch.zeros(n, R, device=dev)
src = {w: torch.randn(n, w, device=dev) for w in (4, 8, 16, 32, 96)}
big = torch.empty(512 << 20, dtype=torch.uint8, device=dev)  # evicts the MALL between runs


def t(fn, reps=10):
    ts = []
    for _ in range(reps):
        big.zero_()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for w in (4, 8, 16, 32, 96):
    us = t(lambda: rec[:, R - w:].copy_(src[w]))
    print(f"write {4 * w:4d} B at the end of each 384-B record: {us:7.1f} us  ({n * 4 * w / us / 1e3:6.0f} GB/s useful)")
us = t(lambda: src[32].copy_(rec[:, 64:96]))
print(f"read  128 B per record: {us:7.1f} us")
