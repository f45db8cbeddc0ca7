"""Phase timeline of the fused hidden-layer backward from the diagnostic stamps build (RSLRL_HB_STAMPS: s_memtime per
workgroup, tile and wave at 7 points; rsl_rl_amd/lib/variants/hbstamps).  Run with
RSLRL_AMD_LIB=rsl_rl_amd/lib/variants/hbstamps/librslrl_amd.so python scripts/hb_stamps.py
Prints the mean cycles per tile of each phase (and their spread over waves) as one JSON line."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rsl_rl_amd import _lib  # noqa: E402
from rsl_rl_amd.networks import fused_mlp  # noqa: E402

PHASES = ["dgrad_loop", "wait_dma_barrier1", "epilogue", "wgrad_loop", "barrier3", "split_store_barrier4"]


def main():
    M = int(os.environ.get("HB_M", "393216"))
    L = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(1)
    dzs = [torch.randn(M, 256, device="cuda", generator=g) * 0.01 for _ in range(2)]
    hs = [torch.nn.functional.elu(torch.randn(M, 256, device="cuda", generator=g)) for _ in range(2)]
    ws = [torch.randn(256, 256, device="cuda", generator=g) / 16 for _ in range(2)]
    imgs = fused_mlp.bimages([(w, True) for w in ws])
    S = L.rslrl_hidden_bwd_slices(M)
    tiles = M // 64
    per = -(-tiles // S)
    buf = torch.zeros(2 * S * per * 8 * 8, dtype=torch.int64, device="cuda")
    for _ in range(20):  # warm: the clock settles under load
        fused_mlp.hidden_bwd_pair(dzs, hs, imgs)
    torch.cuda.synchronize()
    import ctypes
    L.rslrl_hb_debug_stamps.argtypes = [ctypes.c_void_p]
    assert L.rslrl_hb_debug_stamps(buf.data_ptr()) == 0
    fused_mlp.hidden_bwd_pair(dzs, hs, imgs)
    torch.cuda.synchronize()
    L.rslrl_hb_debug_stamps(None)
    st = buf.cpu().numpy().reshape(2 * S, per, 8, 8)[:, :, :, :7].astype(np.int64)
    d = np.diff(st, axis=-1)  # [wg, tile, wave, 6]
    out = {"M": M, "slices_per_problem": S, "tiles_per_slice": per}
    for k, name in enumerate(PHASES):
        x = d[:, 1:-1, :, k]  # steady-state tiles
        out[name] = {"mean_cycles": float(x.mean()), "p10": float(np.percentile(x, 10)),
                     "p90": float(np.percentile(x, 90))}
    tile = np.diff(st[:, :, :, 0], axis=1)[:, :-1]
    out["tile_cycles_mean"] = float(tile.mean())
    out["mfma_cycles_per_tile_per_simd"] = 2 * 384 * 32
    kernel = st[:, :, :, :].max() - st[:, :, :, 0].min()
    out["span_cycles"] = int(kernel)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
