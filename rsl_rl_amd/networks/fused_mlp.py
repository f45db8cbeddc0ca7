"""Actor/critic MLP forward + backward on fused MFMA GEMMs.

For an `MLP` of Linear(+ELU) hidden blocks and a final Linear (rsl_rl/networks/mlp.py:59-114) this
autograd Function runs

    forward   H_l = ELU(H_{l-1} W_l^T + b_l)    one rslrl_linear_fwd launch per hidden layer; the last one
              Y   = H_{L-1} W_L^T + b_L         also computes the (<= 32 wide) output layer from its
                                                register tile (rslrl_linear_fwd_out)
    backward  dW_l = dZ_l^T H_{l-1}             x6 split-K weight-gradient kernel (rslrl_linear_wgrad)
              dZ_{l-1} = (dZ_l W_l) * ELU'(H_{l-1}) and db_{l-1} = column sums of dZ_{l-1}
                                                one rslrl_linear_dgrad_elu launch (+ a tiny fold); for the
                                                output layer together with its dW (rslrl_linear_dgrad_elu_wgrad)

so the pre-activations and dH never reach HBM and the separate ELU / ELU-backward / bias-reduction
kernels disappear.  Parameters, state_dict and the forward values are those of the nn.Sequential (the
MFMA accumulation order differs from hipBLASLt's at fp32 epsilon; tests/test_gpu_fused_mlp.py).
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import weakref

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from ..kernels import timer
from .linear import _splitk_weight_grad

MAX_WIDTH = 256


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


_FUSE_OUT = os.environ.get("RSLRL_FUSE_OUT", "1") == "1"  # output-layer backward in one launch
_FUSE_OUT_FWD = os.environ.get("RSLRL_FUSE_OUT_FWD", "1") == "1"  # output-layer forward in the last hidden GEMM
GEMM_F32 = 0  # v_mfma_f32_32x32x2_f32: exact f32 fma chain
GEMM_X6 = 1   # fp32 split into 3 bf16 planes (24 significant bits), 6 bf16 MFMA products, fp32 accumulation --
#               the default: operands carry fp32's full significand, like the reference's fp32 nn.Linear
GEMM_H3 = 2   # opt-in REDUCED precision: hidden-layer GEMMs on 2 fp16 planes of power-of-two scaled operands
#               (22 significant bits, the a1*b1 product dropped, values far below a tensor's max in fp16
#               subnormals), 3 fp16 MFMA products (include/rslrl_amd.h rslrl_linear_gemm); the first layer and
#               the output layer stay on x6
_MODE_NAMES = {"f32": GEMM_F32, "x6": GEMM_X6, "h3": GEMM_H3}


def _mode_from_env() -> int:
    name = os.environ.get("RSLRL_GEMM_MODE", "x6")
    if name not in _MODE_NAMES:
        raise ValueError(f"RSLRL_GEMM_MODE={name!r}: expected one of {sorted(_MODE_NAMES)}")
    return _MODE_NAMES[name]


_mode = _mode_from_env()


def set_gemm_mode(mode: int) -> int:
    """Select the arithmetic of the fused GEMMs (GEMM_F32 | GEMM_X6 | GEMM_H3); returns the previous mode.  The
    initial mode comes from RSLRL_GEMM_MODE=f32|x6|h3."""
    global _mode
    if mode not in (GEMM_F32, GEMM_X6, GEMM_H3):
        raise ValueError(f"unknown GEMM mode {mode}")
    prev, _mode = _mode, mode
    return prev


def _split() -> bool:
    """A split-precision MFMA mode (x6 or h3): B operands come from images."""
    return _mode in (GEMM_X6, GEMM_H3)


_amax_ws: dict = {}


def _amax_workspace(device, slot: int = 0):
    """Per-device {max bits, ticket} words of the amax reduction (zero once; every launch leaves them zero);
    slot 1: the second problem of a pair launch (rslrl_linear_gemm_pair needs distinct workspaces)."""
    ws = _amax_ws.get((device, slot))
    if ws is None:
        n = max(_lib.lib().rslrl_amax_workspace_bytes() // 4, 4)
        ws = torch.zeros(n, dtype=torch.int32, device=device)
        _amax_ws[(device, slot)] = ws
    return ws


def _amax(t):
    """max |t| as a 1-element device tensor (for an h3 operand whose producer did not publish one)."""
    return t.detach().abs().amax().reshape(1).float()


def _ptr(t):
    return t.data_ptr() if t is not None else None


# B-operand images (include/rslrl_amd.h rslrl_linear_prepare_bimages).  Weights can change in place without
# moving their version counter (fused Adam does not bump it), so images are rebuilt on every use except
# inside a frozen_weights() scope, where the caller promises the weights do not change (the rollout).
_frozen_depth = 0
_frozen_gen = 0  # bumped on entering an outermost frozen_weights() scope (a new rollout: weights may have changed)
_bimage_cache: dict = {}
_pair_memo: dict = {}  # fused_mlp_forward_pair's per-pair plan inside a frozen_weights() scope


@contextlib.contextmanager
def frozen_weights():
    """Scope in which B images of weights are built once and reused (the rollout of on_policy_runner)."""
    global _frozen_depth, _frozen_gen
    if _frozen_depth == 0:
        _frozen_gen += 1
    _frozen_depth += 1
    try:
        yield
    finally:
        _frozen_depth -= 1
        if _frozen_depth == 0:
            _bimage_cache.clear()
            _pair_memo.clear()


_bimage_floats: dict = {}  # (depth, layout) -> image size in floats


def bimages(specs):
    """Images for [(w, transposed[, layout]), ...]: transposed=False -> B = w ([N, K]), True -> B = w^T;
    layout _lib.BIMAGE_LAYOUT_OUT -> the output-layer image of linear_fwd_out.  One launch for every image not
    already cached in a frozen_weights() scope."""
    out = [None] * len(specs)
    todo = []
    for i, spec in enumerate(specs):
        w, tr = spec[0], spec[1]
        layout = spec[2] if len(spec) > 2 else _lib.BIMAGE_LAYOUT_GEMM
        rows, depth = (w.shape[1], w.shape[0]) if tr else (w.shape[0], w.shape[1])
        key = (w.data_ptr(), tr, rows, depth, layout)
        if _frozen_depth:
            hit = _bimage_cache.get(key)
            if hit is not None and hit[0]() is w:
                out[i] = hit[1]
                continue
        todo.append((i, w, tr, rows, depth, key))
    if not todo:
        return out
    L = _lib.lib()
    # (the host side runs once per mini-batch in the update, the first time while the GPU waits: image sizes are
    # looked up once per (depth, layout), the image views come from one split)
    sizes = []
    for (_, _, _, _, depth, key) in todo:
        n = _bimage_floats.get((depth, key[4]))
        if n is None:
            layout = key[4]
            if layout == _lib.BIMAGE_LAYOUT_OUT:
                nb = L.rslrl_linear_out_image_bytes()
            elif layout == _lib.BIMAGE_LAYOUT_H3:
                nb = L.rslrl_linear_bimage_h3_bytes(depth)
            else:
                nb = L.rslrl_linear_bimage_bytes(depth)
            n = _bimage_floats[(depth, key[4])] = nb // 4
        sizes.append(n)
    buf = torch.empty(sum(sizes), dtype=torch.float32, device=todo[0][1].device)
    views = buf.split(sizes)
    base = buf.data_ptr()
    for start in range(0, len(todo), _lib.MAX_BIMAGES):
        part = todo[start:start + _lib.MAX_BIMAGES]
        descs = (_lib.BImageDesc * len(part))()
        off = sum(sizes[:start])
        keep = []
        for j, (d, (i, w, tr, rows, depth, key)) in enumerate(zip(descs, part)):
            src = w.detach()
            if not src.is_contiguous():
                src = src.contiguous()
                keep.append(src)
            d.src, d.image, d.rows, d.depth, d.transposed = src.data_ptr(), base + 4 * off, rows, depth, int(tr)
            d.layout = key[4]
            off += sizes[start + j]
            img = views[start + j]
            out[i] = img
            if _frozen_depth:
                _bimage_cache[key] = (weakref.ref(w), img)
        rc = L.rslrl_linear_prepare_bimages(descs, len(part), _stream(buf))
        _lib.check(rc, "rslrl_linear_prepare_bimages")
    return out


def bimage(w, transposed: bool):
    return bimages([(w, transposed)])[0]


def _gemm_args(op, arith, a, a_amax, N, img, *, bias=None, h=None, c=None, colsum=None, wpart=None, out_img=None,
               out_bias=None, y=None, nout=0, amax_out=None, slot=0):
    M, K = a.shape
    return _lib.LinearArgs(op, arith, a.data_ptr(), _ptr(a_amax), M, K, N, img.data_ptr(), _ptr(bias), _ptr(h),
                           _ptr(c), _ptr(colsum), _ptr(wpart), _ptr(out_img), _ptr(out_bias), _ptr(y), nout,
                           _ptr(amax_out), _ptr(_amax_workspace(a.device, slot)) if amax_out is not None else None)


def _gemm(op, arith, a, a_amax, N, img, **kw):
    args = _gemm_args(op, arith, a, a_amax, N, img, **kw)
    rc = _lib.lib().rslrl_linear_gemm(ctypes.byref(args), _stream(a))
    _lib.check(rc, "rslrl_linear_gemm")


def _tag(arith):
    """Timer-span suffix of the h3 launches (bench.py prices them against the 3-product peak)."""
    return "/h3" if arith == _lib.ARITH_H3 else ""


def linear_fwd_ex(x, b, N: int, elu: bool, img, arith, x_amax=None, want_amax=False):
    """(act(x W^T + b), max |y| or None) on the split MFMA path (arith _lib.ARITH_X6 with a layout-0 image, or
    ARITH_H3 with a layout-H3 image and x_amax = max |x| as a device scalar)."""
    M, K = x.shape
    y = torch.empty(M, N, device=x.device, dtype=torch.float32)
    amax = torch.empty(1, device=x.device, dtype=torch.float32) if want_amax else None
    with timer.span(f"linear_fwd[M={M},K={K},N={N}]{_tag(arith)}", x.device, 4 * M * (K + N), 2 * M * K * N):
        _gemm(_lib.LINEAR_FWD_ELU if elu else _lib.LINEAR_FWD, arith, x, x_amax, N, img, bias=b, c=y, amax_out=amax)
    return y, amax


def linear_fwd_pair(xs, bs, N: int, elu: bool, imgs, arith, x_amaxes, want_amax):
    """linear_fwd_ex of two problems of one shape in one launch (rslrl_linear_gemm_pair): xs, bs, imgs,
    x_amaxes, want_amax are pairs; returns ([y0, y1], [amax0, amax1])."""
    M, K = xs[0].shape
    ys = [torch.empty(M, N, device=x.device, dtype=torch.float32) for x in xs]
    amaxes = [torch.empty(1, device=x.device, dtype=torch.float32) if w else None for x, w in zip(xs, want_amax)]
    op = _lib.LINEAR_FWD_ELU if elu else _lib.LINEAR_FWD
    args = [_gemm_args(op, arith, xs[i], x_amaxes[i], N, imgs[i], bias=bs[i], c=ys[i], amax_out=amaxes[i], slot=i)
            for i in range(2)]
    with timer.span(f"linear_fwd_pair[M={M},K={K},N={N}]{_tag(arith)}", xs[0].device, 8 * M * (K + N),
                    4 * M * K * N):
        rc = _lib.lib().rslrl_linear_gemm_pair(ctypes.byref(args[0]), ctypes.byref(args[1]), _stream(xs[0]))
    _lib.check(rc, "rslrl_linear_gemm_pair")
    return ys, amaxes


def linear_fwd(x, w, b, elu: bool, img=None):
    """act(x w^T + b); img: B image of w (x6 arithmetic) or None (exact f32 MFMA)."""
    M, K = x.shape
    N = w.shape[0]
    y = torch.empty(M, N, device=x.device, dtype=torch.float32)
    with timer.span(f"linear_fwd[M={M},K={K},N={N}]", x.device, 4 * M * (K + N), 2 * M * K * N):
        rc = _lib.lib().rslrl_linear_fwd(x.data_ptr(), M, K, w.data_ptr(), N, b.data_ptr(), 1 if elu else 0,
                                         y.data_ptr(), img.data_ptr() if img is not None else None, _stream(x))
    _lib.check(rc, "rslrl_linear_fwd")
    return y


MAX_OUT_WIDTH = 32


def linear_fwd_out(x, w, b, img, w_out, b_out, out_img, store_h: bool):
    """(h, y): h = ELU(x w^T + b) (None unless store_h) and y = h w_out^T + b_out in one x6 launch; img: B image
    of w, out_img: the BIMAGE_LAYOUT_OUT image of w_out (<= 32 rows)."""
    M, K = x.shape
    N = w.shape[0]
    nout = w_out.shape[0]
    h = torch.empty(M, N, device=x.device, dtype=torch.float32) if store_h else None
    y = torch.empty(M, nout, device=x.device, dtype=torch.float32)
    flops = 2 * M * N * (K + nout)
    with timer.span(f"linear_fwd_out[M={M},K={K},N={N},out={nout}]", x.device,
                    4 * M * (K + nout + (N if store_h else 0)), flops):
        rc = _lib.lib().rslrl_linear_fwd_out(x.data_ptr(), M, K, b.data_ptr(), N, img.data_ptr(),
                                             h.data_ptr() if store_h else None, b_out.data_ptr(), nout,
                                             out_img.data_ptr(), y.data_ptr(), _stream(x))
    _lib.check(rc, "rslrl_linear_fwd_out")
    return h, y


def linear_fwd_out_ex(x, b, N: int, img, arith, x_amax, b_out, out_img, store_h: bool):
    """linear_fwd_out with the hidden GEMM in either split arithmetic (see linear_fwd_ex)."""
    M, K = x.shape
    nout = b_out.shape[0]
    h = torch.empty(M, N, device=x.device, dtype=torch.float32) if store_h else None
    y = torch.empty(M, nout, device=x.device, dtype=torch.float32)
    with timer.span(f"linear_fwd_out[M={M},K={K},N={N},out={nout}]{_tag(arith)}", x.device,
                    4 * M * (K + nout + (N if store_h else 0)), 2 * M * N * (K + nout)):
        _gemm(_lib.LINEAR_FWD_OUT, arith, x, x_amax, N, img, bias=b, c=h, out_img=out_img, out_bias=b_out, y=y,
              nout=nout)
    return h, y


def linear_fwd_out_pair(xs, bs, N: int, imgs, b_outs, out_imgs, store_h: bool):
    """linear_fwd_out_ex (x6) of two problems with the same M, K, N (output widths may differ) in one launch
    (rslrl_linear_gemm_pair, RSLRL_LINEAR_FWD_OUT): the rollout's actor and critic heads.  The library takes the
    pair when its tiles are at most one per CU and otherwise runs the two launches; identical results either way.
    Returns ([h0, h1], [y0, y1])."""
    M, K = xs[0].shape
    hs = [torch.empty(M, N, device=x.device, dtype=torch.float32) if store_h else None for x in xs]
    ys = [torch.empty(M, bo.shape[0], device=x.device, dtype=torch.float32) for x, bo in zip(xs, b_outs)]
    args = [_gemm_args(_lib.LINEAR_FWD_OUT, _lib.ARITH_X6, xs[i], None, N, imgs[i], bias=bs[i], c=hs[i],
                       out_img=out_imgs[i], out_bias=b_outs[i], y=ys[i], nout=b_outs[i].shape[0]) for i in range(2)]
    nout = b_outs[0].shape[0] + b_outs[1].shape[0]
    with timer.span(f"linear_fwd_out_pair[M={M},K={K},N={N},out={nout}]", xs[0].device,
                    4 * M * (2 * K + nout + (2 * N if store_h else 0)), 2 * M * N * (2 * K + nout)):
        rc = _lib.lib().rslrl_linear_gemm_pair(ctypes.byref(args[0]), ctypes.byref(args[1]), _stream(xs[0]))
    _lib.check(rc, "rslrl_linear_gemm_pair")
    return hs, ys


class ValueHead:
    """What the critic's fused head (value_head_fwd_bwd) needs from the PPO loss of the mini-batch: its target values
    and returns and the value-loss configuration (ppo.py:305-313)."""

    __slots__ = ("target_values", "returns", "clip_param", "value_loss_coef", "use_clipped")

    def __init__(self, target_values, returns, clip_param, value_loss_coef, use_clipped):
        self.target_values, self.returns = target_values, returns
        self.clip_param, self.value_loss_coef, self.use_clipped = clip_param, value_loss_coef, use_clipped


_VALUE_HEAD = os.environ.get("RSLRL_VALUE_HEAD", "1") != "0"


def value_head_fwd_bwd(x, b, N: int, img, b_out, out_img, w_out, head: ValueHead):
    """The critic's last hidden layer, value head, d(value loss)/dV and the head's backward in one launch
    (rslrl_value_head_fwd_bwd): returns (dz [M, N], y [M, 1], wpart [tiles, P]) -- dz the gradient at the last hidden
    layer's pre-activation, y the values (the bits linear_fwd_out_ex gives), wpart the head's [dW | db] partials for
    the fold -- or None when the shape is not covered (nothing launched)."""
    M, K = x.shape
    tv, ret = head.target_values, head.returns
    if (w_out.shape[0] != 1 or not w_out.is_contiguous() or w_out.data_ptr() % 16 or tv.numel() != M
            or ret.numel() != M or not tv.is_contiguous() or not ret.is_contiguous()):
        return None
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    P = (N + 1 + 3) // 4 * 4
    dz = torch.empty(M, N, device=x.device, dtype=torch.float32)
    y = torch.empty(M, 1, device=x.device, dtype=torch.float32)
    wpart = torch.empty(tiles, P, device=x.device, dtype=torch.float32)
    args = _gemm_args(_lib.LINEAR_FWD_OUT, _lib.ARITH_X6, x, None, N, img, bias=b, c=dz, out_img=out_img,
                      out_bias=b_out, y=y, nout=1)
    vargs = _lib.ValueHeadArgs(tv.data_ptr(), ret.data_ptr(), w_out.data_ptr(), float(head.clip_param),
                               float(head.value_loss_coef), int(bool(head.use_clipped)), wpart.data_ptr(), None)
    with timer.span(f"linear_value_head[M={M},K={K},N={N}]", x.device, 4 * M * (K + N + 3) + 4 * tiles * P,
                    2 * M * N * (K + 2)):
        rc = L.rslrl_value_head_fwd_bwd(ctypes.byref(args), ctypes.byref(vargs), _stream(x))
    if rc == _lib.E_UNSUPPORTED:
        return None
    _lib.check(rc, "rslrl_value_head_fwd_bwd")
    rows = L.rslrl_value_head_partial_rows(M, 0)  # per slice on the streaming form, else per tile (no colsum passed)
    return dz, y, wpart[:rows]


class ActorHead:
    """What the actor's fused head (actor_head_fwd_bwd) needs for the PPO loss of the mini-batch (ppo.py:259-315): the
    mini-batch fields, the shared std, the loss settings and the destinations of the loss statistics and of
    d loss / d sigma.  `values` (the critic's output of this pass) is filled in by train_forward_pair."""

    __slots__ = ("actions", "old_log_prob", "advantages", "target_values", "returns", "old_mu", "old_sigma", "sigma",
                 "clip_param", "value_loss_coef", "entropy_coef", "use_clipped", "compute_kl", "grad_sigma", "stats",
                 "grad_mu", "values", "done")

    def __init__(self, actions, old_log_prob, advantages, target_values, returns, old_mu, old_sigma, sigma, *,
                 clip_param, value_loss_coef, entropy_coef, use_clipped, compute_kl, grad_sigma, stats, grad_mu=None):
        self.actions, self.old_log_prob, self.advantages = actions, old_log_prob, advantages
        self.target_values, self.returns, self.old_mu, self.old_sigma = target_values, returns, old_mu, old_sigma
        self.sigma = sigma
        self.clip_param, self.value_loss_coef, self.entropy_coef = clip_param, value_loss_coef, entropy_coef
        self.use_clipped, self.compute_kl = use_clipped, compute_kl
        self.grad_sigma, self.stats, self.grad_mu = grad_sigma, stats, grad_mu
        self.values = None
        self.done = False  # set when the fused launch ran (the loss statistics and d sigma are then written)

    def supported(self, M: int) -> bool:
        A = _lib.ACTOR_HEAD_ACTIONS
        flat = (self.old_log_prob, self.advantages, self.target_values, self.returns)
        return (self.sigma.dim() == 1 and self.sigma.numel() == A and self.sigma.is_contiguous()
                and all(t.is_contiguous() and tuple(t.shape) == (M, A) for t in (self.actions, self.old_mu,
                                                                                   self.old_sigma))
                and all(t.is_contiguous() and t.numel() == M for t in flat)
                and self.grad_sigma.is_contiguous() and self.grad_sigma.numel() == A and self.stats.numel() >= 8
                and (self.grad_mu is None or (self.grad_mu.is_contiguous() and tuple(self.grad_mu.shape) == (M, A))))


_ACTOR_HEAD = os.environ.get("RSLRL_ACTOR_HEAD", "1") != "0"
ACTOR_HEAD_ACTIONS = _lib.ACTOR_HEAD_ACTIONS
actor_head_launches = 0  # fused actor-head launches so far (tests check which path an update took)


def actor_head_fwd_bwd(x, b, N: int, img, b_out, out_img, w_t_img, head: ActorHead):
    """The actor's last hidden layer, output layer, the PPO loss and the output layer's backward in one launch
    (rslrl_actor_head_fwd_bwd): returns (dz [M, N], mu [M, A], wpart [tiles, A N + A]) -- dz the gradient at the last
    hidden layer's pre-activation, mu the action means (the bits linear_fwd_out_ex gives), wpart the output layer's
    [dW | db] partials for the fold; head.stats / head.grad_sigma receive what kernels.ppo_loss_fwd_bwd writes.  None
    when the shape is not covered (nothing launched)."""
    M, K = x.shape
    A = _lib.ACTOR_HEAD_ACTIONS
    if head.values is None or head.values.numel() != M or not head.values.is_contiguous() or not head.supported(M):
        return None
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    P = A * N + A
    dz = torch.empty(M, N, device=x.device, dtype=torch.float32)
    mu = torch.empty(M, A, device=x.device, dtype=torch.float32)
    wpart = torch.empty(tiles, P, device=x.device, dtype=torch.float32)
    args = _gemm_args(_lib.LINEAR_FWD_OUT, _lib.ARITH_X6, x, None, N, img, bias=b, c=dz, out_img=out_img,
                      out_bias=b_out, y=mu, nout=A)
    h = _lib.ActorHeadArgs(head.actions.data_ptr(), head.old_log_prob.data_ptr(), head.advantages.data_ptr(),
                           head.values.data_ptr(), head.target_values.data_ptr(), head.returns.data_ptr(),
                           head.old_mu.data_ptr(), head.old_sigma.data_ptr(), head.sigma.data_ptr(), A,
                           float(head.clip_param), float(head.value_loss_coef), float(head.entropy_coef),
                           int(bool(head.use_clipped)), int(bool(head.compute_kl)), w_t_img.data_ptr(),
                           wpart.data_ptr(), head.grad_sigma.data_ptr(), head.stats.data_ptr(),
                           head.grad_mu.data_ptr() if head.grad_mu is not None else None)
    ws = _kernels_ws().get(x.device, "actor_head", L.rslrl_actor_head_workspace_bytes(M))  # zero-filled once
    # algorithmic bytes: read x and the loss's row inputs (actions, old mu, old sigma, 5 scalars), write mu, dz and the
    # per-tile partials
    with timer.span(f"linear_actor_head[M={M},K={K},N={N}]", x.device,
                    4 * M * (K + 3 * A + 5 + A + N) + 4 * tiles * P, 2 * M * N * (K + 3 * A)):
        rc = L.rslrl_actor_head_fwd_bwd(ctypes.byref(args), ctypes.byref(h), ws.data_ptr(), ws.numel(), _stream(x))
    if rc == _lib.E_UNSUPPORTED:
        return None
    _lib.check(rc, "rslrl_actor_head_fwd_bwd")
    head.done = True
    global actor_head_launches
    actor_head_launches += 1
    return dz, mu, wpart


def _fuse_out_fwd(ws) -> bool:
    """The last hidden layer and the output layer run as one linear_fwd_out launch (split modes only)."""
    return _FUSE_OUT_FWD and _split() and len(ws) >= 2 and ws[-1].shape[0] <= MAX_OUT_WIDTH \
        and ws[-1].shape[1] % 4 == 0


def linear_dgrad_elu(dz, w, h, img=None, db_out=None):
    """(dz @ w) * ELU'(h) and its column sums; w is the layer weight [N, K] (dz [M, N], h [M, K]); img: B image
    of w^T (x6 arithmetic) or None (exact f32 MFMA).  db_out: optional [K] destination of the column sums."""
    M, N = dz.shape
    K = w.shape[1]
    wt = w.t().contiguous() if img is None else w  # [K, N]: the f32 kernel's B operand rows are the output columns
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    part = torch.empty(K, tiles, device=dz.device, dtype=torch.float32)
    with timer.span(f"linear_dgrad[M={M},Nred={N},K={K}]", dz.device, 4 * M * (N + 2 * K), 2 * M * K * N):
        rc = L.rslrl_linear_dgrad_elu(dz.data_ptr(), M, N, wt.data_ptr(), K, h.data_ptr(), out.data_ptr(),
                                      part.data_ptr(), img.data_ptr() if img is not None else None, _stream(dz))
    _lib.check(rc, "rslrl_linear_dgrad_elu")
    db = _out_or_empty(db_out, (K,), dz.device)
    rc = L.rslrl_column_sum_fold(part.data_ptr(), tiles, K, db.data_ptr(), _stream(dz))
    _lib.check(rc, "rslrl_column_sum_fold")
    return out, db


def _out_or_empty(out, shape, device):
    """A caller-provided destination (contiguous fp32 of `shape`, e.g. a gradient-arena slot) or a new tensor."""
    if out is None:
        return torch.empty(shape, device=device, dtype=torch.float32)
    if tuple(out.shape) != tuple(shape) or not out.is_contiguous() or out.dtype != torch.float32:
        raise ValueError(f"output slot: expected contiguous fp32 {tuple(shape)}, got {tuple(out.shape)}")
    return out


def linear_dgrad_elu_ex(dz, h, img, arith, dz_amax=None, want_amax=False, db_out=None, want_db=True):
    """((dz W) * ELU'(h), its column sums or None, max |out| or None) on the split path; img: the B image of W^T in
    the layout of arith (see linear_fwd_ex).  want_db=False: no column sums (the previous layer's bias gradient
    comes from its weight-gradient kernel)."""
    M, N = dz.shape
    K = h.shape[1]
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    part = torch.empty(K, tiles, device=dz.device, dtype=torch.float32) if want_db else None
    amax = torch.empty(1, device=dz.device, dtype=torch.float32) if want_amax else None
    with timer.span(f"linear_dgrad[M={M},Nred={N},K={K}]{_tag(arith)}", dz.device, 4 * M * (N + 2 * K),
                    2 * M * K * N):
        _gemm(_lib.LINEAR_DGRAD_ELU, arith, dz, dz_amax, K, img, h=h, c=out, colsum=part, amax_out=amax)
    if not want_db:
        return out, None, amax
    db = _out_or_empty(db_out, (K,), dz.device)
    rc = L.rslrl_column_sum_fold(part.data_ptr(), tiles, K, db.data_ptr(), _stream(dz))
    _lib.check(rc, "rslrl_column_sum_fold")
    return out, db, amax


def linear_dgrad_elu_pair(dzs, hs, imgs, arith, dz_amaxes=(None, None), want_amax=(False, False)):
    """linear_dgrad_elu_ex (want_db=False) of two problems of one shape in one launch (rslrl_linear_gemm_pair) --
    e.g. the actor's and the critic's hidden layer l in the update's backward; bit-identical to two launches.
    Returns ([out0, out1], [amax0, amax1])."""
    M, N = dzs[0].shape
    K = hs[0].shape[1]
    outs = [torch.empty(M, K, device=dz.device, dtype=torch.float32) for dz in dzs]
    amaxes = [torch.empty(1, device=dz.device, dtype=torch.float32) if w else None for dz, w in zip(dzs, want_amax)]
    args = [_gemm_args(_lib.LINEAR_DGRAD_ELU, arith, dzs[i], dz_amaxes[i], K, imgs[i], h=hs[i], c=outs[i],
                       amax_out=amaxes[i], slot=i) for i in range(2)]
    with timer.span(f"linear_dgrad_pair[M={M},Nred={N},K={K}]{_tag(arith)}", dzs[0].device, 8 * M * (N + 2 * K),
                    4 * M * K * N):
        rc = _lib.lib().rslrl_linear_gemm_pair(ctypes.byref(args[0]), ctypes.byref(args[1]), _stream(dzs[0]))
    _lib.check(rc, "rslrl_linear_gemm_pair")
    return outs, amaxes


def linear_dgrad_elu_wgrad(dz, w, h, img, want_amax=False, db_prev_out=None, dwb_out=None, want_db_prev=True):
    """Output-layer backward in one launch (x6; dz [M, Nred <= 16] contiguous -- any Nred, e.g. the value head's
    [M, 1] gradient unpadded): ((dz @ w) * ELU'(h), its column sums, dz^T h).  w is the layer weight [Nred, K] (only
    its image is read).  db_prev_out: optional [K] destination of the column sums; dwb_out: optional [Nred*K + Nred]
    destination of dW (row-major) followed by db -- the layout of a Linear's weight and bias adjacent in a gradient
    arena (used when Nred*K + Nred is a multiple of 4, the kernel's padded partial row)."""
    M, N = dz.shape
    K = h.shape[1]
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    P = (N * K + N + 3) // 4 * 4  # per tile: dW [N, K], then db [N], then zeros
    out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    part = torch.empty(K, tiles, device=dz.device, dtype=torch.float32) if want_db_prev else None
    wpart = torch.empty(tiles, P, device=dz.device, dtype=torch.float32)
    amax = torch.empty(1, device=dz.device, dtype=torch.float32) if want_amax else None
    with timer.span(f"linear_dgrad_wgrad[M={M},Nred={N},K={K}]", dz.device, 4 * M * (N + 2 * K), 4 * M * K * N):
        _gemm(_lib.LINEAR_DGRAD_ELU_WGRAD, _lib.ARITH_X6, dz, None, K, img, h=h, c=out, colsum=part, wpart=wpart,
              amax_out=amax)
    db = None
    if want_db_prev:
        db = _out_or_empty(db_prev_out, (K,), dz.device)
        rc = L.rslrl_column_sum_fold(part.data_ptr(), tiles, K, db.data_ptr(), _stream(dz))
        _lib.check(rc, "rslrl_column_sum_fold")
    dwb = _out_or_empty(dwb_out, (N * K + N,), dz.device)  # the fold writes exactly dW then db (no pad)
    nbytes = L.rslrl_fold_partials_workspace_bytes(tiles, P)
    ws = torch.empty(max(nbytes, 16) // 8, dtype=torch.float64, device=dz.device)
    rc = L.rslrl_fold_partials_ex(wpart.data_ptr(), tiles, P, dwb.data_ptr(), N * K + N, 0, 0, ws.data_ptr(), nbytes,
                                  _stream(dz))
    _lib.check(rc, "rslrl_fold_partials_ex")
    dw, db_out = dwb[: N * K].view(N, K), dwb[N * K:]
    if want_amax:
        return out, db, dw, db_out, amax
    return out, db, dw, db_out


def linear_dgrad_elu_wgrad_pair(dzs, hs, imgs, dwb_outs=(None, None), defer=None):
    """linear_dgrad_elu_wgrad (want_db_prev=False, no amax) of two output layers over the same rows and hidden width
    in one launch (rslrl_linear_gemm_pair, RSLRL_LINEAR_DGRAD_ELU_WGRAD; the reduction widths may differ, e.g. 12
    actions and the value head).  Returns per problem (dz_prev, dw, db).  defer: a _FoldBatch -- the weight-gradient
    folds are queued there (dw, db valid after its run()) instead of launched here."""
    M, K = hs[0].shape
    L = _lib.lib()
    tiles = L.rslrl_linear_tiles(M)
    outs, wparts, dwbs = [], [], []
    for i in range(2):
        N = dzs[i].shape[1]
        P = (N * K + N + 3) // 4 * 4
        outs.append(torch.empty(M, K, device=dzs[i].device, dtype=torch.float32))
        wparts.append(torch.empty(tiles, P, device=dzs[i].device, dtype=torch.float32))
        dwbs.append(_out_or_empty(dwb_outs[i], (N * K + N,), dzs[i].device))
    args = [_gemm_args(_lib.LINEAR_DGRAD_ELU_WGRAD, _lib.ARITH_X6, dzs[i], None, K, imgs[i], h=hs[i], c=outs[i],
                       wpart=wparts[i]) for i in range(2)]
    nred = dzs[0].shape[1] + dzs[1].shape[1]
    with timer.span(f"linear_dgrad_wgrad_pair[M={M},Nred={nred},K={K}]", dzs[0].device, 4 * M * (nred + 4 * K),
                    4 * M * K * nred):
        rc = L.rslrl_linear_gemm_pair(ctypes.byref(args[0]), ctypes.byref(args[1]), _stream(dzs[0]))
    _lib.check(rc, "rslrl_linear_gemm_pair")
    res = []
    for i in range(2):
        N = dzs[i].shape[1]
        P = wparts[i].shape[1]
        if defer is not None:
            defer.add(wparts[i], tiles, P, dwbs[i], N * K + N)
            res.append((outs[i], dwbs[i][: N * K].view(N, K), dwbs[i][N * K:]))
            continue
        nbytes = L.rslrl_fold_partials_workspace_bytes(tiles, P)
        ws = torch.empty(max(nbytes, 16) // 8, dtype=torch.float64, device=dzs[i].device)
        rc = L.rslrl_fold_partials_ex(wparts[i].data_ptr(), tiles, P, dwbs[i].data_ptr(), N * K + N, 0, 0,
                                      ws.data_ptr(), nbytes, _stream(dzs[i]))
        _lib.check(rc, "rslrl_fold_partials_ex")
        res.append((outs[i], dwbs[i][: N * K].view(N, K), dwbs[i][N * K:]))
    return res


def linear_dgrad_elu_wgrad_deferred(dz, h, img, dwb_out, defer):
    """linear_dgrad_elu_wgrad (want_db_prev=False, no amax) of one output layer with its fold queued on `defer` (a
    _FoldBatch); bit-identical input gradient to problem 0 of linear_dgrad_elu_wgrad_pair.  Returns (dz_prev, dw, db)
    (dw, db valid after defer.run())."""
    M, N = dz.shape
    K = h.shape[1]
    tiles = _lib.lib().rslrl_linear_tiles(M)
    P = (N * K + N + 3) // 4 * 4
    out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    wpart = torch.empty(tiles, P, device=dz.device, dtype=torch.float32)
    dwb = _out_or_empty(dwb_out, (N * K + N,), dz.device)
    with timer.span(f"linear_dgrad_wgrad[M={M},Nred={N},K={K}]", dz.device, 4 * M * (N + 2 * K), 4 * M * K * N):
        _gemm(_lib.LINEAR_DGRAD_ELU_WGRAD, _lib.ARITH_X6, dz, None, K, img, h=h, c=out, wpart=wpart)
    defer.add(wpart, tiles, P, dwb, N * K + N)
    return out, dwb[: N * K].view(N, K), dwb[N * K:]


def _head_result(tape, dwb_out, defer):
    """(dz_prev, dw, db) of a tape whose head ran fused (value_head_fwd_bwd: 1 output, actor_head_fwd_bwd: 12): its
    dz, and the fold of its [dW | db] partials queued on `defer`."""
    dz, wpart = tape.head[:2]
    nred = tape.head[2] if len(tape.head) > 2 else 1
    K = dz.shape[1]
    dwb = _out_or_empty(dwb_out, (nred * K + nred,), dz.device)
    defer.add(wpart, wpart.shape[0], wpart.shape[1], dwb, nred * K + nred)
    return dz, dwb[:nred * K].view(nred, K), dwb[nred * K:]


def linear_wgrad(dz, x, arith=_lib.ARITH_X6, dz_amax=None, x_amax=None, out=None, bias_side=0, dwb_out=None):
    """dz^T x ([N, K]) on the split weight-gradient kernel (x6, or h3 with max |dz|, max |x| as device scalars);
    dz [M, N], x [M, K], N, K <= 256 and 4-aligned.  out: optional [N, K] destination.
    bias_side 1 / 2: also the column sums of dz (N values) / of x (K values) from the same kernel -- returns
    (dw, colsum); dwb_out: optional [N*K + E] destination of both (a Linear's adjacent arena slots)."""
    M, N = dz.shape
    K = x.shape[1]
    L = _lib.lib()
    nbytes = L.rslrl_linear_wgrad_bias_workspace_bytes(M, N, K, bias_side)
    ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dz.device)
    E = N if bias_side == 1 else (K if bias_side == 2 else 0)
    if bias_side:
        dwb = _out_or_empty(dwb_out, (N * K + E,), dz.device)
    else:
        dwb = _out_or_empty(out, (N, K), dz.device)
    if arith == _lib.ARITH_H3:
        dz_amax = _amax(dz) if dz_amax is None else dz_amax
        x_amax = _amax(x) if x_amax is None else x_amax
    with timer.span(f"linear_wgrad[M={M},N={N},K={K}]{_tag(arith)}", dz.device, 4 * M * (N + K), 2 * M * K * N):
        rc = L.rslrl_linear_wgrad_bias(dz.data_ptr(), _ptr(dz_amax), x.data_ptr(), _ptr(x_amax), M, N, K, arith,
                                       bias_side, dwb.data_ptr(), ws.data_ptr(), nbytes, _stream(dz))
    _lib.check(rc, "rslrl_linear_wgrad_bias")
    if not bias_side:
        return dwb
    return dwb[: N * K].view(N, K), dwb[N * K:]


def linear_wgrad_pair(dzs, xs, arith=_lib.ARITH_X6, bias_side=0, dwb_outs=(None, None), amaxes=((None, None),) * 2,
                      transpose_out=False, defer=None):
    """linear_wgrad of two problems of one shape in one launch (rslrl_linear_wgrad_bias_pair): returns, per problem,
    dw (bias_side 0) or (dw, colsum).  dwb_outs: optional [N*K + E] destinations (a Linear's adjacent arena slots);
    amaxes: per problem (max |dz|, max |x|) device scalars for h3.  transpose_out: dw is delivered as dw^T ([K, N],
    the first layer's (x^T dz)^T form written straight in W's layout).  defer: a _FoldBatch -- the folds are queued
    there (the results are valid after its run()) instead of launched here."""
    M, N = dzs[0].shape
    K = xs[0].shape[1]
    L = _lib.lib()
    nbytes = L.rslrl_linear_wgrad_bias_pair_workspace_bytes(M, N, K, bias_side)
    E = N if bias_side == 1 else (K if bias_side == 2 else 0)
    wss, dwbs, probs = [], [], []
    for i in range(2):
        ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dzs[i].device)
        dwb = _out_or_empty(dwb_outs[i], (N * K + E,), dzs[i].device)
        da, xa = amaxes[i]
        if arith == _lib.ARITH_H3:
            da = _amax(dzs[i]) if da is None else da
            xa = _amax(xs[i]) if xa is None else xa
        wss.append(ws)
        dwbs.append(dwb)
        probs.append(_lib.WgradProblem(dzs[i].data_ptr(), _ptr(da), xs[i].data_ptr(), _ptr(xa), dwb.data_ptr(),
                                       ws.data_ptr(), nbytes, 1 if transpose_out else 0))
    with timer.span(f"linear_wgrad_pair[M={M},N={N},K={K}]{_tag(arith)}", dzs[0].device, 8 * M * (N + K),
                    4 * M * K * N):
        rc = L.rslrl_linear_wgrad_bias_pair(ctypes.byref(probs[0]), ctypes.byref(probs[1]), M, N, K, arith,
                                            bias_side, _lib.WGRAD_NO_FOLD if defer is not None else 0,
                                            _stream(dzs[0]))
    _lib.check(rc, "rslrl_linear_wgrad_bias_pair")
    if defer is not None:
        S = L.rslrl_linear_wgrad_bias_pair_slices(M, N)
        for i in range(2):
            defer.add(wss[i], S, N * K + E, dwbs[i], N * K + E, (N, K) if transpose_out else None)
    shape = (K, N) if transpose_out else (N, K)
    if not bias_side:
        return [d.view(*shape) for d in dwbs]
    return [(d[: N * K].view(*shape), d[N * K:]) for d in dwbs]


# RSLRL_HIDDEN_BWD=0 keeps the square hidden layers' input and weight gradients in separate launches (A/B)
_HIDDEN_BWD = os.environ.get("RSLRL_HIDDEN_BWD", "1") != "0"
HIDDEN_BWD_WIDTH = 256


def hidden_bwd_ok(dzs, hs) -> bool:
    """hidden_bwd_pair covers the problems: x6, a 256 x 256 hidden layer, M a multiple of 64, contiguous operands."""
    M, N = dzs[0].shape
    return (N == HIDDEN_BWD_WIDTH and hs[0].shape[1] == HIDDEN_BWD_WIDTH and M % 64 == 0 and M >= 64
            and all(t.is_contiguous() and t.shape == (M, HIDDEN_BWD_WIDTH) and t.data_ptr() % 16 == 0
                    for t in list(dzs) + list(hs)))


def hidden_bwd_pair(dzs, hs, imgs, dwb_outs=(None, None), defer=None):
    """The backward of a square hidden layer (Linear(256, 256) + ELU) of one or two problems over the same rows in one
    launch (rslrl_hidden_bwd_pair, csrc/mlp_bwd_fused.hip): per problem dz_prev = (dz W) * ELU'(h) -- the bits of
    linear_dgrad_elu_pair -- and [dW | db] = [dz^T h | sum dz] from the same read of dz and h (the weight gradient of
    linear_wgrad_pair(bias_side=1), summed in another order: fp32-close).  imgs: the x6 images of W^T (the tapes'
    dgrad images).  dwb_outs: optional [256 * 256 + 256] destinations (adjacent arena slots); defer: a _FoldBatch --
    the folds are queued there (dW, db valid after its run()).  Returns per problem (dz_prev, dw, db)."""
    n = len(dzs)
    M = dzs[0].shape[0]
    W = HIDDEN_BWD_WIDTH
    L = _lib.lib()
    S = L.rslrl_hidden_bwd_slices(M)
    NK = L.rslrl_hidden_bwd_partial_floats()
    dev = dzs[0].device
    outs, parts, dwbs, probs = [], [], [], []
    for i in range(n):
        outs.append(torch.empty(M, W, device=dev, dtype=torch.float32))
        parts.append(torch.empty(S, NK, device=dev, dtype=torch.float32))
        dwbs.append(_out_or_empty(dwb_outs[i] if i < len(dwb_outs) else None, (NK,), dev))
        probs.append(_lib.HiddenBwdProblem(dzs[i].data_ptr(), hs[i].data_ptr(), imgs[i].data_ptr(),
                                           outs[i].data_ptr(), parts[i].data_ptr()))
    with timer.span(f"linear_hidden_bwd{'_pair' if n == 2 else ''}[M={M},N={W},K={W}]", dev, n * 4 * M * 3 * W,
                    n * 4 * M * W * W):
        rc = L.rslrl_hidden_bwd_pair(ctypes.byref(probs[0]), ctypes.byref(probs[1]) if n == 2 else None, M, W,
                                     _stream(dzs[0]))
    _lib.check(rc, "rslrl_hidden_bwd_pair")
    res = []
    for i in range(n):
        if defer is not None:
            defer.add(parts[i], S, NK, dwbs[i], NK)
        else:
            nbytes = L.rslrl_fold_partials_workspace_bytes(S, NK)
            ws = torch.empty(max(nbytes, 16) // 8, dtype=torch.float64, device=dev)
            rc = L.rslrl_fold_partials_ex(parts[i].data_ptr(), S, NK, dwbs[i].data_ptr(), NK, 0, 0, ws.data_ptr(),
                                          nbytes, _stream(dzs[i]))
            _lib.check(rc, "rslrl_fold_partials_ex")
        res.append((outs[i], dwbs[i][: W * W].view(W, W), dwbs[i][W * W:]))
    return res


def _weight_grad(dz, x, x6: bool, h3=False, dz_amax=None, x_amax=None, out=None, want_bias=False, db_out=None):
    # the split weight-gradient kernel computes TN x 256 tiles (TN = 32, 64 or 256 rows of its first operand):
    # the square hidden layers run it as dz^T x (h3 when both operands come from h3-layer producers); the first
    # layer (input width <= 64) as (x^T dz)^T on the 64-row tiles (x6); the narrow output layers stay on the
    # split-K batched GEMM (networks/linear.py) unless their backward is fused (linear_dgrad_elu_wgrad).
    # out: optional [N, K] destination (written directly where the kernel's layout allows, else copied).
    # want_bias: also the bias gradient (column sums of dz) from the same kernel where it has one of the two
    # split forms (bias_from_wgrad) -- returns (dw, db or None); db_out: its optional destination.
    def deliver(res):
        if out is None:
            return res if res.is_contiguous() else res.contiguous()
        out.copy_(res)
        return out

    def deliver_b(db):
        if db_out is None:
            return db
        db_out.copy_(db)
        return db_out

    form = _wgrad_form(dz.shape[1], x.shape[1], x6)
    if form == "first":
        pad = (-x.shape[1]) % 4
        xp = F.pad(x, (0, pad)) if pad else x
        if want_bias:  # (x^T dz)^T: the bias is the column sums of dz, here the kernel's K side
            dwt, db = linear_wgrad(xp, dz, bias_side=2)
            return deliver(dwt[: x.shape[1]].t()), deliver_b(db)
        return deliver(linear_wgrad(xp, dz)[: x.shape[1]].t()), None
    if form == "square":
        pad = (-dz.shape[1]) % 4
        if pad:  # the critic's 1-wide output
            return deliver(linear_wgrad(F.pad(dz, (0, pad)), x)[: dz.shape[1]]), None
        arith = _lib.ARITH_H3 if h3 else _lib.ARITH_X6
        if want_bias and dz.shape[1] > 64:
            N, K = dz.shape[1], x.shape[1]
            adjacent = (out is not None and db_out is not None and out.is_contiguous() and db_out.is_contiguous()
                        and db_out.data_ptr() == out.data_ptr() + 4 * out.numel())
            dwb_out = torch.as_strided(out, (N * K + N,), (1,)) if adjacent else None
            dw, db = linear_wgrad(dz, x, arith, dz_amax, x_amax, bias_side=1, dwb_out=dwb_out)
            if adjacent:
                return out, db_out
            return deliver(dw), deliver_b(db)
        return linear_wgrad(dz, x, arith, dz_amax, x_amax, out=out), None
    return deliver(_splitk_weight_grad(dz, x)), None


def _wgrad_form(n_dz: int, n_x: int, x6: bool):
    """Which weight-gradient kernel form _weight_grad takes for an output gradient n_dz wide and an input n_x wide:
    "first" ((x^T dz)^T, input width <= 64), "square" (dz^T x) or None (the split-K fallback)."""
    if x6 and n_dz > 64 and n_x <= 64 and n_dz <= MAX_WIDTH and n_dz % 4 == 0:
        return "first"
    if x6 and n_dz > 32 and n_x > 64 and n_dz <= MAX_WIDTH and n_x <= MAX_WIDTH and n_x % 4 == 0:
        return "square"
    return None


def _bias_from_wgrad(n_dz: int, n_x: int, x6: bool) -> bool:
    """A layer whose output gradient is n_dz wide gets its bias gradient from the weight-gradient kernel (the column
    sums of the dz it stages) instead of from the next layer's input-gradient epilogue + a fold."""
    form = _wgrad_form(n_dz, n_x, x6)
    return form == "first" or (form == "square" and n_dz > 64 and n_dz % 4 == 0)


def _plan(ws):
    """Per-layer arithmetic of a forward/backward pass in the current mode: returns (split, h3 flags per linear
    layer l, fuse_out).  h3[l]: layer l's hidden GEMMs (forward; weight gradient; input gradient) run on h3 --
    every layer whose input is a hidden activation, except the output layer (x6: its narrow GEMMs are
    memory-bound and its fused backward is an x6 kernel)."""
    split = _split()
    nh = len(ws) - 1
    h3 = [_mode == GEMM_H3 and 0 < l < nh for l in range(len(ws))]
    return split, h3, _fuse_out_fwd(ws)


def _forward_images(ws, h3, fuse_out, backward: bool):
    nh = len(ws) - 1
    lay = lambda l: _lib.BIMAGE_LAYOUT_H3 if h3[l] else _lib.BIMAGE_LAYOUT_GEMM  # noqa: E731
    specs = [(w, False, lay(l)) for l, w in enumerate(ws[:-1])]
    if backward:  # transposed images of layers 1..L-1 for the input gradients
        specs += [(w, True, lay(l)) for l, w in enumerate(ws) if l > 0]
    if fuse_out:
        specs.append((ws[-1], False, _lib.BIMAGE_LAYOUT_OUT))
    imgs = bimages(specs)
    fwd = imgs[:nh]
    dgrad = [None] + imgs[nh:2 * nh] if backward else None
    out = imgs[-1] if fuse_out else None
    return fwd, dgrad, out


def _hidden_forward(x, ws, bs, h3, fuse_out, fwd_imgs, out_img, keep: bool):
    """Hidden layers (+ the fused output layer).  Returns (hs, amaxes, y): hs[l] = input of linear l (only
    stored when keep), amaxes[l] = max |hs[l]| when an h3 consumer needs it, y = output (None unless fused)."""
    nh = len(ws) - 1
    arith = lambda l: _lib.ARITH_H3 if h3[l] else _lib.ARITH_X6  # noqa: E731
    hs, amaxes = [x], [None]
    h, y = x, None
    for l in range(nh):
        # max |H_{l+1}| is needed when linear l+1 (a hidden layer) is h3: its forward, and in backward its
        # weight gradient
        want = l + 1 < nh and h3[l + 1]
        if fuse_out and l == nh - 1:
            h, y = linear_fwd_out_ex(h, bs[l], ws[l].shape[0], fwd_imgs[l], arith(l), amaxes[l], bs[-1], out_img,
                                     store_h=keep)
            amax = None
        else:
            h, amax = linear_fwd_ex(h, bs[l], ws[l].shape[0], True, fwd_imgs[l], arith(l), amaxes[l], want)
        hs.append(h)
        amaxes.append(amax)
    return hs, amaxes, y


class MLPTape:
    """What the backward of one MLP pass needs: the layer inputs (hs[l] = input of linear l), the weights, the
    transposed B images of the input gradients, the published max |H| of h3 layers and the per-layer plan."""

    __slots__ = ("hs", "ws", "dgrad_imgs", "amaxes", "h3", "x6", "head")

    def __init__(self, hs, ws, dgrad_imgs, amaxes, h3, x6, head=None):
        self.hs, self.ws, self.dgrad_imgs, self.amaxes, self.h3, self.x6 = hs, ws, dgrad_imgs, amaxes, h3, x6
        self.head = head  # (dz of the last hidden layer, the head's weight-gradient partials): value_head_fwd_bwd


def train_forward(x, ws, bs):
    """y = MLP(x) for hidden ELU(alpha=1) layers (ws/bs: the Linear weights and biases), keeping what the backward
    needs.  Returns (y, MLPTape)."""
    split, h3, fuse_out = _plan(ws)
    nh = len(ws) - 1
    if split:
        fwd_imgs, dgrad_imgs, out_img = _forward_images(ws, h3, fuse_out, backward=True)
        hs, amaxes, y = _hidden_forward(x, ws, bs, h3, fuse_out, fwd_imgs, out_img, keep=True)
    else:
        hs, amaxes, h = [x], [None] * (nh + 1), x
        for l in range(nh):
            h = linear_fwd(h, ws[l], bs[l], elu=True)
            hs.append(h)
        dgrad_imgs, y = [None] * (nh + 1), None
    if y is None:
        y = F.linear(hs[-1], ws[-1], bs[-1])
    return y, MLPTape(hs, list(ws), dgrad_imgs, amaxes, h3, split)


def train_backward(tape, dy, need_dx=False, need_w=None, outs=None, dy_padded=None):
    """Gradients of one MLP pass: returns (dx or None, [dW_l], [db_l]).  need_w[l]: layer l's weight gradient is
    wanted (default: all).  outs[l] = (dW destination, db destination) or None: contiguous fp32 tensors the
    gradients are written into (a gradient arena's slots) instead of new tensors.  dy_padded: optional contiguous
    [B, 4k] tensor whose first columns are dy and the rest zero (the fused output-layer backward's operand; dy
    may then be a strided view of it) -- saves the pad copy of a narrow head such as the value head."""
    hs, ws, h3 = tape.hs, tape.ws, tape.h3
    L = len(ws)
    need_w = [True] * L if need_w is None else need_w
    outs = [None] * L if outs is None else outs
    w_out = lambda l: outs[l][0] if outs[l] is not None else None  # noqa: E731
    b_out = lambda l: outs[l][1] if outs[l] is not None else None  # noqa: E731
    grads_w = [None] * L
    grads_b = [None] * L
    # hidden layers whose bias gradient comes out of their own weight-gradient kernel (x6 forms): the next layer's
    # input-gradient epilogue then skips its column sums and their fold
    bias_wg = [l < L - 1 and need_w[l] and _bias_from_wgrad(ws[l].shape[0], hs[l].shape[1], tape.x6)
               for l in range(L)]
    if dy_padded is not None and not (dy_padded.is_contiguous() and dy_padded.shape[0] == dy.shape[0]
                                      and dy_padded.shape[1] == dy.shape[1] + (-dy.shape[1]) % 4):
        raise ValueError("train_backward: dy_padded must be contiguous [B, round_up(dy width, 4)]")
    dz = dy if dy_padded is not None else dy.contiguous()
    dz_amax = None
    dx = None
    for l in range(L - 1, -1, -1):
        h_in = hs[l]
        fuse_w = (_FUSE_OUT and tape.x6 and l == L - 1 and l > 0 and dz.shape[1] <= 16 and h_in.shape[1] <= MAX_WIDTH
                  and need_w[l])
        if dy_padded is not None and l == L - 1 and not fuse_w:
            dz = dz.contiguous()
        if fuse_w:  # output layer: dgrad + ELU' + bias grad + weight grad over one read of h (one launch)
            nred = dz.shape[1]
            K = h_in.shape[1]
            # the kernel reads any Nred <= 16 (no pad copy) and its fold writes exactly [dW | db]; a caller's padded
            # operand computes the padded rows too (dropped below)
            dzp = dy_padded if dy_padded is not None else dz
            pad = dzp.shape[1] - nred
            want = l - 1 > 0 and h3[l - 1]
            # the kernel's [dW | db] result lands directly in the arena when weight and bias are adjacent there
            dwb_out = None
            wo, bo = w_out(l), b_out(l)
            if not pad and wo is not None and bo is not None and wo.is_contiguous() \
                    and bo.data_ptr() == wo.data_ptr() + 4 * wo.numel():
                dwb_out = torch.as_strided(wo, (nred * K + nred,), (1,))
            res = linear_dgrad_elu_wgrad(dzp, ws[l], h_in, tape.dgrad_imgs[l], want_amax=want,
                                         db_prev_out=b_out(l - 1), dwb_out=dwb_out, want_db_prev=not bias_wg[l - 1])
            dz, grads_b[l - 1], dw, db_out = res[:4]
            dz_amax = res[4] if want else None
            if dwb_out is not None:
                grads_w[l], grads_b[l] = wo, bo
            else:
                grads_w[l], grads_b[l] = dw[:nred], db_out[:nred]
                if wo is not None and bo is not None:  # one multi-tensor copy launch for both
                    torch._foreach_copy_([wo, bo], [grads_w[l], grads_b[l]])
                    grads_w[l], grads_b[l] = wo, bo
                else:
                    if wo is not None:
                        wo.copy_(grads_w[l])
                        grads_w[l] = wo
                    if bo is not None:
                        bo.copy_(grads_b[l])
                        grads_b[l] = bo
            continue
        if l == L - 1:
            grads_b[l] = dz.sum(0) if b_out(l) is None else torch.sum(dz, 0, out=b_out(l))
        if need_w[l]:
            grads_w[l], db = _weight_grad(dz, h_in, tape.x6, h3[l], dz_amax, tape.amaxes[l], out=w_out(l),
                                          want_bias=bias_wg[l], db_out=b_out(l))
            if bias_wg[l]:
                grads_b[l] = db
        if l == 0:
            dx = dz.mm(ws[0]) if need_dx else None
            break
        # dZ_{l-1} = (dZ_l W_l) * ELU'(H_{l-1}), db_{l-1} = column sums; a reduction width that is not a
        # multiple of 4 (the critic's 1-wide output) is zero-padded to the next multiple (the x6 image
        # zero-fills the weight side itself)
        w = ws[l]
        img = tape.dgrad_imgs[l]
        pad = (-dz.shape[1]) % 4
        if pad:
            dz = F.pad(dz, (0, pad))
            if img is None:
                w = F.pad(w, (0, 0, 0, pad))
        want_db = not bias_wg[l - 1]
        if h3[l]:
            want = l - 1 > 0 and h3[l - 1]
            dz_amax = _amax(dz) if dz_amax is None else dz_amax
            dz, db, dz_amax = linear_dgrad_elu_ex(dz, h_in, img, _lib.ARITH_H3, dz_amax, want,
                                                  db_out=b_out(l - 1), want_db=want_db)
        elif img is not None:
            want = l - 1 > 0 and h3[l - 1]
            dz, db, dz_amax = linear_dgrad_elu_ex(dz, h_in, img, _lib.ARITH_X6, None, want, db_out=b_out(l - 1),
                                                  want_db=want_db)
        else:
            dz, db = linear_dgrad_elu(dz, w, h_in, None, db_out=b_out(l - 1))
            dz_amax = None
        if want_db or img is None:
            grads_b[l - 1] = db
    return dx, grads_w, grads_b


def _kernels_ws():
    from ..kernels import _ws
    return _ws


class _FoldBatch:
    """Weight-gradient folds queued during a backward pass and launched together (rslrl_fold_partials_batch): no fold
    is needed before the optimizer step, so the pass's 8 folds (4 layers x 2 networks) take one launch."""

    def __init__(self):
        self.jobs, self.keep, self.after = [], [], []

    def add(self, partials, S, NK, out, out_len, transpose=None):
        t_rows, t_cols = transpose if transpose is not None else (0, 0)
        self.jobs.append(_lib.FoldJob(partials.data_ptr(), S, NK, out.data_ptr(), out_len, t_rows, t_cols))
        self.keep += [partials, out]

    def run(self, device):
        L = _lib.lib()
        for start in range(0, len(self.jobs), _lib.MAX_FOLD_JOBS):
            part = self.jobs[start:start + _lib.MAX_FOLD_JOBS]
            arr = (_lib.FoldJob * len(part))(*part)
            st = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
            nbytes = L.rslrl_fold_partials_batch_workspace_bytes(arr, len(part))
            ws = _kernels_ws().get(device, "fold_batch", nbytes)  # zero-filled once, counters left zero
            _lib.check(L.rslrl_fold_partials_batch(arr, len(part), ws.data_ptr(), ws.numel(), st),
                       "rslrl_fold_partials_batch")
        for fn in self.after:
            fn()
        self.jobs, self.keep, self.after = [], [], []


# ---- the actor and the critic of the PPO update as one pass (same-shape hidden layers batched per launch)
def _pairable(ws_a, ws_c, x_a, x_c) -> bool:
    """Two MLPs whose hidden layers can share launches: the split (x6) arithmetic without h3 layers, the same depth
    and hidden shapes, the same batch, both output layers fused (<= 16 wide, hidden width <= 256)."""
    if _PAIR_TRAIN is False or _mode != GEMM_X6 or not _split():
        return False
    if len(ws_a) != len(ws_c) or len(ws_a) < 3 or x_a.shape[0] != x_c.shape[0]:
        return False
    if any(a.shape != c.shape for a, c in zip(ws_a[:-1], ws_c[:-1])):
        return False
    if not (_fuse_out_fwd(ws_a) and _fuse_out_fwd(ws_c)):
        return False
    return all(w.shape[0] <= 16 and w.shape[1] <= MAX_WIDTH for w in (ws_a[-1], ws_c[-1]))


def train_forward_pair(x_a, ws_a, bs_a, x_c, ws_c, bs_c, value_head: ValueHead | None = None,
                       actor_head: ActorHead | None = None):
    """train_forward of the actor (x_a, ws_a, bs_a) and the critic (x_c, ...) with each same-shape hidden layer of the
    two in one launch (rslrl_linear_gemm_pair) and every B image of both passes in one launch; the output layers run
    as two fused launches.  Values identical to two train_forward calls.  Returns (y_a, tape_a, y_c, tape_c), or None
    when the pair does not qualify (_pairable).

    value_head: the mini-batch's value-loss inputs -- the critic's last launch then also runs the value loss's gradient
    and the value head's backward (value_head_fwd_bwd): its tape carries the last hidden layer's dz instead of that
    layer's activation, and train_backward_pair ignores the critic's dy (the same values the loss kernel writes).
    actor_head (with value_head): the PPO loss inputs -- the critic's launch then runs first and the actor's last
    launch also runs the whole loss and the output layer's backward (actor_head_fwd_bwd; actor_head.done tells whether
    it ran, in which case the loss statistics and d sigma are written and the actor's tape carries its head)."""
    if not _pairable(ws_a, ws_c, x_a, x_c):
        return None
    ws, bs, xs = (ws_a, ws_c), (bs_a, bs_c), (x_a, x_c)
    nh = len(ws_a) - 1
    h3 = [False] * len(ws_a)
    specs = []
    for i in range(2):  # per pass: forward images of layers 0..nh-1, transposed images of 1..nh, the output image
        specs += [(w, False) for w in ws[i][:-1]] + [(w, True) for w in ws[i][1:]]
        specs.append((ws[i][-1], False, _lib.BIMAGE_LAYOUT_OUT))
    imgs = bimages(specs)
    per = 2 * nh + 1
    fwd = [imgs[i * per: i * per + nh] for i in range(2)]
    dgr = [[None] + imgs[i * per + nh: i * per + 2 * nh] for i in range(2)]
    out_img = [imgs[i * per + 2 * nh] for i in range(2)]
    h = [x if x.is_contiguous() else x.contiguous() for x in xs]
    hs = [[h[0]], [h[1]]]
    y = [None, None]
    head = head_a = None
    for l in range(nh):
        if l < nh - 1:
            h, _ = linear_fwd_pair(h, [bs[0][l], bs[1][l]], ws[0][l].shape[0], True, [fwd[0][l], fwd[1][l]],
                                   _lib.ARITH_X6, [None, None], [False, False])
        else:
            # the critic first when the actor's head runs the loss (it reads the values)
            fuse_actor = actor_head is not None and value_head is not None and _VALUE_HEAD and _ACTOR_HEAD
            for i in ((1, 0) if fuse_actor else (0, 1)):
                if i == 1 and value_head is not None and _VALUE_HEAD:
                    res = value_head_fwd_bwd(h[1], bs[1][l], ws[1][l].shape[0], fwd[1][l], bs[1][-1], out_img[1],
                                             ws[1][-1], value_head)
                    if res is not None:
                        head, y[1], h[1] = (res[0], res[2]), res[1], None
                        continue
                if i == 0 and fuse_actor and head is not None:
                    actor_head.values = y[1]
                    res = actor_head_fwd_bwd(h[0], bs[0][l], ws[0][l].shape[0], fwd[0][l], bs[0][-1], out_img[0],
                                             dgr[0][nh], actor_head)
                    if res is not None:
                        head_a, y[0], h[0] = (res[0], res[2], _lib.ACTOR_HEAD_ACTIONS), res[1], None
                        continue
                h[i], y[i] = linear_fwd_out_ex(h[i], bs[i][l], ws[i][l].shape[0], fwd[i][l], _lib.ARITH_X6, None,
                                               bs[i][-1], out_img[i], store_h=True)
        for i in range(2):
            hs[i].append(h[i])
    tapes = [MLPTape(hs[i], list(ws[i]), dgr[i], [None] * (nh + 1), h3, True) for i in range(2)]
    tapes[1].head = head
    tapes[0].head = head_a
    return y[0], tapes[0], y[1], tapes[1]


def train_backward_pair(tape_a, dy_a, outs_a, tape_c, dy_c, outs_c, on_early=None):
    """train_backward of two passes of train_forward_pair, gradients into outs_* (per layer (dW, db) destinations,
    as train_backward's outs): the output layers as two fused launches, then per hidden layer the two weight
    gradients (rslrl_linear_wgrad_bias_pair) and the two input gradients (rslrl_linear_gemm_pair) in one launch each.
    Input gradients are bit-identical to two train_backward calls; a weight gradient's fp32 slice partials cover
    twice the rows (half the slices), so its rounding differs within fp32 accumulation error.  Returns False (nothing
    done) when the tapes do not qualify.  on_early: called after every layer's gradient but the first layers' is
    enqueued (their folds run first, in a launch of their own) -- a multi-GPU update starts its all-reduce there."""
    tapes, dys, outs = (tape_a, tape_c), (dy_a, dy_c), (outs_a, outs_c)
    L = len(tape_a.ws)
    if not (tape_a.x6 and tape_c.x6 and not any(tape_a.h3) and not any(tape_c.h3) and len(tape_c.ws) == L
            and _FUSE_OUT and all(o is not None and all(t is not None for t in o) for ob in outs for o in ob)):
        return False
    if not all(_bias_from_wgrad(t.ws[l].shape[0], t.hs[l].shape[1], True) for t in tapes for l in range(L - 1)):
        return False
    # output layers: dgrad + ELU' + their weight and bias gradients over one read of h, both in one launch
    ds = [d if d.is_contiguous() else d.contiguous() for d in dys]
    K = tape_a.ws[L - 1].shape[1]  # (hs[L - 1] is None behind a fused head)
    dwb_outs, adjacent = [], []
    for i in range(2):
        nred = ds[i].shape[1]
        wo, bo = outs[i][L - 1]
        adj = wo.is_contiguous() and bo.data_ptr() == wo.data_ptr() + 4 * wo.numel()
        adjacent.append(adj)
        dwb_outs.append(torch.as_strided(wo, (nred * K + nred,), (1,)) if adj else None)
    folds = _FoldBatch()
    # RSLRL_FOLD_EAGER=1 (read per call): each weight-gradient launch's folds run right behind it, while its partials
    # are still in the Infinity Cache, instead of one batched fold after the pass (which reads them back from HBM)
    eager = os.environ.get("RSLRL_FOLD_EAGER", "0") == "1"
    if tape_c.head is not None:  # the critic's head ran its backward in the forward launch (value_head_fwd_bwd)
        res = [_head_result(tape_a, dwb_outs[0], folds) if tape_a.head is not None else  # actor_head_fwd_bwd
               linear_dgrad_elu_wgrad_deferred(ds[0], tape_a.hs[L - 1], tape_a.dgrad_imgs[L - 1], dwb_outs[0], folds),
               _head_result(tape_c, dwb_outs[1], folds)]
    else:
        res = linear_dgrad_elu_wgrad_pair(ds, [t.hs[L - 1] for t in tapes], [t.dgrad_imgs[L - 1] for t in tapes],
                                          dwb_outs, defer=folds)
    dz = [r[0] for r in res]
    for i in range(2):
        if not adjacent[i]:
            folds.after.append(lambda o=outs[i][L - 1], r=res[i]: torch._foreach_copy_(list(o), [r[1], r[2]]))
    if eager:
        folds.run(dz[0].device)
    for l in range(L - 2, -1, -1):
        h_in = [t.hs[l] for t in tapes]
        N, K = tapes[0].ws[l].shape
        if l > 0:  # square hidden layer: dW = dz^T h, db = column sums of dz, written into the arena slots
            dwb_outs = []
            for i in range(2):
                wo, bo = outs[i][l]
                adj = wo.is_contiguous() and bo.data_ptr() == wo.data_ptr() + 4 * wo.numel()
                dwb_outs.append(torch.as_strided(wo, (N * K + N,), (1,)) if adj else None)
            if _HIDDEN_BWD and hidden_bwd_ok(dz, h_in):
                # input and weight gradients of the layer from one read of dz and h (csrc/mlp_bwd_fused.hip)
                both = hidden_bwd_pair(dz, h_in, [t.dgrad_imgs[l] for t in tapes], dwb_outs, defer=folds)
                res = [(r[1], r[2]) for r in both]
                dz_next = [r[0] for r in both]
            else:
                res = linear_wgrad_pair(dz, h_in, bias_side=1, dwb_outs=dwb_outs, defer=folds)
                dz_next = None
            for i in range(2):
                if dwb_outs[i] is None:
                    folds.after.append(lambda o=outs[i][l], r=res[i]: torch._foreach_copy_(list(o), list(r)))
            if eager:
                folds.run(dz[0].device)
            if dz_next is None:
                dz, _ = linear_dgrad_elu_pair(dz, h_in, [t.dgrad_imgs[l] for t in tapes], _lib.ARITH_X6)
            else:
                dz = dz_next
        else:  # first layer: (x^T dz)^T on the 64-row tiles, the bias from dz (the kernel's K side)
            if on_early is not None:
                folds.run(dz[0].device)  # every other layer's gradient complete in the arena
                on_early()
                on_early = None
            pad = (-K) % 4
            xp = [F.pad(x, (0, pad)) if pad else x for x in h_in]
            dwb_outs = []
            for i in range(2):  # the fold writes (x^T dz)^T = dW in W's layout, then db: straight into the arena
                wo, bo = outs[i][0]
                adj = not pad and wo.is_contiguous() and bo.data_ptr() == wo.data_ptr() + 4 * wo.numel()
                dwb_outs.append(torch.as_strided(wo, (N * K + N,), (1,)) if adj else None)
            res = linear_wgrad_pair(xp, dz, bias_side=2, dwb_outs=dwb_outs, transpose_out=not pad, defer=folds)
            for i in range(2):
                if dwb_outs[i] is None:
                    def copy(o=outs[i][0], r=res[i]):
                        dwt, db = r
                        torch._foreach_copy_(list(o), [dwt[:, :K] if not pad else dwt[:K].t(), db])
                    folds.after.append(copy)
    folds.run(dz[0].device)
    if on_early is not None:
        on_early()
    return True


class FusedMLPFunction(torch.autograd.Function):
    """y = MLP(x) for hidden ELU(alpha=1) layers; args: (x, W1, b1, ..., WL, bL)."""

    @staticmethod
    def forward(ctx, x, *params):
        ws, bs = params[0::2], params[1::2]
        y, tape = train_forward(x, ws, bs)
        ctx.save_for_backward(*tape.hs, *params)
        tape.hs, tape.ws = None, None  # re-attached from saved_tensors in backward
        ctx.tape = tape
        ctx.n_layers = len(ws)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = ctx.n_layers
        saved = ctx.saved_tensors
        tape = ctx.tape
        tape.hs, tape.ws = list(saved[:L]), list(saved[L:][0::2])
        need_w = [ctx.needs_input_grad[1 + 2 * l] for l in range(L)]
        dx, grads_w, grads_b = train_backward(tape, dy, need_dx=ctx.needs_input_grad[0], need_w=need_w)
        out = [dx]
        for gw, gb in zip(grads_w, grads_b):
            out += [gw, gb]
        return tuple(out)


def fusable_structure(mlp: nn.Sequential) -> bool:
    """Linear, ELU(alpha=1), ..., Linear[, Unflatten] with hidden widths <= 256, all widths 4-aligned."""
    mods = [m for m in mlp if not isinstance(m, nn.Unflatten)]
    if len(mods) < 3 or len(mods) % 2 == 0:
        return False
    for i, m in enumerate(mods):
        if i % 2 == 0:
            if not isinstance(m, nn.Linear) or m.bias is None:
                return False
        elif not (isinstance(m, nn.ELU) and m.alpha == 1.0 and not m.inplace):
            return False
    linears = mods[0::2]
    if linears[0].in_features % 4:
        return False
    return all(m.out_features <= MAX_WIDTH and m.out_features % 4 == 0 for m in linears[:-1])


def fusable(mlp: nn.Sequential, x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and fusable_structure(mlp)


def _unflatten(mlp, y):
    for m in mlp:
        if isinstance(m, nn.Unflatten):
            y = m(y)
    return y


_side_streams: dict = {}
# RSLRL_PAIR_TRAIN=0 keeps the update's actor and critic passes in separate launches (A/B)
_PAIR_TRAIN = os.environ.get("RSLRL_PAIR_TRAIN", "1") != "0"
# RSLRL_OUT_PAIR=0 keeps the rollout's two fused output-layer launches separate (A/B)
_OUT_PAIR = os.environ.get("RSLRL_OUT_PAIR", "1") != "0"
# RSLRL_ROLLOUT_MLP=0 keeps the rollout's forward layer by layer (A/B; the same bits)
_ROLLOUT_MLP = os.environ.get("RSLRL_ROLLOUT_MLP", "1") != "0"
# RSLRL_ROLLOUT_STEP_FUSION=0 (A/B; the same bits): no Normal sample inside the one-launch forward, no single-network
# one-launch forward (compute_returns' last values), no copy-free act graphs for recurring observation buffers
_STEP_FUSION = os.environ.get("RSLRL_ROLLOUT_STEP_FUSION", "1") != "0"
rollout_mlp_launches = 0


def rollout_mlp_pair(xs, ws, bs, imgs, nh: int, sample=None):
    """The rollout's actor and critic forward, every layer in one launch (rslrl_rollout_mlp_pair): y = [y_a, y_b],
    bit-identical to the layer-by-layer launches of fused_mlp_forward_pair; None when the shapes are not covered
    (nothing launched).  xs: the two inputs [M, k0] (or one: a single network, fused_mlp_forward); ws, bs, imgs: per
    network, as fused_mlp_forward_pair holds them (x6 forward images, the output layer's image).  sample: (eps, scale)
    of the first network's Normal sample -- eps [M, nout] standard normals, rewritten in place to eps * scale + y
    (ActorCritic._sample's expression, one launch less per env step); scale: the shared [nout] std.  A sample the
    kernel does not take (other shapes, a per-row scale) returns None before anything launches."""
    P = len(xs)
    M, k0 = xs[0].shape
    if (M % _lib.ROLLOUT_MLP_ROWS or k0 not in (16, 32, 48, 64) or not 2 <= nh <= _lib.ROLLOUT_MLP_MAX_HIDDEN
            or any(x.shape != xs[0].shape for x in xs)):
        return None
    for i in range(P):
        w = ws[i]
        if w[0].shape != (256, k0) or any(w[l].shape != (256, 256) for l in range(1, nh)) or w[nh].shape[1] != 256:
            return None
        if not 1 <= w[nh].shape[0] <= _lib.ROLLOUT_MLP_MAX_OUT or imgs[i][2] is None:
            return None
        if xs[i].data_ptr() % 16 or not xs[i].is_contiguous():
            return None
    if sample is not None:
        eps, scale = sample
        A = ws[0][nh].shape[0]
        if (eps.shape != (M, A) or not eps.is_contiguous() or eps.dtype != torch.float32 or eps.device != xs[0].device
                or scale.shape != (A,) or not scale.is_contiguous() or scale.dtype != torch.float32
                or scale.device != xs[0].device):
            return None
    ys = [torch.empty(M, ws[i][nh].shape[0], device=xs[0].device, dtype=torch.float32) for i in range(P)]
    args = []
    for i in range(P):
        a = _lib.RolloutMlp()
        a.x, a.k0, a.hidden = xs[i].data_ptr(), k0, nh
        for l in range(nh):
            a.bimage[l] = imgs[i][0][l].data_ptr()
            a.bias[l] = bs[i][l].data_ptr()
        a.out_image, a.out_bias = imgs[i][2].data_ptr(), bs[i][nh].data_ptr()
        a.nout, a.y = ws[i][nh].shape[0], ys[i].data_ptr()
        if i == 0 and sample is not None:
            a.sample, a.sample_scale = sample[0].data_ptr(), sample[1].data_ptr()
        args.append(a)
    nout = sum(y.shape[1] for y in ys)
    flops = 2 * M * 256 * (P * k0 + P * 256 * (nh - 1)) + 2 * M * 256 * nout
    with timer.span(f"rollout_mlp_pair[M={M},K={k0},hidden={nh},out={nout}]", xs[0].device, 4 * M * (P * k0 + nout),
                    flops):
        rc = _lib.lib().rslrl_rollout_mlp_pair(ctypes.byref(args[0]), ctypes.byref(args[1]) if P == 2 else None, M,
                                               _stream(xs[0]))
    if rc == _lib.E_UNSUPPORTED:
        return None
    _lib.check(rc, "rslrl_rollout_mlp_pair")
    global rollout_mlp_launches
    rollout_mlp_launches += 1
    return ys


def side_stream(device):
    """A second stream of `device` for independent launches, or None.  Opt-in (RSLRL_TWO_STREAMS=1, read per call):
    the critic's launches beside the actor's measured equal to one stream within run-to-run noise (14.74 / 14.56 M
    vs 14.68 / 14.65 M env-steps/s, alternating 30-iteration benches on one box)."""
    if device.type != "cuda" or os.environ.get("RSLRL_TWO_STREAMS", "0") != "1":
        return None
    s = _side_streams.get(device)
    if s is None:
        s = torch.cuda.Stream(device)
        _side_streams[device] = s
    return s


def fused_mlp_forward_pair(mlp_a: nn.Sequential, x_a: torch.Tensor, mlp_b: nn.Sequential, x_b: torch.Tensor,
                           sample=None):
    """Inference forward of two MLPs (the actor and the critic of the rollout) with their same-shape hidden
    layers batched into one launch each (rslrl_linear_gemm_pair); identical results to two fused_mlp_forward
    calls.  Returns (y_a, y_b), or None when the pair does not qualify (gradients wanted, another GEMM mode,
    different hidden shapes or batch sizes) -- the caller then runs the two forwards.
    sample: (eps, scale) -- the Normal sample of the actor's output (rollout_mlp_pair): the result is then
    (y_a, y_b, sampled), sampled telling whether eps now holds eps * scale + y_a (else the caller samples)."""
    # inside a frozen_weights() scope (the rollout) the weights, their images and the plan are fixed: the
    # structure checks, parameter lists, plans and image lookups run once per scope and pair (host time per
    # rollout step matters when a GPU holds few envs)
    memo_key = (id(mlp_a), id(mlp_b), _mode) if _frozen_depth and not torch.is_grad_enabled() else None
    memo = _pair_memo.get(memo_key) if memo_key is not None else None
    if memo is not None and memo[0]() is mlp_a and memo[1]() is mlp_b:
        ws, bs, h3, fuse, imgs, nh = memo[2]
        if not (x_a.is_cuda and x_b.is_cuda and x_a.dtype == torch.float32 and x_b.dtype == torch.float32
                and x_a.dim() == 2 and x_b.dim() == 2 and x_a.shape[0] == x_b.shape[0]
                and x_a.shape[1] == ws[0][0].shape[1] and x_b.shape[1] == ws[1][0].shape[1]):
            return None
    else:
        if not (_split() and getattr(mlp_a, "_fused", True) and getattr(mlp_b, "_fused", True) and fusable(mlp_a, x_a)
                and fusable(mlp_b, x_b) and x_a.shape[0] == x_b.shape[0]):
            return None
        la = [m for m in mlp_a if isinstance(m, nn.Linear)]
        lb = [m for m in mlp_b if isinstance(m, nn.Linear)]
        params = [p for m in la + lb for p in (m.weight, m.bias)]
        if torch.is_grad_enabled() and any(p.requires_grad for p in params + [x_a, x_b]):
            return None
        if len(la) != len(lb) or any(a.weight.shape != b.weight.shape for a, b in zip(la[:-1], lb[:-1])):
            return None
        ws = ([m.weight for m in la], [m.weight for m in lb])
        bs = ([m.bias for m in la], [m.bias for m in lb])
        plans = [_plan(w) for w in ws]
        h3 = plans[0][1]
        fuse = [plans[0][2], plans[1][2]]
        imgs = [_forward_images(ws[i], h3, fuse[i], backward=False) for i in range(2)]
        nh = len(la) - 1
        if memo_key is not None:
            _pair_memo[memo_key] = (weakref.ref(mlp_a), weakref.ref(mlp_b), (ws, bs, h3, fuse, imgs, nh))
    arith = lambda l: _lib.ARITH_H3 if h3[l] else _lib.ARITH_X6  # noqa: E731
    h = [x_a if x_a.is_contiguous() else x_a.contiguous(), x_b if x_b.is_contiguous() else x_b.contiguous()]
    y = None
    sampled = False
    if _ROLLOUT_MLP and not any(h3) and all(fuse):
        if sample is not None:
            y = rollout_mlp_pair(h, ws, bs, imgs, nh, sample=sample)
            sampled = y is not None
        if y is None:
            y = rollout_mlp_pair(h, ws, bs, imgs, nh)
    if y is not None:
        out = (_unflatten(mlp_a, y[0]), _unflatten(mlp_b, y[1]))
        return out if sample is None else out + (sampled,)
    amax = [None, None]
    y = [None, None]
    for l in range(nh):
        want = l + 1 < nh and h3[l + 1]
        last_fused = [fuse[i] and l == nh - 1 for i in range(2)]
        if not any(last_fused):
            h, amax = linear_fwd_pair(h, [bs[0][l], bs[1][l]], ws[0][l].shape[0], True, [imgs[0][0][l], imgs[1][0][l]],
                                      arith(l), amax, [want, want])
            continue
        if _OUT_PAIR and all(last_fused) and not any(h3) and side_stream(h[1].device) is None:
            # both heads in one launch (different epilogues per output width; two launches past one tile per CU)
            _, y = linear_fwd_out_pair(h, [bs[0][l], bs[1][l]], ws[0][l].shape[0], [imgs[0][0][l], imgs[1][0][l]],
                                       [bs[0][-1], bs[1][-1]], [imgs[0][2], imgs[1][2]], store_h=False)
            h = [None, None]
            continue
        # the output layer's fused launches differ per network (output width): the second network's runs on a
        # side stream beside the first's, so the two launches fill each other's tails
        side = side_stream(h[1].device)
        main = torch.cuda.current_stream(h[1].device) if side is not None else None
        for i in range(2):
            ctx = contextlib.nullcontext()
            if side is not None and i == 1:
                side.wait_stream(main)
                h[1].record_stream(side)
                ctx = torch.cuda.stream(side)
            with ctx:
                if last_fused[i]:
                    h[i], y[i] = linear_fwd_out_ex(h[i], bs[i][l], ws[i][l].shape[0], imgs[i][0][l], arith(l),
                                                   amax[i], bs[i][-1], imgs[i][2], store_h=False)
                else:
                    h[i], amax[i] = linear_fwd_ex(h[i], bs[i][l], ws[i][l].shape[0], True, imgs[i][0][l], arith(l),
                                                  amax[i], want)
        if side is not None:
            main.wait_stream(side)
            for t in (h[1], y[1], amax[1]):
                if t is not None:
                    t.record_stream(main)
    out = []
    for i, mlp in enumerate((mlp_a, mlp_b)):
        yi = y[i] if y[i] is not None else F.linear(h[i], ws[i][-1], bs[i][-1])
        out.append(_unflatten(mlp, yi))
    return (out[0], out[1]) if sample is None else (out[0], out[1], False)


def fused_mlp_forward(mlp: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    linears = [m for m in mlp if isinstance(m, nn.Linear)]
    params = []
    for m in linears:
        params += [m.weight, m.bias]
    x = x if x.is_contiguous() else x.contiguous()
    if torch.is_grad_enabled() and any(p.requires_grad for p in params + [x]):
        y = FusedMLPFunction.apply(x, *params)
    else:
        ws = [m.weight for m in linears]
        bs = [m.bias for m in linears]
        split, h3, fuse_out = _plan(ws)
        if split:  # the last activation never reaches HBM when the output layer is fused
            fwd_imgs, _, out_img = _forward_images(ws, h3, fuse_out, backward=False)
            y = None
            if (_ROLLOUT_MLP and _STEP_FUSION and not any(h3) and fuse_out and x.is_cuda and x.dim() == 2
                    and x.dtype == torch.float32):
                # every layer in one launch (compute_returns' last values, act_inference): the same bits
                r = rollout_mlp_pair([x], [ws], [bs], [(fwd_imgs, None, out_img)], len(ws) - 1)
                y = r[0] if r is not None else None
            if y is None:
                hs, _, y = _hidden_forward(x, ws, bs, h3, fuse_out, fwd_imgs, out_img, keep=False)
                h = hs[-1]
        else:
            h, y = x, None
            for m in linears[:-1]:
                h = linear_fwd(h, m.weight, m.bias, elu=True)
        if y is None:
            y = F.linear(h, linears[-1].weight, linears[-1].bias)
    for m in mlp:
        if isinstance(m, nn.Unflatten):
            y = m(y)
    return y
