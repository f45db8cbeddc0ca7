"""CPU ORACLE for the rsl_rl PPO hot path -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
The product (rsl_rl_amd/) never imports it.  Integer/byte work and the GAE scan are plain C
(oracle/oracle.c via ctypes); the PPO loss is a float32 numpy restatement that evaluates the
reference's expressions in the reference's operation order.

Parity is pinned against tests/golden/ (captured from the reference by tests/golden/make_golden.py);
see tests/test_oracle_golden.py.
"""

from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

f32 = np.float32


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, I64, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float
        L.oracle_gae.argtypes = [P, P, P, P, F, F, I64, I64, P, P]
        L.oracle_adv_stats.argtypes = [P, I64, P, P]
        L.oracle_adv_normalize.argtypes = [P, I64, F]
        L.oracle_randperm.argtypes = [P, I64, P]
        L.oracle_gather_rows.argtypes = [P, I64, P, I64, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------------------------------------
# rollout_storage.py:127-149
# ----------------------------------------------------------------------------------------------
def gae(values, rewards, dones, last_values, gamma, lam):
    """values/rewards [T,N] f32, dones [T,N] u8, last_values [N] f32 -> (returns, raw advantages)."""
    values = np.ascontiguousarray(values, dtype=f32)
    rewards = np.ascontiguousarray(rewards, dtype=f32)
    dones = np.ascontiguousarray(dones, dtype=np.uint8)
    last_values = np.ascontiguousarray(last_values, dtype=f32).reshape(-1)
    T, N = values.shape
    ret = np.empty((T, N), f32)
    adv = np.empty((T, N), f32)
    lib().oracle_gae(_p(values), _p(rewards), _p(dones), _p(last_values), f32(gamma), f32(lam), T, N, _p(ret), _p(adv))
    return ret, adv


def adv_stats(adv):
    a = np.ascontiguousarray(adv, dtype=f32).reshape(-1)
    m = np.zeros(1, f32)
    s = np.zeros(1, f32)
    lib().oracle_adv_stats(_p(a), a.size, _p(m), _p(s))
    return float(m[0]), float(s[0])


def adv_normalize(adv, eps=1e-8):
    a = np.array(adv, dtype=f32, copy=True)
    flat = a.reshape(-1)
    lib().oracle_adv_normalize(_p(flat), flat.size, f32(eps))
    return a


def compute_returns(values, rewards, dones, last_values, gamma, lam, normalize_advantage=True):
    """rollout_storage.py:127-149 -> (returns, advantages)."""
    ret, adv = gae(values, rewards, dones, last_values, gamma, lam)
    if normalize_advantage:
        adv = adv_normalize(adv)
    return ret, adv


# ----------------------------------------------------------------------------------------------
# rollout_storage.py:165  torch.randperm on a CPU generator (mt19937 Fisher-Yates)
# ----------------------------------------------------------------------------------------------
def randperm(state_blob, n):
    """state_blob: uint8 array from torch.Generator.get_state(). Returns (perm int64, new_state)."""
    st = np.array(state_blob, dtype=np.uint8, copy=True)
    perm = np.empty(max(n, 0), np.int64)
    lib().oracle_randperm(_p(st), n, _p(perm))
    return perm, st


def gather_rows(src, idx):
    src = np.ascontiguousarray(src)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    rows = src.shape[0]
    row_bytes = src.nbytes // max(rows, 1)
    out = np.empty((idx.size,) + src.shape[1:], src.dtype)
    lib().oracle_gather_rows(_p(src), row_bytes, _p(idx), idx.size, _p(out))
    return out


# ----------------------------------------------------------------------------------------------
# rollout_storage.py:160-203  mini_batch_generator
# ----------------------------------------------------------------------------------------------
def minibatch_indices(num_envs, num_steps, num_mini_batches, state_blob):
    batch_size = num_envs * num_steps
    mb = batch_size // num_mini_batches
    perm, new_state = randperm(state_blob, num_mini_batches * mb)
    return perm, mb, new_state


def minibatches(fields, perm, mb, num_mini_batches, num_epochs):
    """fields: name -> [T, N, ...] array. Yields dicts name -> gathered [mb, ...] rows."""
    flat = {k: np.ascontiguousarray(v).reshape((v.shape[0] * v.shape[1],) + v.shape[2:]) for k, v in fields.items()}
    for _ in range(num_epochs):
        for i in range(num_mini_batches):
            idx = perm[i * mb:(i + 1) * mb]
            yield {k: gather_rows(v, idx) for k, v in flat.items()}


# ----------------------------------------------------------------------------------------------
# ppo.py:221-315 (+ autograd backward of ppo.py:368 down to mu, sigma, V)
# ----------------------------------------------------------------------------------------------
_LOG_SQRT_2PI = f32(math.log(math.sqrt(2 * math.pi)))  # torch/distributions/normal.py log_prob
_ENT_C = f32(0.5 + 0.5 * math.log(2 * math.pi))  # torch/distributions/normal.py entropy


def _max_grads(a, b, g):
    """torch.max(a, b) backward (derivatives.yaml 'maximum'): ties split the gradient 1/2 : 1/2."""
    ga = np.where(a == b, g / f32(2), g)
    ga = np.where(a < b, f32(0), ga)
    gb = np.where(a == b, g / f32(2), g)
    gb = np.where(a > b, f32(0), gb)
    return ga.astype(f32), gb.astype(f32)


def ppo_loss(mu, sigma, values, actions, old_logp, advantages, target_values, returns, old_mu, old_sigma, *,
             clip_param=0.2, value_loss_coef=1.0, entropy_coef=0.01, use_clipped_value_loss=True,
             compute_kl=True, normalize_advantage_per_mini_batch=False):
    """Forward + backward of the PPO loss for one mini-batch, float32.

    mu, sigma, actions, old_mu, old_sigma: [B, A]; values, old_logp, advantages, target_values, returns:
    [B] or [B, 1].  Returns scalars (surrogate, value, entropy mean, kl_mean, loss) and the gradients of
    the total loss w.r.t. mu [B, A], sigma [B, A] (per sample; sum over B for a shared std) and V [B].
    """
    mu = np.asarray(mu, f32)
    sigma = np.asarray(sigma, f32)
    B, A = mu.shape
    x = np.asarray(actions, f32).reshape(B, A)
    old_logp = np.asarray(old_logp, f32).reshape(B)
    adv = np.asarray(advantages, f32).reshape(B)
    V = np.asarray(values, f32).reshape(B)
    tv = np.asarray(target_values, f32).reshape(B)
    R = np.asarray(returns, f32).reshape(B)
    omu = np.asarray(old_mu, f32).reshape(B, A)
    osig = np.asarray(old_sigma, f32).reshape(B, A)
    eps = f32(clip_param)
    out = {}

    if normalize_advantage_per_mini_batch:  # ppo.py:221-223
        m, s = adv_stats(adv)
        adv = ((adv - f32(m)) / (f32(s) + f32(1e-8))).astype(f32)
        out["adv_mean"], out["adv_std"] = m, s

    # actor_critic.py:170-171 -> Normal.log_prob(actions).sum(-1)
    var = sigma ** 2
    log_scale = np.log(sigma)
    d = x - mu
    num = -(d ** 2)
    den = f32(2) * var
    lp = num / den - log_scale - _LOG_SQRT_2PI
    logp = lp.sum(-1, dtype=f32)
    # actor_critic.py:114-116 -> entropy().sum(-1)
    ent = (_ENT_C + log_scale).sum(-1, dtype=f32)

    if compute_kl:  # ppo.py:262-269
        kl = (np.log(sigma / osig + f32(1e-5)) + (np.square(osig) + np.square(omu - mu)) / (f32(2) * np.square(sigma))
              - f32(0.5)).sum(-1, dtype=f32)
        out["kl_mean"] = float(kl.mean(dtype=np.float64))

    # ppo.py:297-302
    ratio = np.exp(logp - old_logp)
    surr = -adv * ratio
    rc = np.clip(ratio, f32(1.0 - clip_param), f32(1.0 + clip_param))
    surr_c = -adv * rc
    surr_loss = np.maximum(surr, surr_c).mean(dtype=np.float64)
    # ppo.py:305-313
    if use_clipped_value_loss:
        dv = V - tv
        vc = tv + np.clip(dv, -eps, eps)
        vl = (V - R) ** 2
        vlc = (vc - R) ** 2
        v_loss = np.maximum(vl, vlc).mean(dtype=np.float64)
    else:
        v_loss = ((R - V) ** 2).mean(dtype=np.float64)
    ent_mean = ent.mean(dtype=np.float64)
    loss = surr_loss + value_loss_coef * v_loss - entropy_coef * ent_mean
    out.update(surrogate=float(surr_loss), value_function=float(v_loss), entropy=float(ent_mean), loss=float(loss))

    # ---- backward (ppo.py:368), loss -> (logp, entropy, V) -> (mu, sigma)
    gB = f32(1.0 / B)
    g_s, g_sc = _max_grads(surr, surr_c, np.full(B, gB, f32))
    g_ratio = g_s * (-adv)
    in_clip = (ratio >= f32(1.0 - clip_param)) & (ratio <= f32(1.0 + clip_param))
    g_ratio = g_ratio + np.where(in_clip, g_sc * (-adv), f32(0))
    g_logp = (g_ratio * ratio).astype(f32)

    gvB = np.full(B, f32(value_loss_coef) * gB, f32)
    if use_clipped_value_loss:
        g_vl, g_vlc = _max_grads(vl, vlc, gvB)
        dV = g_vl * f32(2) * (V - R)
        in_v = (dv >= -eps) & (dv <= eps)
        dV = dV + np.where(in_v, g_vlc * f32(2) * (vc - R), f32(0))
    else:
        dV = -(gvB * f32(2) * (R - V))
    g_ent = np.full(B, -f32(entropy_coef) * gB, f32)

    g_lp = np.repeat(g_logp[:, None], A, axis=1)
    # lp = num/den - log_scale - c
    g_num = g_lp / den
    g_den = -g_lp * num / (den * den)
    g_d = -g_num * f32(2) * d
    dmu = -g_d
    g_var = f32(2) * g_den
    dsig = g_var * f32(2) * sigma - g_lp / sigma + np.repeat(g_ent[:, None], A, axis=1) / sigma
    out.update(dmu=dmu.astype(f32), dsigma=dsig.astype(f32), dV=dV.astype(f32), dlogp=g_logp)
    return out


# --------------------------------------------------------------------------------------------------
# rollout-side record: act's log-prob + process_env_step's reward + RND (ppo.py:129-169, rnd.py:113-135)
# --------------------------------------------------------------------------------------------------
def normal_log_prob_sum(actions, mu, sigma):
    """torch.distributions.Normal(mu, sigma).log_prob(actions).sum(-1) (normal.py) in fp32:
    -((x - mu) ** 2) / (2 * var) - log(sigma) - log(sqrt(2 pi)), summed over the last axis in order."""
    x, m = actions.astype(f32), mu.astype(f32)
    s = np.broadcast_to(sigma.astype(f32), x.shape)
    d = (x - m).astype(f32)
    num = (-(d * d)).astype(f32)
    den = (f32(2.0) * (s * s).astype(f32)).astype(f32)
    t = ((num / den).astype(f32) - np.log(s).astype(f32)).astype(f32) - f32(math.log(math.sqrt(2 * math.pi)))
    t = t.astype(f32)
    out = np.zeros(x.shape[:-1], f32)
    for a in range(x.shape[-1]):
        out = (out + t[..., a]).astype(f32)
    return out


def _elu(z):
    return np.where(z > 0, z, np.expm1(z.astype(np.float64)).astype(f32)).astype(f32)


def mlp_forward(x, layers):
    """Linear/ELU stack in fp64 accumulation rounded per layer (a GEMM-class fp32 result)."""
    h = x.astype(f32)
    for i, (w, b) in enumerate(layers):
        h = (h.astype(np.float64) @ w.astype(np.float64).T + b.astype(np.float64)).astype(f32)
        if i + 1 < len(layers):
            h = _elu(h)
    return h


def rnd_intrinsic(state, target_layers, predictor_layers, weight, state_mean=None, state_std=None, eps=1e-2):
    """weight * || target(s) - predictor(s) ||_2 with s optionally (s - mean) / (std + eps)."""
    s = state.astype(f32)
    if state_mean is not None:
        s = ((s - state_mean.astype(f32)).astype(f32) / (state_std.astype(f32) + f32(eps)).astype(f32)).astype(f32)
    d = (mlp_forward(s, target_layers) - mlp_forward(s, predictor_layers)).astype(f32)
    ss = np.zeros(d.shape[0], f32)
    for q in range(d.shape[1]):
        ss = (ss + (d[:, q] * d[:, q]).astype(f32)).astype(f32)
    return (np.sqrt(ss).astype(f32) * f32(weight)).astype(f32)


def step_reward(rewards, values, time_outs, gamma, intrinsic=None):
    """(rewards + intrinsic) + gamma * (values * time_outs)  (ppo.py:147-164)."""
    r = rewards.astype(f32).copy()
    if intrinsic is not None:
        r = (r + intrinsic.astype(f32)).astype(f32)
    if time_outs is not None:
        r = (r + (f32(gamma) * (values.reshape(-1).astype(f32) * time_outs.astype(f32)).astype(f32)).astype(f32))
    return r.astype(f32)


# --------------------------------------------------------------------------------------------------
# running normalisers (networks/normalization.py:44-99)
# --------------------------------------------------------------------------------------------------
def normalizer_update(x, mean, var, count, until=None):
    """One EmpiricalNormalization.update: fp64 batch moments, then the reference's fp32 update order.
    Returns (mean, var, std, count) (the inputs unchanged once count >= until)."""
    if until is not None and count >= until:
        return mean, var, np.sqrt(var).astype(f32), count
    n = x.shape[0]
    count = count + n
    rate = f32(f32(n) / f32(count))
    xd = x.astype(np.float64)
    mean_x = xd.mean(0).astype(f32)
    var_x = np.maximum((xd * xd).mean(0) - xd.mean(0) ** 2, 0.0).astype(f32)
    delta = (mean_x - mean).astype(f32)
    mean_new = (mean + (rate * delta).astype(f32)).astype(f32)
    inner = ((var_x - var).astype(f32) + (delta * (mean_x - mean_new).astype(f32)).astype(f32)).astype(f32)
    var_new = (var + (rate * inner).astype(f32)).astype(f32)
    return mean_new, var_new, np.sqrt(var_new).astype(f32), count


def normalizer_apply(x, mean, std, eps=1e-2):
    return ((x.astype(f32) - mean).astype(f32) / (std + f32(eps)).astype(f32)).astype(f32)
