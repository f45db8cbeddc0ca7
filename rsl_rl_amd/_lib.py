"""ctypes binding of librslrl_amd.so (the C ABI declared in include/rslrl_amd.h).

The library is built in-tree (rsl_rl_amd/csrc/Makefile -> rsl_rl_amd/lib/librslrl_amd.so).  torch is
imported first so that the HIP runtime torch ships (libamdhip64.so.7) is the one the library binds to:
the dynamic loader resolves our DT_NEEDED by soname to the already-loaded copy, so torch's streams and
device pointers are valid in both.

There is no fallback: if the library is missing the hot path raises HipLibraryMissing.
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
# RSLRL_AMD_LIB: an alternative in-tree build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("RSLRL_AMD_LIB") or os.path.join(LIB_DIR, "librslrl_amd.so")
ABI_VERSION = 21

# symbols declared in include/rslrl_amd.h (tests/test_capi.py checks the header against this list)
EXPORTED_SYMBOLS = (
    "rslrl_abi_version",
    "rslrl_status_string",
    "rslrl_compute_returns_workspace_bytes",
    "rslrl_compute_returns",
    "rslrl_compute_returns_records",
    "rslrl_compute_returns_slots",
    "rslrl_compute_returns_status_offset",
    "rslrl_compute_returns_slots_form",
    "rslrl_debug_knob",
    "rslrl_normalize_workspace_bytes",
    "rslrl_normalize_advantages",
    "rslrl_randperm_mt19937",
    "rslrl_gather_rows",
    "rslrl_gather_records",
    "rslrl_gather_records_side",
    "rslrl_record_fill_slot",
    "rslrl_ppo_loss_workspace_bytes",
    "rslrl_ppo_loss_fwd_bwd",
    "rslrl_linear_tiles",
    "rslrl_linear_bimage_bytes",
    "rslrl_linear_prepare_bimage",
    "rslrl_linear_prepare_bimages",
    "rslrl_linear_fwd",
    "rslrl_linear_dgrad_elu",
    "rslrl_column_sum_fold",
    "rslrl_linear_out_image_bytes",
    "rslrl_linear_fwd_out",
    "rslrl_linear_wgrad_workspace_bytes",
    "rslrl_linear_wgrad",
    "rslrl_fold_partials_workspace_bytes",
    "rslrl_fold_partials",
    "rslrl_linear_dgrad_wgrad_partial_bytes",
    "rslrl_linear_dgrad_elu_wgrad",
    "rslrl_rollout_record",
    "rslrl_normalizer_workspace_bytes",
    "rslrl_normalizer_update",
    "rslrl_normalizer_apply",
    "rslrl_reward_normalize",
    "rslrl_linear_bimage_h3_bytes",
    "rslrl_amax_workspace_bytes",
    "rslrl_linear_gemm",
    "rslrl_linear_gemm_pair",
    "rslrl_value_head_fwd_bwd",
    "rslrl_value_head_partial_rows",
    "rslrl_actor_head_workspace_bytes",
    "rslrl_actor_head_fwd_bwd",
    "rslrl_linear_wgrad_ex",
    "rslrl_linear_wgrad_bias_workspace_bytes",
    "rslrl_linear_wgrad_bias",
    "rslrl_linear_wgrad_bias_pair_workspace_bytes",
    "rslrl_linear_wgrad_bias_pair",
    "rslrl_fold_partials_ex",
    "rslrl_fold_partials_batch",
    "rslrl_fold_partials_batch_workspace_bytes",
    "rslrl_linear_wgrad_bias_pair_slices",
    "rslrl_normal_affine",
    "rslrl_ppo_update_tail",
    "rslrl_adam_workspace_bytes",
    "rslrl_clip_adam_step",
    "rslrl_clip_adam_step_tail",
    "rslrl_rnd_update_workspace_bytes",
    "rslrl_rnd_update",
    "rslrl_synthetic_env_step",
    "rslrl_launch_timing_enable",
    "rslrl_launch_timing_read_tag",
    "rslrl_launch_timing_read",
    "rslrl_hidden_bwd_slices",
    "rslrl_hidden_bwd_partial_floats",
    "rslrl_hidden_bwd_pair",
    "rslrl_rollout_mlp_pair",
)

MAX_GATHER_FIELDS = 16
MAX_RECORD_FLOATS = 256
PPO_LOSS_MAX_ACTIONS = 64


class HipLibraryMissing(RuntimeError):
    pass


class RslrlError(RuntimeError):
    pass


class GatherField(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("row_bytes", ctypes.c_int64)]


class RecordField(ctypes.Structure):
    """rslrl_record_field_t (include/rslrl_amd.h)."""
    _fields_ = [("offset", ctypes.c_int64), ("width", ctypes.c_int64), ("dst", ctypes.c_void_p)]


class BImageDesc(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("image", ctypes.c_void_p), ("rows", ctypes.c_int32),
                ("depth", ctypes.c_int32), ("transposed", ctypes.c_int32), ("layout", ctypes.c_int32)]


MAX_BIMAGES = 16
BIMAGE_LAYOUT_GEMM = 0
BIMAGE_LAYOUT_OUT = 1
BIMAGE_LAYOUT_H3 = 2

ARITH_X6, ARITH_H3 = 1, 2
LINEAR_FWD, LINEAR_FWD_ELU, LINEAR_DGRAD_ELU, LINEAR_DGRAD_ELU_WGRAD, LINEAR_FWD_OUT = 0, 1, 2, 3, 4
E_INVALID_ARGUMENT = -1  # RSLRL_E_INVALID_ARGUMENT
E_UNSUPPORTED = -3  # RSLRL_E_UNSUPPORTED


ADAM_MAX_TENSORS = 24


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("step", ctypes.c_void_p), ("numel", ctypes.c_int64)]


class AdamArgs(ctypes.Structure):
    """rslrl_adam_args_t (include/rslrl_amd.h)."""
    _fields_ = [("n", ctypes.c_int32), ("max_grad_norm", ctypes.c_float), ("lr", ctypes.c_double),
                ("lr_dev", ctypes.c_void_p), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("offsets", ctypes.c_int64 * (ADAM_MAX_TENSORS + 1)),
                ("t", AdamTensor * ADAM_MAX_TENSORS)]


class PpoTail(ctypes.Structure):
    """rslrl_ppo_tail_t (include/rslrl_amd.h)."""
    _fields_ = [("stats", ctypes.c_void_p), ("kl", ctypes.c_void_p), ("lr", ctypes.c_void_p), ("lr32", ctypes.c_void_p),
                ("round_fp32", ctypes.c_int32), ("kl_hi", ctypes.c_float), ("kl_lo", ctypes.c_float),
                ("sums", ctypes.c_void_p)]


class LinearArgs(ctypes.Structure):
    """rslrl_linear_args_t (include/rslrl_amd.h)."""
    _fields_ = [
        ("op", ctypes.c_int32),
        ("arith", ctypes.c_int32),
        ("a", ctypes.c_void_p),
        ("a_amax", ctypes.c_void_p),
        ("M", ctypes.c_int64),
        ("K", ctypes.c_int32),
        ("N", ctypes.c_int32),
        ("bimage", ctypes.c_void_p),
        ("bias", ctypes.c_void_p),
        ("h", ctypes.c_void_p),
        ("c", ctypes.c_void_p),
        ("colsum_partials", ctypes.c_void_p),
        ("wgrad_partials", ctypes.c_void_p),
        ("out_image", ctypes.c_void_p),
        ("out_bias", ctypes.c_void_p),
        ("y", ctypes.c_void_p),
        ("nout", ctypes.c_int32),
        ("amax_out", ctypes.c_void_p),
        ("amax_workspace", ctypes.c_void_p),
    ]


class ValueHeadArgs(ctypes.Structure):
    """rslrl_value_head_args_t (include/rslrl_amd.h)."""
    _fields_ = [
        ("target_values", ctypes.c_void_p),
        ("returns", ctypes.c_void_p),
        ("out_weight", ctypes.c_void_p),
        ("clip_param", ctypes.c_float),
        ("value_loss_coef", ctypes.c_float),
        ("use_clipped_value_loss", ctypes.c_int32),
        ("wgrad_partials", ctypes.c_void_p),
        ("colsum_partials", ctypes.c_void_p),
    ]


class ActorHeadArgs(ctypes.Structure):
    """rslrl_actor_head_args_t (include/rslrl_amd.h)."""
    _fields_ = [
        ("actions", ctypes.c_void_p),
        ("old_log_prob", ctypes.c_void_p),
        ("advantages", ctypes.c_void_p),
        ("values", ctypes.c_void_p),
        ("target_values", ctypes.c_void_p),
        ("returns", ctypes.c_void_p),
        ("old_mu", ctypes.c_void_p),
        ("old_sigma", ctypes.c_void_p),
        ("sigma", ctypes.c_void_p),
        ("num_actions", ctypes.c_int32),
        ("clip_param", ctypes.c_float),
        ("value_loss_coef", ctypes.c_float),
        ("entropy_coef", ctypes.c_float),
        ("use_clipped_value_loss", ctypes.c_int32),
        ("compute_kl", ctypes.c_int32),
        ("out_weight_t_image", ctypes.c_void_p),
        ("wgrad_partials", ctypes.c_void_p),
        ("grad_sigma", ctypes.c_void_p),
        ("stats", ctypes.c_void_p),
        ("grad_mu", ctypes.c_void_p),
    ]


LAUNCH_TAG_PPO_LOSS, LAUNCH_TAG_ROLLOUT_RECORD, LAUNCH_TAG_GATHER_RECORDS = 0, 1, 2
ACTOR_HEAD_ACTIONS = 12  # the fused actor head's output width (rslrl_actor_head_fwd_bwd)

DTYPE_F32, DTYPE_U8, DTYPE_I32, DTYPE_I64 = 0, 1, 2, 3
ROLLOUT_MAX_OBS = 4


class ObsCopy(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("row_floats", ctypes.c_int64)]


class RolloutArgs(ctypes.Structure):
    _fields_ = [
        ("N", ctypes.c_int64),
        ("A", ctypes.c_int32),
        ("sigma_mode", ctypes.c_int32),
        ("actions", ctypes.c_void_p),
        ("mu", ctypes.c_void_p),
        ("sigma", ctypes.c_void_p),
        ("values", ctypes.c_void_p),
        ("rewards", ctypes.c_void_p),
        ("dones", ctypes.c_void_p),
        ("dones_dtype", ctypes.c_int32),
        ("time_outs_dtype", ctypes.c_int32),
        ("time_outs", ctypes.c_void_p),
        ("gamma", ctypes.c_float),
        ("rnd_weight", ctypes.c_float),
        ("extra_reward", ctypes.c_void_p),
        ("rnd_obs", ctypes.c_void_p),
        ("rnd_obs_stride", ctypes.c_int64),
        ("rnd_in", ctypes.c_int32),
        ("rnd_hidden", ctypes.c_int32),
        ("rnd_out", ctypes.c_int32),
        ("rnd_state_eps", ctypes.c_float),
        ("rnd_target", ctypes.c_void_p),
        ("rnd_predictor", ctypes.c_void_p),
        ("rnd_state_mean", ctypes.c_void_p),
        ("rnd_state_std", ctypes.c_void_p),
        ("intrinsic_out", ctypes.c_void_p),
        ("n_obs", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("obs", ObsCopy * ROLLOUT_MAX_OBS),
        ("out_actions", ctypes.c_void_p),
        ("out_rewards", ctypes.c_void_p),
        ("out_dones", ctypes.c_void_p),
        ("out_values", ctypes.c_void_p),
        ("out_logp", ctypes.c_void_p),
        ("out_mu", ctypes.c_void_p),
        ("out_sigma", ctypes.c_void_p),
        ("record_floats", ctypes.c_int64),
        ("out_records", ctypes.c_void_p),
    ]


class PPOLossArgs(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int64),
        ("A", ctypes.c_int32),
        ("sigma_mode", ctypes.c_int32),
        ("mu", ctypes.c_void_p),
        ("mu_stride", ctypes.c_int64),
        ("sigma", ctypes.c_void_p),
        ("sigma_stride", ctypes.c_int64),
        ("values", ctypes.c_void_p),
        ("actions", ctypes.c_void_p),
        ("old_logp", ctypes.c_void_p),
        ("advantages", ctypes.c_void_p),
        ("target_values", ctypes.c_void_p),
        ("returns", ctypes.c_void_p),
        ("old_mu", ctypes.c_void_p),
        ("old_sigma", ctypes.c_void_p),
        ("clip_param", ctypes.c_float),
        ("value_loss_coef", ctypes.c_float),
        ("entropy_coef", ctypes.c_float),
        ("use_clipped_value_loss", ctypes.c_int32),
        ("compute_kl", ctypes.c_int32),
        ("normalize_advantage", ctypes.c_int32),
        ("grad_mu", ctypes.c_void_p),
        ("grad_mu_stride", ctypes.c_int64),
        ("grad_sigma", ctypes.c_void_p),
        ("grad_sigma_stride", ctypes.c_int64),
        ("grad_values", ctypes.c_void_p),
        ("stats", ctypes.c_void_p),
        ("grad_values_stride", ctypes.c_int64),
    ]


class RndUpdateArgs(ctypes.Structure):
    """include/rslrl_amd.h rslrl_rnd_update_args_t"""
    _fields_ = [
        ("B", ctypes.c_int64),
        ("in_", ctypes.c_int32),
        ("hidden", ctypes.c_int32),
        ("out", ctypes.c_int32),
        ("state_eps", ctypes.c_float),
        ("state", ctypes.c_void_p),
        ("state_stride", ctypes.c_int64),
        ("state_mean", ctypes.c_void_p),
        ("state_std", ctypes.c_void_p),
        ("pred_w1", ctypes.c_void_p),
        ("pred_b1", ctypes.c_void_p),
        ("pred_w2", ctypes.c_void_p),
        ("pred_b2", ctypes.c_void_p),
        ("target_w1", ctypes.c_void_p),
        ("target_b1", ctypes.c_void_p),
        ("target_w2", ctypes.c_void_p),
        ("target_b2", ctypes.c_void_p),
        ("target_embedding", ctypes.c_void_p),
        ("grad", ctypes.c_void_p),
        ("loss_sum", ctypes.c_void_p),
        ("loss", ctypes.c_void_p),
    ]


class FoldJob(ctypes.Structure):
    """include/rslrl_amd.h rslrl_fold_job_t"""
    _fields_ = [
        ("partials", ctypes.c_void_p),
        ("S", ctypes.c_int64),
        ("NK", ctypes.c_int64),
        ("out", ctypes.c_void_p),
        ("out_len", ctypes.c_int64),
        ("t_rows", ctypes.c_int32),
        ("t_cols", ctypes.c_int32),
    ]


MAX_FOLD_JOBS = 16
WGRAD_NO_FOLD = 1


class WgradProblem(ctypes.Structure):
    """include/rslrl_amd.h rslrl_wgrad_problem_t"""
    _fields_ = [
        ("dz", ctypes.c_void_p),
        ("dz_amax", ctypes.c_void_p),
        ("x", ctypes.c_void_p),
        ("x_amax", ctypes.c_void_p),
        ("dw_db", ctypes.c_void_p),
        ("workspace", ctypes.c_void_p),
        ("workspace_bytes", ctypes.c_size_t),
        ("transpose_out", ctypes.c_int32),
    ]


class HiddenBwdProblem(ctypes.Structure):
    """include/rslrl_amd.h rslrl_hidden_bwd_problem_t"""
    _fields_ = [
        ("dz", ctypes.c_void_p),
        ("h", ctypes.c_void_p),
        ("bimage", ctypes.c_void_p),
        ("dz_prev", ctypes.c_void_p),
        ("partials", ctypes.c_void_p),
    ]


class RolloutMlp(ctypes.Structure):
    """include/rslrl_amd.h rslrl_rollout_mlp_t"""
    _fields_ = [
        ("x", ctypes.c_void_p),
        ("k0", ctypes.c_int32),
        ("hidden", ctypes.c_int32),
        ("bimage", ctypes.c_void_p * 4),
        ("bias", ctypes.c_void_p * 4),
        ("out_image", ctypes.c_void_p),
        ("out_bias", ctypes.c_void_p),
        ("nout", ctypes.c_int32),
        ("y", ctypes.c_void_p),
        ("sample", ctypes.c_void_p),
        ("sample_scale", ctypes.c_void_p),
    ]


ROLLOUT_MLP_MAX_HIDDEN, ROLLOUT_MLP_MAX_OUT, ROLLOUT_MLP_ROWS = 4, 16, 64

RND_MAX_IN, RND_MAX_HIDDEN, RND_MAX_OUT = 64, 64, 8

_lib = None
_lock = threading.Lock()


def _declare(L):
    P, I32, I64, F, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_size_t
    L.rslrl_abi_version.restype = ctypes.c_int
    L.rslrl_abi_version.argtypes = []
    L.rslrl_status_string.restype = ctypes.c_char_p
    L.rslrl_status_string.argtypes = [ctypes.c_int]
    L.rslrl_compute_returns_workspace_bytes.restype = SZ
    L.rslrl_compute_returns_workspace_bytes.argtypes = [I64, I64]
    L.rslrl_compute_returns.restype = ctypes.c_int
    L.rslrl_compute_returns.argtypes = [P, P, P, P, F, F, I64, I64, I32, P, P, P, SZ, P]
    L.rslrl_compute_returns_records.restype = ctypes.c_int
    L.rslrl_compute_returns_records.argtypes = [P, P, P, P, F, F, I64, I64, P, P, P, P, I64, I64, P, SZ, P]
    L.rslrl_normalize_workspace_bytes.restype = SZ
    L.rslrl_normalize_workspace_bytes.argtypes = [I64]
    L.rslrl_normalize_advantages.restype = ctypes.c_int
    L.rslrl_normalize_advantages.argtypes = [P, I64, F, P, SZ, P]
    L.rslrl_randperm_mt19937.restype = ctypes.c_int
    L.rslrl_randperm_mt19937.argtypes = [P, SZ, I64, P]
    L.rslrl_gather_rows.restype = ctypes.c_int
    L.rslrl_gather_rows.argtypes = [ctypes.POINTER(GatherField), I32, P, I64, P]
    L.rslrl_gather_records.restype = ctypes.c_int
    L.rslrl_gather_records.argtypes = [P, I64, ctypes.POINTER(RecordField), I32, P, I64, P]
    L.rslrl_gather_records_side.restype = ctypes.c_int
    L.rslrl_gather_records_side.argtypes = [P, I64, ctypes.POINTER(RecordField), I32, P, ctypes.POINTER(RecordField),
                                            I32, P, I64, P]
    L.rslrl_compute_returns_slots.restype = ctypes.c_int
    L.rslrl_compute_returns_slots.argtypes = [P, P, P, P, F, F, I64, I64, P, P, P, P, P, SZ, P]
    L.rslrl_compute_returns_status_offset.restype = SZ
    L.rslrl_compute_returns_status_offset.argtypes = []
    L.rslrl_compute_returns_slots_form.restype = ctypes.c_int
    L.rslrl_compute_returns_slots_form.argtypes = [I64, I64, P, P, P, P, P, P]
    L.rslrl_debug_knob.restype = ctypes.c_int
    L.rslrl_debug_knob.argtypes = [ctypes.c_char_p, I64, ctypes.POINTER(I64)]
    L.rslrl_record_fill_slot.restype = ctypes.c_int
    L.rslrl_record_fill_slot.argtypes = [P, I64, I64, I32, P, I32, ctypes.POINTER(ctypes.c_void_p), I32, I64, P]
    L.rslrl_ppo_loss_workspace_bytes.restype = SZ
    L.rslrl_ppo_loss_workspace_bytes.argtypes = [I64, I32]
    L.rslrl_ppo_loss_fwd_bwd.restype = ctypes.c_int
    L.rslrl_ppo_loss_fwd_bwd.argtypes = [ctypes.POINTER(PPOLossArgs), P, SZ, P]
    L.rslrl_linear_tiles.restype = I64
    L.rslrl_linear_tiles.argtypes = [I64]
    L.rslrl_linear_fwd.restype = ctypes.c_int
    L.rslrl_linear_bimage_bytes.restype = SZ
    L.rslrl_linear_bimage_bytes.argtypes = [I32]
    L.rslrl_linear_prepare_bimage.restype = ctypes.c_int
    L.rslrl_linear_prepare_bimage.argtypes = [P, I32, I32, I32, P, P]
    L.rslrl_linear_prepare_bimages.restype = ctypes.c_int
    L.rslrl_linear_prepare_bimages.argtypes = [ctypes.POINTER(BImageDesc), I32, P]
    L.rslrl_linear_fwd.argtypes = [P, I64, I32, P, I32, P, I32, P, P, P]
    L.rslrl_linear_out_image_bytes.restype = SZ
    L.rslrl_linear_out_image_bytes.argtypes = []
    L.rslrl_linear_fwd_out.restype = ctypes.c_int
    L.rslrl_linear_fwd_out.argtypes = [P, I64, I32, P, I32, P, P, P, I32, P, P, P]
    L.rslrl_linear_dgrad_elu.restype = ctypes.c_int
    L.rslrl_linear_dgrad_elu.argtypes = [P, I64, I32, P, I32, P, P, P, P, P]
    L.rslrl_linear_wgrad_workspace_bytes.restype = SZ
    L.rslrl_linear_wgrad_workspace_bytes.argtypes = [I64, I32, I32]
    L.rslrl_fold_partials.restype = ctypes.c_int
    L.rslrl_fold_partials.argtypes = [P, I64, I64, P, P, SZ, P]
    L.rslrl_normal_affine.restype = ctypes.c_int
    L.rslrl_normal_affine.argtypes = [P, P, I64, P, I64, I64, I32, P]
    L.rslrl_fold_partials_ex.restype = ctypes.c_int
    L.rslrl_fold_partials_ex.argtypes = [P, I64, I64, P, I64, I32, I32, P, SZ, P]
    L.rslrl_fold_partials_workspace_bytes.restype = SZ
    L.rslrl_fold_partials_workspace_bytes.argtypes = [I64, I64]
    L.rslrl_linear_dgrad_wgrad_partial_bytes.restype = SZ
    L.rslrl_linear_dgrad_wgrad_partial_bytes.argtypes = [I64, I32, I32]
    L.rslrl_linear_dgrad_elu_wgrad.restype = ctypes.c_int
    L.rslrl_linear_dgrad_elu_wgrad.argtypes = [P, I64, I32, I32, P, P, P, P, P, P]
    L.rslrl_linear_wgrad.restype = ctypes.c_int
    L.rslrl_linear_wgrad.argtypes = [P, P, I64, I32, I32, P, P, SZ, P]
    L.rslrl_normalizer_workspace_bytes.restype = SZ
    L.rslrl_normalizer_workspace_bytes.argtypes = [I64, I32]
    L.rslrl_normalizer_update.restype = ctypes.c_int
    L.rslrl_normalizer_update.argtypes = [P, I64, I32, I64, P, P, P, P, I64, P, SZ, P]
    L.rslrl_normalizer_apply.restype = ctypes.c_int
    L.rslrl_normalizer_apply.argtypes = [P, I64, I32, I64, P, P, F, P, P]
    L.rslrl_reward_normalize.restype = ctypes.c_int
    L.rslrl_reward_normalize.argtypes = [P, I64, F, P, I32, P, P, P, P, I64, I32, P, P, SZ, P]
    L.rslrl_rollout_record.restype = ctypes.c_int
    L.rslrl_rollout_record.argtypes = [ctypes.POINTER(RolloutArgs), P]
    L.rslrl_column_sum_fold.restype = ctypes.c_int
    L.rslrl_column_sum_fold.argtypes = [P, I64, I32, P, P]
    L.rslrl_linear_bimage_h3_bytes.restype = SZ
    L.rslrl_linear_bimage_h3_bytes.argtypes = [I32]
    L.rslrl_amax_workspace_bytes.restype = SZ
    L.rslrl_amax_workspace_bytes.argtypes = []
    L.rslrl_linear_gemm.restype = ctypes.c_int
    L.rslrl_linear_gemm.argtypes = [ctypes.POINTER(LinearArgs), P]
    L.rslrl_linear_gemm_pair.restype = ctypes.c_int
    L.rslrl_linear_gemm_pair.argtypes = [ctypes.POINTER(LinearArgs), ctypes.POINTER(LinearArgs), P]
    L.rslrl_value_head_fwd_bwd.restype = ctypes.c_int
    L.rslrl_value_head_fwd_bwd.argtypes = [ctypes.POINTER(LinearArgs), ctypes.POINTER(ValueHeadArgs), P]
    L.rslrl_value_head_partial_rows.restype = ctypes.c_int64
    L.rslrl_value_head_partial_rows.argtypes = [ctypes.c_int64, ctypes.c_int32]
    L.rslrl_actor_head_workspace_bytes.restype = ctypes.c_size_t
    L.rslrl_actor_head_workspace_bytes.argtypes = [I64]
    L.rslrl_actor_head_fwd_bwd.restype = ctypes.c_int
    L.rslrl_actor_head_fwd_bwd.argtypes = [ctypes.POINTER(LinearArgs), ctypes.POINTER(ActorHeadArgs), P, ctypes.c_size_t, P]
    L.rslrl_adam_workspace_bytes.restype = SZ
    L.rslrl_adam_workspace_bytes.argtypes = []
    L.rslrl_clip_adam_step.restype = ctypes.c_int
    L.rslrl_clip_adam_step.argtypes = [ctypes.POINTER(AdamArgs), P, SZ, P]
    L.rslrl_clip_adam_step_tail.restype = ctypes.c_int
    L.rslrl_clip_adam_step_tail.argtypes = [ctypes.POINTER(AdamArgs), ctypes.POINTER(PpoTail), P, SZ, P]
    L.rslrl_ppo_update_tail.restype = ctypes.c_int
    L.rslrl_ppo_update_tail.argtypes = [P, P, P, P, I32, F, F, P, P]
    L.rslrl_linear_wgrad_ex.restype = ctypes.c_int
    L.rslrl_linear_wgrad_ex.argtypes = [P, P, P, P, I64, I32, I32, I32, P, P, SZ, P]
    L.rslrl_linear_wgrad_bias_workspace_bytes.restype = SZ
    L.rslrl_linear_wgrad_bias_workspace_bytes.argtypes = [I64, I32, I32, I32]
    L.rslrl_linear_wgrad_bias.restype = ctypes.c_int
    L.rslrl_linear_wgrad_bias.argtypes = [P, P, P, P, I64, I32, I32, I32, I32, P, P, SZ, P]
    L.rslrl_linear_wgrad_bias_pair_workspace_bytes.restype = SZ
    L.rslrl_linear_wgrad_bias_pair_workspace_bytes.argtypes = [I64, I32, I32, I32]
    L.rslrl_hidden_bwd_slices.restype = I64
    L.rslrl_hidden_bwd_slices.argtypes = [I64]
    L.rslrl_hidden_bwd_partial_floats.restype = SZ
    L.rslrl_hidden_bwd_partial_floats.argtypes = []
    L.rslrl_hidden_bwd_pair.restype = ctypes.c_int
    L.rslrl_hidden_bwd_pair.argtypes = [ctypes.POINTER(HiddenBwdProblem), ctypes.POINTER(HiddenBwdProblem), I64, I32, P]
    L.rslrl_rollout_mlp_pair.restype = ctypes.c_int
    L.rslrl_rollout_mlp_pair.argtypes = [ctypes.POINTER(RolloutMlp), ctypes.POINTER(RolloutMlp), I64, P]
    L.rslrl_linear_wgrad_bias_pair.restype = ctypes.c_int
    L.rslrl_linear_wgrad_bias_pair.argtypes = [ctypes.POINTER(WgradProblem), ctypes.POINTER(WgradProblem), I64, I32,
                                               I32, I32, I32, I32, P]
    L.rslrl_linear_wgrad_bias_pair_slices.restype = I64
    L.rslrl_linear_wgrad_bias_pair_slices.argtypes = [I64, I32]
    L.rslrl_fold_partials_batch.restype = ctypes.c_int
    L.rslrl_fold_partials_batch.argtypes = [ctypes.POINTER(FoldJob), I32, P, SZ, P]
    L.rslrl_fold_partials_batch_workspace_bytes.restype = SZ
    L.rslrl_fold_partials_batch_workspace_bytes.argtypes = [ctypes.POINTER(FoldJob), I32]
    L.rslrl_rnd_update_workspace_bytes.restype = SZ
    L.rslrl_rnd_update_workspace_bytes.argtypes = [I64, I32, I32, I32]
    L.rslrl_rnd_update.restype = ctypes.c_int
    L.rslrl_rnd_update.argtypes = [ctypes.POINTER(RndUpdateArgs), P, SZ, P]
    L.rslrl_synthetic_env_step.restype = ctypes.c_int
    L.rslrl_synthetic_env_step.argtypes = [P, I32, P, P, P, P, I64, ctypes.c_uint64, ctypes.c_uint32, F, F, I64, P]
    L.rslrl_launch_timing_enable.restype = ctypes.c_int
    L.rslrl_launch_timing_enable.argtypes = [I32]
    L.rslrl_launch_timing_read.restype = ctypes.c_int
    L.rslrl_launch_timing_read.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    L.rslrl_launch_timing_read_tag.restype = ctypes.c_int
    L.rslrl_launch_timing_read_tag.argtypes = [I32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]


def lib():
    """Load (once) and return the ctypes handle; raises HipLibraryMissing if the .so is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipLibraryMissing(
                    f"{LIB_PATH} not found: build it with `make -C rsl_rl_amd/csrc` (or "
                    "`python -c 'import __graft_entry__ as g; g.build()'`). The rsl_rl_amd hot path has "
                    "no CPU fallback."
                )
            L = ctypes.CDLL(LIB_PATH)
            _declare(L)
            v = L.rslrl_abi_version()
            if v != ABI_VERSION:
                raise HipLibraryMissing(f"{LIB_PATH} has ABI version {v}, expected {ABI_VERSION}; rebuild it")
            _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().rslrl_status_string(rc)
        raise RslrlError(f"{what} failed with status {rc}: {msg.decode() if msg else '?'}")
