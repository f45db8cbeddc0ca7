/*
 * rslrl_amd.h -- C ABI of the MI355X (gfx950) PPO hot-path library  librslrl_amd.so
 *
 * The reference (kaixi287/rsl_rl, rsl-rl-lib 3.1.0) is pure Python/PyTorch and has no FFI; each
 * entry point below replaces one group of ATen ops on the PPO hot path, named by the reference
 * file:line it takes over.  The Python host side (rsl_rl_amd/_lib.py) binds these with ctypes and is
 * what RolloutStorage / PPO call; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Device pointers are HIP device memory (e.g. torch CUDA/HIP
 *     tensors' data_ptr()); "host" marks host memory.  `stream` is a hipStream_t (NULL = legacy
 *     default stream); every device call is stream-ordered, never synchronises the host and
 *     allocates nothing (capturable into a hipGraph).  Workspaces are caller-owned, sized by the
 *     matching *_workspace_bytes() query.
 *   - Return value: 0 = success; < 0 = rslrl argument error (RSLRL_E_*); > 0 = hipError_t of the
 *     failed launch.  rslrl_status_string() describes a code.  No exceptions cross the ABI.
 *   - Layouts follow the reference buffers (rollout_storage.py:47-68): [T, N, ...] row-major fp32,
 *     dones uint8; flat row index = t * N + n (flatten(0, 1), rollout_storage.py:168-177).
 *   - Determinism: every reduction uses a fixed partition and a fixed combine order, so results are
 *     bitwise identical run to run for the same inputs and sizes.
 */
#ifndef RSLRL_AMD_H_
#define RSLRL_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* rslrl_stream_t; /* == hipStream_t */

#define RSLRL_ABI_VERSION 21

enum {
    RSLRL_OK = 0,
    RSLRL_E_INVALID_ARGUMENT = -1,
    RSLRL_E_WORKSPACE_TOO_SMALL = -2,
    RSLRL_E_UNSUPPORTED = -3,
    RSLRL_E_MISALIGNED = -4,
    RSLRL_E_BAD_GENERATOR_STATE = -5,
};

int rslrl_abi_version(void);
const char* rslrl_status_string(int status);

/* ------------------------------------------------------------------------------------------------
 * RolloutStorage.compute_returns(last_values, gamma, lam, normalize_advantage)
 *   replaces rsl_rl/storage/rollout_storage.py:127-149 (GAE reverse scan :128-142, advantages
 *   :145, normalisation :148-149).
 * values, rewards: [T, N] fp32; dones: [T, N] uint8; last_values: [N] fp32 (device).
 * returns, advantages: [T, N] fp32 outputs (device).  returns and the un-normalised advantages are
 * bit-identical to the reference's fp32 evaluation; with normalize_advantage the advantages are
 * (adv - mean) / (std_unbiased + 1e-8) over all T*N elements (statistics accumulated in fp64).
 * ----------------------------------------------------------------------------------------------*/
size_t rslrl_compute_returns_workspace_bytes(int64_t T, int64_t N);
int rslrl_compute_returns(const float* values, const float* rewards, const uint8_t* dones,
                          const float* last_values, float gamma, float lam, int64_t T, int64_t N,
                          int32_t normalize_advantage, float* returns, float* advantages,
                          void* workspace, size_t workspace_bytes, rslrl_stream_t stream);

/* rslrl_compute_returns with normalize_advantage = 1 whose normalisation pass also fills every env-step's
 * transition-record slot (see rslrl_record_fill_slot below): records[i][slot_offset : slot_offset + 8] =
 * {values[i], log_prob[i], returns[i], advantages[i] (normalised), 0, 0, 0, 0}, i < T*N.  The storage then needs no
 * slot copy per update (rollout_storage.py:127-149 then :168-197; values identical to rslrl_compute_returns
 * followed by rslrl_record_fill_slot).  records: [T*N, record_floats] fp32, 16-byte aligned, record_floats and
 * slot_offset multiples of 4, slot_offset + 8 <= record_floats; log_prob: [T, N] fp32. */
int rslrl_compute_returns_records(const float* values, const float* rewards, const uint8_t* dones,
                                  const float* last_values, float gamma, float lam, int64_t T, int64_t N,
                                  float* returns, float* advantages, const float* log_prob, float* records,
                                  int64_t record_floats, int64_t slot_offset, void* workspace,
                                  size_t workspace_bytes, rslrl_stream_t stream);

/* rslrl_compute_returns with normalize_advantage = 1 whose normalisation pass also writes the update's scalar slot
 * array (ABI 12): slots[i] = {values[i], log_prob[i], returns[i], advantages[i] (normalised)}, i < T*N, one contiguous
 * 16-byte unit per env-step (slots: [T*N, 4] fp32, 16-byte aligned) -- coalesced stores where the in-record slots
 * of rslrl_compute_returns_records are 32-byte pieces at the record stride.  The mini-batch gather reads each drawn
 * row's slot beside its record (rslrl_gather_records_side).  Replaces rollout_storage.py:127-149 like
 * rslrl_compute_returns.
 * ABI 16: for T in {8, 16, 24, 32} and N <= 131072 whose blocks the device holds at once, the scan, the statistics and
 * the normalisation run as ONE launch (a grid barrier between the scan and the normalisation; same bits as the
 * two-launch form, RSLRL_GAE_FUSED=0 forces that).  The barrier words sit after the partials in the workspace:
 * a workspace must be zero-filled before its first use with this entry point (the library leaves it so).
 * ABI 18: the one launch takes one env per lane in 256-thread blocks (the fastest of the three one-launch forms at
 * every size measured; the LDS-staged and 64-thread forms stay selectable through rslrl_debug_knob("gae_form"), the
 * same bits).  RSLRL_GAE_COOP=1 runs it as a cooperative launch (a refused launch runs the two-launch form; off by
 * default: +6-17 us per call on this runtime).  A workspace serves one stream at a time (the barrier's ticket).  If the
 * grid barrier ever times out (blocks not co-resident) the call writes NaN advantages and sets the uint32 status word
 * at rslrl_compute_returns_status_offset() in the workspace to nonzero; the caller reads it at its next
 * synchronisation and clears it (PPO.update raises on it). */
int rslrl_compute_returns_slots(const float* values, const float* rewards, const uint8_t* dones,
                                const float* last_values, float gamma, float lam, int64_t T, int64_t N,
                                float* returns, float* advantages, const float* log_prob, float* slots,
                                void* workspace, size_t workspace_bytes, rslrl_stream_t stream);

/* ABI 18: byte offset of the uint32 barrier status word in a compute_returns workspace (0 = ok). */
size_t rslrl_compute_returns_status_offset(void);
/* ABI 18: which form rslrl_compute_returns_slots takes for these arguments on the current device: 0 = scan + normaliser
 * (two launches), 1 = one launch, one env per lane, 2 = one launch, LDS-staged tiles of 64 envs (the algorithmic bytes
 * of forms 1 and 2: read 13 B + write 24 B per env-step, + 4 B per env; form 0 also writes and re-reads the raw
 * advantages). */
int rslrl_compute_returns_slots_form(int64_t T, int64_t N, const float* values, const float* rewards,
                                     const uint8_t* dones, const float* log_prob, const float* returns,
                                     const float* advantages);
/* ABI 18: test / diagnostic knobs (not a reference interface).  "gae_form": -1 auto, else that
 * rslrl_compute_returns_slots form where it fits, the two-launch path otherwise (0 forces it; 3 = one env per lane in
 * 64-thread blocks); "gae_coop": -1 auto (RSLRL_GAE_COOP), 0 plain launch, 1
 * cooperative launch; "gae_spin_limit": polls before a grid-barrier wait gives up (default 2^22).  Writes the old
 * value into *previous (may be NULL). */
int rslrl_debug_knob(const char* name, int64_t value, int64_t* previous);

/* Advantage statistics + in-place normalisation of an arbitrary fp32 vector (the normalisation half
 * of rollout_storage.py:148-149; ppo.py:221-223 uses the same expression per mini-batch).          */
size_t rslrl_normalize_workspace_bytes(int64_t n);
int rslrl_normalize_advantages(float* advantages, int64_t n, float eps, void* workspace,
                               size_t workspace_bytes, rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * torch.randperm(n) on a CPU generator -- rollout_storage.py:165.  HOST code.
 * state: the torch CPU generator state blob (torch.Generator.get_state(), 5056 bytes, host); it is
 * read and advanced in place exactly as torch's randperm_cpu advances it, so the caller writes it
 * back with Generator.set_state().  out: host int32 [n].  Requires 0 <= n < 2^31.
 * ----------------------------------------------------------------------------------------------*/
int rslrl_randperm_mt19937(uint8_t* state, size_t state_bytes, int64_t n, int32_t* out);

/* ------------------------------------------------------------------------------------------------
 * Multi-field row gather -- rollout_storage.py:168-197 (`field.flatten(0,1)[batch_idx]` for every
 * field of the mini-batch in one launch).  dst[r] = src[indices[r]] row by row for each field.
 * row_bytes must be a multiple of 4; rows with row_bytes % 16 == 0 and 16-byte aligned pointers
 * move in 16-byte units.  indices: device int32 [num_rows], each in [0, rows of src).
 * ----------------------------------------------------------------------------------------------*/
#define RSLRL_MAX_GATHER_FIELDS 16
typedef struct {
    const void* src; /* device, [rows, row_bytes] */
    void* dst;       /* device, [num_rows, row_bytes] */
    int64_t row_bytes;
} rslrl_gather_field_t;

int rslrl_gather_rows(const rslrl_gather_field_t* fields /* host array */, int32_t num_fields,
                      const int32_t* indices, int64_t num_rows, rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Transition records -- the same mini-batch assembly (rollout_storage.py:168-197) over a storage whose
 * gathered fields live side by side in one fp32 record per env-step ([T*N, record_floats], record_floats
 * % 4 == 0, records 16-byte aligned; RolloutStorage's record layout).  A random row then costs the record's
 * whole 128-byte lines instead of one line per field, and the scalar fields no line each.
 *
 * rslrl_gather_records: for each field f, dst_f[r] = records[indices[r]][offset_f : offset_f + width_f]
 *   (dst_f contiguous [num_rows, width_f]); the record's first max(offset_f + width_f) floats (<= 256)
 *   are read once per row.  indices: device int32 [num_rows], each in [0, number of records).
 * rslrl_record_fill_slot: records[i][offset : offset + slot_floats] = row_src[i][0 : row_width] (contiguous
 *   [n, row_width]), then columns[j][i] for j < num_columns (<= 4), then zeros -- the slot written whole.
 *   RolloutStorage's slot is {value, log-prob, return, advantage, 0, 0, 0, 0}, a 32-byte piece of its own
 *   filled once per update (written whole: no partial-piece writes).
 *   offset, slot_floats % 4 == 0, slot_floats <= 64.
 * ----------------------------------------------------------------------------------------------*/
#define RSLRL_MAX_RECORD_FLOATS 256
typedef struct {
    int64_t offset; /* floats from the record start */
    int64_t width;  /* floats */
    float* dst;     /* device, [num_rows, width] */
} rslrl_record_field_t;

int rslrl_gather_records(const float* records, int64_t record_floats, const rslrl_record_field_t* fields /* host */,
                         int32_t num_fields, const int32_t* indices, int64_t num_rows, rslrl_stream_t stream);
/* rslrl_gather_records plus one 16-byte unit per row from a side array (ABI 12): for each side field g,
 * dst_g[r] = side[indices[r]][offset_g : offset_g + width_g] (offset_g + width_g <= 4; side: [n, 4] fp32, 16-byte
 * aligned) -- RolloutStorage's scalar slot array {value, log-prob, return, advantage} (rslrl_compute_returns_slots).
 * num_fields + num_side_fields <= RSLRL_MAX_GATHER_FIELDS. */
int rslrl_gather_records_side(const float* records, int64_t record_floats, const rslrl_record_field_t* fields,
                              int32_t num_fields, const float* side, const rslrl_record_field_t* side_fields,
                              int32_t num_side_fields, const int32_t* indices, int64_t num_rows,
                              rslrl_stream_t stream);
int rslrl_record_fill_slot(float* records, int64_t record_floats, int64_t offset, int32_t slot_floats,
                           const float* row_src, int32_t row_width,
                           const float* const* columns /* host array of device pointers */, int32_t num_columns,
                           int64_t n, rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Fused PPO loss forward + backward for one mini-batch -- rsl_rl/algorithms/ppo.py:221-223
 * (optional per-mini-batch advantage normalisation), :259-269 (KL), :297-302 (clipped surrogate),
 * :305-313 (clipped value loss), :315 (total), and autograd's backward of :368 down to the policy
 * outputs (the Normal log_prob / entropy of actor_critic.py:106-171 included).
 *
 * Inputs, all device fp32, B rows:
 *   mu [B, A] (row stride mu_stride elements)   sigma: sigma_mode 0 -> [A] shared by all rows;
 *   values V [B]                                         sigma_mode 1 -> [B, A] (row stride sigma_stride)
 *   actions, old_mu, old_sigma [B, A] contiguous; old_logp, advantages, target_values, returns [B]
 * Outputs:
 *   grad_mu [B, A] (row stride grad_mu_stride); grad_sigma: mode 0 -> [A] (summed over rows),
 *   mode 1 -> [B, A] (row stride grad_sigma_stride); grad_values [B]; all are d(loss)/d(input) for
 *   a unit upstream gradient.
 *   stats [8] fp32: loss, surrogate_loss, value_loss, entropy_mean, kl_mean, adv_mean, adv_std, 0.
 * ----------------------------------------------------------------------------------------------*/
typedef struct {
    int64_t B;
    int32_t A;
    int32_t sigma_mode; /* 0: shared [A]; 1: per-row [B, A] */
    const float* mu;
    int64_t mu_stride;
    const float* sigma;
    int64_t sigma_stride;
    const float* values;
    const float* actions;
    const float* old_logp;
    const float* advantages;
    const float* target_values;
    const float* returns;
    const float* old_mu;
    const float* old_sigma;
    float clip_param;
    float value_loss_coef;
    float entropy_coef;
    int32_t use_clipped_value_loss;
    int32_t compute_kl;
    int32_t normalize_advantage; /* ppo.py:221-223 */
    float* grad_mu;
    int64_t grad_mu_stride;
    float* grad_sigma;
    int64_t grad_sigma_stride;
    float* grad_values;
    float* stats;
    int64_t grad_values_stride; /* elements between rows of grad_values (0 or 1: contiguous [B]); e.g. 4 writes
                                   column 0 of a zero-padded [B, 4] buffer, the value head's padded gradient */
} rslrl_ppo_loss_args_t;

#define RSLRL_PPO_LOSS_MAX_ACTIONS 64
/* The workspace starts with an arrival counter that must be ZERO when the workspace is first used
 * (e.g. hipMemset once after allocation); every call leaves it zero again.  The partial sums are folded
 * by the last-arriving workgroup inside the one loss launch (no separate reduction kernel). */
size_t rslrl_ppo_loss_workspace_bytes(int64_t B, int32_t A);
int rslrl_ppo_loss_fwd_bwd(const rslrl_ppo_loss_args_t* args /* host struct */, void* workspace,
                           size_t workspace_bytes, rslrl_stream_t stream);

/* Per-mini-batch tail of PPO.update on device scalars (one launch): when lr is non-NULL, the adaptive-KL rule
 * of ppo.py:280-284 -- fp32 kl = *kl (stats[4], or the all-reduced mean), kl > kl_hi (= fp32(2 kl*)):
 * lr = max(lr / 1.5, 1e-5); 0 < kl < kl_lo (= fp32(kl* / 2)): lr = min(lr * 1.5, 1e-2); lr is fp64 (the
 * reference's Python float), rounded through fp32 when round_fp32 (multi-GPU broadcast, ppo.py:288-290);
 * *lr32 = fp32(lr) (the optimizer's tensor lr); and when sums is non-NULL, sums[0..2] += (value, surrogate,
 * entropy) of stats (ppo.py:387-395, fp64).  Replaces the reference's host-side logic and .item() syncs. */
int rslrl_ppo_update_tail(const float* stats, const float* kl, double* lr, float* lr32, int32_t round_fp32,
                          float kl_hi, float kl_lo, double* sums, rslrl_stream_t stream);

/* Gradient-norm clipping + Adam step over a parameter list (ppo.py:373-374: clip_grad_norm_ then
 * optimizer.step() of torch.optim.Adam(fused), no weight decay / amsgrad / maximize), two launches:
 * ||g||_2 over every tensor (fp64, fixed order), coef = min(1, max_grad_norm / (||g|| + 1e-6)) (NaN stays
 * NaN like torch.clamp; no clipping when max_grad_norm <= 0), every step += 1; then per element grad = g * coef
 * (written back, as clip_grad_norm_ leaves .grad) and torch's fused-Adam arithmetic on it.
 * lr_dev (fp32 device scalar) overrides lr when non-NULL.  offsets are filled by the call.  workspace:
 * rslrl_adam_workspace_bytes(), zero-filled once (an arrival counter every call leaves zero). */
#define RSLRL_ADAM_MAX_TENSORS 24
typedef struct {
    float* param;
    float* grad; /* read, then overwritten with the clipped gradient */
    float* exp_avg;
    float* exp_avg_sq;
    float* step; /* fp32 device scalar (torch's fused-Adam state["step"]) */
    int64_t numel;
} rslrl_adam_tensor_t;
typedef struct {
    int32_t n;
    float max_grad_norm;
    double lr;
    const float* lr_dev;
    double beta1;
    double beta2;
    double eps;
    int64_t offsets[RSLRL_ADAM_MAX_TENSORS + 1];
    rslrl_adam_tensor_t t[RSLRL_ADAM_MAX_TENSORS];
} rslrl_adam_args_t;
size_t rslrl_adam_workspace_bytes(void);
int rslrl_clip_adam_step(const rslrl_adam_args_t* args /* host struct */, void* workspace, size_t workspace_bytes,
                         rslrl_stream_t stream);

/* ABI 21: rslrl_ppo_update_tail and rslrl_clip_adam_step in the clip-and-Adam launches (one launch less per
 * mini-batch): the tail's arguments as a struct (the meanings of rslrl_ppo_update_tail's); its lr rule and loss sums
 * run in the norm launch before the step sizes are derived from the new lr (args->lr_dev is then normally tail->lr32).
 * The same values as the two calls in sequence. */
typedef struct {
    const float* stats;
    const float* kl;   /* with lr */
    double* lr;        /* NULL: no lr rule (the loss sums only) */
    float* lr32;       /* with lr */
    int32_t round_fp32;
    float kl_hi;
    float kl_lo;
    double* sums;      /* NULL: no loss sums */
} rslrl_ppo_tail_t;
int rslrl_clip_adam_step_tail(const rslrl_adam_args_t* args, const rslrl_ppo_tail_t* tail, void* workspace,
                              size_t workspace_bytes, rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Actor/critic MLP layers on MFMA -- rsl_rl/networks/mlp.py:59-114
 * (nn.Linear + ELU(alpha=1) blocks) and their autograd backward.
 *   rslrl_linear_fwd:       y[M,N] = act(x[M,K] weight[N,K]^T + bias[N]); act 0 = identity, 1 = ELU.
 *   rslrl_linear_dgrad_elu: dz_prev[M,K] = (dz[M,Nred] weight_t[K,Nred]^T) * ELU'(h[M,K]), where h is the
 *                           ELU output feeding this layer (ELU'(z) = 1 if h > 0 else h + 1), and the
 *                           per-128-row-tile column sums of dz_prev into colsum_partials
 *                           [rslrl_linear_tiles(M), K] (one row per tile; -> the previous layer's bias
 *                           gradient); weight_t is the layer weight transposed ([K, Nred] row-major).
 *   rslrl_column_sum_fold:  out[N] = sum over tiles of partials[tiles, N] (fixed order, fp64; two launches).
 *                           The partials are scratch: the fold overwrites them.
 *   bimage (both calls): NULL -> exact f32 arithmetic (v_mfma_f32_32x32x2_f32, a k-ordered f32 fma
 *                           chain) on weight / weight_t.  Non-NULL -> the "x6" split-bf16 path: the B
 *                           operand comes from an image built by rslrl_linear_prepare_bimage (weight / weight_t
 *                           may then be NULL), every fp32 operand is split into three bf16 planes and six bf16
 *                           MFMA products per k step accumulate in fp32 -- the error of an fp32 GEMM at 2.67x
 *                           fewer MFMA cycles (tests/test_gpu_fused_mlp.py: error vs fp64 next to torch fp32).
 *   rslrl_linear_prepare_bimage: image of the B operand B[n][k], n < rows <= 256, k < depth:
 *                           B[n][k] = transposed ? src[k * rows + n] : src[n * depth + k].  For linear_fwd
 *                           pass the weight [N, K] (rows N, depth K, transposed 0); for linear_dgrad_elu the
 *                           weight [Nred, K] itself with rows K, depth Nred, transposed 1.  The image is
 *                           rslrl_linear_bimage_bytes(depth) bytes, 16-byte aligned; it stays valid until the
 *                           weight changes.
 *   rslrl_linear_prepare_bimages: the same for n <= 16 images in one launch (one descriptor each).
 * Requirements: N (resp. K) <= 256; K (resp. Nred) % 4 == 0; x/dz and the weights 16-byte aligned.
 * ----------------------------------------------------------------------------------------------*/
int64_t rslrl_linear_tiles(int64_t M);
size_t rslrl_linear_bimage_bytes(int32_t depth);
int rslrl_linear_prepare_bimage(const float* src, int32_t rows, int32_t depth, int32_t transposed, void* image,
                                rslrl_stream_t stream);
typedef struct {
    const float* src;
    void* image;
    int32_t rows;
    int32_t depth;
    int32_t transposed;
    int32_t layout; /* RSLRL_BIMAGE_LAYOUT_GEMM (0) or RSLRL_BIMAGE_LAYOUT_OUT (1, see rslrl_linear_fwd_out) */
} rslrl_bimage_desc_t;
#define RSLRL_BIMAGE_LAYOUT_GEMM 0
#define RSLRL_BIMAGE_LAYOUT_OUT 1
#define RSLRL_BIMAGE_LAYOUT_H3 2 /* h3 arithmetic (rslrl_linear_gemm): rslrl_linear_bimage_h3_bytes(depth) bytes */
#define RSLRL_MAX_BIMAGES 16
int rslrl_linear_prepare_bimages(const rslrl_bimage_desc_t* descs, int32_t n, rslrl_stream_t stream);
int rslrl_linear_fwd(const float* x, int64_t M, int32_t K, const float* weight, int32_t N, const float* bias,
                     int32_t activation, float* y, const void* bimage, rslrl_stream_t stream);
int rslrl_linear_dgrad_elu(const float* dz, int64_t M, int32_t Nred, const float* weight_t, int32_t K,
                           const float* h, float* dz_prev, float* colsum_partials, const void* bimage,
                           rslrl_stream_t stream);
int rslrl_column_sum_fold(float* partials, int64_t tiles, int32_t N, float* out, rslrl_stream_t stream);

/* Last hidden layer and output layer in one x6 launch (the MLP's final Linear, rsl_rl/networks/mlp.py:106-114,
 * 1-32 outputs): h = ELU(x[M,K] W[N,K]^T + bias[N]) -- written to h_out[M,N] unless h_out is NULL (inference:
 * the activation then never reaches HBM) -- and y[M,Nout] = h W_out[Nout,N]^T + out_bias[Nout].  bimage is W's
 * image (layout 0); out_image (rslrl_linear_out_image_bytes() bytes) is W_out's image built with a descriptor
 * {src = W_out, rows = Nout <= 32, depth = N, transposed = 0, layout = RSLRL_BIMAGE_LAYOUT_OUT}.  N % 4 == 0. */
size_t rslrl_linear_out_image_bytes(void);
int rslrl_linear_fwd_out(const float* x, int64_t M, int32_t K, const float* bias, int32_t N, const void* bimage,
                         float* h_out, const float* out_bias, int32_t Nout, const void* out_image, float* y,
                         rslrl_stream_t stream);

/* Weight gradient of a linear layer on the x6 path: dw[N,K] = dz[M,N]^T x[M,K] (the autograd backward of
 * nn.Linear.weight; the reference's cuBLAS GEMM).  N, K <= 256 and % 4 == 0; dz, x 16-byte aligned.  The
 * rows are split over workgroups whose partial tiles go to the workspace
 * (rslrl_linear_wgrad_workspace_bytes) and are added in a fixed order in fp64: deterministic. */
size_t rslrl_linear_wgrad_workspace_bytes(int64_t M, int32_t N, int32_t K);
/* out[NK] = sum over s < S of partials[s][NK] in fp64, in an order fixed by (S, NK) (NK % 4 == 0; 16-byte
 * aligned).  Many slices over few columns fold in two stages through an fp64 workspace of
 * rslrl_fold_partials_workspace_bytes(S, NK) bytes (0: none needed, workspace may be NULL). */
size_t rslrl_fold_partials_workspace_bytes(int64_t S, int64_t NK);
int rslrl_fold_partials(const float* partials, int64_t S, int64_t NK, float* out, void* workspace,
                        size_t workspace_bytes, rslrl_stream_t stream);
/* rslrl_fold_partials writing only the first out_len (<= NK) sums, and the leading t_rows x t_cols block of them
 * transposed (sum e = r * t_cols + c -> out[c * t_rows + r]; t_rows = t_cols = 0: none) -- a weight gradient
 * computed as (x^T dz) lands in W's [t_cols, t_rows] layout with its bias sums after it, and a partial row padded to
 * a multiple of 4 lands in an exact-size destination.  out needs 4-byte alignment only. */
int rslrl_fold_partials_ex(const float* partials, int64_t S, int64_t NK, float* out, int64_t out_len, int32_t t_rows,
                           int32_t t_cols, void* workspace, size_t workspace_bytes, rslrl_stream_t stream);
/* Up to 16 folds in one launch, each as rslrl_fold_partials_ex (64 columns per workgroup; a narrow job with more
 * than 256 slices is also split into up to 16 slice groups whose fp64 sums the last-arriving group adds in order;
 * fp64 in a fixed order that depends on S alone).  The folds of one backward pass (every layer of the actor and the
 * critic) run as one launch instead of one or two each.  Workspace: rslrl_fold_partials_batch_workspace_bytes(jobs,
 * n) bytes, 256-byte aligned, ZERO-FILLED before its first use (its leading arrival counters are left zero by every
 * call; reuse one buffer per stream); NULL when that size is <= 256. */
typedef struct {
    const float* partials; /* [S][NK], 16-byte aligned */
    int64_t S;
    int64_t NK;            /* multiple of 4 */
    float* out;
    int64_t out_len;
    int32_t t_rows, t_cols;
} rslrl_fold_job_t;
size_t rslrl_fold_partials_batch_workspace_bytes(const rslrl_fold_job_t* jobs, int32_t n);
int rslrl_fold_partials_batch(const rslrl_fold_job_t* jobs, int32_t n, void* workspace, size_t workspace_bytes,
                              rslrl_stream_t stream);

/* Output-layer backward in one launch (1 <= Nred <= 16, dz rows of Nred floats -- a 1-wide value head's [M, 1]
 * gradient as it is; fp32 FMAs on the VALU, W rebuilt exactly from its x6 image -- RSLRL_OUT_BWD=mfma selects the
 * x6 MFMA kernel, Nred % 4 == 0 only): rslrl_linear_dgrad_elu's outputs plus this layer's weight gradient
 * dW[Nred, K] = dz^T h and bias gradient db[Nred] = column sums of dz, as per-128-row-tile partials
 * [rslrl_linear_tiles(M)][P], P = Nred * K + Nred rounded up to a multiple of 4 (dW row-major, then db, then
 * zeros; rslrl_linear_dgrad_wgrad_partial_bytes), folded by rslrl_fold_partials over P columns.
 * The reference runs these as three autograd GEMM/elementwise steps over the same h (mlp.py:106-114). */
size_t rslrl_linear_dgrad_wgrad_partial_bytes(int64_t M, int32_t Nred, int32_t K);
int rslrl_linear_dgrad_elu_wgrad(const float* dz, int64_t M, int32_t Nred, int32_t K, const float* h, float* dz_prev,
                                 float* colsum_partials, const void* bimage, float* wgrad_partials,
                                 rslrl_stream_t stream);
int rslrl_linear_wgrad(const float* dz, const float* x, int64_t M, int32_t N, int32_t K, float* dw, void* workspace,
                       size_t workspace_bytes, rslrl_stream_t stream);

/* "h3" arithmetic (opt-in, REDUCED precision: 22-bit operands) and the generic entry point of the fused linear
 * ops.  The default path (networks/fused_mlp.py, RSLRL_GEMM_MODE unset) calls it with arith = X6 only.
 * h3: every fp32 operand x is scaled by a power of two s (max |s x| < 2^15) and split into two fp16 planes
 * x0 + x1 (22 significant bits); three fp16 MFMA products a0b0 + a0b1 + a1b0 accumulate in fp32 and the
 * result is divided by the scales (exact) -- half the MFMA work of x6 at an fp32 GEMM's normwise error
 * (tests/test_gpu_h3.py measures it against fp64 next to torch's fp32 GEMM).  The A operand's scale comes
 * from a_amax, a device scalar max |A| that A's producer wrote through amax_out (every op here can write
 * one; the first layer's input has no producer and stays on x6); the B image (layout H3) carries a scale
 * per row of B.
 *   op                         A (a, [M, K])  output                      B image (rows = N, depth = K)
 *   RSLRL_LINEAR_FWD[_ELU]     x              c = act(x W^T + bias) [M,N]  W [N, K]
 *   RSLRL_LINEAR_DGRAD_ELU     dz             c = (dz W) * ELU'(h) [M,N]   W^T (transposed image of W [K, N])
 *                                             + colsum_partials [rslrl_linear_tiles(M), N] (optional: NULL skips)
 *   RSLRL_LINEAR_DGRAD_ELU_WGRAD  (x6 only)   as rslrl_linear_dgrad_elu_wgrad (K = Nred <= 16)
 *   RSLRL_LINEAR_FWD_OUT       x              c = h (nullable), y = h W_out^T + out_bias (rslrl_linear_fwd_out)
 * amax_out (optional, not for FWD_OUT): max |c| over the output, published by the launch's last workgroup;
 * needs amax_workspace (rslrl_amax_workspace_bytes(), zero-filled once; every launch leaves it zero; one
 * workspace per stream).
 * rslrl_linear_wgrad_ex: rslrl_linear_wgrad with arith = X6 | H3 (H3: dz_amax, x_amax = max |dz|, max |x|). */
#define RSLRL_ARITH_X6 1
#define RSLRL_ARITH_H3 2
#define RSLRL_LINEAR_FWD 0
#define RSLRL_LINEAR_FWD_ELU 1
#define RSLRL_LINEAR_DGRAD_ELU 2
#define RSLRL_LINEAR_DGRAD_ELU_WGRAD 3
#define RSLRL_LINEAR_FWD_OUT 4
typedef struct {
    int32_t op;
    int32_t arith;
    const float* a;
    const float* a_amax;
    int64_t M;
    int32_t K;
    int32_t N;
    const void* bimage;
    const float* bias;
    const float* h;
    float* c;
    float* colsum_partials;
    float* wgrad_partials;
    const void* out_image;
    const float* out_bias;
    float* y;
    int32_t nout;
    float* amax_out;
    void* amax_workspace;
} rslrl_linear_args_t;
size_t rslrl_linear_bimage_h3_bytes(int32_t depth);
size_t rslrl_amax_workspace_bytes(void);
int rslrl_linear_gemm(const rslrl_linear_args_t* args /* host struct */, rslrl_stream_t stream);
/* Two RSLRL_LINEAR_FWD[_ELU] or RSLRL_LINEAR_DGRAD_ELU problems of the same op, arithmetic, M, K and N in one
 * launch (the actor's and the critic's layer l: the rollout's forward, where one problem fills half of the
 * workgroup slots at M = 65536, and the update's hidden-layer input gradients, where a problem's tile count is
 * not a whole number of slot rounds at M <= 98,304).  Results are identical to two rslrl_linear_gemm calls; distinct
 * amax workspaces when both write an amax. */
int rslrl_linear_gemm_pair(const rslrl_linear_args_t* a0, const rslrl_linear_args_t* a1, rslrl_stream_t stream);

/* The critic's last hidden layer, value head, value-loss gradient and the value head's backward in one launch:
 * rsl_rl/networks/mlp.py:106-114 (the critic's last Linear + ELU and the 1-wide output Linear), ppo.py:305-313 (value
 * loss, clipped or not) and the backward of ppo.py:367 through the value head.  a: an RSLRL_LINEAR_FWD_OUT problem
 * (x6, nout = 1, N = K = 256, M a multiple of 128) whose `y` receives V = the critic's output and whose `c` receives
 * dZ = (dV w) * ELU'(H), the gradient at the last hidden layer's pre-activation (H itself is not stored); with
 * g = value_loss_coef / M, dV is the loss kernel's d loss / dV (rslrl_ppo_loss_fwd_bwd; same bits).
 * wgrad_partials: [M / 128][260] per-tile rows [sum dV H (256) | sum dV | 0 0 0] -- the layout of the
 * RSLRL_LINEAR_DGRAD_ELU_WGRAD partials, folded by rslrl_fold_partials* into the head's [dW | db].
 * colsum_partials: optional [M / 128][256] per-tile column sums of dZ (the last hidden layer's bias gradient).
 * RSLRL_E_UNSUPPORTED (nothing launched) for any other shape. */
typedef struct {
    const float* target_values; /* [M] */
    const float* returns;       /* [M] */
    const float* out_weight;    /* [256] the value head's weight row, 16-byte aligned */
    float clip_param;
    float value_loss_coef;
    int32_t use_clipped_value_loss;
    float* wgrad_partials;  /* [M / 128][260] */
    float* colsum_partials; /* [M / 128][256] or NULL */
} rslrl_value_head_args_t;
int rslrl_value_head_fwd_bwd(const rslrl_linear_args_t* a, const rslrl_value_head_args_t* v, rslrl_stream_t stream);
/* ABI 17: how many rows of wgrad_partials the call above fills: one row per workgroup slice of the streaming form (the
 * default since round 5; at most 256), M / 128 for the tiled kernel (RSLRL_VALUE_HEAD_STREAM=0, or any call with
 * colsum_partials, which only the tiled kernel writes) -- the fold's row count.  ABI 18: with_colsum says whether the
 * call passes colsum_partials, so the count follows the same dispatch as rslrl_value_head_fwd_bwd. */
int64_t rslrl_value_head_partial_rows(int64_t M, int32_t with_colsum);

/* The actor's last hidden layer, its 12-wide output layer (the action mean), the whole PPO loss of the mini-batch and
 * the backward through the output layer in one launch (ABI 13): rsl_rl/networks/mlp.py:106-114 (the actor's last
 * Linear + ELU and the output Linear), ppo.py:259-315 (KL for the adaptive schedule, clipped surrogate, value loss
 * and entropy terms, total loss; the statistics rslrl_ppo_loss_fwd_bwd writes, d loss / d sigma of the shared std)
 * and the backward of ppo.py:367 down to the actor's last hidden pre-activation.  Replaces, for that shape, the
 * sequence rslrl_linear_gemm(RSLRL_LINEAR_FWD_OUT) -> rslrl_ppo_loss_fwd_bwd -> rslrl_linear_gemm(
 * RSLRL_LINEAR_DGRAD_ELU_WGRAD): H and d loss / d mu never reach HBM.
 * a: an RSLRL_LINEAR_FWD_OUT problem (x6, nout = 12, N = K = 256, M a multiple of 128, at most 4096 tiles) whose
 * `y` receives mu [M, 12] (the bits rslrl_linear_gemm gives) and whose `c` receives dZ [M, 256] = (d mu W_out) *
 * ELU'(H).  d mu is the loss kernel's (same bits); dZ comes from x6 products of d mu and W_out (fp32-faithful, the
 * separate output-layer backward's fp32 FMA chain differs in rounding).  Shared std only (sigma [12]); per-mini-batch
 * advantage normalisation is not fused (RSLRL_E_UNSUPPORTED: use the separate launches).
 * wgrad_partials: [M / 128][3084] per-tile rows [sum d mu^T H (12 x 256) | sum d mu (12)] -- the
 * RSLRL_LINEAR_DGRAD_ELU_WGRAD partial layout, folded by rslrl_fold_partials* into the output layer's [dW | db].
 * stats [8] and grad_sigma [12] as rslrl_ppo_loss_fwd_bwd writes them (loss-term sums fold in fp64 per 128-row tile:
 * within fp32 rounding of the loss kernel's).  grad_mu: optional [M, 12] copy of d loss / d mu (tests).
 * workspace: rslrl_actor_head_workspace_bytes(M), 16-byte aligned, zero-filled before its first use (the launch
 * leaves it re-armed). */
typedef struct {
    const float* actions;        /* [M, 12] */
    const float* old_log_prob;   /* [M] */
    const float* advantages;     /* [M] */
    const float* values;         /* [M] V of the mini-batch (the critic's output of this pass) */
    const float* target_values;  /* [M] */
    const float* returns;        /* [M] */
    const float* old_mu;         /* [M, 12] */
    const float* old_sigma;      /* [M, 12] */
    const float* sigma;          /* [12] the shared std */
    int32_t num_actions;         /* 12 */
    float clip_param;
    float value_loss_coef;
    float entropy_coef;
    int32_t use_clipped_value_loss;
    int32_t compute_kl;
    const void* out_weight_t_image; /* x6 B image (layout 0) of W_out^T: rslrl_linear_prepare_bimage(W_out, 12, 256, 1) */
    float* wgrad_partials;       /* [M / 128][3084] */
    float* grad_sigma;           /* [12] */
    float* stats;                /* [8] */
    float* grad_mu;              /* [M, 12] or NULL */
} rslrl_actor_head_args_t;
size_t rslrl_actor_head_workspace_bytes(int64_t M);
int rslrl_actor_head_fwd_bwd(const rslrl_linear_args_t* a, const rslrl_actor_head_args_t* h, void* workspace,
                             size_t workspace_bytes, rslrl_stream_t stream);
int rslrl_linear_wgrad_ex(const float* dz, const float* dz_amax, const float* x, const float* x_amax, int64_t M,
                          int32_t N, int32_t K, int32_t arith, float* dw, void* workspace, size_t workspace_bytes,
                          rslrl_stream_t stream);
/* rslrl_linear_wgrad_ex plus the bias gradient of the layer from the same staged rows: bias_side 1 -> the column
 * sums of dz (N values; N > 64), 2 -> of x (K values; the first layer's (x^T dz)^T form), 0 -> none.  dw_db
 * receives dw [N, K] followed by the column sums -- a Linear's weight and bias gradients when they are adjacent
 * (a gradient arena).  Replaces rslrl_linear_dgrad_elu's colsum partials + rslrl_column_sum_fold for that layer
 * (pass colsum_partials = NULL there).  Workspace: rslrl_linear_wgrad_bias_workspace_bytes. */
size_t rslrl_linear_wgrad_bias_workspace_bytes(int64_t M, int32_t N, int32_t K, int32_t bias_side);
int rslrl_linear_wgrad_bias(const float* dz, const float* dz_amax, const float* x, const float* x_amax, int64_t M,
                            int32_t N, int32_t K, int32_t arith, int32_t bias_side, float* dw_db, void* workspace,
                            size_t workspace_bytes, rslrl_stream_t stream);
/* Two rslrl_linear_wgrad_bias problems of one shape (M, N, K, arith, bias_side) in one launch -- the actor's and
 * the critic's layer l in the update's backward.  Each problem takes half the row slices of a single launch (the
 * grid stays one workgroup per CU), so its partials and their fold are half as large.  Deterministic; the slice
 * boundaries differ from rslrl_linear_wgrad_bias's, so the fp32 partial sums (not the fp64 fold) round
 * differently.  Workspace per problem: rslrl_linear_wgrad_bias_pair_workspace_bytes. */
typedef struct {
    const float* dz;
    const float* dz_amax; /* h3 only */
    const float* x;
    const float* x_amax;  /* h3 only */
    float* dw_db;
    void* workspace;
    size_t workspace_bytes;
    int32_t transpose_out; /* 1: dw_db receives dw^T ([K, N] row-major), then the column sums */
} rslrl_wgrad_problem_t;
size_t rslrl_linear_wgrad_bias_pair_workspace_bytes(int64_t M, int32_t N, int32_t K, int32_t bias_side);
/* flags RSLRL_WGRAD_NO_FOLD: leave each problem's [S][N * K + E] fp32 partials at the start of its workspace
 * (S = rslrl_linear_wgrad_bias_pair_slices(M, N)) for the caller to fold (rslrl_fold_partials_batch: the folds of a
 * whole backward pass in one launch); transpose_out / dw_db are then unused. */
#define RSLRL_WGRAD_NO_FOLD 1
int64_t rslrl_linear_wgrad_bias_pair_slices(int64_t M, int32_t N);
int rslrl_linear_wgrad_bias_pair(const rslrl_wgrad_problem_t* p0, const rslrl_wgrad_problem_t* p1, int64_t M,
                                 int32_t N, int32_t K, int32_t arith, int32_t bias_side, int32_t flags,
                                 rslrl_stream_t stream);

/* Backward of a square hidden layer (Linear(256, 256) + ELU; rsl_rl/networks/mlp.py:106-114 via ppo.py:367) in one
 * pass over the rows (ABI 15): the input gradient dz_prev = (dz W) * ELU'(h) -- the bits rslrl_linear_gemm
 * (RSLRL_LINEAR_DGRAD_ELU, x6) gives -- and the slice partials of the weight and bias gradients, [S][256 * 256 + 256]
 * rows [sum dz^T h | sum dz] (rslrl_linear_wgrad_bias bias_side 1's partial layout: rslrl_fold_partials* folds them
 * into [dW | db]), reading dz and h from HBM once instead of once per GEMM.  Replaces, for this shape, the pair
 * rslrl_linear_wgrad_bias_pair(bias_side 1) + rslrl_linear_gemm_pair(RSLRL_LINEAR_DGRAD_ELU).  M a multiple of 64
 * (else RSLRL_E_UNSUPPORTED, nothing launched); S = rslrl_hidden_bwd_slices(M) slices per problem (<= 128: a pair
 * fills 256 CUs with one workgroup each).  bimage: the x6 image of W^T (rslrl_linear_prepare_bimage(W, 256, 256, 1)).
 * p1 may be NULL (one problem).  All pointers 16-byte aligned. */
typedef struct {
    const float* dz;      /* [M, 256] gradient at this layer's pre-activation */
    const float* h;       /* [M, 256] this layer's input (the previous layer's ELU output) */
    const void* bimage;   /* x6 image of W^T */
    float* dz_prev;       /* [M, 256] */
    float* partials;      /* [S][256 * 256 + 256] */
} rslrl_hidden_bwd_problem_t;
int64_t rslrl_hidden_bwd_slices(int64_t M);
size_t rslrl_hidden_bwd_partial_floats(void);
int rslrl_hidden_bwd_pair(const rslrl_hidden_bwd_problem_t* p0, const rslrl_hidden_bwd_problem_t* p1, int64_t M,
                          int32_t width, rslrl_stream_t stream);

/* ABI 19: the rollout's actor and critic forward in one launch -- policy.act + policy.evaluate of an env step
 * (rsl_rl/algorithms/ppo.py:155-156, rsl_rl/networks/mlp.py:106-114): for each of the two problems, `hidden` Linear +
 * ELU layers of width 256 (the first on the k0-wide input x) and the output Linear, y = MLP(x), on x6 arithmetic.  The
 * hidden activations stay on chip.  y is bit-identical to the layer-by-layer path (rslrl_linear_gemm_pair per hidden
 * layer, then RSLRL_LINEAR_FWD_OUT for the last hidden layer and the output layer).  bimage[l]: layer l's layout-0
 * image (RSLRL_BIMAGE_LAYOUT_GEMM), out_image: the output layer's RSLRL_BIMAGE_LAYOUT_OUT image.  Both problems share
 * M, k0 and hidden.  RSLRL_E_UNSUPPORTED (nothing launched) unless M is a multiple of 64, k0 in {16, 32, 48, 64},
 * 2 <= hidden <= 4 and 1 <= nout <= 16.
 * ABI 20: a1 may be NULL (one network: policy.evaluate of compute_returns' last values, ppo.py:171-173, or
 * act_inference, actor_critic.py:148-151); and a problem may carry the Normal sample of ActorCritic.act
 * (actor_critic.py:142-146, distribution.sample() = normal_(0, 1) * scale + loc): with `sample` non-NULL it also rewrites
 * sample[r][o] <- sample[r][o] * sample_scale[o] + y[r][o] with torch's two roundings (mul_, then add_) -- the
 * standard normals in, the actions out, bit-identical to rslrl_normal_affine on y. */
typedef struct {
    const float* x;         /* [M, k0], 16-byte aligned */
    int32_t k0;
    int32_t hidden;
    const void* bimage[4];  /* layers 0 .. hidden - 1 */
    const float* bias[4];   /* [256] each, 16-byte aligned */
    const void* out_image;
    const float* out_bias;  /* [nout] */
    int32_t nout;
    float* y;               /* [M, nout] */
    float* sample;              /* [M, nout] standard normals in, actions out; NULL: no sample (ABI 20) */
    const float* sample_scale;  /* [nout] the shared std (required with sample) */
} rslrl_rollout_mlp_t;
int rslrl_rollout_mlp_pair(const rslrl_rollout_mlp_t* a0, const rslrl_rollout_mlp_t* a1, int64_t M,
                           rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Rollout-side record: for environment step t, in one launch,
 *   logp   = sum_a Normal(mu, sigma).log_prob(actions)           (actor_critic.py:150-151, ppo.py:135)
 *   r_int  = rnd_weight * || target(s) - predictor(s) ||_2       (rnd.py:113-135; optional)
 *   reward = (rewards + extra_reward + r_int) + gamma * (values * time_outs)   (ppo.py:147-164)
 * and writes storage row t: obs groups, actions, reward, uint8(dones), values, logp, mu, sigma
 * (rollout_storage.py:77-103).  out_* point at row t of each [T, N, d] buffer (contiguous [N, d]).
 * record_floats > 0: the copied fields (obs groups, actions, mu, sigma) live in transition records
 * (rslrl_gather_records) starting at out_records: each destination is a field of record 0 (in that order,
 * not overlapping) with row stride record_floats; record_floats, A and every obs width must be multiples
 * of 4 with 16-byte aligned pointers.  The launch writes the records whole: units outside the fields get 0
 * (no partial-line writes).
 * RND nets: Linear(in -> hidden) + ELU + Linear(hidden -> out), in, hidden <= 64, out <= 8, packed per
 * net as [W1 (hidden x in) | b1 | W2 (out x hidden) | b2]; optional state normalisation
 * (s - mean) / (std + eps).  dones / time_outs dtype: RSLRL_DTYPE_*; time_outs may be NULL.
 * ----------------------------------------------------------------------------------------------*/
#define RSLRL_DTYPE_F32 0
#define RSLRL_DTYPE_U8 1 /* also bool */
#define RSLRL_DTYPE_I32 2
#define RSLRL_DTYPE_I64 3
#define RSLRL_ROLLOUT_MAX_OBS 4
typedef struct {
    const float* src;
    float* dst;
    int64_t row_floats; /* % 4 == 0, both 16-byte aligned */
} rslrl_obs_copy_t;
typedef struct {
    int64_t N;
    int32_t A;
    int32_t sigma_mode; /* 0: sigma [A] shared; 1: [N, A] */
    const float* actions;
    const float* mu;
    const float* sigma;
    const float* values;
    const float* rewards;
    const void* dones;
    int32_t dones_dtype;
    int32_t time_outs_dtype;
    const void* time_outs;
    float gamma;
    float rnd_weight;
    const float* extra_reward; /* optional [N], added before the RND reward */
    const float* rnd_obs;      /* RND state rows (row stride rnd_obs_stride) */
    int64_t rnd_obs_stride;
    int32_t rnd_in;
    int32_t rnd_hidden;
    int32_t rnd_out;
    float rnd_state_eps;
    const float* rnd_target; /* NULL: no RND */
    const float* rnd_predictor;
    const float* rnd_state_mean; /* NULL: no state normalisation */
    const float* rnd_state_std;
    float* intrinsic_out; /* optional [N] */
    int32_t n_obs;
    int32_t reserved;
    rslrl_obs_copy_t obs[RSLRL_ROLLOUT_MAX_OBS];
    float* out_actions;
    float* out_rewards;
    uint8_t* out_dones;
    float* out_values;
    float* out_logp;
    float* out_mu;
    float* out_sigma;
    int64_t record_floats; /* 0: contiguous destinations; > 0: record row stride (floats) */
    float* out_records;    /* record mode: the first record of step t ([N, record_floats], 16-byte aligned) */
} rslrl_rollout_args_t;
int rslrl_rollout_record(const rslrl_rollout_args_t* args /* host struct */, rslrl_stream_t stream);
/* The rollout's action sample (actor_critic.py act(): Normal(mu, sigma).sample()): x [N, A] (contiguous standard
 * normals drawn by the framework's generator, so the random stream is the reference's) <- x * scale + loc, rounded
 * as torch's mul_ then add_ -- one launch for the pair.  scale / loc row strides in floats (0: one row for all rows). */
int rslrl_normal_affine(float* x, const float* scale, int64_t scale_row_stride, const float* loc,
                        int64_t loc_row_stride, int64_t N, int32_t A, rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Running normalisers, rsl_rl/networks/normalization.py.
 *   rslrl_normalizer_update: EmpiricalNormalization.update (:44-66) of the running (mean, var, std, count)
 *     [D] fp32 buffers (count: device int64) with the batch x [N, D] (row stride row_stride); no-op when
 *     until >= 0 and count >= until (tested on the device).  Workspace: rslrl_normalizer_workspace_bytes.
 *   rslrl_normalizer_apply: y [N, D] = (x - mean) / (std + eps)  (forward, :40-42).
 *   rslrl_reward_normalize: EmpiricalDiscountedVariationNormalization.forward (:84-99) over rewards [N]:
 *     when training, disc_avg = first ? r : disc_avg * gamma + r, then the update above with D = 1; then
 *     out = r / std if std > 0 else r.
 * ----------------------------------------------------------------------------------------------*/
size_t rslrl_normalizer_workspace_bytes(int64_t N, int32_t D);
int rslrl_normalizer_update(const float* x, int64_t N, int32_t D, int64_t row_stride, float* mean, float* var,
                            float* std, int64_t* count, int64_t until, void* workspace, size_t workspace_bytes,
                            rslrl_stream_t stream);
int rslrl_normalizer_apply(const float* x, int64_t N, int32_t D, int64_t row_stride, const float* mean,
                           const float* std, float eps, float* y, rslrl_stream_t stream);
int rslrl_reward_normalize(const float* rewards, int64_t N, float gamma, float* disc_avg, int32_t first, float* mean,
                           float* var, float* std, int64_t* count, int64_t until, int32_t training, float* out,
                           void* workspace, size_t workspace_bytes, rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * RND predictor loss + backward of one mini-batch (the update leg), replacing
 * rsl_rl/algorithms/ppo.py:352-363 (state extraction + normalisation, predictor / detached target forward,
 * MSE) and :369-372 (rnd_loss.backward() into the predictor's .grad) -- rsl_rl/modules/rnd.py:85-95 networks.
 *   state [B, in] rows (row stride state_stride); optional (s - mean) / (std + eps) (normalization.py:40-42);
 *   predictor / target: Linear(in -> hidden) + ELU + Linear(hidden -> out) given as four tensors each
 *   (w1 [hidden, in], b1 [hidden], w2 [out, hidden], b2 [out]); in, hidden <= 64, out <= 8.
 *   target_w1 != NULL: the target forward runs here and, when target_embedding != NULL, its [B, out] values are
 *   stored there; target_w1 == NULL: target_embedding is read instead (the target is constant within update()).
 *   grad: the predictor's gradient, packed [dW1 | db1 | dW2 | db2] (the order of predictor.parameters() -- a
 *   contiguous span of the gradient arena), overwritten with d(mse)/d(params); per-workgroup fp32 partials are
 *   folded in fp64 in a fixed order (deterministic).  loss_sum (fp64, optional) += (double)(float)mse, the
 *   reference's rnd_loss.item() accumulation (ppo.py:391-392); loss (fp32, optional) = mse.
 *   Workspace: rslrl_rnd_update_workspace_bytes.
 * ----------------------------------------------------------------------------------------------*/
#define RSLRL_RND_MAX_IN 64
#define RSLRL_RND_MAX_HIDDEN 64
#define RSLRL_RND_MAX_OUT 8
typedef struct {
    int64_t B;
    int32_t in;
    int32_t hidden;
    int32_t out;
    float state_eps;
    const float* state;
    int64_t state_stride;
    const float* state_mean; /* NULL: no state normalisation */
    const float* state_std;
    const float* pred_w1;
    const float* pred_b1;
    const float* pred_w2;
    const float* pred_b2;
    const float* target_w1; /* NULL: read target_embedding */
    const float* target_b1;
    const float* target_w2;
    const float* target_b2;
    float* target_embedding; /* [B, out] */
    float* grad;             /* [hidden*in + hidden + out*hidden + out] */
    double* loss_sum;        /* optional */
    float* loss;             /* optional */
} rslrl_rnd_update_args_t;
size_t rslrl_rnd_update_workspace_bytes(int64_t B, int32_t in, int32_t hidden, int32_t out);
int rslrl_rnd_update(const rslrl_rnd_update_args_t* args /* host struct */, void* workspace, size_t workspace_bytes,
                     rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Benchmark environment (SURVEY.md §8d synthetic VecEnv; not a reference interface): one env step for N envs in
 * one launch -- obs [N, num_obs] ~ N(0,1) (num_obs % 4 == 0, 16-byte aligned), rewards [N] ~ N(0,1), then with
 * u ~ U[0,1): episode_length += 1, over = episode_length >= max_episode_length, dones (int64) = over or
 * u < done_prob, time_outs (fp32) = over or u < done_prob * timeout_prob, episode_length = 0 where done.
 * Counter-based (philox4x32-10 keyed by seed, counter by step and env): deterministic for (seed, step).
 * ----------------------------------------------------------------------------------------------*/
int rslrl_synthetic_env_step(float* obs, int32_t num_obs, float* rewards, int64_t* dones, float* time_outs,
                             int64_t* episode_length, int64_t N, uint64_t seed, uint32_t step, float done_prob,
                             float timeout_prob, int64_t max_episode_length, rslrl_stream_t stream);

/* ------------------------------------------------------------------------------------------------
 * Live launch timing (measurement, not a reference interface; ABI 11): rslrl_launch_timing_enable(capacity > 0)
 * arms the next `capacity` launches of the PPO loss kernel (rslrl_ppo_loss_fwd_bwd's quad-layout path) to carry a
 * (start, stop) HIP event pair bound to the dispatch itself (hipExtLaunchKernel), so each elapsed time is the
 * kernel's begin-to-end duration as rocprofv3 reports it; launches on a capturing stream are never bound.
 * capacity 0 disarms and keeps the recorded launches.  rslrl_launch_timing_read synchronises the recorded
 * events and returns their summed duration (ms) and count.
 * ----------------------------------------------------------------------------------------------*/
int rslrl_launch_timing_enable(int32_t capacity);
int rslrl_launch_timing_read(double* total_ms, int64_t* launches);
/* ABI 14: the armed launches are those of the PPO loss kernel (tag 0), the rollout record (tag 1,
 * rslrl_rollout_record) and the transition-record gather (tag 2, rslrl_gather_records[_side]); this reads one tag's
 * summed duration and count (rslrl_launch_timing_read = tag 0). */
#define RSLRL_LAUNCH_TAG_PPO_LOSS 0
#define RSLRL_LAUNCH_TAG_ROLLOUT_RECORD 1
#define RSLRL_LAUNCH_TAG_GATHER_RECORDS 2
int rslrl_launch_timing_read_tag(int32_t tag, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif

#endif /* RSLRL_AMD_H_ */
