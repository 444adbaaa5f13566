/* pldepth_hip.h — C ABI of the MI355X-native (gfx950 / CDNA4) PLDepth training hot path.
 *
 * libpldepth_hip.so exports exactly the functions below. Conventions:
 *   - every entry point returns an int status (PLD_OK = 0); pld_last_error() gives the text;
 *   - all tensors are CALLER-OWNED DEVICE pointers, fp32 unless stated; activations are NHWC,
 *     filters are Keras HWIO [kh][kw][cin][cout] unless a function names a native layout;
 *   - `stream` is a hipStream_t (NULL = default stream); every call is stream-ordered and
 *     asynchronous, performs no allocation (workspaces are caller-provided, sized by the
 *     matching *_workspace_size call) and no host synchronisation, so a whole training step can
 *     be captured into one hipGraph (pld_graph_*);
 *   - no global mutable state: the library is reentrant across streams and devices.
 *
 * The reference (praneeth-b/PLDepth) is pure Python on TF2/Keras and has no FFI; each function
 * below replaces the TF/Keras op(s) named in its comment (reference file:line). INTEGRATION.md
 * shows the ctypes binding the reference-side Python would add.
 */
#ifndef PLDEPTH_HIP_H
#define PLDEPTH_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { PLD_OK = 0, PLD_ERR_ARG = 1, PLD_ERR_HIP = 2, PLD_ERR_UNSUPPORTED = 3 };

/* activation selectors (Keras 'relu', 'swish', 'sigmoid') */
enum { PLD_ACT_NONE = 0, PLD_ACT_RELU = 1, PLD_ACT_SWISH = 2, PLD_ACT_SIGMOID = 3 };

/* sampler strategies (pldepth/data/sampling.py) */
enum {
  PLD_SAMPLER_PURE = 0,   /* PurelyMaskedRandomSamplingStrategy     sampling.py:106-150, f=0.8 */
  PLD_SAMPLER_MASKED = 1, /* MaskedRandomSamplingStrategy           sampling.py:153-170, f=1.5 */
  PLD_SAMPLER_THRESH = 2, /* ThresholdedMaskedRandomSamplingStrategy sampling.py:172-208, f=1.5 */
  PLD_SAMPLER_INFO = 3    /* InformationScoreBasedSampling          sampling.py:211-242, f=5   */
};

const char* pld_last_error(void);
int pld_version(void);

/* ------------------------------------------------------------------------------------------
 * Loss: replaces prepare_fully_fledged_loss_input (pldepth/data/depth_utils.py:39-61) +
 * FullyFledgedMetaBatchListMLELoss.compute_unreduced_loss (pldepth/losses/nll_loss.py:51-62) +
 * tfr ListMLELoss + Keras SUM_OVER_BATCH_SIZE, i.e. HourglassNegativeLogLikelihood.__call__
 * (nll_loss.py:32-40) forward AND its gradient.
 *   pred   [B][HW]            predicted depth map (y_pred [B,H,W,1])
 *   y_true [B][R][L][2]       col 0 = flat pixel index as float32, col 1 = gt depth
 *   nll    [B*R]              per-list negative log-likelihood (workspace/output)
 *   loss   [1]                mean over the B*R lists
 *   dpred  [B][HW]            d loss / d pred; zeroed first when zero_dpred != 0, else added to
 * L may be 1..512. Ties keep a deterministic order (oracle/listmle.py).
 * ------------------------------------------------------------------------------------------ */
int pld_listmle_fwd_bwd(const float* pred, const float* y_true, int B, int HW, int R, int L,
                        float* nll, float* loss, float* dpred, int zero_dpred, void* stream);

/* ------------------------------------------------------------------------------------------
 * Optimizer: replaces keras.optimizers.Adam(lr, amsgrad=True) (pldepth/PLDepth.py:133), i.e. TF
 * ResourceApplyAdamWithAmsgrad on every trainable variable, fused over one flat buffer:
 *   alpha = lr*sqrt(1-b2^t)/(1-b1^t); g' = grad*grad_scale; m += (g'-m)(1-b1);
 *   v += (g'^2-v)(1-b2); vhat = max(vhat, v); p -= alpha*m/(sqrt(vhat)+eps)
 * grad_scale lets a data-parallel caller fold the 1/world averaging into the update.
 * ------------------------------------------------------------------------------------------ */
int pld_adam_amsgrad(float* param, const float* grad, float* m, float* v, float* vhat, int64_t n,
                     float lr, float beta1, float beta2, float eps, int64_t step, float grad_scale,
                     void* stream);

/* graph-replayable form: lr and the step counter are read from device memory at run time
 * (lr_dev[0], step_dev[0] >= 1), so one captured hipGraph serves every step */
int pld_adam_amsgrad_dev(float* param, const float* grad, float* m, float* v, float* vhat,
                         int64_t n, const float* lr_dev, const int64_t* step_dev, float beta1,
                         float beta2, float eps, float grad_scale, void* stream);
/* step_dev[0] += 1 (the in-graph step counter) */
int pld_step_increment(int64_t* step_dev, void* stream);
/* dev[0] = value (stream-ordered; sets the per-step learning rate ahead of a graph replay) */
int pld_set_scalar_f32(float* dev, float value, void* stream);

/* ------------------------------------------------------------------------------------------
 * Convolution (implicit GEMM on MFMA, fp32 in/out; see pld_conv_args.math): replaces Keras Conv2D /
 * TF Conv2D + Conv2DBackpropInput + Conv2DBackpropFilter (pl_hourglass.py:59-96 decoder, the
 * EfficientNetB0 1x1/3x3 convs, redweb.py convs). The input may be the channel concatenation of
 * two NHWC tensors (layers.Concatenate, pl_hourglass.py:66,75,84) — no concat is materialised.
 * Padding is explicit (TF 'same' = pad_t = ((oh-1)*sh + kh - h)/2 rounded down, rest at the
 * bottom; ZeroPadding2D(correct_pad) likewise).
 * ------------------------------------------------------------------------------------------ */
typedef struct pld_conv_args {
  const float* x1;  /* [n][h][w][c1] */
  const float* x2;  /* [n][h][w][c2] or NULL (c2 = 0) */
  int c1, c2;
  int n, h, w;
  int kh, kw, sh, sw, pad_t, pad_l;
  int oh, ow;
  int cout;
  /* optional input prologue applied to in-bounds pixels of x1 (fuses BN-apply + act of the
   * producer): x' = act(x*in_scale[c] + in_shift[c]); NULL scale = identity */
  const float* in_scale;
  const float* in_shift;
  int in_act;
  /* implicit-GEMM schedule: -1 = built-in heuristic, else an index < pld_conv_num_tiles()
   * selecting a block tile and whether the GEMM's K is split across workgroups (callers
   * autotune per layer shape; every schedule computes the same result up to fp32 summation
   * order) */
  int tile;
  /* caller workspace for split-K partial slabs of the forward / dgrad GEMMs (size from
   * pld_conv2d_{fwd,dgrad}_workspace_size; may be NULL when that size is 0) */
  void* ws;
  size_t ws_bytes;
  /* product arithmetic (PLD_MATH_*): FP32 = v_mfma_f32_32x32x2_f32, exact fp32 fmaf chains;
   * BF16X3 = each fp32 operand split into bf16 hi + lo and a.b = a_hi.b_hi + a_hi.b_lo +
   * a_lo.b_hi on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (|error| <= ~2^-16 |a.b| per
   * product; 5.3x the fp32 MFMA rate). Shapes the BF16X3 kernel does not take (channel counts
   * not a multiple of 8 for fwd/dgrad, of 4 for wgrad) run on the FP32 path. */
  int math;
  /* optional, BF16X3 fwd/dgrad only: the filter operand (w_ohwi for fwd, w_dgrad for dgrad)
   * already split by pld_filter_split, so the kernel stages it without converting; NULL = the
   * kernel splits the fp32 filter itself. Ignored on the FP32 path. */
  const void* w_split;
} pld_conv_args;

enum { PLD_MATH_FP32 = 0, PLD_MATH_BF16X3 = 1 };

/* conv forward (as pld_conv2d_fwd, no accumulate) followed by the training-mode batch statistics
 * of its output for the BatchNormalization after it (as pld_bn_stats: eps, momentum, mean,
 * invstd, optional moving statistics). Where the conv's kernel can gather the per-channel sums
 * as it stores its tile (thin 1x1 convs: the early EfficientNet expand convs, pl_hourglass.py
 * via keras efficientnet block()), the output is not read back; otherwise the two calls.
 * Workspace: pld_conv2d_fwd_bn_stats_workspace_size (besides a->ws for split-K). */
size_t pld_conv2d_fwd_bn_stats_workspace_size(const pld_conv_args* a);
int pld_conv2d_fwd_bn_stats(const pld_conv_args* a, const float* w_ohwi, const float* bias,
                            float* y, float eps, float momentum, float* mean, float* invstd,
                            float* moving_mean, float* moving_var, void* ws, size_t ws_bytes,
                            void* stream);

/* number of implicit-GEMM schedules selectable through pld_conv_args.tile (FP32 math) */
int pld_conv_num_tiles(void);
/* the same for a given PLD_MATH_* */
int pld_conv_num_schedules(int math);
/* what schedule `idx` of pld_conv_num_schedules(math) is (for a caller-side tuner): a bf16x3
 * tile, a bf16x3 tile with split-K, the bf16x3 patch kernel (3x3 convs of 32-channel inputs;
 * other shapes run the default tile), an fp32 tile, an fp32 tile with split-K, a bf16x3 tile
 * stream (a 1-D grid of persistent workgroups walking (tile, K-step) ranges: whole tiles when
 * they fill the GPU, else an even cut of the K steps with a fixup pass over the cut tiles; no
 * input prologue: such calls run the default tile), a bf16x3 row-band halo kernel (3x3 stride-1
 * 'same' convs on maps up to 56 pixels wide, forward view: each 32-channel chunk of the input
 * band staged once for its 9 taps; "x3halo/BMxBN", with split-K over whole chunks
 * "x3halosplit/BMxBN"; other shapes run the default tile); -1 if out of range. WGRAD sizes its
 * own split: only the tile classes are distinct for it. */
enum { PLD_SCHED_X3 = 0, PLD_SCHED_X3_SPLIT = 1, PLD_SCHED_X3_PATCH = 2, PLD_SCHED_FP32 = 3,
       PLD_SCHED_FP32_SPLIT = 4, PLD_SCHED_X3_STREAM = 5, PLD_SCHED_X3_HALO = 6 };
int pld_conv_schedule_class(int math, int idx);
/* a stable text name of schedule `idx` ("x3/128x128", "x3split/256x64", "x3patch/32",
 * "fp32/128x96", "fp32split/256x32"; NULL if out of range): a persisted tuning table keys its
 * choices by this name, so it stays valid across library builds whose schedule tables keep
 * the same entries (bench.py / pldepth_amd/schedules/). */
const char* pld_conv_schedule_desc(int math, int idx);
/* which kernel family a conv call runs (mode 0 = fwd, 1 = dgrad, 2 = wgrad) for its math and
 * tile: PLD_KIND_FP32 (v_mfma_f32_32x32x2_f32), PLD_KIND_BF16X3 (v_mfma_f32_32x32x16_bf16 x3) or
 * PLD_KIND_DIRECT (VALU kernels: single-output-channel 3x3 convs, thin 1x1 convs with GEMM K <= 48,
 * K x N <= 4096 — HBM-bound); -1 on bad arguments. For roofline
 * accounting (each family has its own peak). */
enum { PLD_KIND_FP32 = 0, PLD_KIND_BF16X3 = 1, PLD_KIND_DIRECT = 2 };
int pld_conv_kernel_kind(const pld_conv_args* a, int mode);
/* the name of the main kernel that call launches ("conv_x3_kernel", "conv_x3_patch_wgrad_kernel",
 * "conv_igemm_kernel", "thin1x1_kernel", "skinny_fwd_kernel", ...; "" on bad arguments): lets a
 * caller attribute HIP-event timings to rocprof kernel names (bench.py roofline.dominant). */
const char* pld_conv_kernel_name(const pld_conv_args* a, int mode);
size_t pld_conv2d_fwd_workspace_size(const pld_conv_args* a);
size_t pld_conv2d_dgrad_workspace_size(const pld_conv_args* a);

/* forward: y[n][oh][ow][cout] (+)= conv(x, W) + bias.  w_ohwi = native layout
 * [cout][kh][kw][c1+c2] (pld_filter_to_native).  bias may be NULL. */
int pld_conv2d_fwd(const pld_conv_args* a, const float* w_ohwi, const float* bias, float* y,
                   int accumulate, void* stream);

/* input gradient: dx = conv^T(dy, W) for stride-1 convolutions and for strided 1x1 unpadded
 * ones (the ResNet-50 downsampling / projection convs, redweb.py:410 -> keras resnet block1;
 * computed as a GEMM into workspace then scattered to the stride grid).  w_dgrad = native layout
 * [c1+c2][kh][kw][cout] with the taps flipped (pld_filter_to_dgrad).  dx1 receives channels
 * [0,c1), dx2 channels [c1,c1+c2); each is overwritten or accumulated per its flag. */
int pld_conv2d_dgrad(const pld_conv_args* a, const float* dy, const float* w_dgrad, float* dx1,
                     int accumulate1, float* dx2, int accumulate2, void* stream);

/* filter gradient: dw[kh][kw][c1+c2][cout] (HWIO) (+)= sum over pixels of x (x) dy.
 * Deterministic split-K: partial slabs in `ws`, then an ordered reduction. */
size_t pld_conv2d_wgrad_workspace_size(const pld_conv_args* a);
int pld_conv2d_wgrad(const pld_conv_args* a, const float* dy, float* dw, int accumulate, void* ws,
                     size_t ws_bytes, void* stream);

/* bf16x3 operand split of a row-major [rows][K] fp32 matrix (K % 8 == 0), e.g. a native or
 * dgrad filter: every 8 consecutive values v become 8 bf16 hi = rne(v) then 8 bf16 lo =
 * rne(v - hi) — 32 bytes, the size and offset of the 8 fp32 values they replace (pld_conv_args
 * .w_split). */
int pld_filter_split(const float* w, int64_t rows, int K, void* out, void* stream);

/* HWIO [kh][kw][cin][cout] -> forward native [cout][kh][kw][cin] */
int pld_filter_to_native(const float* w_hwio, int kh, int kw, int cin, int cout, float* w_ohwi,
                         void* stream);
/* HWIO -> dgrad native [cin][kh][kw][cout] with flipped taps (kh-1-i, kw-1-j) */
int pld_filter_to_dgrad(const float* w_hwio, int kh, int kw, int cin, int cout, float* w_dgrad,
                        void* stream);
/* Per-step refresh of a trainable conv's filter copies after the optimizer (replaces the
 * Keras variable read of pl_hourglass.py:56-96's decoder Conv2D kernels): forward native
 * [cout][kh][kw][cin] and, if w_dgrad is given, the flipped dgrad [cin][kh][kw][cout], each with
 * its bf16x3 split (pld_filter_split layout) when the split pointer is non-NULL — the same
 * bytes as pld_filter_to_native + pld_filter_to_dgrad + pld_filter_split, in two coalesced
 * passes (a 64x64 LDS-tiled transpose and a row permutation). */
int pld_filter_refresh(const float* w_hwio, int kh, int kw, int cin, int cout, float* w_ohwi,
                       void* w_ohwi_split, float* w_dgrad, void* w_dgrad_split, void* stream);

/* The refresh of many filters in one launch (every trainable conv after the optimizer step):
 * the caller builds a device table of descriptors once (the buffers do not move), blk0 = the
 * running sum of the nblk of the entries before it, nblk = pld_filter_refresh_plan(...) (> 0:
 * the filter takes the batched path; 0: refresh it with pld_filter_refresh). Same bytes as
 * pld_filter_refresh per filter. */
typedef struct pld_filter_refresh_desc {
  const float* w;        /* HWIO [taps][cin][cout] */
  float* w_nat;          /* [cout][taps][cin] */
  void* w_nat_split;     /* or NULL */
  float* w_dgrad;        /* [cin][taps'][cout] or NULL */
  void* w_dgrad_split;   /* or NULL */
  int taps, cin, cout;
  int blk0, nblk;
  int reserved;
} pld_filter_refresh_desc;
int pld_filter_refresh_plan(int kh, int kw, int cin, int cout, const void* w_hwio,
                            const void* w_ohwi, const void* w_ohwi_split, const void* w_dgrad,
                            const void* w_dgrad_split);
int pld_filter_refresh_multi(const pld_filter_refresh_desc* table_dev, int count,
                             int total_blocks, void* stream);

/* per-channel column sum over `rows` rows of an [rows][c] tensor: out[c] (+)= sum_r x[r][c]
 * (bias gradient of Conv2D). ws >= pld_channel_reduce_workspace_size(rows, c). */
size_t pld_channel_reduce_workspace_size(int64_t rows, int c);
int pld_channel_sum(const float* x, int64_t rows, int c, float* out, int accumulate, void* ws,
                    void* stream);

/* ------------------------------------------------------------------------------------------
 * BatchNormalization in training mode (Keras BatchNormalization, TF FusedBatchNormV3 + grad):
 * every BN of pl_hourglass.py:60-92, the 49 EfficientNet BNs (trainable, :52-57), redweb.py BNs.
 * Batch statistics over all rows of an NHWC tensor viewed as [rows][c]; biased variance for the
 * normalisation, unbiased for the moving-variance update (momentum as Keras: new = old*mom +
 * batch*(1-mom)). Statistics accumulate in fp64.
 * ------------------------------------------------------------------------------------------ */
int pld_bn_stats(const float* x, int64_t rows, int c, float eps, float momentum, float* mean,
                 float* invstd, float* moving_mean, float* moving_var, void* ws, void* stream);
/* y = act(((x-mean)*invstd)*gamma + beta) [* gate[img][c]]  (gate = SE excitation, may be NULL;
 * hw = rows per image, used only with gate) */
int pld_bn_apply(const float* x, int64_t rows, int c, const float* mean, const float* invstd,
                 const float* gamma, const float* beta, int act, const float* gate, int hw,
                 float* y, void* stream);
/* backward of y = act(bn(x)):  dy_eff = dy*(gate?gate[img][c]:1) + (addn?addn[img][c]:0);
 * dz = dy_eff*act'(z); dgamma (+)= sum dz*xhat; dbeta (+)= sum dz;
 * dx (=|+=) invstd*gamma*(dz - mean(dz) - xhat*mean(dz*xhat)). */
int pld_bn_bwd(const float* x, const float* dy, int64_t rows, int c, const float* mean,
               const float* invstd, const float* gamma, const float* beta, int act,
               const float* gate, const float* addn, int hw, float* dx, int dx_accumulate,
               float* dgamma, float* dbeta, int param_accumulate, void* ws, void* stream);

/* pld_bn_bwd's channel reductions + finalize only: dgamma/dbeta (=|+=) and k12 [2][c] =
 * [mean(dz) | mean(dz xhat)], for a consumer that forms dx on the fly (pld_pgemm_bn_bwd).
 * Workspace as pld_bn_bwd. */
int pld_bn_bwd_coeffs(const float* x, const float* dy, int64_t rows, int c, const float* mean,
                      const float* invstd, const float* gamma, const float* beta, int act,
                      float* dgamma, float* dbeta, int param_accumulate, float* k12, void* ws,
                      void* stream);

/* 1x1 convs with a small output width (N <= 48) whose input is formed on the fly by the op
 * before them (K % 4 == 0, K <= 240; x, dy, w, BN vectors 16-byte aligned; exact fp32 FMAs):
 *   pld_pgemm_bn_act: y (=|+=) (act(bn(x)) * gate[img]) . w^T — an EfficientNet block's
 *       project_conv over bn -> swish -> SE multiply (keras efficientnet block(), used by
 *       pl_hourglass.py:52-57), replacing pld_bn_apply(gate) + pld_conv2d_fwd; gate [n][K] per
 *       image of hw rows, or NULL;
 *   pld_pgemm_bn_bwd: y (=|+=) bnbwd(x, dy) . w^T with bnbwd = pld_bn_bwd's dx for the
 *       coefficients k12 from pld_bn_bwd_coeffs — the expand_conv's input gradient through the
 *       expand BN's backward, replacing pld_bn_bwd's apply + pld_conv2d_dgrad.
 * x, dy [rows][K]; w [N][K] (the native fwd filter, or the dgrad filter [cin][cout]); y [rows][N]. */
int pld_pgemm_ok(int k, int n);
int pld_pgemm_bn_act(const float* x, int64_t rows, int k, const float* mean, const float* invstd,
                     const float* gamma, const float* beta, int act, const float* gate, int hw,
                     const float* w, int n, float* y, int accumulate, void* stream);
int pld_pgemm_bn_bwd(const float* x, const float* dy, int64_t rows, int k, const float* mean,
                     const float* invstd, const float* gamma, const float* beta, int act,
                     const float* k12, const float* w, int n, float* y, int accumulate,
                     void* stream);

/* residual forms (ResNet-50 blocks `Add -> ReLU`, keras resnet block1; ReDWeb
 * BottleneckConvLayer `out += residual; relu` redweb.py:137-165 and FeatureFusionLayer
 * `x_left + x_up` redweb.py:270):  y = act(bn(x) + res);  backward: dz = dy*act'(bn(x)+res),
 * dgamma/dbeta/dx as pld_bn_bwd, and dres (=|+=) dz (the residual branch's gradient; NULL to
 * skip).  dx may be NULL when only dres and the parameter gradients are wanted. */
int pld_bn_add_apply(const float* x, int64_t rows, int c, const float* mean, const float* invstd,
                     const float* gamma, const float* beta, const float* res, int act, float* y,
                     void* stream);
int pld_bn_add_bwd(const float* x, const float* dy, int64_t rows, int c, const float* mean,
                   const float* invstd, const float* gamma, const float* beta, const float* res,
                   int act, float* dx, int dx_accumulate, float* dres, int dres_accumulate,
                   float* dgamma, float* dbeta, int param_accumulate, void* ws, void* stream);

/* EfficientNet's residual MBConv output (keras efficientnet.block: project BN -> Dropout(
 * drop_rate, noise_shape=(None, 1, 1, 1)) -> add([x, inputs]), the blocks pl_hourglass.py:48's
 * EfficientNetB0 stacks): y = act(bn(x) * sample_scale[img] + res), img = row / hw, in one pass
 * (the product and the sum rounded separately, as bn_apply + pld_residual_add); sample_scale
 * from pld_dropconnect_scales, NULL = pld_bn_add_apply.  Backward: the BN(+act) backward of
 * dy * sample_scale[img] (the scaled copy of dy never written); the residual branch's gradient
 * is dy itself. */
int pld_bn_scale_add_apply(const float* x, int64_t rows, int c, const float* mean,
                           const float* invstd, const float* gamma, const float* beta,
                           const float* sample_scale, int hw, const float* res, int act, float* y,
                           void* stream);
int pld_bn_bwd_scaled(const float* x, const float* dy, int64_t rows, int c, const float* mean,
                      const float* invstd, const float* gamma, const float* beta, int act,
                      const float* sample_scale, int hw, float* dx, int dx_accumulate,
                      float* dgamma, float* dbeta, int param_accumulate, void* ws, void* stream);

/* inference-mode BN (Keras BatchNormalization, training=False): scale = gamma/sqrt(mvar+eps),
 * shift = beta - mmean*scale, for pld_channel_affine_act / the conv prologue */
int pld_bn_inference_coeffs(const float* gamma, const float* beta, const float* moving_mean,
                            const float* moving_var, int c, float eps, float* scale, float* shift,
                            void* stream);
/* training-mode BN as a per-channel affine map of its input, from the batch statistics:
 * scale = gamma*invstd, shift = beta - mean*scale (the conv input prologue: the consuming conv
 * applies act(x*scale + shift) while staging its operand, so the BN output is never
 * materialised; replaces the FusedBatchNormV3 output write + the next Conv2D's read of it) */
int pld_bn_train_coeffs(const float* mean, const float* invstd, const float* gamma,
                        const float* beta, int c, float* scale, float* shift, void* stream);

/* ------------------------------------------------------------------------------------------
 * Elementwise / resampling
 * ------------------------------------------------------------------------------------------ */
/* y[r][0..cin) = x[r][c]*scale[c] + shift[c] (scale/shift NULL: identity), y[r][cin..cout) = 0,
 * cout = 4 or 8: a 3-channel network input widened for the stem conv's vector / bf16x3 kernels
 * (TF zero-pads the normalised map, so padding taps stay zero either way); replaces the
 * Rescaling + Normalization (EfficientNetB0) of the input before its stem Conv2D */
int pld_channel_pad_affine(const float* x, int64_t rows, int cin, int cout, const float* scale,
                           const float* shift, float* y, void* stream);
/* y = act(x*scale[c] + shift[c]) (input normalisation, bias+act) over [rows][c] */
int pld_channel_affine_act(const float* x, int64_t rows, int c, const float* scale,
                           const float* shift, int act, float* y, void* stream);
/* ZeroPadding2D(pad) + MaxPooling2D(k, s) (ResNet-50 stem pool1, redweb.py:410): windows read
 * zeros outside the input; argmax [n][oh][ow][c] u8 = first maximal tap (row-major) or NULL;
 * bwd gathers dy onto those taps: dx [n][h][w][c] (=|+=). */
int pld_maxpool2d_fwd(const float* x, int n, int h, int w, int c, int k, int s, int pad_t,
                      int pad_l, int oh, int ow, float* y, uint8_t* argmax, void* stream);
int pld_maxpool2d_bwd(const float* dy, const uint8_t* argmax, int n, int h, int w, int c, int k,
                      int s, int pad_t, int pad_l, int oh, int ow, float* dx, int accumulate,
                      void* stream);

/* UpSampling2D(interpolation='bilinear') x2, half-pixel centres (pl_hourglass.py:62..94):
 * x [n][h][w][c] -> y [n][2h][2w][c];  bwd: dx [n][h][w][c] (=|+=) adjoint(dy) */
int pld_upsample2x_fwd(const float* x, int n, int h, int w, int c, float* y, void* stream);
/* Same, with the decoder's training-mode BatchNormalization + Activation (pl_hourglass.py:88-90)
 * applied to each tap as it is read: x is the pre-BN conv output, act as pld_bn_apply. mean == NULL
 * is the plain upsample. */
int pld_upsample2x_fwd_bn(const float* x, int n, int h, int w, int c, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, int act,
                          float* y, void* stream);
int pld_upsample2x_bwd(const float* dy, int n, int h, int w, int c, float* dx, int accumulate,
                       void* stream);

/* The ff_effnet decoder's last stage fused (pl_hourglass.py:92-96: BatchNormalization -> ReLU ->
 * UpSampling2D(bilinear) -> Conv2D(1, 3x3, 'same') + bias), without forming the 2x map:
 * x [n][h][w][c] is the pre-BN map (c % 4 == 0, c <= 32), BN with the batch statistics
 * (mean, invstd) and gamma/beta (16-byte aligned); wt [3][3][c] (HWIO, cout 1); y / dy
 * [n][2h][2w]. The one-channel conv commutes with the per-channel upsampling: the kernels work
 * on the 9 tap maps z_t = sum_c w_t[c] relu(bn(x))_c (forward) and G_t = up^T(shift_t^T dy)
 * (backward) at 1x resolution.
 *   fwd  : y = conv(up(relu(bn(x)))) + bias    (replaces pld_upsample2x_fwd_bn + pld_conv2d_fwd)
 *   bwd  : dact [n][h][w][c] = up^T(conv^T(dy)) (the gradient w.r.t. relu(bn(x)); NULL = not
 *          wanted), dw [3][3][c] = d loss / d wt (NULL = not wanted), and, when dx is given, the
 *          whole BatchNormalization + ReLU backward of x as pld_bn_bwd(x, dact, ..., act relu)
 *          computes it (dx =|+= , dgamma/dbeta =|+= by param_accumulate), its channel
 *          reductions accumulated inside the same pass (dact must then be given: the apply reads
 *          it). Caller workspace: pld_upconv_bwd_workspace_size(c) when dw or dx is wanted.
 *   wgrad / dgrad: pld_upconv_bwd with only dw / only dact (wgrad's workspace size is bwd's). */
size_t pld_upconv_bwd_workspace_size(int c);
size_t pld_upconv_wgrad_workspace_size(int c);
int pld_upconv_fwd(const float* x, int n, int h, int w, int c, const float* mean,
                   const float* invstd, const float* gamma, const float* beta, const float* wt,
                   const float* bias, float* y, void* stream);
int pld_upconv_bwd(const float* x, int n, int h, int w, int c, const float* mean,
                   const float* invstd, const float* gamma, const float* beta, const float* wt,
                   const float* dy, float* dact, float* dw, float* dx, int dx_accumulate,
                   float* dgamma, float* dbeta, int param_accumulate, void* ws, size_t ws_bytes,
                   void* stream);
int pld_upconv_wgrad(const float* x, int n, int h, int w, int c, const float* mean,
                     const float* invstd, const float* gamma, const float* beta, const float* dy,
                     float* dw, void* ws, size_t ws_bytes, void* stream);
int pld_upconv_dgrad(const float* dy, int n, int h, int w, int c, const float* wt, float* dact,
                     void* stream);
/* y = a * sample_scale[img] + b  (EfficientNet drop-connect Dropout(noise_shape=(N,1,1,1)) +
 * residual add; the product and the sum rounded separately, as Keras' two layers);
 * sample_scale may be NULL (=1). rows_per_img*c elements per image. */
int pld_residual_add(const float* a, const float* sample_scale, const float* b, int n,
                     int64_t elems_per_img, float* y, void* stream);
/* Dropout(rate, noise_shape=(N,1,1,1)) keep factors for drop-connect: scales[i] = keep ? 1/(1-rate)
 * : 0 with keep ~ Bernoulli(1-rate) from Philox4x32-10 keyed by (seed), counter (layer,
 * image_offset+i, step). */
int pld_dropconnect_scales(float* scales, int n, float rate, uint64_t seed, uint64_t step,
                           int layer, int image_offset, void* stream);
int pld_dropconnect_scales_dev(float* scales, int n, float rate, uint64_t seed,
                               const int64_t* step_dev, int layer, int image_offset,
                               void* stream);
/* The same keep factors for nl <= 32 layers in one launch: scales[s * n + i] = the factor of
 * layer layers[s] at rate rates[s] (host arrays); the step from step_dev when it is non-NULL
 * (graph replay), else from step. */
int pld_dropconnect_scales_multi(float* scales, int n, int nl, const float* rates,
                                 const int* layers, uint64_t seed, uint64_t step,
                                 const int64_t* step_dev, int image_offset, void* stream);
/* y[i] = x[i] * sample_scale[img] (+ y[i] when accumulate) */
int pld_scale_per_sample(const float* x, const float* sample_scale, int n, int64_t elems_per_img,
                         float* y, int accumulate, void* stream);

/* ------------------------------------------------------------------------------------------
 * EfficientNet depthwise conv (DepthwiseConv2D, no bias) fwd and input gradient; filter
 * [k][k][c]; any stride, explicit (possibly asymmetric) padding.
 * ------------------------------------------------------------------------------------------ */
int pld_dwconv_fwd(const float* x, int n, int h, int w, int c, const float* wdw, int k, int s,
                   int pad_t, int pad_l, int oh, int ow, float* y, void* stream);
/* forward with the producer's training-mode BN + activation fused into the input read:
 * x' = act(((x - mean) * invstd) * gamma + beta) on in-image pixels (padding stays 0, as TF pads
 * the activated tensor); the pre-activation tensor is read instead of a materialised
 * activation (pl_hourglass.py:48 EfficientNet expand_bn -> expand_activation -> dwconv). */
int pld_dwconv_fwd_bn(const float* x, int n, int h, int w, int c, const float* wdw, int k, int s,
                      int pad_t, int pad_l, int oh, int ow, const float* mean,
                      const float* invstd, const float* gamma, const float* beta, int act,
                      float* y, void* stream);
/* pld_dwconv_fwd_bn + the training-mode batch statistics of its output y for the block's
 * BatchNormalization after the depthwise conv (eps, momentum, y_mean, y_invstd, optional moving
 * statistics: as pld_bn_stats), gathered in the conv's epilogue where the tiled kernel runs
 * (c % 16 == 0), else a pld_bn_stats pass. Workspace: pld_dwconv_fwd_bn_stats_workspace_size. */
size_t pld_dwconv_fwd_bn_stats_workspace_size(int n, int oh, int ow, int c, int s);
int pld_dwconv_fwd_bn_stats(const float* x, int n, int h, int w, int c, const float* wdw, int k,
                            int s, int pad_t, int pad_l, int oh, int ow, const float* mean,
                            const float* invstd, const float* gamma, const float* beta, int act,
                            float* y, float eps, float momentum, float* y_mean, float* y_invstd,
                            float* y_moving_mean, float* y_moving_var, void* ws, size_t ws_bytes,
                            void* stream);
int pld_dwconv_dgrad(const float* dy, int n, int h, int w, int c, const float* wdw, int k, int s,
                     int pad_t, int pad_l, int oh, int ow, float* dx, int accumulate,
                     void* stream);
/* pld_dwconv_dgrad into dact (= d act(bn(x)), the gradient at the depthwise input) fused with
 * the backward of that BatchNormalization + activation (the MBConv expand BN,
 * pl_hourglass.py:52-57 via Keras EfficientNetB0 block{i}expand_bn / expand_activation): its
 * reductions (sum dz, sum dz xhat, dz = dact act'(bn(x))) are gathered as dact is stored, then
 * dgamma / dbeta (param_accumulate) and k12 = [mean dz | mean dz xhat] (2c floats) are
 * finalized, and, when dx != NULL, dx (= the BN input gradient, dx_accumulate) is written as
 * pld_bn_bwd does. dx == NULL: coefficients only (for pld_pgemm_bn_bwd). x / mean / invstd /
 * gamma / beta 16-byte aligned. Workspace: pld_dwconv_dgrad_bn_bwd_workspace_size. */
size_t pld_dwconv_dgrad_bn_bwd_workspace_size(int n, int h, int w, int c, int s);
int pld_dwconv_dgrad_bn_bwd(const float* dy, int n, int h, int w, int c, const float* wdw, int k,
                            int s, int pad_t, int pad_l, int oh, int ow, float* dact,
                            int accumulate, const float* x, const float* mean,
                            const float* invstd, const float* gamma, const float* beta, int act,
                            float* dx, int dx_accumulate, float* dgamma, float* dbeta,
                            int param_accumulate, float* k12, void* ws, size_t ws_bytes,
                            void* stream);

/* ------------------------------------------------------------------------------------------
 * EfficientNet squeeze-and-excitation (frozen FCs, gradient flows to the input):
 *   pooled = mean_hw(a); z1 = pooled@w1 + b1; h1 = swish(z1); z2 = h1@w2 + b2; gate = sigmoid(z2)
 * (the caller applies a*gate, e.g. via pld_bn_apply's gate). w1 [c][cse], w2 [cse][c].
 * pld_se_bwd: given dy (grad of a*gate) and a, produces gate (unchanged) and addn[n][c] =
 * d(pooled)/hw so that da = dy*gate + addn (consumed by pld_bn_bwd's gate/addn).
 * ------------------------------------------------------------------------------------------ */
size_t pld_se_workspace_size(int n, int hw, int c, int cse);
int pld_se_fwd(const float* a, int n, int hw, int c, int cse, const float* w1, const float* b1,
               const float* w2, const float* b2, float* pooled, float* z1, float* gate, void* ws,
               void* stream);
int pld_se_bwd(const float* dy, const float* a, int n, int hw, int c, int cse, const float* w1,
               const float* w2, const float* z1, const float* gate, float* addn, void* ws,
               void* stream);
/* the same with a = act(((x - mean) * invstd) * gamma + beta) computed on the fly from the
 * block's pre-BN depthwise output x (the activation need not be materialised in training) */
int pld_se_fwd_bn(const float* x, const float* mean, const float* invstd, const float* gamma,
                  const float* beta, int act, int n, int hw, int c, int cse, const float* w1,
                  const float* b1, const float* w2, const float* b2, float* pooled, float* z1,
                  float* gate, void* ws, void* stream);
int pld_se_bwd_bn(const float* dy, const float* x, const float* mean, const float* invstd,
                  const float* gamma, const float* beta, int act, int n, int hw, int c, int cse,
                  const float* w1, const float* w2, const float* z1, const float* gate,
                  float* addn, void* ws, void* stream);
/* pld_se_bwd_bn + the block's BatchNormalization + activation backward in one sweep
 * (pl_hourglass.py:52-57 via Keras EfficientNet block: bn -> swish -> SE -> project): the SE
 * squeeze over (x, dy) also gathers per (image, channel) sum dy act'(z), sum act'(z) and their
 * xhat-weighted sums, from which, once addn is known, the BN's reductions follow exactly
 * (dz = (dy gate + addn) act'(z) is affine in the per-image constants gate, addn); then
 * dx (=|+=) the pre-BN gradient as pld_bn_bwd(x, dy, ..., gate, addn) computes it, and
 * dgamma/dbeta (=|+= by param_accumulate). Replaces pld_se_bwd_bn + pld_bn_bwd (one fewer pass
 * over x and dy). Workspace: pld_se_bwd_bn_full_workspace_size. */
size_t pld_se_bwd_bn_full_workspace_size(int n, int hw, int c, int cse);
int pld_se_bwd_bn_full(const float* dy, const float* x, const float* mean, const float* invstd,
                       const float* gamma, const float* beta, int act, int n, int hw, int c,
                       int cse, const float* w1, const float* w2, const float* z1,
                       const float* gate, float* addn, float* dx, int dx_accumulate,
                       float* dgamma, float* dbeta, int param_accumulate, void* ws,
                       size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Ranking sampler (pldepth/data/sampling.py), split into draws and a deterministic part.
 *   pld_sampler_compact: mask [B][H][W] (>0 valid) -> valid_idx [B][H*W] (row-major flat
 *       positions, np.where order), nvalid [B]; also gt min/max per image (Info strategy).
 *   pld_sampler_draw: Philox4x32-10 draws[b][cand][slot] in [0, nvalid[b]) keyed by
 *       (seed, step, image_offset + b, cand*L + slot) — independent of the GPU count.
 *   pld_sampler_rank: gather + per-list descending sort + strategy score + top-R selection,
 *       bit-identical to oracle/sampler.py for the same draws. out [B][R_out][L][2] float32
 *       (R_out = R, or floor(0.8R) for PURE).
 * ------------------------------------------------------------------------------------------ */
size_t pld_sampler_workspace_size(int B, int H, int W, int R, int L, int strategy);
int pld_sampler_compact(const float* mask, int B, int H, int W, const float* gt, int* valid_idx,
                        int* nvalid, float* gt_minmax, void* ws, void* stream);
/* workspace of pld_sampler_compact (per-segment counts and gt min/max) */
size_t pld_sampler_compact_workspace_size(int B, int H, int W);
int pld_sampler_draw(const int* nvalid, int B, int n_cand, int L, uint64_t seed, uint64_t step,
                     int image_offset, int* draws, void* stream);
/* graph-replayable form: the Philox step counter is read from step_dev[0] */
int pld_sampler_draw_dev(const int* nvalid, int B, int n_cand, int L, uint64_t seed,
                         const int64_t* step_dev, int image_offset, int* draws, void* stream);
int pld_sampler_rank(const float* gt, const int* valid_idx, const int* nvalid,
                     const float* gt_minmax, const int* draws, int B, int H, int W, int R, int L,
                     int strategy, float* out, void* ws, void* stream);
int pld_sampler_candidates(int R, int strategy); /* int(R * factor) */

/* ------------------------------------------------------------------------------------------
 * HR-WSI data access: tf.image.resize of decoded images / depth maps (bilinear)
 * and validity masks (nearest), TF2 semantics (half-pixel centres, no antialias),
 * pldepth/data/dao/hr_wsi.py:65-74. NHWC float32 [n][h][w][c] -> [n][oh][ow][c].
 * ------------------------------------------------------------------------------------------ */
int pld_resize_bilinear(const float* x, int n, int h, int w, int c, int oh, int ow, float* y,
                        void* stream);
int pld_resize_nearest(const float* x, int n, int h, int w, int c, int oh, int ow, float* y,
                       void* stream);

/* ------------------------------------------------------------------------------------------
 * Test-pass metrics, one workgroup per image. Pixel pairs / lists are drawn on
 * the host exactly as the reference draws them and passed as int32 flat pixel indices.
 * ------------------------------------------------------------------------------------------ */
/* pldepth/active_learning/metrics.py:60-70 ordinal_error, for n images of hw pixels:
 * err[i] = 1 - #{j : (pred[idx0[j]] > pred[idx1[j]]) == (gt[idx0[j]] > gt[idx1[j]])} / num */
int pld_ordinal_error(const float* pred, const float* gt, int n, int64_t hw, const int32_t* idx0,
                      const int32_t* idx1, int num, double* err, void* stream);
/* metrics.py:92-109 calc_d: pred min-max normalised over the image (cv2 NORM_MINMAX to [0,1]),
 * the list_size (<= 1024) listed pixels of pred and gt sorted ascending, out[i] = DCG(pred) /
 * DCG(gt) with DCG = sum_k (1 / (v_k + 1)) / log2(k + 2) (metrics.py:83-89 calcDCG) */
int pld_dcg_ratio(const float* pred, const float* gt, int n, int64_t hw, const int32_t* ids,
                  int list_size, double* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * hipGraph capture of a whole stream-ordered step (replaces Keras' per-op dispatch)
 * ------------------------------------------------------------------------------------------ */
int pld_graph_begin(void* stream);
int pld_graph_end(void* stream, void** graph_exec);
int pld_graph_launch(void* graph_exec, void* stream);
int pld_graph_destroy(void* graph_exec);

#ifdef __cplusplus
}
#endif
#endif /* PLDEPTH_HIP_H */
