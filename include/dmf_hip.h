/*
 * dmf_hip.h -- C-ABI of the MI355X (gfx950) hot path for the DCE-MRI x DWI
 * fusion classifier.
 *
 * The reference (simhelgithub/Deep-Multimodal-Fusion-..., pure Python on
 * PyTorch) has no FFI: its "plugin interface" is the nn.Module API of
 * code/model_module.py, code/foundation_model.py and code/loss.py. The
 * Python package next to this header mirrors that API and binds the entry
 * points below through ctypes (argtypes are parsed from THIS file; see
 * INTEGRATION.md). Every function:
 *   - takes plain device pointers, sizes and a hipStream_t passed as void*;
 *   - never allocates, never synchronises (hipGraph-capture safe);
 *   - returns 0 on success, <0 on error with dmf_last_error() describing it
 *     (the Python layer raises RuntimeError -- SURVEY.md 8(b) "Errors").
 *
 * Layout conventions
 *   activations : NHWC ("channels_last"); element type selected by `dtype`
 *                 (DMF_F32 = float, DMF_BF16 = bfloat16 bits in uint16);
 *                 `ld*` arguments are channel strides (elements per pixel)
 *   conv weights: forward  [Cout][KH][KW][CinP]  (dmf_conv_weight_prep mode 0)
 *                 dgrad    [CinP][KH][KW][Cout]  (mode 1)
 *                 dgrad as a forward conv of dY (stride 1): mode 1 with the
 *                 filter taps flipped (mode 2)
 *                 gradients are produced in torch layout [Cout][Cin][KH][KW]
 *   BN partials : float [tiles][C][2] (sum, sum of squares)
 *   scale_shift : float [2][C] (y = x*scale + shift)
 *   dropout rng : unsigned long long [2] = (seed, per-step offset) in device memory
 *
 * Reference interfaces each group replaces are cited per entry point.
 */
#ifndef DMF_HIP_H
#define DMF_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define DMF_ABI_VERSION 3

/* compute / storage dtypes: f32, bf16 and IEEE f16 (the reference's "16-mixed" autocast) */
enum { DMF_F32 = 0, DMF_BF16 = 1, DMF_F16 = 2 };
enum { DMF_ACT_NONE = 0, DMF_ACT_RELU = 1, DMF_ACT_GELU = 2, DMF_ACT_SIGMOID = 3 };

/* ------------------------------------------------------------- runtime */
const char* dmf_last_error(void);
int dmf_abi_version(void);
int dmf_iota_f32(float* y, long long n, float a, float b, void* stream);
/* state[1] += inc (per-step dropout offset; graph-replay safe) */
int dmf_rng_advance(unsigned long long* state, unsigned long long inc, void* stream);

/* ---------------------------------------------------- convolution engine
 * Replaces every nn.Conv2d forward/backward on the path: timm ResNet-50
 * OS8 (foundation_model.py:260-267), BackboneAdapter necks
 * (model_module.py:440-447), ResNetLiteBlock_withRecon (:259-280), ReconHead
 * (:113-118), MaskHeadResize (:150-187), Projector (:337-345),
 * FeatureDownAlign (:386-390), FusionModel.proj_in_* / reduce (:857-862,
 * :788-792), PatchEmbed.proj (transformer_model.py:17-22). */
int dmf_conv_m_tile(void);
/* the kernel body of the most recent conv launch (forward, fused-BN forward or
 * dgrad) made from this host thread: one of DMF_FORM_* (-1 before any) */
enum { DMF_FORM_IGEMM = 0, DMF_FORM_BUF = 1, DMF_FORM_BUF_INA = 2, DMF_FORM_WIDE = 3, DMF_FORM_SQ = 4,
       DMF_FORM_PS = 5, DMF_FORM_PP = 6, DMF_FORM_STEM = 7 };
int dmf_conv_last_form(void);
/* forward-conv tuning knobs, set only from code (benchmarks / A-B runs; the
 * library reads no environment): 0 = 256x256 LDS-DMA tile on (1, default) / off;
 * 1 = its scheduling variant 0..3; 2 = forced tile; 3 = statistics accumulation
 * mode; 4 = persistent 256x256 form on / off; 6 = benchmark-only skip bits of the
 * persistent form; 7 = ping-pong form mode 0..2; 8 = ping-pong persistent grid;
 * 10 = 7x7 stem kernel; 11 = statistics-only epilogue; 14 / 15 = tiles a launch
 * needs for the 256x128 / 256x256 forms; 16 = persistent-form output stores
 * nontemporal for outputs of at least this many MiB (0 = off).
 * Documented with their tests in DESIGN.md "Knobs". */
int dmf_conv_tune(int key, int value);
/* In-kernel timing stamps of the forward-conv launches (tools/stream_stamps.py): dmf_stamp_arm(buf, n)
 * arms a zeroed device buffer of n launch regions of 4096 blocks x 8 waves x [start, end] u64 (NULL
 * disarms and clears the record); each following forward-conv launch from this process takes the next
 * region, into which lane 0 of each wave writes its start and end in s_memrealtime ticks (100 MHz) --
 * graph captures keep the regions, so one replay fills them. dmf_stamp_info(i, ...): launch i's stream
 * handle, DMF_FORM_* and GEMM shape (M, N, K). */
int dmf_stamp_arm(unsigned long long* buf, int capacity);
int dmf_stamp_count(void);
int dmf_stamp_info(int i, void** stream, int* form, int* m, int* n, int* k);
/* Benchmark knobs of the weight-gradient engine: key 0 = LDS-DMA staging of the
 * bf16 transposed-read kernel on (1, default) / off; key 1 = its 128x256 tile
 * (one workgroup per CU) where K >= 256 on (1, default) / off; key 2 = the
 * transposed-read kernels 1 (default) / 2 (register-staged 128x256) / 0 (off);
 * key 3 = the 256x256 LDS-DMA tile where Cout and KH*KW*Cin are multiples of 256:
 * 0 off / 1 (default) for weights of >= 2^18 entries / 2 wherever legal;
 * key 4 = split-lane reducers of dmf_conv2d_wgrad_reduce at >= 16 splits on (1) / off;
 * key 5 = blocks the pixel splits aim for, percent of one chip-filling wave (10..400, default 50). */
int dmf_conv_wgrad_tune(int key, int value);
/* rows (M tiles) of the bn_partials slab that dmf_conv2d_fwd / _fwd_bn write
 * for this shape (the launcher picks 64- or 128-row tiles per shape) */
int dmf_conv2d_fwd_stat_tiles(int dtype, int N, int H, int W, int Cin, int ldx, int Cin2, int ldx2, int Cout, int KH,
                              int KW, int stride, int pad, int Ho, int Wo, int has_in_affine);
/* 1 when a plain 1x1 conv (Cin -> Cout over N x H x W) fed by
 * in_scale_shift runs on the same tile family as the unfused conv, so fusing
 * the producer's BN apply + activation into it saves that pass (the 256-wide
 * LDS-DMA tiles have no input-affine form); 0 -> apply the BN separately */
int dmf_conv2d_fwd_input_affine_fusable(int dtype, int N, int H, int W, int Cin, int Cout);
/* x2 (nullable): second input concatenated along channels after the Cin
 * channels of x (BackboneAdapter chain [C4, C5], model_module.py:471) */
/* in_scale_shift (nullable, single source only): the producer's batch-norm
 * apply + activation fused into the A loads, x <- in_act(x*ss[c] + ss[C+c])
 * on in-bounds elements (Bottleneck conv1->bn1->relu->conv2, adapter
 * conv->BN->GELU->conv; model_module.py:440-447). in_act is DMF_ACT_*. */
int dmf_conv2d_fwd(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* x2, int Cin2,
                   int ldx2, const void* w, int Cout, int KH, int KW, int stride, int pad, int dil, const float* bias,
                   void* y, int Ho, int Wo, int ldy, float* bn_partials, int act, const float* in_scale_shift,
                   int in_act, void* stream);
/* conv + training-mode BatchNorm2d finalize in ONE launch: every block
 * writes its per-channel (sum, sum^2) into bn_partials [mtiles][Cout][2]
 * and takes a ticket of its output-channel tile; the last block of each
 * tile reduces that tile's columns (fixed order, double) into scale_shift
 * [2][Cout] (+ save_mean_invstd, running stats, num_batches_tracked, as
 * dmf_bn_finalize) and re-zeroes its ticket. bn_tickets: >= ceil(Cout/128)
 * counters, zero on the first call (persistent per BatchNorm site). */
int dmf_conv2d_fwd_bn(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* x2, int Cin2,
                      int ldx2, const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                      const float* bias, void* y, int Ho, int Wo, int ldy, const float* in_scale_shift, int in_act,
                      float* bn_partials, unsigned* bn_tickets, double count, double unbias_count, const float* gamma,
                      const float* beta, float* running_mean, float* running_var, long long* num_batches_tracked,
                      float momentum, float eps, float* scale_shift, float* save_mean_invstd, void* stream);
/* dmf_conv2d_fwd whose epilogue ADDS each block's per-channel (sum, sum^2)
 * into bn_acc [replicas][Cout][2] -- replica (M tile % replicas), float64
 * atomics: arrival order does not show at fp32, and the replicas keep the
 * same-address contention of many M tiles off the epilogue; bn_acc zeroed by
 * the caller, one slice per BatchNorm use. No slab and no finalize launch:
 * the consumer dmf_bn_apply finalizes the statistics (training-mode
 * BatchNorm2d after every conv of timm Bottleneck, the necks, ResNetLite,
 * projectors). */
int dmf_conv2d_fwd_acc(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* x2, int Cin2,
                       int ldx2, const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                       const float* bias, void* y, int Ho, int Wo, int ldy, double* bn_acc, int replicas,
                       const float* in_scale_shift, int in_act, void* stream);
/* Two-pass conv -> BatchNorm2d (batch statistics) -> + shortcut -> ReLU of a 1x1 conv that the forward
 * never differentiates (frozen encoders, mode A: timm Bottleneck conv3 / bn3 / residual / act3,
 * foundation_model.py:260-267): the first pass accumulates the BN statistics into an arena slice
 * WITHOUT writing the conv output (dmf_conv2d_fwd_stats; finalized by dmf_bn_finalize_acc), the
 * second recomputes the conv and writes relu(y * scale_shift + shortcut) once (dmf_conv2d_fwd_affine;
 * res_scale_shift nullable: the shortcut's own BatchNorm, a projection shortcut's raw conv output).
 * Replaces the raw conv output's write and the separate BN-apply pass (its read of the raw output) by
 * a second K loop. dmf_conv2d_fwd_affine_ok: 1 when a 1x1 conv of this shape runs the persistent
 * 256x256 form both passes need (16-bit dtype, Cout % 256 == 0, N*Ho*Wo % 256 == 0). */
int dmf_conv2d_fwd_affine_ok(int dtype, int N, int H, int W, int Cin, int Cout, int stride);
/* a 1x1 conv (a token linear over its rows' NHWC view) -> bias -> GELU -> dropout(p) in one launch on
 * the persistent 256x256 form (forward-only transformer blocks' fc1 under MLP dropout,
 * transformer_model.py:128-134); keep masks on element m * Cout + n with (rng, site), the token GEMM's
 * index, so the masks equal dmf_gemm_bf16's. dmf_conv2d_fwd_drop_ok: 1 when the shape takes that form. */
int dmf_conv2d_fwd_drop_ok(int dtype, int N, int H, int W, int Cin, int Cout);
int dmf_conv2d_fwd_drop(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w, int Cout,
                        const float* bias, void* y, int ldy, int act, float dropout_p, const unsigned long long* rng,
                        int site, void* stream);
int dmf_conv2d_fwd_stats(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w, int Cout,
                         int stride, int Ho, int Wo, double* bn_acc, int replicas, void* stream);
int dmf_conv2d_fwd_affine(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w, int Cout,
                          int stride, void* y, int Ho, int Wo, int ldy, const float* scale_shift, const void* res,
                          int ldr, const float* res_scale_shift, void* stream);
/* conv (+ bias) -> + res -> act in one launch on the forms that stage the C tile through LDS (buffer-
 * load / 256x128 / 256x256 / general implicit GEMM): an eval-mode Bottleneck conv3 -> bn3 -> + shortcut
 * -> act3 (foundation_model.py:260-267) with the BatchNorm folded into w and bias by the caller, where
 * the persistent dmf_conv2d_fwd_affine form does not take the shape. res / y: NHWC rows, 16-B aligned,
 * whole 16-B channel chunks. dmf_conv2d_fwd_res_ok: 1 when the planner gives this shape such a form
 * (dmf_conv2d_fwd_res refuses the others). */
/* a token linear (1x1 conv over the rows' NHWC view) -> + bias -> dropout(p) -> x colscale -> + res, f32
 * out, on the persistent 256x256 form: the proj / fc2 linears of a transformer block that is never
 * differentiated (transformer_model.py:83-134), with k_gemm_bf16's epilogue and Philox masks (element
 * m * Cout + n, (rng, site)). res: the f32 residual stream (ldr), y: f32 (ldy), may not alias res.
 * dmf_conv2d_fwd_tokres_ok: 1 when the shape takes that form. */
int dmf_conv2d_fwd_tokres_ok(int dtype, int N, int H, int W, int Cin, int Cout);
int dmf_conv2d_fwd_tokres(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w, int Cout,
                          const float* bias, const float* colscale, const float* res, int ldr, float dropout_p,
                          const unsigned long long* rng, int site, float* y, int ldy, void* stream);
int dmf_conv2d_fwd_res_ok(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                          int dil);
int dmf_conv2d_fwd_res(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w, int Cout,
                       int KH, int KW, int stride, int pad, int dil, const float* bias, const void* res, int ldr,
                       int act, void* y, int Ho, int Wo, int ldy, void* stream);
int dmf_conv2d_dgrad(int dtype, const void* dy, int N, int Ho, int Wo, int Cout, int lddy, const void* wt, int Cin,
                     int KH, int KW, int stride, int pad, int dil, void* dx, int H, int W, int lddx, void* stream);
int dmf_conv_weight_prep(int dtype, const float* w, void* out, int Cout, int Cin, int CinP, int KH, int KW, int mode,
                         void* stream);
/* Batched re-layout: every conv weight a training step uses, in one launch
 * (replaces one dmf_conv_weight_prep per conv per step). jobs: device array of
 * dmf_wprep_job; blk: device array of nblocks block codes (job index << 40) |
 * unit, unit = first element of a 4096-element run (mode 0) or index of a
 * 64x64 output tile, K-tile major (modes 1/2). No reference
 * counterpart: the reference lets cuDNN read the torch-layout weights. */
typedef struct {
  const float* w; /* torch layout [Cout][Cin][KH][KW], fp32 */
  void* out;      /* re-laid-out copy, DMF_BF16 or DMF_F32 */
  int dtype, Cout, Cin, CinP, KH, KW, mode, pad_;
} dmf_wprep_job;
int dmf_conv_weight_prep_multi(const dmf_wprep_job* jobs, const long long* blk, long long nblocks, void* stream);
int dmf_conv2d_wgrad_splits(int dtype, int Cout, int Cin, int KH, int KW, long long M);
int dmf_conv2d_wgrad(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* x2, int Cin2,
                     int ldx2, const void* dy, int Ho, int Wo, int Cout, int lddy, int KH, int KW, int stride, int pad,
                     int dil, int splits, float* workspace, void* stream);
int dmf_conv2d_wgrad_reduce(const float* workspace, int splits, int Cout, int Cin, int CinP, int KH, int KW,
                            float* dw, int accumulate, void* stream);
/* gate gradient of a channel-gated conv input y = x*gate[N][Cin] from
 * per-sample weight-gradient slabs (dmf_conv2d_wgrad with splits = N and
 * Ho*Wo a multiple of dmf_conv2d_wgrad_pixel_step): dgate[n][c] =
 * sum_{co,r,s} W[co][c][r][s] * slab_n[co][r][s][c] / gate[n][c], w the fp32
 * torch-layout weight (SE input gate, model_module.py:584-591) */
int dmf_conv2d_wgrad_gate(const float* workspace, int N, int Cout, int Cin, int CinP, int KH, int KW, const float* w,
                          const float* gate, float* dgate, void* stream);
/* pixels per K-step of dmf_conv2d_wgrad (splits cover whole multiples of it) */
int dmf_conv2d_wgrad_pixel_step(int dtype);
/* single-output-channel convs: ReconHead.conv[3] (model_module.py:117),
 * MaskHeadResize.out (:187); weights [KH][KW][Cin] fp32 */
int dmf_conv_cout1_fwd(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const float* w,
                       const float* bias, int KH, int KW, int stride, int pad, int dil, void* y, int Ho, int Wo,
                       int ldy, int act, void* stream);
int dmf_conv_cout1_dgrad(int dtype, const void* dy, int lddy, const float* w, int N, int H, int W, int Cin, int KH,
                         int KW, int stride, int pad, int dil, int Ho, int Wo, void* dx, int lddx, void* stream);
int dmf_conv_cout1_wgrad_splits(long long M);
int dmf_conv_cout1_wgrad(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* dy, int lddy,
                         int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, int splits, float* workspace,
                         float* dw, float* db, void* stream);
/* the same with dw in torch layout [1][Cin][KH][KW] (accumulated: a parameter's .grad) */
int dmf_conv_cout1_wgrad_torch(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* dy,
                               int lddy, int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, int splits,
                               float* workspace, float* dw, float* db, void* stream);
/* single-input-channel 1x1 convs: mask_processor[0] (model_module.py:68),
 * proj_r1/proj_r2 first conv (:639-640) */
int dmf_conv_cin1_fwd(int dtype, const void* x, int ldx, const float* w, const float* bias, void* y, int ldy,
                      long long M, int Cout, int act, void* stream);
int dmf_conv_cin1_dgrad(int dtype, const void* dy, int lddy, const float* w, void* dx, int lddx, long long M,
                        int Cout, void* stream);
int dmf_conv_cin1_wgrad_tiles(long long M);
int dmf_conv_cin1_wgrad(int dtype, const void* x, int ldx, const void* dy, int lddy, long long M, int Cout,
                        float* workspace, float* dw, float* db, void* stream);

/* ---------------------------------------------------- batch norm & acts
 * nn.BatchNorm2d train/eval semantics + fused residual/activation/dropout
 * (timm Bottleneck, ResNetLite :259-307, necks, heads, projectors). */
/* workspace: dmf_bn_finalize_ws_size(ntiles, C) doubles (two-stage reduction when ntiles > 64) */
int dmf_bn_finalize_ws_size(int ntiles, int C);
int dmf_bn_finalize(const float* partials, int ntiles, int C, double count, double unbias_count,
                    const float* gamma, const float* beta, float* running_mean, float* running_var,
                    long long* num_batches_tracked, float momentum, float eps, int training, float* scale_shift,
                    float* save_mean_invstd, double* workspace, void* stream);
/* a training-mode BatchNorm2d whose batch statistics a dmf_conv2d_fwd_acc
 * launch accumulated: finalized inside dmf_bn_apply (torch semantics as
 * dmf_bn_finalize: biased batch variance, running stats with momentum and
 * the unbiased variance over unbias_count (0 -> count) rows) */
typedef struct dmf_bn_desc {
  const double* acc;            /* [replicas][C][2] (sum, sum^2) */
  const float* gamma;           /* nullable (affine=False) */
  const float* beta;
  float* running_mean;          /* nullable (no running statistics) */
  float* running_var;
  long long* num_batches_tracked; /* nullable */
  float* scale_shift;           /* out [2][C] */
  float* save_mean_invstd;      /* out [2][C], nullable */
  double count;
  double unbias_count;
  float momentum;
  float eps;
  int replicas;                 /* of acc (dmf_conv2d_fwd_acc) */
} dmf_bn_desc;
/* dmf_conv2d_fwd_affine with the BatchNorm finalized inside the launch: every block reads the
 * (sum, sum^2) replicas of bn->acc (<= 8) for the channels it stages and block 0 moves the running
 * statistics and num_batches_tracked (bn->scale_shift / save_mean_invstd are not written): the
 * dmf_bn_finalize_acc launch between the two passes of the two-pass conv3 folded in. */
int dmf_conv2d_fwd_affine_acc(int dtype, const void* x, int N, int H, int W, int Cin, int ldx, const void* w,
                              int Cout, int stride, void* y, int Ho, int Wo, int ldy, const dmf_bn_desc* bn,
                              const void* res, int ldr, const float* res_scale_shift, void* stream);
/* y = drop(act(x*a + [res*r | res])) with a = finalize(bn) when bn is given
 * (else scale_shift, else identity) and r likewise from res_bn /
 * res_scale_shift (residual optional). One launch replaces
 * dmf_bn_finalize (x2 for a projection shortcut) + dmf_affine_act; the
 * finalized scale_shift / save_mean_invstd are written for the backward.
 * C and the strides multiples of 8, 16-byte aligned tensors. */
int dmf_bn_apply(int dtype, const void* x, int ldx, const dmf_bn_desc* bn, const float* scale_shift,
                 const void* res, int ldr, const dmf_bn_desc* res_bn, const float* res_scale_shift, int act,
                 float dropout_p, const unsigned long long* rng, int site, void* y, int ldy, long long M, int C,
                 void* stream);
/* finalize (as dmf_bn_finalize, training mode) of batch statistics accumulated into an arena slice
 * [replicas][C][2] (dmf_conv2d_fwd_acc / dmf_conv2d_fwd_stats) */
int dmf_bn_finalize_acc(const double* acc, int replicas, int C, double count, double unbias_count, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, long long* num_batches_tracked,
                        float momentum, float eps, float* scale_shift, float* save_mean_invstd, void* stream);
int dmf_affine_act(int dtype, const void* x, int ldx, const float* scale_shift, const void* res, int ldr,
                   const float* res_scale_shift, int act, float dropout_p, const unsigned long long* rng, int site,
                   void* y, int ldy, long long M, int C, void* stream);
int dmf_act_bwd(int dtype, const void* dy, int lddy, const void* x, int ldx, const float* scale_shift,
                const void* res, int ldr, const float* res_scale_shift, int act, float dropout_p,
                const unsigned long long* rng, int site, void* dz, int lddz, long long M, int C, void* stream);
int dmf_bn_bwd_tiles(long long M);
int dmf_bn_bwd_reduce(int dtype, const void* dz, int lddz, const void* x, int ldx, const float* save_mean_invstd,
                      long long M, int C, float* partials, void* stream);
int dmf_bn_bwd_finalize(const float* partials, int ntiles, int C, double count, int training, const float* gamma,
                        const float* save_mean_invstd, float* dgamma, float* dbeta, float* coef, void* stream);
int dmf_bn_bwd_apply(int dtype, const void* dz, int lddz, const void* x, int ldx, const float* coef, void* dx,
                     int lddx, long long M, int C, void* stream);
/* dmf_act_bwd + dmf_bn_bwd_reduce in one pass: dz = act/dropout backward of
 * y = drop(act(x*scale_shift + residual)) written once, plus the BN column
 * partials [dmf_bn_bwd_tiles(M)][C][2] of x (the BN input) with the saved
 * (mean, invstd); ResNetLite/Bottleneck conv->BN->act backward
 * (model_module.py:259-280, timm Bottleneck). dy2 (may be null; then lddy2
 * is ignored): a second gradient of the same output, summed with dy in fp32
 * -- the next Bottleneck's shortcut gradient, handed over by that block's
 * backward instead of an autograd add pass (needs 8-channel vectors). */
int dmf_act_bwd_bn_reduce(int dtype, const void* dy, int lddy, const void* dy2, int lddy2, const void* x, int ldx,
                          const float* scale_shift,
                          const void* res, int ldr, const float* res_scale_shift, int act, float dropout_p,
                          const unsigned long long* rng, int site, const float* save_mean_invstd, void* dz, int lddz,
                          long long M, int C, float* partials, void* stream);
/* BatchNorm backward without a finalize launch: the column sums (sum dz,
 * sum dz*xhat) go by float64 atomics into [replicas][C][2] (zeroed; a slice of
 * the forward's statistics arena), and the apply finalizes them per 64-channel
 * block (dgamma / dbeta added once) -- the backward of conv -> BatchNorm2d ->
 * act of timm Bottleneck / BackboneAdapter (foundation_model.py:260-267,
 * model_module.py:440-447). C and strides multiples of 8. */
int dmf_act_bwd_bn_reduce_acc(int dtype, const void* dy, int lddy, const void* dy2, int lddy2, const void* x, int ldx,
                              const float* scale_shift,
                              const void* res, int ldr, const float* res_scale_shift, int act, float dropout_p,
                              const unsigned long long* rng, int site, const float* save_mean_invstd, void* dz,
                              int lddz, long long M, int C, double* acc, int replicas, void* stream);
int dmf_bn_bwd_apply_acc(int dtype, const void* dz, int lddz, const void* x, int ldx, const double* acc, int replicas,
                         double count, int training, const float* gamma, const float* save_mean_invstd, float* dgamma,
                         float* dbeta, void* dx, int lddx, long long M, int C, void* stream);
int dmf_col_stats_tiles(long long M);
int dmf_col_stats(int dtype, const void* x, int ldx, long long M, int C, float* partials, void* stream);

/* -------------------------------------------------- encoder elementwise
 * SEBlock (model_module.py:25-43), GroupNorm(C,C) mix (:673-675, :688-690),
 * maxpool (timm stem), proj_pool (:531-534), F.interpolate bilinear
 * (:81-87, :206-211), MaskGuidedSpatialAttention (:49-97). */
int dmf_input_prep(int dtype, const float* x, int N, int C, int H, int W, const float* gate, void* y, int Cp,
                   float* chan_mean, void* stream);
int dmf_nchw_mean(const float* x, int NC, long long HW, float* out, void* stream);
/* out[n][c] (+)= scale * sum_hw a*(b or 1); out_sq (nullable, b == NULL only)
 * also gets scale * sum_hw a^2 in the same pass. workspace (nullable):
 * dmf_nhwc_reduce_ws_size(N, HW, C) floats enable the chip-wide split form
 * (partials + ordered combine, deterministic). out == NULL (vector layout,
 * no out_sq): stage 1 only -- workspace receives dmf_nhwc_reduce_splits(N,
 * HW, C) partial planes [S][N][C] (unscaled) for a consumer that sums them
 * (dmf_se_mlp). */
int dmf_nhwc_reduce_ws_size(int N, int HW, int C);
int dmf_nhwc_reduce_splits(int N, int HW, int C);
int dmf_nhwc_reduce(int dtype, const void* a, int lda, const void* b, int ldb, int N, int HW, int C, float scale,
                    float* out, float* out_sq, int accumulate, float* workspace, void* stream);
int dmf_channel_scale(int dtype, const void* x, int ldx, const float* gate, void* y, int ldy, int N, int HW, int C,
                      void* stream);
int dmf_mix(int dtype, const void* a, int lda, const void* b, int ldb, const float* wlogit, void* z, int ldz,
            long long M, int C, void* stream);
int dmf_gn_apply(int dtype, const void* z, int ldz, const float* mean, const float* m2, const float* gamma,
                 const float* beta, float eps, void* y, int ldy, int N, int HW, int C, void* stream);
int dmf_gn_bwd(int dtype, const void* dy, int lddy, const void* z, int ldz, const float* mean, const float* m2,
               const float* gamma, float eps, float* s1, float* s2, void* dz, int lddz, int N, int HW, int C,
               void* stream);
int dmf_maxpool2d(int dtype, const void* x, int N, int H, int W, int C, int ldx, void* y, int Ho, int Wo, int ldy,
                  int k, int s, int p, void* stream);
/* 2x2 average pool of timm's ResNet-D shortcut (resnet50d, downsample_avg; reference dispatch
 * foundation_model.py:503 -> timm.create_model("resnet50d", ...) at :29): same = 0 is
 * AvgPool2d(2, s, ceil_mode=True, count_include_pad=False), same = 1 (s = 1) AvgPool2dSame(2, 1) of a
 * dilated stage (one zero row / column padded at the end, divisor 4). NHWC; Ho / Wo must be the
 * pool's output size. The backward scatters dy / divisor to every input of each window. */
int dmf_avgpool2d(int dtype, const void* x, int N, int H, int W, int C, int ldx, void* y, int Ho, int Wo, int ldy,
                  int s, int same, void* stream);
int dmf_avgpool2d_bwd(int dtype, const void* dy, int N, int H, int W, int C, int Ho, int Wo, int lddy, void* dx,
                      int lddx, int s, int same, void* stream);
int dmf_maxpool2d_bwd(int dtype, const void* x, int N, int H, int W, int C, int ldx, const void* dy, int Ho, int Wo,
                      int lddy, void* dx, int lddx, int k, int s, int p, void* stream);
/* Max pool forward that also records each output element's window position
 * of its maximum (one byte per element, [N*Ho*Wo][C]; first in scan order,
 * first NaN wins), and the backward from those positions (no window re-scan).
 * Same results as dmf_maxpool2d / dmf_maxpool2d_bwd (nn.MaxPool2d, timm stem
 * foundation_model.py:260-267). C and strides multiples of 8, idx 8-B aligned. */
int dmf_maxpool2d_idx(int dtype, const void* x, int N, int H, int W, int C, int ldx, void* y, int Ho, int Wo, int ldy,
                      void* idx, int k, int s, int p, void* stream);
int dmf_maxpool2d_bwd_idx(int dtype, const void* dy, int N, int H, int W, int C, int Ho, int Wo, int lddy,
                          const void* idx, void* dx, int lddx, int k, int s, int p, void* stream);
int dmf_upsample_nearest(int dtype, const void* x, int ldx, void* y, int N, int H, int W, int C, int r,
                         void* stream);
/* nn.AdaptiveAvgPool2d((Ho, Wo)) on NHWC, any ratio (proj_pool, model_module.py:534) */
int dmf_adaptive_avgpool2d(int dtype, const void* x, int N, int H, int W, int C, int ldx, void* y, int Ho, int Wo,
                           int ldy, void* stream);
int dmf_adaptive_avgpool2d_bwd(int dtype, const void* dy, int N, int Ho, int Wo, int C, int lddy, void* dx, int H,
                               int W, int lddx, void* stream);
int dmf_upsample_nearest_bwd(int dtype, const void* dy, void* dx, int N, int H, int W, int C, int r, void* stream);
int dmf_bilinear(int dtype, const void* x, int N, int Hi, int Wi, int C, int ldx, void* y, int Ho, int Wo, int ldy,
                 void* stream);
int dmf_bilinear_bwd(int dtype, const void* dy, int N, int Ho, int Wo, int C, int lddy, void* dx, int Hi, int Wi,
                     int lddx, void* stream);
int dmf_channel_affine(int dtype, const void* x, int ldx, const float* gate, const float* add, float add_scale,
                       void* y, int ldy, int N, int HW, int C, void* stream);
int dmf_broadcast_hw(int dtype, const float* vec, float scale, void* y, int ldy, int N, int HW, int C,
                     int accumulate, void* stream);
int dmf_gate_grad_nchw(int dtype, const void* dy, int lddy, const float* x, int N, int C, int HW, float* out,
                       void* stream);
int dmf_mask_attn_fwd(int dtype, const void* f, int ldf, const void* m, int N, int HW, int C, const float* w1,
                      const float* gn_w, const float* gn_b, const float* w2, const float* b2, const float* gamma,
                      int hidden, float eps, float* stats, void* out, int ldo, void* A_out, void* stream);
/* floats of the dmf_mask_attn_bwd workspace */
int dmf_mask_attn_bwd_ws_size(int N, int HW, int hidden);
/* workspace: dmf_mask_attn_bwd_ws_size floats; grads (accumulated):
 * [hidden] dw1, [hidden] dgn_w, [hidden] dgn_b, [hidden] dw2, [1] db2, [1] dgamma */
int dmf_mask_attn_bwd(int dtype, const void* dout, int lddo, const void* f, int ldf, const void* m, int N, int HW,
                      int C, const float* w1, const float* gn_w, const float* gn_b, const float* w2, const float* b2,
                      const float* gamma, int hidden, float eps, const float* stats, void* df, int lddf, void* dm,
                      float* workspace, float* grads, void* stream);
/* dw (accumulated) = the per-block partials in ws (>= DMF_MIX_BWD_WS floats) summed in block order */
#define DMF_MIX_BWD_WS 4096
int dmf_mix_bwd(int dtype, const void* dz, int lddz, const void* a, int lda, const void* b, int ldb,
                const float* wlogit, void* da, void* db, int ldd, float* dw, long long M, int C, float* ws,
                void* stream);

/* ------------------------------------------- cross-modal fusion op (fp32)
 * FusionModel.forward (model_module.py:919-1000): GatingAttention
 * (:745-780), _to_tokens (:903-917), CrossAttentionBlock (:799-818: MHA +
 * LayerNorm/Linear FFN), gated combine + bilinear upsample-add (:952-973);
 * nn.Linear layers (classifier, SE excitations) via dmf_sgemm. */
/* workspace (nullable): dmf_sgemm_ws_size(M, N, K) floats enable a
 * deterministic split-K (partial tiles + ordered reduce, which also applies
 * beta * C) for small-output, long-K problems; without it one pass over K. */
int dmf_sgemm_ws_size(int M, int N, int K);
int dmf_sgemm(int transA, int transB, int M, int N, int K, float alpha, const float* A, int lda, const float* B,
              int ldb, float beta, float* C, int ldc, const float* bias, int act, float* workspace, void* stream);
/* 1 (default): dmf_sgemm's small GEMMs (M * N <= 512^2, K <= 8192) on 16 x 16 fp32-MFMA output tiles, one
 * workgroup per tile with the K-steps split over its 4 waves (no split-K workspace); 0: the 64 x 64 VALU
 * tile with split-K (A/B runs) */
int dmf_sgemm_tune(int mfma);
int dmf_colsum_f32(const float* X, int ldx, int M, int N, float* out, int accumulate, void* stream);
int dmf_act_grad_f32(const float* dy, const float* z, float* dx, long long n, int act, void* stream);
int dmf_act_f32(const float* x, float* y, long long n, int act, void* stream);
int dmf_sig_grad_f32(const float* dg, const float* s, float* dz, long long n, void* stream);
/* SEBlock excitation (model_module.py:25-43; the modality attention of
 * :584-591) in <= 3 launches: pooled[n] = scale * sum_z ws[z][n][:] over S
 * partial planes of [N][C] (dmf_nhwc_reduce's stage-1 layout; S = 1, scale = 1
 * for a finished pool), hpre = pooled w1^T + b1 ([mid][C]), hact = gelu(hpre),
 * gate = sigmoid(hact w2^T + b2) ([C][mid]). pooled (required when S > 1 or
 * scale != 1), hpre, b1, b2 nullable; C, mid <= 2048; weights and vectors
 * 16-B aligned. */
int dmf_se_mlp(const float* ws, int S, int N, int C, float scale, const float* w1, const float* b1, int mid,
               const float* w2, const float* b2, float* pooled, float* hpre, float* hact, float* gate, void* stream);
/* dmf_se_mlp's form (A/B runs): 1 (default) two launches of 16 x 16 fp32-MFMA output tiles, the squeeze
 * summed on the fly (C and mid multiples of 4); 2 one workgroup for both layers where N <= 64 and
 * N*(C+mid) floats fit 96 KiB; 0 the three-launch form. */
int dmf_se_mlp_tune(int mode);
int dmf_row_l2norm(const float* x, int R, int C, float eps, float* y, float* norms, void* stream);
int dmf_row_l2norm_bwd(const float* dy, const float* y, const float* norms, int R, int C, float eps, float* dx,
                       void* stream);
int dmf_layernorm_fwd(const float* x, int R, int E, const float* gamma, const float* beta, float eps, float* y,
                      float* save, void* stream);
int dmf_layernorm_bwd(const float* dy, const float* x, const float* save, int R, int E, const float* gamma,
                      float* dx, float* dgamma, float* dbeta, void* stream);
/* avg_weights (nullable, needs probs): the mean over heads of probs, summed in head order */
int dmf_attn_fwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, int B, int Nq, int Nk,
                 int H, int D, float scale, float* out, int ldo, float* probs, float* avg_weights, void* stream);
int dmf_attn_bwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, const float* probs,
                 const float* dout, int lddo, int B, int Nq, int Nk, int H, int D, float scale, float* dq, int lddq,
                 float* dk, int lddk, float* dv, int lddv, void* stream);
int dmf_tokens_fwd(int dtype, const void* x, int ldx, int B, int H, int W, int C, int Hp, int Wp, float* tokens,
                   void* stream);
int dmf_tokens_bwd(int dtype, const float* dtokens, int B, int H, int W, int C, int Hp, int Wp, void* dx, int lddx,
                   int accumulate, void* stream);
int dmf_fusion_combine_fwd(int dtype, const void* p_dwi, const void* p_dce, int ld, const float* gates,
                           const float* lowres, int B, int H, int W, int C, int Hp, int Wp, void* y, int ldy,
                           void* stream);
int dmf_fusion_combine_bwd(int dtype, const void* dy, int lddy, const void* p_dwi, const void* p_dce, int ld,
                           const float* gates, int B, int H, int W, int C, int Hp, int Wp, void* dp_dwi,
                           void* dp_dce, int ldd, float* dgates, float* dlowres, void* stream);
int dmf_gate_fwd(const float* pv_dwi, const float* pv_dce, const float* conf_dwi, const float* conf_dce, int B,
                 int C, const float* W, const float* b, float* gates, void* stream);
int dmf_gate_bwd(const float* pv_dwi, const float* pv_dce, const float* conf_dwi, const float* conf_dce, int B,
                 int C, const float* W, const float* gates, const float* dgates, float* dW, float* db,
                 float* dpv_dwi, float* dpv_dce, float* dconf_dwi, float* dconf_dce, void* stream);

/* ------------------------------------------------------------ criteria
 * loss.py:45-62 (SoftDiceLoss), :157-187 (SoftWeightedFocalLoss), :190-213
 * (LabelSmoothing); train_fusion.py:709-744 (compute_recon_list_loss);
 * train.py:1033-1048 (mimic_feat_loss, recon_image_loss, charbonnier).
 * Forward writes the loss and the unit-upstream gradient in one pass. */
/* targets: soft_targets [B][K] (nullable) else labels; reduction 0 mean, 1 sum, 2 none */
int dmf_focal_loss(const float* logits, const long long* labels, const float* soft_targets, int B, int K,
                   float smoothing, int use_smoothing, const float* class_weights, float gamma, int reduction,
                   float* loss, float* per_row, float* dlogits, void* stream);
int dmf_label_smooth(const long long* labels, int B, int K, float smoothing, float* out, void* stream);
int dmf_soft_dice(int dtype, const void* logits, const float* target, int B, int P, float eps, float* sums_ws,
                  float* loss, float* dlogits, void* stream);
int dmf_recon_loss(int dtype, int nterms, const void* r0, const void* r1, const void* r2, const void* r3,
                   const void* r4, int ldr0, int ldr1, int ldr2, int ldr3, int ldr4, int sel0, int sel1, int sel2,
                   int sel3, int sel4, const float* tA, const float* tB, float ca, float cb, int B, int h, int w,
                   int S, float* sums, float* g0, float* g1, float* g2, float* g3, float* g4, float* ws,
                   void* stream);
/* recon workspace (floats) of the two-pass streaming form (deterministic; sums and
 * gradients written, not accumulated); 0 = not applicable: pass ws = NULL with zeroed
 * sums / gradients (atomic one-pass forms) */
int dmf_recon_ws_floats(int nterms, int B, int h, int w, int S);
/* loss (accumulated) += the per-(pair, channel) terms, written to ws (npairs * C floats) and
 * summed in a fixed order (deterministic) */
int dmf_mimic_loss(int dtype, const void* student, const void* teacher, long long sstride, long long tstride, int ld,
                   int HW, int C, int npairs, float* loss, void* dstudent, long long dstride, float* ws,
                   void* stream);
int dmf_scale_by(const float* src, long long n, const float* scalar, float mul, float* dst, void* stream);
int dmf_scale_by_cast(int dtype, const float* src, long long M, int C, const float* scalar, float mul, void* dst,
                      int ldd, void* stream);
/* Loss assembly of LightningFusionModel._shared_step (train_fusion.py:246-300):
 * total = sum_i coef[i] * v_i * (w if flags[i] & 1) over n <= DMF_LOSS_MAX scalar
 * criterion values v_i = *ptrs[i]; groups[g] = sum of gcoef[i] * v_i over the
 * elements of group g = (flags[i] >> 1) - 1 (the logged mask / recon / mimic
 * values). ptrs, coef, flags, gcoef are HOST arrays (ptrs holds device
 * addresses); w (nullable = 1) is the device aux-loss weight. The backward
 * writes grads[i] = *dtotal * coef[i] * (w or 1). */
#define DMF_LOSS_MAX 16
int dmf_loss_combine(int n, const unsigned long long* ptrs, const float* coef, const int* flags, const float* gcoef,
                     int ngroups, const float* w, float* total, float* groups, void* stream);
int dmf_loss_combine_bwd(int n, const float* coef, const int* flags, const float* w, const float* dtotal, float* grads,
                         void* stream);
/* mean over rows of (argmax(logits[b]) == labels[b]), torch's argmax rule (first
 * maximum, NaN is the maximum); logits fp32 [B][K] (train_fusion.py:302-303) */
int dmf_batch_accuracy(const float* logits, const long long* labels, int B, int K, float* out, void* stream);

/* ------------------------------------------ batched bf16 GEMM, attention
 * Hybrid TransformerStage, configuration 5 (transformer_model.py:68-134):
 * nn.Linear (qkv, proj, fc1, fc2) forward/backward and the
 * MultiHeadSelfAttention core at 576 tokens (:83-116) as GEMMs.
 *   op(A)[m][k] = ta ? A[k*lda+m] : A[m*lda+k]; op(B)[k][n] = tb ? B[k*ldb+n] : B[n*ldb+k]
 *   z = z1*batch2 + z2, operand offset z1*s?1 + z2*s?2 (elements; aux/pre use C's).
 * Fused epilogue, in order (each step optional):
 *   t = alpha * sum_k op(A) op(B) + bias[n]
 *   aux[m][n] = bf16(t)                         (pre-activation saved for backward)
 *   pre == NULL: t = dropout(act(t), p)         (forward; Philox index z*M*N + m*N + n at `site`)
 *   pre != NULL: t = dropout_mask(t) * act'(pre[m][n])   (gradient of that forward)
 *   t *= colscale[n]; t += res[m][n] (f32, unbatched; may alias C); C = t; dbias[n] += t
 *   (dbias: unbatched only; per-128-row-tile column sums into dbias_ws [cdiv(M,128)][N],
 *   then summed in tile order -- deterministic)
 * A, B bf16; C f32 or bf16 (out_dtype). */
int dmf_gemm_bf16(int out_dtype, int ta, int tb, int M, int N, int K, float alpha, const void* A, int lda,
                  long long sA1, long long sA2, const void* B, int ldb, long long sB1, long long sB2, void* C,
                  int ldc, long long sC1, long long sC2, int batch1, int batch2, const float* bias, int act,
                  const float* colscale, const float* res, int ldr, void* aux, int ldaux, const void* pre, int ldpre,
                  float dropout_p, const unsigned long long* rng, int site, float* dbias, float* dbias_ws,
                  void* stream);
/* the same GEMM with f32 A, B, aux and pre on the 16x16x4 f32 MFMA (exact
 * f32 products): the fp32 parity mode of the transformer stage
 * (set_compute_dtype(float32)); K, lda, ldb multiples of 4. */
int dmf_gemm_f32(int out_dtype, int ta, int tb, int M, int N, int K, float alpha, const float* A, int lda,
                 long long sA1, long long sA2, const float* B, int ldb, long long sB1, long long sB2, void* C,
                 int ldc, long long sC1, long long sC2, int batch1, int batch2, const float* bias, int act,
                 const float* colscale, const float* res, int ldr, float* aux, int ldaux, const float* pre, int ldpre,
                 float dropout_p, const unsigned long long* rng, int site, float* dbias, float* dbias_ws,
                  void* stream);
/* attention probabilities (transformer_model.py:104-110): per row of L f32
 * scores, probs = softmax(scale * s) (bf16, kept for backward) and
 * probs_dropped = dropout(probs, p) (bf16, the P operand of P v); Philox
 * element index row*L + col at dropout site `site`. Columns >= Lv are key
 * padding (token counts rounded up to the GEMM granule): probability 0. */
/* Fused attention forward for a block that builds no autograd graph (frozen encoders, mode A;
 * transformer_model.py:100-116): o = dropout(softmax(q k^T * scale)) v per (batch item, head) from the
 * packed qkv rows [batch*n][ldq] (q | k | v, E columns each, head h at columns h*128), bf16, fp32
 * accumulation; keys >= nv are padding; the dropout mask is dmf_softmax_dropout's (element index
 * ((b*heads + h)*n + query)*n + key, Philox site `site`), the row sum keeps the pre-dropout
 * probabilities. o [batch*n][ldo] bf16, head h at columns h*128. Head dim 128 only (E = 128*heads);
 * the scores and probabilities never reach HBM (csrc/attn.hip). */
int dmf_flash_attn_fwd(const void* qkv, int ldq, int batch, int n, int nv, int E, int heads, float scale,
                       float dropout_p, const unsigned long long* rng, int site, void* o, int ldo, void* stream);
/* dmf_flash_attn_fwd variant (A/B only): 1 = 64 queries per block, 64-key tiles, one tile in flight;
 * 2 (default) = 128 queries per block, 64-key tiles, one in flight; 3 = 128 queries, 32-key tiles,
 * two in flight */
int dmf_flash_attn_tune(int var);
int dmf_softmax_dropout(const float* S, int lds, long long rows, int L, int Lv, float scale, float dropout_p,
                        const unsigned long long* rng, int site, void* probs, void* probs_dropped, int ldp,
                        void* stream);
/* dscores = scale * P * (g - sum(P g)), g = dropout_mask(dprobs_dropped) (bf16 out) */
int dmf_softmax_dropout_bwd(const void* probs, int ldp, const float* dprobs_dropped, int ldg, long long rows, int L,
                            float scale, float dropout_p, const unsigned long long* rng, int site, void* dscores,
                            int lds, void* stream);
/* f32 probs / dscores (parity mode) */
int dmf_softmax_dropout_f32(const float* S, int lds, long long rows, int L, int Lv, float scale, float dropout_p,
                            const unsigned long long* rng, int site, float* probs, float* probs_dropped, int ldp,
                            void* stream);
int dmf_softmax_dropout_bwd_f32(const float* probs, int ldp, const float* dprobs_dropped, int ldg, long long rows,
                                int L, float scale, float dropout_p, const unsigned long long* rng, int site,
                                float* dscores, int lds, void* stream);

/* token-stream kernels (transformer_model.py:29, :71-80, :115, :133); rows R = B*N,
 * E % 256 == 0 and E <= 1024. LayerNorm: y bf16, save = (mean, rstd) per row. */
int dmf_tok_layernorm_fwd(int x_dtype, const void* x, int ldx, long long R, int E, const float* gamma,
                          const float* beta, float eps, int y_dtype, void* y, int ldy, float* save, void* stream);
/* workspace floats of the token backward column sums (dmf_tok_layernorm_bwd,
 * dmf_tok_scale_dropout_bwd*): one slab row per 32-row block and sum, summed in
 * block order (deterministic) */
long long dmf_tok_bwd_ws_floats(long long R, int E);
/* dx (f32) = LN'(dy) (+ dres; dx may alias dres); dgamma/dbeta accumulated (nullable; ws needed with either) */
int dmf_tok_layernorm_bwd(const float* dy, int x_dtype, const void* x, int ldx, const float* save, long long R,
                          int E, const float* gamma, const float* dres, float* dx, float* dgamma, float* dbeta,
                          float* ws, void* stream);
/* backward of out = res + dropout(y) * gamma: dy (bf16) = mask * gamma * gout,
 * dgamma += sum gout * dropout(y), dbias += sum dy (accumulated, nullable) */
int dmf_tok_scale_dropout_bwd(const float* gout, const void* yaux, long long R, int E, const float* gamma,
                              float dropout_p, const unsigned long long* rng, int site, void* dy, float* dgamma,
                              float* dbias, float* ws, void* stream);
/* f32 yaux / dy (parity mode) */
int dmf_tok_scale_dropout_bwd_f32(const float* gout, const float* yaux, long long R, int E, const float* gamma,
                                  float dropout_p, const unsigned long long* rng, int site, float* dy, float* dgamma,
                                  float* dbias, float* ws, void* stream);
/* out (accumulated) += column sums of bf16 X [R][ldx]: 64-row band sums into ws
 * (dmf_colsum_bf16_ws_floats), then the bands in order */
long long dmf_colsum_bf16_ws_floats(long long R, int C);
int dmf_colsum_bf16(const void* X, int ldx, long long R, int C, float* out, float* ws, void* stream);
int dmf_cast_bf16(const float* x, long long n, void* y, void* stream);
int dmf_cast_f32(const void* x, long long n, float* y, void* stream);
/* keep[i] (0/1) of element i at dropout site `site` -- the mask every fused
 * dropout of this library draws (test/inspection helper; n % 4 == 0) */
int dmf_dropout_keep_mask(const unsigned long long* rng, int site, long long n, float p, unsigned char* keep,
                          void* stream);

/* ------------------------------------------------- fp8 patch embed (cfg 5)
 * PatchEmbed.proj (conv, kernel = stride = P; transformer_model.py:7-32) on
 * OCP e4m3 MFMA (v_mfma_f32_16x16x32_fp8_fp8, fp32 accumulation).
 * dmf_patch_quant_fp8: NHWC bf16 x [N][H][W][ldx] -> q [N*(H/P)*(W/P)][ldq]
 *   e4m3 patch rows in (r, s, c) order, row_scale[m] = amax_m / 448.
 * dmf_weight_quant_fp8: torch weight [E][C][P][P] fp32 -> q [E][P*P*C] e4m3,
 *   col_scale[e] = amax_e / 448.
 * dmf_gemm_fp8: C (bf16) [M][ldc] = a_scale[m] * b_scale[n] * A[m].B[n] + bias[n]
 *   (A [M][lda], B [N][ldb], K-contiguous e4m3; K, lda, ldb multiples of 16).
 *   Where N >= 256 and the 144x256 tiles fill the chip: the block-scaled
 *   v_mfma_scale_f32_16x16x128_f8f6f4 (unit scales, twice the non-scaled rate),
 *   LDS-DMA staged; otherwise the 128x128 non-scaled form.
 * dmf_gemm_fp8_tune: 1 (default) allows the block-scaled form, 0 forces the
 *   128x128 form (A/B runs). dmf_gemm_fp8_last_form: the form of the last
 *   launch (0 / 1; -1 before any). */
int dmf_patch_quant_fp8(const void* x, int N, int H, int W, int C, int ldx, int P, void* q, int ldq,
                        float* row_scale, void* stream);
int dmf_weight_quant_fp8(const float* w, int E, int C, int P, void* q, float* col_scale, void* stream);
int dmf_gemm_fp8(int M, int N, int K, const void* A, int lda, const float* a_scale, const void* B, int ldb,
                 const float* b_scale, const float* bias, void* C, int ldc, void* stream);
int dmf_gemm_fp8_tune(int var);
int dmf_gemm_fp8_last_form(void);

/* ------------------------------------------------------------ data path
 *  fp32 NCHW-contiguous planes [N*C][HW].
 * dmf_dwi_normalize: DWINormalize (dataset.py:9-41), ADC slot zero if adc.
 * dmf_adc_map: compute_adc_map (preprocess_helpers.py:133-167) -> [N][HW];
 *   preprocess != 0 fuses preprocess_adc (:39-49).
 * dmf_plane_select: the ranks[T] (ascending, T <= 64) order statistics of
 *   every plane -> vals [planes][T] (exact; multi-target radix select).
 * dmf_plane_percentiles: numpy 'linear' percentiles from them: perc
 *   [planes][L] (float64) = _lerp(vals[lo_idx[l]], vals[hi_idx[l]], gamma[l]).
 * dmf_nyul_apply: NyulStandardizer.transform (preprocess_helpers.py:94-120):
 *   y = interp(interp(x, perc[plane], avg[c]), avg[c], scale), np.interp
 *   semantics, float64 arithmetic, L <= 32. */
int dmf_dwi_normalize(const float* x, int N, int C, long long HW, int adc, float z_lo, float z_hi, float* y,
                      void* stream);
int dmf_adc_map(const float* dwi, int N, int C, long long HW, const float* bvals, float eps, int preprocess,
                float* adc, void* stream);
int dmf_plane_select(const float* x, int planes, long long HW, const int* ranks, int T, float* vals, void* stream);
int dmf_plane_percentiles(const float* vals, int T, const int* lo_idx, const int* hi_idx, const double* gamma, int L,
                          int planes, double* perc, void* stream);
int dmf_nyul_apply(const float* x, int planes, int C, long long HW, const double* perc, const double* avg,
                   const double* scale, int L, float* y, void* stream);
/* training augmentation (prepare_single_model.py:107-113), NCHW f32:
 * dmf_affine_flip: torchvision RandomAffine (nearest, fill 0) then the
 *   horizontal / vertical flips, one gather; params [N][8] per volume =
 *   the inverse affine matrix m0..m5 (_get_inverse_affine_matrix, centred
 *   pixel coordinates), hflip, vflip (0 / 1). y must not alias x.
 * dmf_resize_aa: Resize (bilinear, antialias; aten _upsample_bilinear2d_aa)
 *   of [planes][Hin][Win] -> [planes][Hout][Wout], W pass then H pass; tmp
 *   [planes][Hin][Wout] when both axes change. */
int dmf_affine_flip(const float* x, int N, int C, int H, int W, const float* params, float* y, void* stream);
int dmf_resize_aa(const float* x, long long planes, int Hin, int Win, int Hout, int Wout, float* tmp, float* y,
                  void* stream);

/* ------------------------------------------------------------ optimizer
 * torch.optim.AdamW as built by LightningFusionOptimizerFactory
 * (selector_helpers.py:632-685, :617-629) -- multi-tensor, one launch. */
int dmf_adamw_multi(int nchunks, const long long* chunks, const long long* tensors, const float* hyper,
                    const int* steps, float grad_scale, void* stream);
int dmf_steps_inc(int* steps, int n, void* stream);
/* dynamic loss scaling ("16-mixed", torch.amp.GradScaler under Lightning;
 * parameters_generate.py:211): amp = {scale, found_inf} (device f32[2]).
 * dmf_amp_nonfinite: found_inf = 1 if any gradient of the AdamW table is
 *   inf / nan; dmf_adamw_multi_amp: steps += 1 and the AdamW update with
 *   g * grad_scale / scale, both skipped entirely when found_inf;
 * dmf_amp_update: torch._amp_update_scale_ (backoff on found_inf, growth
 *   every `interval` clean steps), then found_inf = 0. */
int dmf_adamw_multi_amp(int nchunks, const long long* chunks, const long long* tensors, const float* hyper, int* steps,
                        int nsteps, float grad_scale, const float* amp, void* stream);
int dmf_amp_nonfinite(int nchunks, const long long* chunks, const long long* tensors, float* amp, void* stream);
int dmf_amp_update(float* amp, int* tracker, float growth, float backoff, int interval, void* stream);
int dmf_multi_copy(int nchunks, const long long* chunks, const long long* pairs, float scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DMF_HIP_H */
