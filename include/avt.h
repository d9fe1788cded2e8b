/* libavt — MI355X (gfx950) C-ABI for the audio-visual hard-way train step.
 *
 * Every entry point takes plain device pointers + sizes and a hipStream_t (as void*), launches
 * asynchronously on that stream, never allocates, never synchronises the host, and returns
 * AVT_OK (0) or a negative code; avt_last_error() returns a thread-local message.
 * Buffers are owned by the caller (PyTorch's caching allocator in the Python host).
 *
 * Layouts: activations NHWC bf16 (raw uint16 bits); statistics/head fp32;
 * conv master weights fp32 in OHWI order (== channels_last OIHW parameters).
 *
 * Reference interface each entry point replaces (tonymisic/audio-visual-tubes):
 *   avt_conv2d_fwd/dgrad/wgrad   nn.Conv2d fwd + autograd bwd of conv3x3/conv1x1/stems
 *                                (models/base_models.py:23-30, 135-138; called at 53-69, 195-210)
 *   avt_bn_finalize/apply/bwd    nn.BatchNorm2d train mode + nn.ReLU(inplace) + residual add
 *                                (models/base_models.py:39, 46-49, 58-67, 120-121, 141)
 *   avt_maxpool3s2_fwd/bwd       nn.MaxPool2d(3, 2, 1) (models/base_models.py:143, 203)
 *   avt_stem_*                   stem bn1 -> relu -> maxpool fused fwd/bwd (models/base_models.py:200-203)
 *   avt_bn_relu_bwd              BasicBlock bn1+relu backward, mask from the pre-activation (base_models.py:47-48)
 *   avt_bn_apply_mask,           BasicBlock output relu(bn2(c2) + residual) (base_models.py:64-67) with its ReLU
 *   avt_bn_bwd_mask,             mask kept as bits; the backward of bn2 (+ downsample.1) from those bits, and the
 *   avt_conv2d_dgrad_mask        identity block's input gradient dgrad(conv1) + g * mask without a stored g'
 *   (avt_set_*: A/B knobs between measured kernel variants, in avt_tuning.h -- not part of this boundary)
 *   avt_audio_pool_norm_fwd/bwd  nn.AdaptiveMaxPool2d((1,1)) + F.normalize(dim=1) (model.py:96, 120-122)
 *   avt_hardway_fwd/bwd          AVENet.forward head: normalize, A/A0 einsums, sigmoid trimap,
 *                                sim1/sim/sim2, logits/0.07, weighted_A (model.py:114-154);
 *                                HardWayAttention.forward (model.py:46-60)
 *   avt_hardway_ce               nn.CrossEntropyLoss()(logits, zeros) (train_hardway_1frame.py:113, 130-131)
 *   avt_adam_step                torch.optim.Adam(lr, weight_decay) step (train_hardway_1frame.py:116, 134)
 *   avt_conv3d_fwd               nn.Conv3d fwd of the R3D-18 video trunk (models/resnet3D.py:14-28 conv3x3x3 /
 *                                conv1x1x1, called from BasicBlock.forward 45-61; FullModel.vidnet, model.py:20)
 *   avt_video_stem_im2col,       the R3D stem Conv3d(3,64,(7,7,7),s(1,2,2),p3) (models/resnet3D.py:122-127) as a
 *   avt_pack_conv3d_weight       32-channel Conv2d over the frames (temporal taps folded into channels);
 *   (+ _weights_batched)         the other Conv3d weights' bf16 operands in one launch
 *   avt_maxpool3d_fwd            the R3D stem's nn.MaxPool3d(3, 2, 1) when no_max_pool=False (resnet3D.py:129, 200-201)
 *   avt_bn_finalize_rep          BatchNorm2d over the t-fold repeated spectrogram batch (train_3D.py:128-130)
 *                                computed once per distinct clip
 *   avt_twoview_loss             the 16-frame two-view loss of train_hardway.py:134-142: lw*CE x2, (100-lw)*
 *                                nn.MSELoss(weighted, weighted2), PropagationLoss x2 (losses.py:16-23)
 *   avt_propagation_loss         PropagationLoss.forward (losses.py:22-23) + its gradient
 *   avt_npratio_loss             NPRatio.forward (losses.py:13-14) + its gradient (train_3D.py:113, 135)
 *   avt_flip_l1_loss             FlipLoss.forward (losses.py:34-36) + its gradients
 *   avt_ncthw_to_nhwc_bf16       einops 'b c t h w -> (b t) c h w' of the frames (train_hardway.py:130-131)
 *   avt_localize_ciou,           the test loops' heatmap -> cIoU protocol (train_hardway_1frame.py:195-206,
 *   avt_pair_ciou                utils.Evaluator.cal_CIOU utils.py:209-214, utils.mTC 311-318)
 *   avt_spectrogram              the dataset's scipy.signal.spectrogram + log + Normalize(0, 12)
 *   avt_frames_transform         the dataset's frame transform: PIL BICUBIC Resize + crop + flip + ToTensor +
 *                                Normalize (datasets/dataloader.py:47-62)
 *                                (datasets/dataloader.py:86-96, 252-274)
 */
#ifndef AVT_H_
#define AVT_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVT_OK 0
#define AVT_EINVAL -1
#define AVT_EHIP -2

const char* avt_last_error(void);
int avt_abi_version(void);
/* bit mask of how this library was built: AVT_BUILD_DIAG = the timing-diagnostics build (-DAVT_DIAG:
 * environment knobs that drop launches or loads and give WRONG results); bench.py refuses such a build */
#define AVT_BUILD_DIAG 1
int avt_build_flags(void);

/* ---- measured peaks (bench.py's roofline denominators, re-measured in the same run) ---- */
/* back-to-back bf16 MFMA on pseudo-random register operands, one wave per SIMD (256-thread blocks):
 * shape 0 = v_mfma_f32_32x32x16_bf16 (4 accumulators), 1 = v_mfma_f32_16x16x32_bf16 (8); sink:
 * float[blocks*256] (one value per lane, keeps the loop live).  avt_peak_mfma_flops: the FLOPs of one
 * such launch (-1 on bad arguments). */
int avt_peak_mfma(float* sink, int shape, int blocks, int iters, unsigned seed, void* stream);
long long avt_peak_mfma_flops(int shape, int blocks, int iters);
/* dst = src, 16-byte vector loads/stores in a grid-stride loop of `blocks` 256-thread blocks (bytes % 16 == 0) */
int avt_copy16(void* dst, const void* src, size_t bytes, int blocks, void* stream);

/* ---- convolution (implicit GEMM on bf16 MFMA, fp32 accumulate) ---- */
/* BatchNorm statistics (deterministic).  A BN's fp64 accumulator holds a small header and one slot of
 * partial sums per row tile (or persistent block / reduce block) of the launch that accumulates it, each
 * slot element written by exactly one block with plain stores (the column tiles of a row tile write
 * disjoint channel ranges of its slot) -- no atomics, nothing to zero between uses, any
 * contents on entry.  The finalize sums the slots in slot order, so identical inputs give bitwise identical
 * statistics, gradients and updates on every run (model.py:112-154's CPU path is deterministic too).
 * Forward: avt_bn_acc_doubles(rows, C) doubles; backward: avt_bn_bwd_workspace(rows, C) bytes.
 *
 * y[N,P,Q,K] = conv(x[N,H,W,Cp], wpack[K][Kg]); if bn_acc != NULL the fp32 results' batch-norm
 * statistics are stored into bn_acc (avt_bn_acc_doubles(N*P*Q, K) doubles), for avt_bn_finalize.
 * Cp is 1 or 4 (stems, Kg = R*S*Cp rounded up to 32) or a multiple of 32 (Kg = R*S*Cp). */
size_t avt_bn_acc_doubles(long long rows, int C);
int avt_conv2d_fwd(const void* x, const void* wpack, void* y, double* bn_acc, int N, int H, int W, int Cp, int K,
                   int R, int S, int stride, int pad, int Kg, void* stream);
/* dx[N,H,W,C] = dgrad(dy[N,P,Q,K], wt[C][R*S*K]) (+ add[N,H,W,C] if add != NULL; add may alias dx) */
int avt_conv2d_dgrad(const void* dy, const void* wt, void* dx, const void* add, int N, int H, int W, int C, int K,
                     int R, int S, int stride, int pad, void* stream);
/* dx = dgrad(dy, wt) + add * mask: an identity BasicBlock's input gradient (base_models.py:64-67), the
 * residual branch entering as g * [out > 0] with the bits of avt_bn_apply_mask ([N*H*W][C/8] u8) --
 * the masked copy of g is never stored.  add must not alias dx. */
int avt_conv2d_dgrad_mask(const void* dy, const void* wt, void* dx, const void* add, const void* add_mask, int N,
                          int H, int W, int C, int K, int R, int S, int stride, int pad, void* stream);
/* Split-K form of the 3x3/s1 fwd / dgrad at short grids (a few clips per GPU: layer3/4 of BASELINE
 * configs[2]'s 32-clip shard), same results to fp32 summation order.  avt_conv2d_splitk_plan gives
 * the workspace of one call: part = float[*part_floats] (any contents), cnt = int[*counters] zeroed
 * once (the kernel leaves it zero; one per concurrently running call); both 0 = no split for this
 * shape (the _ws calls then behave as avt_conv2d_fwd / avt_conv2d_dgrad[_mask]).  dgrad: 0 fwd, 1 dgrad.
 * avt_set_halo_splitk(s, blocks): s > 0 forces the split count (largest chunk-count divisor <= s),
 * 0 plans it as the smallest divisor whose grid reaches `blocks` (0: two per CU). */
int avt_conv2d_splitk_plan(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int dgrad,
                           long long* part_floats, int* counters);
/* part_floats / counters: the sizes of part and cnt as allocated; the plan is re-made at every call from the
 * current knobs, and a call whose plan needs more than the workspace holds runs without split-K. */
int avt_conv2d_fwd_ws(const void* x, const void* wpack, void* y, double* bn_acc, int N, int H, int W, int Cp, int K,
                      int R, int S, int stride, int pad, int Kg, float* part, long long part_floats, int* cnt,
                      int counters, void* stream);
int avt_conv2d_dgrad_ws(const void* dy, const void* wt, void* dx, const void* add, const void* add_mask, int N,
                        int H, int W, int C, int K, int R, int S, int stride, int pad, float* part,
                        long long part_floats, int* cnt, int counters, void* stream);
/* avt_conv2d_dgrad with the backward of the BatchNorm (+ReLU) that produced dx's positions fused into
 * its store epilogue (BasicBlock.forward, base_models.py:46-49, 58-67): the result g (after `add`) is
 * masked, g' = g * [y > 0] (y given: the block output) or g * [fma(xc, scale, shift) > 0] (y NULL:
 * BasicBlock.bn1's ReLU), dx = g' is stored, and sum g', sum g' * (xc - mean) * invstd are stored into
 * acc (an avt_bn_bwd_workspace(N*H*W, C) workspace); xc2/stats2/acc2 (optional) a second BN fed by the
 * same g' (a first block's downsample.1).  skip_class00: for a stride-2 dgrad, the (even, even) pixels are
 * stored plain (a later in-place downsample dgrad finishes them).  append_slots: this call's partial sums
 * go after those of the call before it on acc (that skip_class00 call: the downsample dgrad finishing the
 * same BN's reduction); 0: this call's sums replace whatever acc held. */
typedef struct {
  const void* xc;      /* [N,H,W,C] bf16 pre-BN activations */
  const void* y;       /* [N,H,W,C] bf16 ReLU output, or NULL */
  const float* stats;  /* [4][C] fp32: scale, shift, mean, invstd (avt_bn_finalize outputs) */
  double* acc;
  const void* xc2;
  const float* stats2;
  double* acc2;
  int skip_class00;
  int append_slots;
} avt_dgrad_bn_epi;
int avt_conv2d_dgrad_bn(const void* dy, const void* wt, void* dx, const void* add, int N, int H, int W, int C, int K,
                        int R, int S, int stride, int pad, const avt_dgrad_bn_epi* epi, void* stream);
/* dw[K][R][S][Creal] += wgrad(x[N,H,W,Cp], dy[N,P,Q,K]).  Split-K partials go through an fp32 slab
 * in `workspace` (>= avt_conv2d_wgrad_workspace(...) bytes; deterministic) or, if it is NULL/too
 * small or for the stems, are added with fp32 atomics. */
size_t avt_conv2d_wgrad_workspace(int N, int H, int W, int Cp, int Creal, int K, int R, int S, int stride, int pad);
int avt_conv2d_wgrad(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal, int K, int R,
                     int S, int stride, int pad, void* workspace, size_t ws_bytes, void* stream);
/* Deferred split-K reduce: avt_conv2d_wgrad_defer runs the wgrad kernel and, where avt_conv2d_wgrad would launch its
 * separate slab reduce (one wave per slab position), leaves it: *desc describes the slab (desc->splits > 0; keep the
 * workspace alive) and dw is incomplete until avt_wgrad_reduce_batch(descs, n) sums any number of such slabs in one
 * launch (blockIdx.y = the slab), in the same split order (the same bits).  desc->splits == 0: dw is complete. */
typedef struct {
  const float* slab;
  float* dw;
  int splits, tiles, nnt, Mg, ldw;
  int wm, wn, tm, tn;  /* the wgrad tile's wave grid and 32x32 blocks per wave (register order of the partials) */
} avt_slab_reduce_desc;
int avt_conv2d_wgrad_defer(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal, int K,
                           int R, int S, int stride, int pad, void* workspace, size_t ws_bytes, avt_slab_reduce_desc* desc,
                           void* stream);
int avt_wgrad_reduce_batch(const avt_slab_reduce_desc* descs, int n, void* stream);
/* The same with the slab summed inside the wgrad kernel: the last block of each output tile to take its ticket adds
 * the tile's split partials into dw in split order (the separate reduce's order: the same bits), so the reduce launch
 * goes.  `tickets`: >= avt_conv2d_wgrad_tickets(...) ints, zero on entry, left zero (keep them for the next call);
 * NULL or a count of 0: avt_conv2d_wgrad.  avt_conv2d_wgrad_tickets() is 0 unless avt_set_wgrad_fused(1) -- the fused
 * form measured slower than the separate reduce (an A/B knob, include/avt_tuning.h). */
int avt_conv2d_wgrad_tickets(int N, int H, int W, int Cp, int Creal, int K, int R, int S, int stride, int pad);
int avt_conv2d_wgrad_tk(const void* x, const void* dy, float* dw, int N, int H, int W, int Cp, int Creal, int K, int R,
                        int S, int stride, int pad, void* workspace, size_t ws_bytes, int* tickets, int n_tickets,
                        void* stream);

/* Input gradient of the 7x7 / stride 2 / pad 3 stem conv (base_models.py:135-138, the reference's autograd through
 * conv1 / conv1_a when the trunk input requires grad): gx[N][Cin][H][W] fp32 (NCHW, the input's layout) =
 * conv2d_input(gy[N,P,Q,64] bf16, w fp32 OHWI [64][7][7][Cin]); Cin <= 4; fp32 sums over (r, s, k) in a fixed order. */
int avt_conv_stem_dgrad(const void* gy, const float* w, float* gx, int N, int H, int W, int Cin, void* stream);

/* Conv3d, temporal stride 1: y[N,T',P,Q,K] = conv3d(x[N,T,H,W,Cp], wpack[K][(kt,r,s,c)]),
 * T' = T + 2*pad_t - KT + 1, spatial stride 1 or 2; Cp % 32 == 0; KT*R*S <= 27; bn_acc as conv2d_fwd */
int avt_conv3d_fwd(const void* x, const void* wpack, void* y, double* bn_acc, int N, int T, int H, int W, int Cp,
                   int K, int KT, int R, int S, int stride, int pad_t, int pad, void* stream);
/* R3D stem input: x fp32 NCDHW [N][C<=4][T][H][W] -> bf16 [N][T][H][W][32], channel kt*4+c = x[c][t+kt-pad_t]
 * (zero outside the clip / for c >= C / channels >= 4*KT) */
int avt_video_stem_im2col(const float* x, void* out, int N, int C, int T, int H, int W, int KT, int pad_t,
                          void* stream);
/* w fp32 OIDHW [K][C][KT][R][S] -> bf16 [K][(kt,r,s,c)] (fold 0) or the stem layout
 * [K][(r,s)][kt*4+c] with 32 channels per (r,s) (fold 1) */
int avt_pack_conv3d_weight(const float* w, void* out, int K, int C, int KT, int R, int S, int fold, void* stream);
/* every non-stem Conv3d weight in one launch: descs = device array of n records {const float* w; void* out; int K,
 * C, T, pad} (avt_pack3d_desc_bytes() bytes each), out[k][t*C + c] = bf16(w[k][c][t]) (T = KT*R*S, the fold-0 layout
 * of avt_pack_conv3d_weight); max_k = the largest K, max_row = the largest C*T (<= 15360) */
size_t avt_pack3d_desc_bytes(void);
int avt_pack_conv3d_weights_batched(const void* descs, int n, int max_k, int max_row, void* stream);
/* nn.MaxPool3d(kernel_size=3, stride=2, padding=1) over bf16 NDHWC [N][T][H][W][C], C % 8 == 0 ->
 * [N][(T-1)/2+1][(H-1)/2+1][(W-1)/2+1][C] (the winning input's bits; NaN propagates) */
int avt_maxpool3d_fwd(const void* x, void* y, int N, int T, int H, int W, int C, void* stream);

/* tube-step audio de-duplication: out[b*rep+k][:] = in[b][:]  /  out[b][:] = sum_k in[b*rep+k][:] */
int avt_repeat_rows_f32(const float* in, float* out, int B, int rep, int C, void* stream);
int avt_sum_rep_rows_f32(const float* in, float* out, int B, int rep, int C, void* stream);

/* ---- batch norm (train mode) ---- */
/* merge bn_acc (see avt_conv2d_fwd) over `rows` rows -> scale, shift, mean, invstd (fp32 [C]);
 * running stats updated if non-NULL (momentum, unbiased var); bn_acc is read, not modified */
int avt_bn_finalize(double* acc, long long rows, int C, const float* gamma, const float* beta, float* running_mean,
                    float* running_var, float momentum, float eps, float* scale, float* shift, float* save_mean,
                    float* save_invstd, void* stream);
/* avt_bn_finalize for a logical batch in which each accumulated row occurs `rep` times: the running
 * variance uses the unbiased factor of rows*rep rows (mean/variance are those of the distinct rows) */
int avt_bn_finalize_rep(double* acc, long long rows, long long rep, int C, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, float momentum, float eps, float* scale,
                        float* shift, float* save_mean, float* save_invstd, void* stream);
/* out = [relu](x*scale+shift + [residual*rscale+rshift | residual]) over rows x C (NHWC rows) */
int avt_bn_apply(const void* x, const float* scale, const float* shift, const void* residual, const float* rscale,
                 const float* rshift, void* out, long long rows, int C, int relu, void* stream);
/* avt_bn_apply with relu, also writing the ReLU mask of out as bits: mask [rows][C/8] u8, bit e of byte
 * j = out[.][8j+e] > 0 (the stored bf16 value) -- what the backward's relu mask reads instead of out */
int avt_bn_apply_mask(const void* x, const float* scale, const float* shift, const void* residual, const float* rscale,
                      const float* rshift, void* out, void* mask, long long rows, int C, void* stream);
/* bytes of the BN-backward workspace for up to `rows` rows (any contents on entry) */
size_t avt_bn_bwd_workspace(long long rows, int C);
/* g' = g*[y>0] (y may be NULL: no mask); dgamma += sum g'*xhat; dbeta += sum g';
 * gc = gamma*invstd*(g' - mean(g') - xhat*mean(g'*xhat)); gmask_out (optional) = g' */
int avt_bn_bwd(const void* g, const void* y, const void* xc, const float* mean, const float* invstd,
               const float* gamma, float* dgamma, float* dbeta, void* gc, void* gmask_out, void* workspace,
               long long rows, int C, void* stream);
/* one BatchNorm fed by g' (see avt_bn_bwd_mask) */
typedef struct {
  const void* xc;         /* [rows][C] bf16 pre-BN activations */
  const float* mean;      /* [C] batch mean / invstd (avt_bn_finalize save_mean / save_invstd) */
  const float* invstd;
  const float* gamma;
  float* dgamma;          /* [C] accumulated (+=), may be NULL */
  float* dbeta;
  void* gc;               /* [rows][C] bf16 output: gradient of xc */
  void* workspace;        /* avt_bn_bwd_workspace(rows, C) bytes (any contents on entry) */
} avt_bn_bwd_target;
/* BasicBlock output backward (base_models.py:64-67): g' = g * mask (bits of avt_bn_apply_mask), then the
 * BN backward of t1 and -- if t2 != NULL -- of t2 (a first block's bn2 and downsample.1, which share g'),
 * reading g and the mask once for both */
int avt_bn_bwd_mask(const void* g, const void* mask, const avt_bn_bwd_target* t1, const avt_bn_bwd_target* t2,
                    long long rows, int C, void* stream);
/* avt_bn_bwd for a g' that is already masked and whose reductions a dgrad epilogue already added
 * into the workspace (avt_conv2d_dgrad_bn): finalize + apply only */
int avt_bn_bwd_premasked(const void* gm, const void* xc, const float* mean, const float* invstd, const float* gamma,
                         float* dgamma, float* dbeta, void* gc, void* workspace, long long rows, int C, void* stream);
/* as avt_bn_bwd with g' = g*[fma(xc, scale, shift) > 0] -- the ReLU mask the forward's avt_bn_apply
 * produced from the same (scale, shift), recomputed instead of read */
int avt_bn_relu_bwd(const void* g, const void* xc, const float* scale, const float* shift, const float* mean,
                    const float* invstd, const float* gamma, float* dgamma, float* dbeta, void* gc, void* workspace,
                    long long rows, int C, void* stream);
/* stem: y = maxpool3s2(relu(c*scale + shift)) without storing the full-resolution activation; idx = window
 * argmax (as avt_maxpool3s2_fwd), carg = c at the argmax.  y/idx/carg are [N,P,Q,C] */
int avt_stem_bn_relu_maxpool_fwd(const void* c, const float* scale, const float* shift, void* y, void* idx,
                                 void* carg, int N, int H, int W, int C, void* stream);
/* gc = bn_bwd(relu_bwd(maxpool_bwd(gy))) over the [N,H,W,C] pre-activation c (workspace: avt_bn_bwd_workspace) */
int avt_stem_maxpool_bn_relu_bwd(const void* gy, const void* idx, const void* carg, const void* c, const float* scale,
                                 const float* shift, const float* mean, const float* invstd, const float* gamma,
                                 float* dgamma, float* dbeta, void* gc, void* workspace, int N, int H, int W, int C,
                                 void* stream);

/* ---- pooling ---- */
int avt_maxpool3s2_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, void* stream);
int avt_maxpool3s2_bwd(const void* gy, const void* idx, void* gx, int N, int H, int W, int C, void* stream);
int avt_audio_pool_norm_fwd(const void* a, float* an, int* amax, float* anorm, int B, int HW, int C, void* stream);
int avt_audio_pool_norm_bwd(const float* gan, const float* an, const int* amax, const float* anorm, void* ga, int B,
                            int HW, int C, void* stream);

/* ---- hard-way head (fp32) ---- */
size_t avt_hardway_save_floats(int B);
int avt_hardway_fwd(const void* v, const float* an, int B, int P, int C, float eps1, float eps2, float tau, int trimap,
                    int use_neg, float* inv, float* vsum, float* A0, float* save, float* logits, float* Aout,
                    float* Pos, float* Neg, float* wA, void* stream);
int avt_hardway_ce(const float* logits, int B, int L, float scale, float* loss, float* dlogits, void* stream);
/* dvh = gv = NULL: no vision gradient (detached video features of the tube head).
 * dwA [B][P] (or NULL): upstream gradient of weighted_A (model.py:148-152; train_hardway.py:138-141
 * back-propagates it), needs the forward's vsum and a dm [B][P] workspace.
 * gan_accumulate = 1: gan += (two views sharing one audio batch) instead of gan = */
int avt_hardway_bwd(const void* v, const float* an, const float* inv, const float* A0, const float* save,
                    const float* dlogits, int B, int P, int C, float eps1, float eps2, float tau, int trimap,
                    int use_neg, const float* dwA, const float* vsum, float* dm, float* dA0, float* dvh, void* gv,
                    float* gan, int gan_accumulate, void* stream);
/* avt_hardway_bwd plus the gradients arriving through the returned maps A, Pos, Neg (model.py:154;
 * gA/gPos/gNeg [B][P] fp32, each may be NULL) */
int avt_hardway_bwd_ex(const void* v, const float* an, const float* inv, const float* A0, const float* save,
                       const float* dlogits, int B, int P, int C, float eps1, float eps2, float tau, int trimap,
                       int use_neg, const float* dwA, const float* vsum, float* dm, const float* gA, const float* gPos,
                       const float* gNeg, float* dA0, float* dvh, void* gv, float* gan, int gan_accumulate,
                       float* ws, void* stream);
/* ws (avt_hardway_bwd_ex / avt_hardway_attention_bwd): avt_hardway_bwd_ws_floats(B, C) floats for the split-K
 * partials of the audio-vector gradient, summed in split order (deterministic); NULL: one split (slow).
 * avt_hardway_bwd runs without it. */
size_t avt_hardway_bwd_ws_floats(int B, int C);
/* Standalone HardWayAttention()(audio_features, video_features) -> (A, logits) (model.py:38-60): fp32
 * features taken as given (the module does not normalise them; FullModel normalises before the call,
 * model.py:31-35), tri-map and Neg on.  v [B][P][C] fp32 = '(b t) (h w) c' of video_features,
 * an [B][C] fp32.  inv/vsum [B][P], A0 [B][P][B], save [B*(2B+4)] are saved for the backward; Pos, Neg,
 * wA [B][P] are scratch. */
int avt_hardway_attention_fwd(const float* v, const float* an, int B, int P, int C, float eps1, float eps2, float tau,
                              float* inv, float* vsum, float* A0, float* save, float* logits, float* Aout, float* Pos,
                              float* Neg, float* wA, void* stream);
/* Its backward: dlogits [B][B+2] and gA [B][P] (or NULL) -> gv [B][P][C] fp32 (d video features,
 * '(b t) (h w) c'), gan [B][C] fp32 (d audio features).  dA0 [B][P][B], dvh [B][P][C] fp32: workspace. */
int avt_hardway_attention_bwd(const float* v, const float* an, const float* inv, const float* A0, const float* save,
                              const float* dlogits, const float* gA, int B, int P, int C, float eps1, float eps2,
                              float tau, float* dA0, float* dvh, float* gv, float* gan, float* ws, void* stream);
/* train_hardway.py:134-142 loss combination of the 16-frame two-view step: given the two CE values
 * (avt_hardway_ce outputs; their dlogits use scale loss_weight/2) and weighted_A of both views
 * ([b*t][P], '(b t)' clip-major), out[5] = {combined, hardway, aug, l2, consistency} and
 * dwA1/dwA2 = d(combined)/d(weighted_A).  losses.py:16-23 PropagationLoss + nn.MSELoss. */
int avt_twoview_loss(const float* ce1, const float* ce2, const float* wA1, const float* wA2, int b, int t, int P,
                     float loss_weight, float* out, float* dwA1, float* dwA2, void* stream);
/* Scratch (floats) of the three losses below for n elements / `rows` rows (NPRatio: b*t): per-block
 * partial sums, summed by one block in a fixed order (deterministic) -- and NPRatio's row sums */
size_t avt_loss_workspace_floats(long long n, long long rows);
/* PropagationLoss (losses.py:16-23) of x [b][t][P]; dx (or NULL) = d(loss)/dx */
int avt_propagation_loss(const float* x, int b, int t, int P, float* loss, float* dx, float* ws, void* stream);
/* NPRatio (losses.py:7-14) of x [b][t][P]: mean |diff_t sum_p x|; dx (or NULL) = d(loss)/dx */
int avt_npratio_loss(const float* x, int b, int t, int P, float* loss, float* dx, float* ws, void* stream);
/* FlipLoss (losses.py:25-36): nn.L1Loss()(y, hflip(x)) over `rows` rows of W; dx, dy (or NULL) gradients */
int avt_flip_l1_loss(const float* x, const float* y, long long rows, int W, float* loss, float* dx, float* dy,
                     float* ws, void* stream);

/* ---- localisation metrics (test loops of train_hardway*.py / test.py; utils.py:203-239, 311-318) ---- */
/* A [N][h][w] heatmaps -> cv2 INTER_LINEAR resize to S x S, normalize_img(-.), 1 - ., median
 * binarisation, cIoU(., gt, 0.5): out [N][3] fp64 = (cIoU, intersection, denominator) when gt
 * [N][S][S] is given; pred_out [N][S][S] u8 binary maps (either may be NULL, not both) */
int avt_localize_ciou(const float* A, int N, int h, int w, int S, const float* gt, double* out, void* pred_out,
                      void* stream);
/* out[k] = cIoU(p[k], p[k+1], 0.5) of binary maps p [N][n] u8, k < N-1 (utils.mTC) */
int avt_pair_ciou(const void* p, int N, int n, double* out, void* stream);

/* ---- audio front end (datasets/dataloader.py:86-96): waveform -> normalised log-spectrogram ---- */
/* segments of a length-N waveform at hop = nperseg - noverlap (the reference: 512 - 1) */
int avt_spectrogram_segments(long long n_samples, int hop);
/* x [B][N] fp32 -> out [B][1][257][nseg] = log(PSD + 1e-7) / 12 with scipy.signal.spectrogram's
 * defaults (periodic Tukey(0.25), constant detrend, one-sided density scaling), input clipped to [-1,1] */
int avt_spectrogram(const float* x, int B, long long N, int hop, float fs, float* out, void* stream);

/* ---- frame transform (datasets/dataloader.py:47-62): decoded RGB frames -> normalised tensors ----
 * src: uint8 HWC frames packed at byte offsets; desc: DEVICE int64 [n][8] = {offset, H, W, resized_h,
 * resized_w, crop_top, crop_left, flip}; tmp: device scratch of n*3*Hmax*S bytes; mean/std: HOST
 * float[3]; out: float32 [n][3][S][S].  The resize is bit-identical to Pillow's Image.resize(BICUBIC)
 * (fixed-point separable resampler); S <= 256, downscale factor <= 7.5 (checked by the caller). */
int avt_frames_transform(const void* src, const long long* desc, int n, int S, int Hmax, void* tmp,
                         const float* mean, const float* std, float* out, void* stream);

/* ---- optimizer / layout ---- */
int avt_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n, float grad_scale,
                  float lr, float beta1, float beta2, float eps, float weight_decay, int step, void* stream);
/* avt_adam_step with the step count AND the hyper-parameters on the device: hyper = device float[5]
 * {lr, beta1, beta2, eps, weight_decay}, read at every launch (a schedule or a restored checkpoint
 * writes it; a captured graph follows); *step is incremented first and the bias corrections computed
 * there into coef[AVT_ADAM_COEF_FLOATS] (scratch) — graph-capturable */
#define AVT_ADAM_COEF_FLOATS 8
int avt_adam_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                      float grad_scale, const float* hyper, int* step, float* coef, void* stream);
/* avt_adam_step_dev in two parts (the same update): prep increments *step and writes coef once per
 * step; apply updates one region of the flat buffers from coef (train.py: each trunk's region at the
 * end of that trunk's backward branch) */
int avt_adam_prep_dev(const float* hyper, int* step, float* coef, void* stream);
int avt_adam_apply_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                       float grad_scale, const float* coef, void* stream);
int avt_pack_conv_weight(const float* w, int K, int R, int S, int C, int Cp, int Kg, void* out_fwd, void* out_dgrad,
                         void* stream);
/* two launches (fwd copy, dgrad transpose) for many convs: descs = device array of n records
 * {const float* w; void* fwd; void* dgrad; int K, RS, C, Cp, Kg, pad;} (avt_pack_desc_bytes() each) */
size_t avt_pack_desc_bytes(void);
int avt_pack_conv_weights_batched(const void* descs, int n, long long max_elems, void* stream);
/* one of its two launches: which = 1 the fwd images, 2 the dgrad images */
int avt_pack_conv_weights_part(const void* descs, int n, long long max_elems, int which, void* stream);
int avt_nchw_to_nhwc_bf16(const float* x, void* y, int N, int C, int H, int W, int Cp, void* stream);
/* x [N][C][T][H][W] fp32 -> y [(N T)][H][W][Cp] bf16: the 'b c t h w -> (b t) c h w' fold of
 * train_hardway.py:130-131 fused with the NHWC/bf16 conversion */
int avt_ncthw_to_nhwc_bf16(const float* x, void* y, int N, int C, int T, int H, int W, int Cp, void* stream);
int avt_nhwc_bf16_to_nchw(const void* x, float* y, int N, int C, int HW, void* stream);

#include "avt_tuning.h"  /* A/B knobs (process-global; not part of the drop-in path) */

#ifdef __cplusplus
}
#endif
#endif /* AVT_H_ */
