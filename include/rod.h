/*
 * rod.h — C ABI of librod.so, the MI355X (gfx950) hot path of the
 * road-object detector (RefineDet-style MobileNet-v2 detector of
 * YoungYoung619/road-object-detection-for-bdd100k).
 *
 * The reference is pure TensorFlow-1.x/slim Python with no FFI; every entry
 * point below replaces the TF graph op(s) that the cited reference line builds
 * (paths relative to the reference root).  Callers (rod/_abi.py, ctypes) own
 * every device buffer; the library never allocates device memory, never keeps
 * a pointer past the call, and never synchronises the stream.
 *
 * Conventions
 *   - tensors are NHWC row-major (C innermost); "rows" = N*H*W pixels;
 *   - dtype: ROD_F32 (0) or ROD_BF16 (1) = storage type of activations;
 *     arithmetic and accumulation are fp32; weights/statistics/grads of
 *     parameters are fp32 unless stated;
 *   - return 0 on success, ROD_EINVAL (-1) on a bad shape/dtype/argument,
 *     or a positive hipError_t; the message is in rod_last_error()
 *     (thread-local).  Device faults surface at the caller's next sync;
 *   - `stream` is a hipStream_t passed as void* (0 = null stream).
 */
#ifndef ROD_H_
#define ROD_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ROD_ABI_VERSION 23
#define ROD_EINVAL (-1)

enum { ROD_F32 = 0, ROD_BF16 = 1, ROD_I32 = 2 /* collectives only (ABI 19) */ };
/* activation applied after BatchNorm:
 *   NONE  = identity (project conv, conv_blocks.py:294)
 *   RELU6 = tf.nn.relu6 (mobilenet_v2.py:47)
 *   LEAKY = tf.nn.leaky_relu, alpha 0.2 (catch_net.py:302)
 *   RELU  = tf.nn.relu (vgg_arg_scope activation_fn, nets/backbone/vgg.py:58; ABI 9) */
enum { ROD_ACT_NONE = 0, ROD_ACT_RELU6 = 1, ROD_ACT_LEAKY = 2, ROD_ACT_RELU = 3 };

/* BatchNorm-apply prologue (ABI 3).  rod_conv_fwd, rod_conv_wgrad, rod_dw3x3_fwd and
 * rod_dw3x3_bwd_filter take, right after their input x, the five arguments
 *     const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
 *     const float* pro_beta, int pro_act
 * With pro_mean == NULL x is used as is.  Otherwise x is the PRE-BatchNorm tensor y of the
 * layer below and the kernel reads, wherever the reference reads that layer's BatchNorm +
 * activation output (slim.batch_norm then relu6 / leaky_relu, mobilenet.py:417-420,
 * catch_net.py:302), z = act(y*scale + offset) (one fma; scale = rstd*gamma, offset =
 * beta - mean*scale, TF's fused batch-norm form) rounded to the storage
 * dtype — bit for bit the tensor rod_bn_apply would have written — formed in registers as
 * y is loaded (padding taps stay 0).  gamma / beta may be NULL (1 / 0), as in rod_bn_apply.
 * The normalised activation therefore never crosses HBM in forward or in the weight
 * gradients; channel count <= 2048 for the GEMM prologues. */

int rod_abi_version(void);
const char* rod_last_error(void);

/* ---------------------------------------------------------------- ingest */
/* out = (2/255)*img - 1 from uint8 pixels (train.py:126, predict.py:98). */
int rod_normalize_image(const void* img_u8, void* out, long n, int out_dtype, void* stream);
/* dst = src converted between storage dtypes (tf.cast). */
int rod_cast(const void* src, int src_dtype, void* dst, int dst_dtype, long n, void* stream);

/* ------------------------------------------------ training augmentation (A17)
 * process_raw_data_train (utils/data_pileline_tools.py:76-108) on a batch of decoded uint8
 * RGB images of any sizes: image b is src_hw[b] = (H, W) pixels at byte offset src_off[b] of
 * src (rows of 3*W bytes).  Per image, with parameters sampled on the host:
 *   crop[b]   = (y0, x0, h, w)   tf.slice window of sample_distorted_bounding_box (process.py:117-127)
 *   mode[b]   = (flip, ordering) random_flip_left_right (tf_image.py:281-305); colour ordering
 *               0..3 of distort_color(fast_mode=False) (process.py:59-77), -1 = no colour ops
 *   colour[b] = (brightness delta, saturation factor, contrast factor)
 * out[b] = colour(flip(resize_bilinear_legacy(crop(src_b), Ho x Wo))) on the 0-255 scale, no
 * clamping (process.py:79), then (2/255)x - 1 when normalize != 0 (train.py:126), stored in
 * dtype as [B, Ho, Wo, 3].  Contrast uses the per-image channel mean of the image it receives.
 * prepare_data_test (data_pileline_tools.py:18-43) is crop = whole image, mode = (0, -1).
 * workspace: rod_augment_workspace(B, Ho, Wo) bytes.  out 16-byte aligned. */
size_t rod_augment_workspace(int B, int Ho, int Wo);
int rod_augment_images(const void* src, const int64_t* src_off, const int32_t* src_hw, const int32_t* crop,
                       const int32_t* mode, const float* colour, void* workspace, void* out, int B, int Ho, int Wo,
                       int normalize, int dtype, void* stream);
/* Box side of the same step, boxes [B][G][4] (ymin, xmin, ymax, xmax), first n[b] valid:
 * bboxes_resize to ref[b] (the crop as a normalised box, bboxes.py:139-163), keep boxes whose
 * intersection / own area with [0,0,1,1] is > threshold (bboxes_filter_overlap, bboxes.py:408-428;
 * 0.3 = BBOX_CROP_OVERLAP, process.py:6) compacted in order (tf.boolean_mask), flip when
 * mode[b][0] (tf_image.py:284-289; mode may be NULL), clip to [0,1] (data_pileline_tools.py:106-107).
 * Outputs padded with zeros past n_out[b]. */
int rod_augment_boxes(const float* boxes, const int32_t* labels, const int32_t* n, const float* ref,
                      const int32_t* mode, float* boxes_out, int32_t* labels_out, int32_t* n_out, int B, int G,
                      float threshold, void* stream);

/* --------------------------------------------------- depthwise 3x3 (A1)
 * slim.separable_conv2d(num_outputs=None, depth_multiplier=1), padding SAME
 * (conv_blocks.py:238-247): y[n,ho,wo,c] = sum_ij x[n,ho*s+i-pt,wo*s+j-pl,c]*w[i,j,c].
 * w is fp32 [3][3][C] (TF depthwise_weights [3,3,C,1]). */
/* stat_parts (nullable): BatchNorm partial statistics of y ([nparts][3][C], see
 * rod_bn_finalize) with nparts = rod_dw3x3_fwd_stat_parts(), reduced in the epilogue from
 * the rounded outputs (the depthwise BatchNorm, conv_blocks.py:247 + mobilenet.py:417). */
int rod_dw3x3_fwd_stat_parts(int N, int Ho, int Wo, int C, int stride, int dtype);
int rod_dw3x3_fwd(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                  const float* pro_beta, int pro_act, const float* w, void* y, float* stat_parts, int N, int H,
                  int W, int C, int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream);
/* The same forward with its input recomputed, not read (ABI 23; conv_blocks.py:263-270 expand +
 * mobilenet.py:417-420 + 238-247): the depthwise input is ReLU6(BN_e(ye)) with ye =
 * bf16(x_act . wt0^T) the expand conv's output, x [N,H,W,Cin] the block input (x_act: its pending
 * BatchNorm prologue x_mean.. / x_act, or x itself when x_mean is NULL), wt0 = the expand's forward
 * operand [C][Cin] bf16, e_* the expand BatchNorm (e_act ReLU6).  Each block forms ye for its input
 * rows with the expand forward's MFMA and rounding, so y and stat_parts (same count,
 * rod_dw3x3_fwd_stat_parts) are bit-identical to rod_dw3x3_fwd over the stored ye with that
 * prologue, while the C-wide ye is never read (1.42 GB at 720p b8, block 1).  bf16, stride 1 / 2,
 * Cin 16 / 24 / 32, TF-SAME pads; rod_dw3x3_fwd_rc_supported() tells which shapes. */
int rod_dw3x3_fwd_rc_supported(int N, int H, int W, int C, int Cin, int stride, int dtype);
int rod_dw3x3_fwd_rc(const void* x, const float* x_mean, const float* x_rstd, const float* x_gamma,
                     const float* x_beta, int x_act, const void* wt0, int Cin, const float* e_mean,
                     const float* e_rstd, const float* e_gamma, const float* e_beta, int e_act, const float* w,
                     void* y, float* stat_parts, int N, int H, int W, int C, int stride, int pad_t, int pad_l,
                     int Ho, int Wo, int dtype, void* stream);
/* dx = d y / d x  (DepthwiseConv2dNativeBackpropInput).
 * gred_* (nullable, ABI 4): when x was read through a BatchNorm-apply prologue, dx is the
 * gradient of that BatchNorm's output and the kernel also reduces its backward partial
 * sums in the epilogue: gred_y = the pre-BatchNorm tensor (x's storage, [N,H,W,C]),
 * gred_mean/rstd/gamma/beta/act its BatchNorm, gred_parts [nparts][2][C] with
 * nparts = rod_dw3x3_bwd_data_gred_parts(); see rod_bn_bwd_finalize. */
int rod_dw3x3_bwd_data_gred_parts(int N, int H, int W, int C, int stride, int dtype);
int rod_dw3x3_bwd_data(const void* dy, const float* w, void* dx, const void* gred_y, const float* gred_mean,
                       const float* gred_rstd, const float* gred_gamma, const float* gred_beta, int gred_act,
                       float* gred_parts, int N, int H, int W, int C, int stride, int pad_t, int pad_l,
                       int Ho, int Wo, int dtype, void* stream);
/* dw[3][3][C] (fp32, overwritten) (DepthwiseConv2dNativeBackpropFilter).
 * workspace: rod_dw3x3_bwd_filter_workspace() bytes. */
size_t rod_dw3x3_bwd_filter_workspace(int N, int Ho, int Wo, int C);
int rod_dw3x3_bwd_filter(const void* x, const float* pro_mean, const float* pro_rstd,
                         const float* pro_gamma, const float* pro_beta, int pro_act, const void* dy,
                         float* dw, void* workspace, int N, int H, int W, int C, int stride, int pad_t,
                         int pad_l, int Ho, int Wo, int dtype, void* stream);
/* Fused depthwise backward (ABI 12 stride 1; ABI 13 adds stride 2): for x = act_e(BN_e(ye))
 * (the input's BatchNorm-prologue form, pro_*) -> yd = DepthwiseConv2dNative(x, w, stride,
 * padding pad_t / pad_l) -> act_d(BN_d(yd)) (bn_*, with coef [3][C] from rod_bn_bwd_reduce over
 * (dz, yd)), ONE pass over ye, dz, yd (conv_blocks.py:238-247 backward, FusedBatchNormGrad
 * under mobilenet.py:417-420):
 *   dx = DepthwiseConv2dNativeBackpropInput(dy, w)  (T, [N,H,W,C]; bit-identical to
 *        rod_bn_bwd_apply -> rod_dw3x3_bwd_data),
 *   dw = DepthwiseConv2dNativeBackpropFilter(x, dy) (fp32 [3][3][C]),
 * with dy = rod_bn_bwd_apply(dz, yd, ...) ([N,Ho,Wo,C]) formed in registers and never stored;
 * gparts (nullable; needs pro_*) receives BN_e's backward sums over (dx, ye) as
 * [rod_dw3x3_bwd_fused_parts()][2][C] for rod_bn_bwd_finalize (the producer's
 * rod_bn_bwd_reduce pass disappears).  stride 1: pad 1, Ho = H, Wo = W; stride 2: pad 0 | 1.
 * C % 4 == 0; bf16 tensors 8-byte, fp32 16-byte aligned; workspace =
 * rod_dw3x3_bwd_fused_workspace bytes (both 0 for an unsupported geometry). */
int rod_dw3x3_bwd_fused_parts(int N, int H, int W, int C, int stride, int pad_t, int pad_l);
size_t rod_dw3x3_bwd_fused_workspace(int N, int H, int W, int C, int stride, int pad_t, int pad_l);
int rod_dw3x3_bwd_fused(const void* ye, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                        const float* pro_beta, int pro_act, const void* dz, const void* yd, const float* bn_mean,
                        const float* bn_rstd, const float* bn_gamma, const float* bn_beta, int bn_act,
                        const float* coef, const float* w, void* dx, float* dw, float* gparts, void* workspace, int N,
                        int H, int W, int C, int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype,
                        void* stream);
/* The stride-2 fused backward with its input recomputed, not read (ABI 23; conv_blocks.py:263-270
 * expand + mobilenet.py:417-420 + 238-247): rod_dw3x3_bwd_fused with ye (the expand conv's output,
 * C-wide) replaced by the block input x [N,H,W,Cin] (x_mean.. / x_act: its pending BatchNorm
 * prologue, NULL mean = none) and the expand's forward operand wt0 [C][Cin] bf16; e_* = the expand
 * BatchNorm (the depthwise input prologue, pro_* of rod_dw3x3_bwd_fused; ReLU6).  Each block forms
 * the ye values of its row steps in LDS with the expand forward's MFMA and rounding one step ahead,
 * so dx, dw and gparts (required: the BN_e sums) are bit-identical to rod_dw3x3_bwd_fused over the
 * stored ye, while ye is never read (1.42 GB at 720p b8, block 1).  bf16, stride 2, both BatchNorms
 * ReLU6, Cin 16 / 24 / 32; parts / workspace: rod_dw3x3_bwd_fused_parts / _workspace. */
int rod_dw3x3_bwd_fused_rc_supported(int N, int H, int W, int C, int Cin, int stride, int pad_t, int pad_l,
                                     int dtype);
int rod_dw3x3_bwd_fused_rc(const void* x, const float* x_mean, const float* x_rstd, const float* x_gamma,
                           const float* x_beta, int x_act, const void* wt0, int Cin, const float* e_mean,
                           const float* e_rstd, const float* e_gamma, const float* e_beta, int e_act, const void* dz,
                           const void* yd, const float* bn_mean, const float* bn_rstd, const float* bn_gamma,
                           const float* bn_beta, int bn_act, const float* coef, const float* w, void* dx, float* dw,
                           float* gparts, void* workspace, int N, int H, int W, int C, int stride, int pad_t,
                           int pad_l, int Ho, int Wo, int dtype, void* stream);
/* The same stride-1 pass without a materialised dz (ABI 20): in the inverted-residual block dz is
 * the project conv's input gradient dy_p . W_p (conv_blocks.py:287-294 backward), so the kernel
 * reads the cout-wide dy_p ([N*H*W][cout] bf16: the project BatchNorm's backward output, written
 * by rod_pw_bwd_gred_dyp) and wt1 = W_p^T ([C][cout] bf16, the conv's mode-1 layout) and forms dz
 * per row tile with the MFMA rod_pw_bwd_gred uses for it, rounded to bf16 once — dx, dw and gparts
 * bit-identical to rod_pw_bwd_gred -> rod_dw3x3_bwd_fused, minus the 2*es*M*C bytes of dz.  Plans:
 * rod_dw3x3_bwd_fused_pw_supported (bf16, both activations ReLU6, cout % 8 == 0 and <= 32, the
 * stride-1 tile <= 32 columns x 48 channels); pad 1, Ho = H, Wo = W; workspace as
 * rod_dw3x3_bwd_fused_workspace(N, H, W, C, 1, 1, 1); gparts as rod_dw3x3_bwd_fused_parts. */
int rod_dw3x3_bwd_fused_pw_supported(int N, int H, int W, int C, int cout, int pro_act, int bn_act, int dtype);
int rod_dw3x3_bwd_fused_pw(const void* ye, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                           const float* pro_beta, int pro_act, const void* dyp, const void* wt1, int cout,
                           const void* yd, const float* bn_mean, const float* bn_rstd, const float* bn_gamma,
                           const float* bn_beta, int bn_act, const float* coef, const float* w, void* dx, float* dw,
                           float* gparts, void* workspace, int N, int H, int W, int C, int dtype, void* stream);

/* The BatchNorm backward of the depthwise's output fused into its filter gradient (ABI 10):
 * dy = FusedBatchNormGrad-apply of (dz, y) with the coefficients coef[3][C] of
 * rod_bn_bwd_reduce (exactly rod_bn_bwd_apply's arithmetic; y = this depthwise's output before
 * its BatchNorm, bn_act its activation) is formed as the kernel streams dz / y, written to dy
 * (for rod_dw3x3_bwd_data), and contracted with x into dw — the separate apply pass over the
 * widest backbone tensors is never run (ref conv_blocks.py:238-247 + mobilenet.py:417-420).
 * Same workspace as rod_dw3x3_bwd_filter. */
int rod_dw3x3_bwd_filter_bn(const void* x, const float* pro_mean, const float* pro_rstd,
                            const float* pro_gamma, const float* pro_beta, int pro_act, const void* dz,
                            const void* y, const float* bn_mean, const float* bn_rstd, const float* bn_gamma,
                            const float* bn_beta, int bn_act, const float* coef, void* dy, float* dw,
                            void* workspace, int N, int H, int W, int C, int stride, int pad_t, int pad_l,
                            int Ho, int Wo, int dtype, void* stream);

/* ------------------------------------------------ BatchNorm (A4)
 * slim.batch_norm, fused, NHWC (mobilenet.py:417-420; catch_net.py:302).
 * Training statistics over all M rows of x[M, C] (row stride ldx):
 *   mean, biased var -> rstd = 1/sqrt(var + eps) used to normalise;
 *   moving_mean -= (moving_mean - mean)*(1-decay);
 *   moving_var  -= (moving_var  - var*M/(M-1))*(1-decay)   (FusedBatchNorm
 *   reports the Bessel-corrected variance to the moving average).
 * moving_* may be NULL (no update). */
size_t rod_bn_stats_workspace(long M, int C);
int rod_bn_stats(const void* x, long M, int C, int ldx, float eps, float decay,
                 float* mean, float* rstd, float* moving_mean, float* moving_var,
                 void* workspace, int dtype, void* stream);
/* The same statistics (and moving-average update) from partial statistics written by a
 * producer's epilogue: parts [nparts][3][C] = (count, mean, M2) per part; parts with
 * count 0 are ignored; M = total count.  Chan's merge in f64, fixed order (two levels when
 * nparts > 2048: workspace = rod_bn_finalize_workspace() bytes, else may be NULL). */
size_t rod_bn_finalize_workspace(int nparts, int C);
int rod_bn_finalize(const float* parts, int nparts, long M, int C, float eps, float decay,
                    float* mean, float* rstd, float* moving_mean, float* moving_var,
                    void* workspace, void* stream);
/* Partial statistics of x[M, C] (dense rows) as exactly nparts chunks of ceil(M/nparts) rows,
 * parts [nparts][3][C] in the rod_bn_finalize format (ABI 8).  For a BatchNorm whose
 * statistics span more rows than this process holds: data-parallel ranks all-gather their
 * parts and each merges the same array (SyncBN; the reference normalises over its whole
 * single-device batch, mobilenet.py:417-420). */
int rod_bn_stat_parts(const void* x, long M, int C, float* parts, int nparts, int dtype, void* stream);
/* inference: mean = moving_mean, rstd = 1/sqrt(moving_var + eps). */
int rod_bn_eval_stats(const float* moving_mean, const float* moving_var, float eps,
                      float* mean, float* rstd, int C, void* stream);
/* y = act(x*scale + offset) + residual, scale = rstd*gamma, offset = beta - mean*scale
 * (one fma, TF's fused batch-norm form; gamma NULL => 1,
 * beta NULL => 0, residual NULL => none; residual added after act, as
 * expanded_conv's `net += input_tensor`, conv_blocks.py:311). */
int rod_bn_apply(const void* x, const float* mean, const float* rstd, const float* gamma,
                 const float* beta, const void* residual, void* y, long M, int C, int ldx,
                 int ldr, int ldy, int act, int dtype, void* stream);
/* Backward of bn_apply (without the residual term, which the caller routes).
 * dy: grad of the activation output (row stride lddy); dx: grad wrt x (ldx);
 * dgamma/dbeta fp32 [C] are overwritten (dgamma may be NULL when gamma is). */
size_t rod_bn_bwd_workspace(long M, int C);
int rod_bn_bwd(const void* dy, const void* x, const float* mean, const float* rstd,
               const float* gamma, const float* beta, void* dx, float* dgamma, float* dbeta,
               void* workspace, long M, int C, int lddy, int ldx, int lddx, int act,
               int dtype, void* stream);
/* The same backward split at its reduction (ABI 4), for a BatchNorm applied in a
 * consumer's load prologue: the consumer's backward-data kernel (rod_conv_fwd /
 * rod_dw3x3_bwd_data "gred_*" arguments) writes dz = d/d(act output) and, from the same
 * registers plus the pre-BatchNorm y, the partial sums parts [nparts][2][C] =
 * (sum g, sum g*yhat), g = dz*act'(y*scale + offset), yhat = (y - mean)*rstd (the
 * reduction of FusedBatchNormGrad).  rod_bn_bwd_finalize merges them (f64, fixed order)
 * into dbeta, dgamma (either may be NULL) and coef[3][C] = (rstd*gamma, mean g,
 * mean g*yhat); rod_bn_bwd_apply writes dy = coef0*(g - coef1 - yhat*coef2) [M, C] dense,
 * bit for bit the rod_bn_bwd result for the same sums. */
int rod_bn_bwd_finalize(const float* parts, int nparts, long M, int C, const float* rstd,
                        const float* gamma, float* dgamma, float* dbeta, float* coef, void* stream);
int rod_bn_bwd_apply(const void* dz, const void* y, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, const float* coef, void* dy, long M, int C,
                     int act, int dtype, void* stream);
/* The reduction of FusedBatchNormGrad (ref mobilenet.py:417-420; catch_net.py:302) without
 * the apply pass (ABI 5): reads dz and the pre-BatchNorm y once, writes dbeta, dgamma
 * (either may be NULL) and coef[3][C] as rod_bn_bwd_finalize.  The consumer of coef applies
 * dy = coef0*(g - coef1 - yhat*coef2) as it loads (rod_pw_bwd), so dy never crosses HBM.
 * workspace: rod_bn_bwd_workspace(M, C) bytes. */
int rod_bn_bwd_reduce(const void* dz, const void* y, const float* mean, const float* rstd,
                      const float* gamma, const float* beta, float* dgamma, float* dbeta, float* coef,
                      void* workspace, long M, int C, int act, int dtype, void* stream);
/* The backward partial sums alone (ABI 8): parts [nparts][2][C] = (sum g, sum g*yhat) over
 * exactly nparts chunks of ceil(M/nparts) rows, for rod_bn_bwd_finalize — after an
 * all-gather over data-parallel ranks under SyncBN (FusedBatchNormGrad over the global batch). */
int rod_bn_bwd_parts(const void* dz, const void* y, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, int act, float* parts, int nparts, long M, int C,
                     int dtype, void* stream);

/* ------------------------------------------------ VGG-16 backbone (F3, ABI 9)
 * nets/backbone/vgg.py:67-137 (vgg_16 with the SSD extra blocks 6-10).  C % 8 == 0 (bf16) /
 * C % 4 == 0 (fp32) for all of these.
 * slim.max_pool2d([2, 2]) — stride 2, VALID (vgg.py:93-101): Ho = H/2, Wo = W/2 (floor);
 * argmax [N][Ho][Wo][C] uint8 = window position 0..3 (row-major) of the first maximum. */
int rod_maxpool2x2(const void* x, void* y, uint8_t* argmax, int N, int H, int W, int C, int dtype, void* stream);
/* MaxPoolGrad: dx[N][H][W][C] = dy at each window's argmax position, 0 elsewhere. */
int rod_maxpool2x2_bwd(const void* dy, const uint8_t* argmax, void* dx, int N, int H, int W, int C, int dtype,
                       void* stream);
/* tf.layers.dropout(rate, training=True) (vgg.py:106, 111; rate = the reference's
 * dropout_keep_prob = 0.5): binary = floor(keep_prob + U[0,1)), y = x / keep_prob * binary;
 * U from a counter-based hash of (seed, element index), mask[n] = binary for the backward. */
int rod_dropout(const void* x, void* y, uint8_t* mask, long n, float keep_prob, uint64_t seed, int dtype,
                void* stream);
int rod_dropout_bwd(const void* dy, const uint8_t* mask, void* dx, long n, float keep_prob, int dtype, void* stream);
/* 3x3 convolution as an explicit column matrix, for the strides / paddings rod_conv_fwd does
 * not take: custom_layers.pad2d(1) + VALID stride 2 (vgg.py:116-118, 123-125) and VALID stride 1
 * (vgg.py:131): col[M = N*Ho*Wo][(i*3 + j)*C + c] = x[n, ho*stride + i - pad_t, wo*stride + j -
 * pad_l, c] (0 outside), read through the optional BatchNorm / activation prologue (ABI 3).
 * rod_conv_fwd / rod_conv_wgrad with ksize 1 and Cin = 9*C then run the GEMMs. */
int rod_im2col3x3(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                  const float* pro_beta, int pro_act, void* col, int N, int H, int W, int C, int stride, int pad_t,
                  int pad_l, int Ho, int Wo, int dtype, void* stream);
/* dx[N][H][W][C] = the sum of the column-matrix entries that read each input (col2im). */
int rod_col2im3x3(const void* col, void* dx, int N, int H, int W, int C, int stride, int pad_t, int pad_l, int Ho,
                  int Wo, int dtype, void* stream);

/* ------------------------------------- PREORDER_MSF feature augmentation (F4, ABI 9)
 * process_backbone_method.PREORDER_MSF (nets/catch_net.py:115-152).  rod_se_*: C % 8 (bf16) / 4
 * (fp32); pad and space_to_depth take any C (16-byte vectors when C allows).
 * tf.pad(x, [[0,0],[top,0],[left,0],[0,0]]) into y [N][Hp][Wp][C] (zeros elsewhere);
 * inverse != 0: the gradient, y [N][H][W][C] = x[n, h+top, w+left] of a padded x [N][Hp][Wp][C]. */
int rod_pad2d(const void* x, void* y, int N, int H, int W, int C, int top, int left, int Hp, int Wp, int inverse,
              int dtype, void* stream);
/* tf.space_to_depth(x [N][H][W][C], block): y[n, i, j, (di*block + dj)*C + c] = x[n, i*block + di,
 * j*block + dj, c]; inverse != 0: depth_to_space (x [N][H/block][W/block][block^2*C] -> y [N][H][W][C]). */
int rod_space_to_depth(const void* x, void* y, int N, int H, int W, int C, int block, int inverse, int dtype,
                       void* stream);
/* se_block (nets/attention_module.py:3-33) on x [N][HW][C]: sq = mean over HW [N][C] fp32,
 * hid = relu(sq . w1 + b1) [N][C8], e = sigmoid(hid . w2 + b2) [N][C], y = x * e.
 * w1 [C][C8], w2 [C8][C] (tf.layers.dense kernels), fp32. */
int rod_se_fwd(const void* x, const float* w1, const float* b1, const float* w2, const float* b2, float* sq,
               float* hid, float* e, void* y, int N, long HW, int C, int C8, int dtype, void* stream);
/* Its backward: de = sum_HW dy*x, the dense layers' gradients (dw1 / db1 / dw2 / db2 overwritten,
 * each may be NULL; summed over the N images), dx = dy*e + dsq/HW.  de, dsq: [N][C] scratch. */
int rod_se_bwd(const void* dy, const void* x, const float* w1, const float* w2, const float* sq, const float* hid,
               const float* e, float* de, float* dsq, float* dw1, float* db1, float* dw2, float* db2, void* dx, int N,
               long HW, int C, int C8, int dtype, void* stream);

/* -------------------------------------- dense conv as implicit GEMM (A2 A3 A5)
 * y[m, co] = sum_k A[m, k] * wt[co, k] (+ bias[co]), fp32 accumulation,
 *   ksize 1: A = x rows [M = N*H*W, Cin] (slim.conv2d [1,1], conv_blocks.py:343)
 *   ksize 3: A = 3x3 im2col of x, stride 1, TF-SAME (pad 1/1), k = (i*3+j)*Cin + ci
 *            (stem mobilenet_v2.py:58; heads catch_net.py:303, 336)
 * wt: [Cout][ksize*ksize*Cin] in the activation dtype; bias fp32 or NULL.
 * ldx / ldy: row strides of x / y in elements (0 => Cin / Cout), so a conv can
 * read or write a channel slice of a concatenated buffer (catch_net.py:211).
 * workspace: rod_conv_fwd_workspace() bytes; non-zero when the output has too few
 * 128-row tiles to fill the chip and K is deep (head convs on the small pyramid levels):
 * K is then split over workgroups into fp32 partial slabs summed in fixed order.  NULL
 * is accepted and disables the split.
 * stat_parts (nullable): BatchNorm partial statistics of y for rod_bn_finalize, as
 * [ceil(M/128)][3][Cout] (count, mean, M2) per 128-row tile, computed in the epilogue from
 * the rounded outputs (the BatchNorm that follows every conv, mobilenet.py:417,
 * catch_net.py:302) so no separate statistics pass re-reads y. */
size_t rod_conv_fwd_workspace(int N, int H, int W, int Cin, int Cout, int ksize);
/* gred_* (nullable, ABI 4): used as a backward-data (x = dy, wt mode 1) whose input went
 * through a BatchNorm-apply prologue in the forward, the output is that BatchNorm's dz and
 * the epilogue also writes its backward partial sums [ceil(M/128)][2][Cout] (gred_y = the
 * pre-BatchNorm tensor [M, Cout], dense; see rod_bn_bwd_finalize). */
int rod_conv_fwd(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                 const float* pro_beta, int pro_act, const void* wt, const float* bias, void* y,
                 void* workspace, float* stat_parts, const void* gred_y, const float* gred_mean,
                 const float* gred_rstd, const float* gred_gamma, const float* gred_beta, int gred_act,
                 float* gred_parts, int N, int H, int W, int Cin, int Cout, int ksize, int ldx, int ldy,
                 int dtype, void* stream);
/* ABI 14: 1 when rod_conv_fwd of this 1x1 shape (no bias, no prologue, 16-byte aligned dense
 * rows) takes the streaming kernel, whose gred epilogue costs about one extra read of gred_y —
 * the caller then asks for the gred sums instead of running rod_bn_bwd_reduce over (dz, y)
 * afterwards (the project conv's backward-data and the depthwise BatchNorm it feeds,
 * conv_blocks.py:287-294 -> 238-247); 0 otherwise.  M = N*H*W rows, K = Cin. */
int rod_conv_fwd_stream_ok(long M, int K, int Cout, int dtype);
/* Statistics only (ABI 23): the BatchNorm statistics parts of y = x_act . wt^T ([ceil(M/128)][3][Cout],
 * the stat_parts contract of rod_conv_fwd, bit-identical to it) with y NOT written — the expand conv
 * of an inverted-residual block whose consumers recompute y from x (rod_dw3x3_fwd_rc,
 * rod_dw3x3_bwd_fused_rc, rod_pw_bwd(_gred)_rc): the C-wide expanded tensor never crosses HBM.
 * 1x1, no bias, bf16, Cin <= 32 on the streaming kernel's shapes (rod_conv_fwd_stats_supported). */
int rod_conv_fwd_stats_supported(long M, int Cin, int Cout, int dtype);
int rod_conv_fwd_stats(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                       const float* pro_beta, int pro_act, const void* wt, float* stat_parts, long M, int Cin, int Cout,
                       int dtype, void* stream);
/* Inference conv + BatchNorm-apply epilogue (ABI 21): rod_conv_fwd whose output is
 *   z = act(fma(y, scale, offset)) (+ res),  y = the conv output rounded to bf16,
 *   scale = bn_rstd*bn_gamma, offset = bn_beta - bn_mean*scale (bn_affine),
 * rounded once — exactly what rod_conv_fwd followed by rod_bn_apply(y, ..., res, z) writes
 * (slim.conv2d + slim.batch_norm(is_training=False) + act (+ the block's residual add),
 * mobilenet.py:417-420, conv_blocks.py:302-311, catch_net.py:301-305), without y crossing HBM.
 * bf16 only; res (nullable) [M][ldr] with 16-byte rows; the other arguments as rod_conv_fwd
 * (no statistics / gred epilogue: inference). */
int rod_conv_fwd_bnact(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                       const float* pro_beta, int pro_act, const void* wt, const float* bias, void* z, void* workspace,
                       const float* bn_mean, const float* bn_rstd, const float* bn_gamma, const float* bn_beta,
                       int bn_act, const void* res, int ldr, int N, int H, int W, int Cin, int Cout, int ksize,
                       int ldx, int ldy, int dtype, void* stream);
/* Backward-data of a 1x1 conv through its BatchNorm (ABI 22): the BatchNorm-backward apply
 *   dy = rod_bn_bwd_apply(dz, y, mean, rstd, gamma, beta, coef, act)   [M][Cout], bf16, written
 * formed in the GEMM's operand loader, and dx[M][Cin] = dy . wt1^T — bit for bit what
 * rod_bn_bwd_apply followed by rod_conv_fwd(dy, wt1 (mode 1), ..., Cin = Cout, Cout = Cin, 1x1)
 * writes (FusedBatchNormGrad + Conv2DBackpropInput of slim.conv2d + slim.batch_norm,
 * conv_blocks.py:263-294 expand convs), in one launch: the deep expands' dy is produced where it
 * is first consumed; the weight gradient then reads it (rod_conv_wgrad).  bf16, Cout % 8 == 0,
 * Cin % 8 == 0, 16-byte aligned dense rows.  workspace: rod_conv_fwd_workspace(1, 1, M, Cout,
 * Cin, 1) bytes (split-K partials; NULL when 0). */
int rod_conv_bwd_data_bn_supported(int Cout, int Cin, int dtype);
int rod_conv_bwd_data_bn(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                         const float* beta, int act, const float* coef, const void* wt1, void* dy, void* dx,
                         void* workspace, long M, int Cout, int Cin, int dtype, void* stream);
/* Weight layouts derived from the fp32 master weight w[Cout][ksize][ksize][Cin]:
 *   mode 0: forward operand      wt[co][i][j][ci]           (cast to dtype)
 *   mode 1: backward-data operand wt[ci][2-i][2-j][co]       (transposed, flipped)
 * so dx = rod_conv_fwd(dy, wt_mode1) (Conv2DBackpropInput, stride 1 SAME). */
int rod_conv_weight_prep(const float* w, void* wt, int Cout, int Cin, int ksize, int mode,
                         int dtype, void* stream);
/* Every weight of a step in one launch: table is a DEVICE array of n entries
 *   struct { const float* w; void* wt; long start; int Cout, Cin, ksize, mode; }  (40 bytes)
 * each as rod_conv_weight_prep(w, wt, Cout, Cin, ksize, mode); start = the sum of
 * Cout*ksize*ksize*Cin over the entries before it (ascending), total = the sum over all. */
int rod_conv_weight_prep_batch(const void* table, int n, long total, int dtype, void* stream);
/* dw[co][k] = sum_m dy[m, co] * A[m, k]  (Conv2DBackpropFilter), fp32 out,
 * db[co] = sum_m dy[m, co] when db != NULL.  workspace: see query. */
size_t rod_conv_wgrad_workspace(int N, int H, int W, int Cin, int Cout, int ksize);
int rod_conv_wgrad(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                   const float* pro_beta, int pro_act, const void* dy, float* dw, float* db,
                   void* workspace, int N, int H, int W, int Cin, int Cout, int ksize, int ldx,
                   int lddy, int dtype, void* stream);

/* -------------------------------------- fused inverted-residual block, inference (ABI 6)
 * out = BN_p(project(relu6(BN_d(dw3x3_s(relu6(BN_e(expand(x)))))))) (+ x when residual)
 * — expanded_conv (ref conv_blocks.py:163-312) with eval-mode BatchNorms (mean / rstd from
 * rod_bn_eval_stats; gamma / beta as in rod_bn_apply), in ONE kernel: the expanded tensor
 * stays in LDS (chunks of 32 channels).  we = expand weights [inner][Cin]
 * and wp = project weights [Cout][inner] in bf16 (rod_conv_weight_prep mode 0), wd fp32
 * [3][3][inner].  x [N,H,W,Cin] -> out [N,ceil(H/s),ceil(W/s),Cout], bf16, TF-SAME padding.
 * Bit-identical to the unfused chain rod_conv_fwd -> rod_dw3x3_fwd -> rod_conv_fwd ->
 * rod_bn_apply (same roundings, same MFMA k order) where those run without split-K.
 * rod_ir_block_supported: stride 1 with Cin, Cout <= 160; stride 2 with Cin <= 96,
 * Cout <= 320; channels multiples of 8; residual only for stride 1 and Cin == Cout. */
int rod_ir_block_supported(int Cin, int inner, int Cout, int stride, int residual, int dtype);
int rod_ir_block_fwd(const void* x, const void* we, const float* e_mean, const float* e_rstd,
                     const float* e_gamma, const float* e_beta, const float* wd, const float* d_mean,
                     const float* d_rstd, const float* d_gamma, const float* d_beta, const void* wp,
                     const float* p_mean, const float* p_rstd, const float* p_gamma, const float* p_beta,
                     int residual, void* y, int N, int H, int W, int Cin, int inner, int Cout, int stride,
                     int dtype, void* stream);
/* Variant switch (process-wide; returns the previous value).  Bit 0 (set by default): a
 * persistent launch — every chunk's parameters resident in LDS, each workgroup walking tiles
 * with the next tile's input window in flight — wherever those parameters fit in LDS; clear:
 * one tile per workgroup (identical output).  Bit 1 (ABI 14, clear by default): the exact
 * rounding of the unfused eval chain (each conv output rounded to bf16 before its BatchNorm),
 * bit-identical to it; clear: the accumulators go through BatchNorm (+ ReLU6) in fp32 and are
 * rounded once. */
int rod_ir_block_set_mode(int mode);
/* 1 when the block runs the persistent variant (all of its parameters fit in LDS). */
int rod_ir_block_persistent(int Cin, int inner, int Cout, int stride, int residual, int dtype);

/* -------------------------------------- fused 1x1-conv backward through its BatchNorm (ABI 5)
 * The backward of  z = act(BN(y)), y = conv1x1(a) + bias,  a = act_x(BN_x(x)) or x, in ONE
 * pass over the rows (ref: Conv2DBackpropInput + Conv2DBackpropFilter + FusedBatchNormGrad of
 * slim.conv2d + slim.batch_norm, conv_blocks.py:263-294, catch_net.py:301-304):
 *   dy = coef0*(dz*act'(y*sc + sh) - coef1 - yhat*coef2)   (coef from rod_bn_bwd_reduce,
 *        rounded to bf16 as rod_bn_bwd_apply would store it, kept in LDS only)
 *   dx = dy . W            (W = the mode-1 operand wt1[Cin][Cout], bf16) -> dx [M, Cin]
 *   dw = a^T . dy  -> dw fp32 [Cout][Cin] (overwritten), db = sum_m dy (when db != NULL)
 * a = the conv input with the optional BatchNorm-apply prologue (xmean NULL => none).  One
 * read of dz, y and x, one write of dx: the dy tensor of the unfused path (write + 3 reads)
 * does not exist.  bf16 only; rod_pw_bwd_supported() tells which (Cin, Cout) it takes (Cin,
 * Cout multiples of 8, Cin*Cout <= 16384, Cin <= 192, Cout <= 512).  dx may be NULL (input
 * gradient not needed).  workspace: rod_pw_bwd_workspace() bytes. */
int rod_pw_bwd_supported(int Cin, int Cout, int dtype);
size_t rod_pw_bwd_workspace(long M, int Cin, int Cout);
int rod_pw_bwd(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
               const float* beta, int act, const float* coef, const void* x, const float* xmean,
               const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1,
               void* dx, float* dw, float* db, void* workspace, long M, int Cin, int Cout, int dtype,
               void* stream);
/* Project form (ABI 17): the same backward for a 1x1 conv whose input is the ReLU6(BatchNorm) of
 * a depthwise output — the inverted-residual block's project conv (conv_blocks.py:287-294 after
 * 238-247) — and, in the same pass, the backward sums of THAT input BatchNorm over (dx, x):
 *   xparts[p][0][c] = sum g, xparts[p][1][c] = sum g*xhat,  g = dx*act_x'(x*sc_x + sh_x),
 *   xhat = (x - xmean)*xrstd  (the [nparts][2][Cin] contract of rod_bn_bwd_finalize)
 * so the depthwise BatchNorm's rod_bn_bwd_reduce pass over (dz, y) is not needed: x is read once
 * for the weight gradient's prologue and for the sums, dx is summed as it is written.  No bias;
 * xmean / xrstd, dx and wt1 required.  rod_pw_bwd_gred_parts() is the part count (0: shape not taken —
 * bf16, Cout in {16, 24, 32, 64}, Cin a multiple of 32 or 48; or the expand shape 16 -> 96, whose
 * input is the previous block's project output: its linear BatchNorm's sums, ABI 18); workspace:
 * rod_pw_bwd_gred_workspace() bytes.  dx is rod_pw_bwd's bit for bit. */
long rod_pw_bwd_gred_parts(long M, int Cin, int Cout, int dtype);
size_t rod_pw_bwd_gred_workspace(long M, int Cin, int Cout);
int rod_pw_bwd_gred(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                    const float* beta, int act, const float* coef, const void* x, const float* xmean,
                    const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1,
                    void* dx, float* dw, float* xparts, void* workspace, long M, int Cin, int Cout, int dtype,
                    void* stream);
/* The same pass handing the consumer the project BatchNorm's backward output instead of dx
 * (ABI 20): dyp [M][Cout] bf16 = dy (the values dx = dy . W is formed from, written once by the
 * first column group), dx NOT written; dw and xparts exactly as rod_pw_bwd_gred (they are formed
 * from the same in-register dx).  For a depthwise that recomputes dx = dy . W itself
 * (rod_dw3x3_bwd_fused_pw): the Cin-wide dx never crosses HBM.  The shapes of rod_pw_bwd_gred
 * other than the expand form (16 -> 96). */
int rod_pw_bwd_gred_dyp(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                        const float* beta, int act, const float* coef, const void* x, const float* xmean,
                        const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1,
                        void* dyp, float* dw, float* xparts, void* workspace, long M, int Cin, int Cout, int dtype,
                        void* stream);
/* Expanded tensor recomputed, not read (ABI 23; ref conv_blocks.py:263-270 expand + 238-247): the
 * same backward of an inverted-residual block's expand conv with y (its pre-BatchNorm output, the
 * C-wide expanded tensor) NOT passed: each 16-row tile of it is recomputed as bf16(a . wt0^T) from
 * the conv input a (x with the optional prologue) the kernel already reads for the weight gradient,
 * with the forward's MFMA and rounding — bit for bit the y the forward would have stored.
 * wt0 = the forward operand [Cout][Cin] bf16 (rod_conv_weight_prep mode 0).  The M x Cout y stream
 * (1.42 GB at 720p b8 for 16 -> 96) is gone.  rod_pw_bwd_rc: the streaming shapes 16 -> 96 and
 * 24 -> 144 (rod_pw_bwd_rc_supported), no bias, outputs identical to rod_pw_bwd; rod_pw_bwd_gred_rc:
 * the 16 -> 96 expand form of rod_pw_bwd_gred (its parts / workspace queries apply). */
int rod_pw_bwd_rc_supported(long M, int Cin, int Cout, int dtype);
int rod_pw_bwd_rc(const void* dz, const void* wt0, const float* mean, const float* rstd, const float* gamma,
                  const float* beta, int act, const float* coef, const void* x, const float* xmean,
                  const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1, void* dx,
                  float* dw, void* workspace, long M, int Cin, int Cout, int dtype, void* stream);
int rod_pw_bwd_gred_rc(const void* dz, const void* wt0, const float* mean, const float* rstd, const float* gamma,
                       const float* beta, int act, const float* coef, const void* x, const float* xmean,
                       const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1,
                       void* dx, float* dw, float* xparts, void* workspace, long M, int Cin, int Cout, int dtype,
                       void* stream);

/* Stem weight gradient through its BatchNorm (ABI 18): rod_conv_wgrad of the 3x3, 3 -> 32 stem
 * (mobilenet_v2.py:58 conv + mobilenet.py:417-420 batch_norm) with dy formed in the loader from
 * the BatchNorm's (dz, y) by rod_bn_bwd_apply's arithmetic (coef from rod_bn_bwd_reduce or
 * rod_bn_bwd_finalize) instead of read: the [M, 32] dy of the unfused path is never written or
 * read.  dw fp32 [32][3][3][3] (overwritten); workspace: rod_conv_wgrad_workspace() of the same
 * shape; x bf16 NHWC [N,H,W,3]; dz / y bf16 [N,H,W,32].  bf16, ksize 3, Cin 3, Cout 32 only
 * (rod_stem_wgrad_bn_supported). */
int rod_stem_wgrad_bn_supported(int Cin, int Cout, int ksize, int dtype);
int rod_stem_wgrad_bn(const void* x, const void* dz, const void* y, const float* mean, const float* rstd,
                      const float* gamma, const float* beta, int act, const float* coef, float* dw, void* workspace,
                      int N, int H, int W, int Cin, int Cout, int ksize, int dtype, void* stream);

/* ------------------------------------------------ targets and losses
 * Anchor matching, JACCARD_BIGGER (utils/net_tools.py:270-428, branch 382-421).
 * anc_corner/anc_center: [A,4] fp32 = (ymin,xmin,ymax,xmax) / (cy,cx,h,w) of
 * every anchor, levels concatenated in (fh,fw,A) order; lvl_off[L+1] anchor
 * offset of each level; thr[L] refine_pos_jac_val_all_layers (config.py:79).
 * gt: [B,G,4] centre boxes (cy,cx,h,w) normalised (train.py:109); gt_lbl [B,G];
 * gt_n [B] valid boxes per image (>= 1, net_tools.py:398 reads box 0).
 * Outputs [B,A,4] / [B,A]: encoded offsets (net_tools.py:147-179), matched
 * centre box, label, positive mask — zero where not positive. */
int rod_match_anchors(const float* anc_corner, const float* anc_center, const int* lvl_off,
                      const float* thr, int L, const float* gt, const int* gt_lbl,
                      const int* gt_n, float* out_off, float* out_cbox, int* out_lbl,
                      int* out_pos, int B, int A, int G, void* stream);
/* NEAREST_NEIGHBOR (net_tools.py:354-380, ABI 9): the box of least sum of squared encoded
 * offsets (tf.argmin, first minimum wins) is matched to EVERY anchor (pos_mask = ones);
 * same arrays as rod_match_anchors without the thresholds. */
int rod_match_anchors_nn(const float* anc_corner, const float* anc_center, const int* lvl_off, int L, const float* gt,
                         const int* gt_lbl, const int* gt_n, float* out_off, float* out_cbox, int* out_lbl,
                         int* out_pos, int B, int A, int G, void* stream);
/* Masked smooth-L1 (net_tools.py:478-516): per-level sums of
 * smooth_l1((target - pred)*mask) / scale written to loss_lvl[0..L-1] and their
 * sum (accumulated in level order) to loss_lvl[L] (fp32, device, L+1 entries),
 * and grad = d(sum/scale)/d pred when grad != NULL; grad_target (nullable, fp32) =
 * d(sum/scale)/d target = -grad (the ODM target det_gt depends on refine_out when the refine
 * net is trained, net_tools.py:471).  pred [B,A,4] in dtype, target fp32 [B,A,4], mask int [B,A]. */
size_t rod_smoothl1_workspace(int B, int A);
int rod_smoothl1_masked(const void* pred, const float* target, const int* mask,
                        const int* lvl_off, int L, float scale, float* loss_lvl, void* grad,
                        float* grad_target, void* workspace, int B, int A, int dtype, void* stream);

/* Box conversions on [n,4] fp32 (utils/common_tools.py:16-56):
 * to_center=1: (ymin,xmin,ymax,xmax) -> (cy,cx,h,w); 0: the inverse. */
int rod_boxes_convert(const float* in, float* out, long n_boxes, int to_center, void* stream);
/* Strided block copy: rows x cols_bytes from src (row stride src_ld_bytes) to dst
 * (dst_ld_bytes); used for tf.concat of per-level tensors (net_tools.py:557-565). */
int rod_copy2d(const void* src, long src_ld_bytes, void* dst, long dst_ld_bytes, long rows, long cols_bytes,
               void* stream);

/* ------------------------------------------------ deconvolution pyramid (A6)
 * Legacy TF1 bilinear resize, align_corners=False: src = dst * in/out, no half-pixel
 * offset (tf.image.resize_images; catch_net.py:207, tf_image.py:266-278), NHWC. */
int rod_resize_bilinear(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo,
                        int dtype, void* stream);
/* ResizeBilinearGrad: dx [N,H,W,C] from dy [N,Ho,Wo,C] (deterministic gather). */
int rod_resize_bilinear_bwd(const void* dy, void* dx, int N, int H, int W, int C, int Ho, int Wo,
                            int dtype, void* stream);
/* conv2d_transpose(k=2, s=2, SAME) = 1x1 rod_conv_fwd to z [N,h,w,4F] (channel (a*2+b)*F+f,
 * weight [2,2,F,Cin] read as [4F,Cin]) followed by this scatter into out [N,Ho,Wo,ldo]
 * (rows/cols >= Ho/Wo cropped; catch_net.py:196).  space_to_depth2 is its adjoint. */
int rod_depth_to_space2(const void* z, void* out, int N, int h, int w, int F, int Ho, int Wo,
                        int ldo, int dtype, void* stream);
int rod_space_to_depth2(const void* dout, void* dz, int N, int h, int w, int F, int Ho, int Wo,
                        int ldo, int dtype, void* stream);
/* c = a + b elementwise (ADD merge catch_net.py:269). */
int rod_add(const void* a, const void* b, void* c, long n, int dtype, void* stream);

/* ------------------------------------------------ decode / ODM targets / classification loss
 * decode_locations_one_layer (net_tools.py:182-234) of off_a (+ off_b, NULL = none) against
 * the anchor centres, levels concatenated: out fp32 [B,A,4] centre boxes, or corners when
 * to_corner (centerBboxes_2_cornerBboxes, predict.py:133). */
int rod_decode(const float* anc_center, const void* off_a, const void* off_b, float* out, int B,
               int A, int to_corner, int dtype, void* stream);
/* det_groundtruth (net_tools.py:431-475): IoU of the refined anchor with its matched box,
 * det_pos = (iou >= thr[level]) & refine_pos, det_gt = (refine_gt - refine_out)*det_pos,
 * det_lbl = label*det_pos; iou [B,A] fp32 is also returned for the IoU factor.
 * lvl_off[L+1], thr[L] (det_pos_jac_val_all_layers) are host arrays. */
int rod_det_targets(const float* anc_center, const void* refine_out, const float* refine_gt,
                    const float* cbox, const int* label, const int* refine_pos, const int* lvl_off,
                    const float* thr, int L, float* det_gt, int* det_pos, int* det_lbl, float* iou,
                    int B, int A, int dtype, void* stream);
/* Backward of rod_det_targets wrt refine_out, for training the refine net through the ODM
 * loss (train.py fix_refine=False; the reference has no stop-gradient, net_tools.py:459-471):
 * g_refine_out = -g_det_gt * det_pos + d iou / d refine_out * g_iou (decode -> corners ->
 * jaccard with TF's max/min gradient rules).  g_det_gt / g_iou fp32 nullable; output in the
 * refine_out dtype, overwritten. */
int rod_det_targets_bwd(const float* anc_center, const void* refine_out, const float* cbox,
                        const int* det_pos, const float* g_det_gt, const float* g_iou,
                        void* g_refine_out, int B, int A, int dtype, void* stream);
/* d clf_loss / d iou through the per-(image, level) IoU focal factor (net_tools.py:590-607:
 * tf.nn.moments standardisation, min-shift, max-normalise, ^4; reduce_min/max gradients
 * split over ties as TF does), for the positives' cross-entropy recomputed from logits.
 * g_iou fp32 [B*A] overwritten. */
int rod_iou_factor_bwd(const void* logits, const int* det_lbl, const int* det_pos, const float* iou,
                       const int* lvl_off, int L, float bs, float* g_iou, int B, int A, int K,
                       int dtype, void* stream);
/* probs[r, k] = softmax(logits[r, :]) over K <= 16 classes, fp32 out (slim.softmax). */
int rod_softmax(const void* logits, float* probs, long rows, int K, int dtype, void* stream);
/* Classification half of det_clf_loss with global hard-negative mining (net_tools.py:551-615),
 * all on the device: nvalues, k = min(int(3*n_pos)+B, n_neg), exact radix select of the
 * k-th smallest nvalue, strict '<' negative mask, per-(image,level) IoU factor, CE losses.
 * logits [B*A, K] (dtype), det_lbl/det_pos int [B*A], iou fp32 [B*A], lvl_off host [L+1].
 * out fp32 [8] (device): pos_loss, neg_loss, clf_loss, max_hard_pred, n_pos, k,
 * n_neg_selected, 0.  grad (nullable, dtype [B*A, K]) = d clf_loss / d logits. */
size_t rod_softmax_ce_hnm_workspace(int B, int A, int L);
int rod_softmax_ce_hnm(const void* logits, const int* det_lbl, const int* det_pos, const float* iou,
                       const int* lvl_off, int L, float bs, float* out, void* grad, void* workspace,
                       int B, int A, int K, int dtype, void* stream);
/* The same, split at its exchange points for data parallelism (the reference
 * selects negatives over the WHOLE batch, net_tools.py:557-587).  Per rank, on its B images:
 *   rod_hnm_rows        -> counts[2] = (n_pos, n_neg) of its rows  [caller: all-reduce SUM]
 *   rod_hnm_begin       -> state (k from the global counts, B_global = the global batch)
 *   for shift = 24, 16, 8, 0:
 *     rod_hnm_radix_hist -> hist[256] of its rows                 [caller: all-reduce SUM]
 *     rod_hnm_radix_scan -> the next digit of the k-th smallest nvalue (clears hist)
 *   rod_hnm_loss        -> out / grad of its rows; bs = the GLOBAL batch; out[6] counts
 *                          this rank's selected negatives
 * counts (int[2]), state (int[8]) and hist (unsigned[256]) are caller-owned device arrays;
 * every call is stream-ordered (the all-reduces go on the same stream).  Integer sums make
 * k and the threshold bit-identical to rod_softmax_ce_hnm on the concatenated batch.
 * workspace: rod_hnm_workspace() bytes (per rank, kept from rod_hnm_rows to rod_hnm_loss). */
size_t rod_hnm_workspace(int B, int A, int L);
int rod_hnm_rows(const void* logits, const int* det_pos, void* workspace, int* counts, int B, int A,
                 int K, int L, int dtype, void* stream);
int rod_hnm_begin(const int* counts, int B_global, int* state, unsigned* hist, void* stream);
int rod_hnm_radix_hist(const void* workspace, int B, int A, int L, int shift, const int* state,
                       unsigned* hist, void* stream);
int rod_hnm_radix_scan(int shift, int* state, unsigned* hist, void* stream);
int rod_hnm_loss(const void* logits, const int* det_lbl, const int* det_pos, const float* iou,
                 const int* lvl_off, int L, float bs, const int* state, float* out, void* grad,
                 void* workspace, int B, int A, int K, int dtype, void* stream);

/* ------------------------------------------------ post-processing (A15)
 * detected_bboxes (net_tools.py:739-758) for every image and class 1..K-1: select
 * (p >= select_threshold), top_k sort (score desc, ties by index), greedy NMS (IoU >
 * nms_threshold, tf.image.non_max_suppression semantics), zero-pad to keep_top_k.
 * probs fp32 [B,A,K]; boxes fp32 corner [B,A,4];
 * out_scores [B,K-1,keep_top_k], out_boxes [B,K-1,keep_top_k,4]; top_k, keep_top_k <= 1024.
 * workspace (ABI 7; rod_select_topk_nms_workspace bytes, may be NULL): with it and
 * select_threshold > 0 (K - 1 <= 32) probs is read ONCE, row-wise, and every class's selected
 * scores are compacted into per-(image, class) candidate lists that are sorted / radix-selected
 * on their own; otherwise each (image, class) reads its probs column directly.  Same output. */
size_t rod_select_topk_nms_workspace(int B, int A, int K);
int rod_select_topk_nms(const float* probs, const float* boxes, int B, int A, int K,
                        float select_threshold, int top_k, int keep_top_k, float nms_threshold,
                        float* out_scores, float* out_boxes, void* workspace, void* stream);

/* ------------------------------------------------ optimiser (A14)
 * Plain SGD with clip by value (net_tools.py:645-651):
 *   p -= lr * clamp(g, -clip, clip)   over one flat fp32 buffer. */
int rod_sgd_clip(float* param, const float* grad, long n, float lr, float clip, void* stream);

/* ------------------------------------------------ deferred parameter-gradient sums (ABI 11)
 * The weight / bias gradients of rod_conv_wgrad, rod_dw3x3_bwd_filter(_bn) and rod_pw_bwd end in
 * a fixed-order f64 sum of per-workgroup fp32 partial slabs, whose only readers are the
 * optimizer (ApplyGradientDescent under net_tools.py:645-651) and the data-parallel all-reduce.
 * rod_slab_defer(1) makes the library (process-wide: autograd may run the backward on another
 * thread) queue those sums instead of launching them (the
 * ONE exception to "no pointer kept past the call": the caller keeps the partial slabs and
 * the gradient outputs alive, unmodified, until the flush); rod_slab_flush runs every queued
 * sum on `stream` as one batched launch per 32 sums, bit-identical to the immediate launches;
 * rod_slab_defer(0) stops queueing (queued sums stay queued until flushed).  rod_slab_defer
 * returns the previous mode, rod_slab_pending the queue length.
 * rod_slab_flush_range (ABI 15) runs only the queued sums whose output lies entirely in the
 * byte range [lo, hi) — the data-parallel bucket about to be all-reduced (the reduce point,
 * net_tools.py:645-651) — and leaves the others queued, so a bucket launched from inside
 * backward does not split the rest of the step's batched sums. */
int rod_slab_defer(int on);
int rod_slab_pending(void);
int rod_slab_flush(void* stream);
int rod_slab_flush_range(const void* lo, const void* hi, void* stream);

/* ------------------------------------------------ data-parallel reduce point (ABI 16)
 * The exchange the reference's single-device optimizer step becomes under data parallelism
 * (net_tools.py:645-651: the gradient is summed over the ranks before the clip + SGD).  One
 * RCCL communicator per process (RCCL bound at run time: the process's already loaded
 * librccl.so.1 is reused).  rod_rccl_unique_id writes the 128-byte id rank 0 creates; the
 * caller distributes it (any rendezvous) and every rank calls rod_rccl_init with it.
 * rod_allreduce_bucket sums `count` elements (ROD_F32 / ROD_BF16; ABI 19: ROD_I32) in place
 * over all ranks, ordered on `stream` (capturable into a HIP graph).  rod_rccl_destroy frees
 * the communicator.
 * ABI 19 — every collective a captured data-parallel step holds goes through this
 * communicator, so no host-side watchdog ever polls a stream while it is being captured:
 * the gradient buckets (rod_allreduce_bucket on a side stream, overlapping backward), the
 * hard-negative counts / radix histograms (ROD_I32 sums; ref net_tools.py:557-587 selects
 * over the whole batch) and SyncBatchNorm's partial statistics: rod_allgather concatenates
 * every rank's `count` elements of `send` into `recv` ([world][count], rank order).
 * rod_rccl_world returns the communicator's rank count (0: none). */
int rod_rccl_unique_id(void* uid128);
int rod_rccl_init(int rank, int world, const void* uid128);
int rod_allreduce_bucket(void* ptr, long count, int dtype, void* stream);
int rod_allgather(const void* send, void* recv, long count, int dtype, void* stream);
int rod_rccl_world(void);
int rod_rccl_destroy(void);

#ifdef __cplusplus
}
#endif
#endif /* ROD_H_ */
