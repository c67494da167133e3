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

#define ROD_ABI_VERSION 1
#define ROD_EINVAL (-1)

enum { ROD_F32 = 0, ROD_BF16 = 1 };
/* activation applied after BatchNorm:
 *   NONE  = identity (project conv, conv_blocks.py:294)
 *   RELU6 = tf.nn.relu6 (mobilenet_v2.py:47)
 *   LEAKY = tf.nn.leaky_relu, alpha 0.2 (catch_net.py:302) */
enum { ROD_ACT_NONE = 0, ROD_ACT_RELU6 = 1, ROD_ACT_LEAKY = 2 };

int rod_abi_version(void);
const char* rod_last_error(void);

/* ---------------------------------------------------------------- ingest */
/* out = (2/255)*img - 1 from uint8 pixels (train.py:126, predict.py:98). */
int rod_normalize_image(const void* img_u8, void* out, long n, int out_dtype, void* stream);
/* dst = src converted between storage dtypes (tf.cast). */
int rod_cast(const void* src, int src_dtype, void* dst, int dst_dtype, long n, void* stream);

/* --------------------------------------------------- depthwise 3x3 (A1)
 * slim.separable_conv2d(num_outputs=None, depth_multiplier=1), padding SAME
 * (conv_blocks.py:238-247): y[n,ho,wo,c] = sum_ij x[n,ho*s+i-pt,wo*s+j-pl,c]*w[i,j,c].
 * w is fp32 [3][3][C] (TF depthwise_weights [3,3,C,1]). */
int rod_dw3x3_fwd(const void* x, const float* w, void* y, int N, int H, int W, int C,
                  int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream);
/* dx = d y / d x  (DepthwiseConv2dNativeBackpropInput) */
int rod_dw3x3_bwd_data(const void* dy, const float* w, void* dx, int N, int H, int W, int C,
                       int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream);
/* dw[3][3][C] (fp32, overwritten) (DepthwiseConv2dNativeBackpropFilter).
 * workspace: rod_dw3x3_bwd_filter_workspace() bytes. */
size_t rod_dw3x3_bwd_filter_workspace(int N, int Ho, int Wo, int C);
int rod_dw3x3_bwd_filter(const void* x, const void* dy, float* dw, void* workspace,
                         int N, int H, int W, int C, int stride, int pad_t, int pad_l,
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
/* inference: mean = moving_mean, rstd = 1/sqrt(moving_var + eps). */
int rod_bn_eval_stats(const float* moving_mean, const float* moving_var, float eps,
                      float* mean, float* rstd, int C, void* stream);
/* y = act((x - mean)*rstd*gamma + beta) + residual   (gamma NULL => 1,
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

/* -------------------------------------- dense conv as implicit GEMM (A2 A3 A5)
 * y[m, co] = sum_k A[m, k] * wt[co, k] (+ bias[co]), fp32 accumulation,
 *   ksize 1: A = x rows [M = N*H*W, Cin] (slim.conv2d [1,1], conv_blocks.py:343)
 *   ksize 3: A = 3x3 im2col of x, stride 1, TF-SAME (pad 1/1), k = (i*3+j)*Cin + ci
 *            (stem mobilenet_v2.py:58; heads catch_net.py:303, 336)
 * wt: [Cout][ksize*ksize*Cin] in the activation dtype; bias fp32 or NULL.
 * ldx / ldy: row strides of x / y in elements (0 => Cin / Cout), so a conv can
 * read or write a channel slice of a concatenated buffer (catch_net.py:211). */
int rod_conv_fwd(const void* x, const void* wt, const float* bias, void* y, int N, int H,
                 int W, int Cin, int Cout, int ksize, int ldx, int ldy, int dtype, void* stream);
/* Weight layouts derived from the fp32 master weight w[Cout][ksize][ksize][Cin]:
 *   mode 0: forward operand      wt[co][i][j][ci]           (cast to dtype)
 *   mode 1: backward-data operand wt[ci][2-i][2-j][co]       (transposed, flipped)
 * so dx = rod_conv_fwd(dy, wt_mode1) (Conv2DBackpropInput, stride 1 SAME). */
int rod_conv_weight_prep(const float* w, void* wt, int Cout, int Cin, int ksize, int mode,
                         int dtype, void* stream);
/* dw[co][k] = sum_m dy[m, co] * A[m, k]  (Conv2DBackpropFilter), fp32 out,
 * db[co] = sum_m dy[m, co] when db != NULL.  workspace: see query. */
size_t rod_conv_wgrad_workspace(int N, int H, int W, int Cin, int Cout, int ksize);
int rod_conv_wgrad(const void* x, const void* dy, float* dw, float* db, void* workspace,
                   int N, int H, int W, int Cin, int Cout, int ksize, int ldx, int lddy,
                   int dtype, void* stream);

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
/* Masked smooth-L1 (net_tools.py:478-516): per-level sums of
 * smooth_l1((target - pred)*mask) / scale written to loss_lvl[0..L-1] and their
 * sum (accumulated in level order) to loss_lvl[L] (fp32, device, L+1 entries),
 * and grad = d(sum/scale)/d pred when grad != NULL.  pred [B,A,4] in dtype,
 * target fp32 [B,A,4], mask int [B,A]. */
size_t rod_smoothl1_workspace(int B, int A);
int rod_smoothl1_masked(const void* pred, const float* target, const int* mask,
                        const int* lvl_off, int L, float scale, float* loss_lvl, void* grad,
                        void* workspace, int B, int A, int dtype, void* stream);

/* Box conversions on [n,4] fp32 (utils/common_tools.py:16-56):
 * to_center=1: (ymin,xmin,ymax,xmax) -> (cy,cx,h,w); 0: the inverse. */
int rod_boxes_convert(const float* in, float* out, long n_boxes, int to_center, void* stream);
/* Strided block copy: rows x cols_bytes from src (row stride src_ld_bytes) to dst
 * (dst_ld_bytes); used for tf.concat of per-level tensors (net_tools.py:557-565). */
int rod_copy2d(const void* src, long src_ld_bytes, void* dst, long dst_ld_bytes, long rows, long cols_bytes,
               void* stream);

/* ------------------------------------------------ optimiser (A14)
 * Plain SGD with clip by value (net_tools.py:645-651):
 *   p -= lr * clamp(g, -clip, clip)   over one flat fp32 buffer. */
int rod_sgd_clip(float* param, const float* grad, long n, float lr, float clip, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ROD_H_ */
