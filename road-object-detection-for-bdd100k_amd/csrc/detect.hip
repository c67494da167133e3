// detect.hip — deconvolution-pyramid helpers and the ODM (det) target path.
//
//   legacy bilinear resize   tf.image.resize_images(BILINEAR, align_corners=False), TF1
//                            scaling src = dst * (in/out) (catch_net.py:207; tf_image.py:275)
//   depth-to-space 2x2       conv2d_transpose(k=2, s=2, SAME) = 1x1 GEMM [M, i_c] x [i_c, 4 f_c]
//                            followed by this scatter (catch_net.py:196); cropping of odd outputs
//   add                      ADD merge (catch_net.py:269), refine_out + det_out (predict.py:132)
//   decode                   decode_locations_one_layer (net_tools.py:182-234) [+ centre->corner]
//   det targets              det_groundtruth (net_tools.py:431-475)
//   softmax                  slim.softmax over the class axis (predict.py:128)
// Compiled with -ffp-contract=off: each expression rounds per op like the TF op chain.
#include <math.h>

#include "rod_common.h"

namespace rod {

constexpr int MAXLV = 8;
struct Levels {
  int off[MAXLV + 1];
  float thr[MAXLV];
  int L;
};

// ---------------------------------------------------------------- legacy bilinear
struct Lerp {
  int lo, hi;
  float f;
};
__device__ __forceinline__ Lerp legacy_lerp(int o, float scale, int n_in) {
  const float in = (float)o * scale;  // LegacyScaler: out * scale, no half-pixel offset
  const float fl = floorf(in);
  Lerp r;
  r.lo = max((int)fl, 0);
  r.hi = min((int)ceilf(in), n_in - 1);
  r.f = in - fl;
  return r;
}

template <typename T>
__global__ void resize_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int Ho,
                                  int Wo, float sy, float sx) {
  const long total = (long)N * Ho * Wo * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int xo = (int)(t % Wo);
    t /= Wo;
    const int yo = (int)(t % Ho);
    const int n = (int)(t / Ho);
    const Lerp ly = legacy_lerp(yo, sy, H), lx = legacy_lerp(xo, sx, W);
    const T* b = x + (long)n * H * W * C + c;
    const float tl = to_f32(b[((long)ly.lo * W + lx.lo) * C]);
    const float tr = to_f32(b[((long)ly.lo * W + lx.hi) * C]);
    const float bl = to_f32(b[((long)ly.hi * W + lx.lo) * C]);
    const float br = to_f32(b[((long)ly.hi * W + lx.hi) * C]);
    const float top = tl + (tr - tl) * lx.f;  // compute_lerp (resize_bilinear_op.cc)
    const float bot = bl + (br - bl) * lx.f;
    y[i] = from_f32<T>(top + (bot - top) * ly.f);
  }
}

// ResizeBilinearGrad as a gather: every input pixel sums the weights of the output pixels
// whose lo/hi taps land on it (deterministic; no atomics).
template <typename T>
__global__ void resize_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                  int Wo, float sy, float sx) {
  const long total = (long)N * H * W * C;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long t = i / C;
    const int xi = (int)(t % W);
    t /= W;
    const int yi = (int)(t % H);
    const int n = (int)(t / H);
    // output rows whose taps can touch yi: in = yo*sy in (yi-1, yi+1]
    const int y_lo = max(0, (int)floorf((float)(yi - 1) / sy) - 1);
    const int y_hi = min(Ho - 1, (int)ceilf((float)(yi + 1) / sy) + 1);
    const int x_lo = max(0, (int)floorf((float)(xi - 1) / sx) - 1);
    const int x_hi = min(Wo - 1, (int)ceilf((float)(xi + 1) / sx) + 1);
    float acc = 0.f;
    for (int yo = y_lo; yo <= y_hi; ++yo) {
      const Lerp ly = legacy_lerp(yo, sy, H);
      float wy = 0.f;
      if (ly.lo == yi) wy += 1.f - ly.f;
      if (ly.hi == yi) wy += ly.f;
      if (wy == 0.f) continue;
      for (int xo = x_lo; xo <= x_hi; ++xo) {
        const Lerp lx = legacy_lerp(xo, sx, W);
        float wx = 0.f;
        if (lx.lo == xi) wx += 1.f - lx.f;
        if (lx.hi == xi) wx += lx.f;
        if (wx == 0.f) continue;
        acc = fmaf(to_f32(dy[(((long)n * Ho + yo) * Wo + xo) * C + c]), wy * wx, acc);
      }
    }
    dx[i] = from_f32<T>(acc);
  }
}

// ---------------------------------------------------------------- deconv scatter / gather
// out[n, 2i+a, 2j+b, f] = z[n, i, j, (a*2+b)*F + f]   (rows/cols beyond Ho/Wo cropped)
template <typename T>
__global__ void d2s_kernel(const T* __restrict__ z, T* __restrict__ out, int N, int h, int w, int F, int Ho, int Wo,
                           int ldo) {
  const long total = (long)N * Ho * Wo * F;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int f = (int)(i % F);
    long t = i / F;
    const int xo = (int)(t % Wo);
    t /= Wo;
    const int yo = (int)(t % Ho);
    const int n = (int)(t / Ho);
    const int a = yo & 1, b = xo & 1;
    out[(((long)n * Ho + yo) * Wo + xo) * ldo + f] =
        z[(((long)n * h + (yo >> 1)) * w + (xo >> 1)) * 4 * F + (a * 2 + b) * F + f];
  }
}

template <typename T>
__global__ void s2d_kernel(const T* __restrict__ dout, T* __restrict__ dz, int N, int h, int w, int F, int Ho, int Wo,
                           int ldo) {
  const long total = (long)N * h * w * 4 * F;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int q = (int)(i % (4 * F));
    long t = i / (4 * F);
    const int j = (int)(t % w);
    t /= w;
    const int ii = (int)(t % h);
    const int n = (int)(t / h);
    const int ab = q / F, f = q - ab * F;
    const int yo = 2 * ii + (ab >> 1), xo = 2 * j + (ab & 1);
    dz[i] = (yo < Ho && xo < Wo) ? dout[(((long)n * Ho + yo) * Wo + xo) * ldo + f] : (T)0.f;
  }
}

template <typename T>
__global__ void add_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ c, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    c[i] = from_f32<T>(to_f32(a[i]) + to_f32(b[i]));
}

// ---------------------------------------------------------------- decode
// out = decode(anchor, a (+ b)), centre form or corner form, fp32 [B, A, 4]
template <typename T>
__global__ void decode_kernel(const float* __restrict__ anc_center, const T* __restrict__ oa,
                              const T* __restrict__ ob, float* __restrict__ out, long BA, int A, int to_corner) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < BA; i += (long)gridDim.x * blockDim.x) {
    const int a = (int)(i % A);
    const f32x4 az = *(const f32x4*)(anc_center + (long)a * 4);
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = to_f32(oa[i * 4 + k]);
      if (ob) o[k] = o[k] + to_f32(ob[i * 4 + k]);  // refine_out + det_out (predict.py:132)
    }
    const float cy = o[0] * az[2] + az[0];   // bboxes_cy = off * anchor_h + anchor_cy
    const float cx = o[1] * az[3] + az[1];
    const float h = exp_cr(o[2]) * az[2];
    const float w = exp_cr(o[3]) * az[3];
    f32x4 r;
    if (to_corner) {  // centerBboxes_2_cornerBboxes (common_tools.py:30-33)
      r[0] = cy - h / 2.f;
      r[1] = cx - w / 2.f;
      r[2] = cy + h / 2.f;
      r[3] = cx + w / 2.f;
    } else {
      r[0] = cy; r[1] = cx; r[2] = h; r[3] = w;
    }
    *(f32x4*)(out + i * 4) = r;
  }
}

// ---------------------------------------------------------------- det targets
template <typename T>
__global__ void det_targets_kernel(const float* __restrict__ anc_center, const T* __restrict__ refine_out,
                                   const float* __restrict__ refine_gt, const float* __restrict__ cbox,
                                   const int* __restrict__ label, const int* __restrict__ refine_pos, Levels lv,
                                   float* __restrict__ det_gt, int* __restrict__ det_pos, int* __restrict__ det_lbl,
                                   float* __restrict__ iou_out, long BA, int A) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < BA; i += (long)gridDim.x * blockDim.x) {
    const int a = (int)(i % A);
    int l = 0;
#pragma unroll
    for (int k = 1; k < MAXLV; ++k)
      if (k < lv.L && a >= lv.off[k]) l = k;
    const f32x4 az = *(const f32x4*)(anc_center + (long)a * 4);
    float ro[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ro[k] = to_f32(refine_out[i * 4 + k]);
    // adjusted anchor = corner(decode(anchor, refine_out))   (net_tools.py:459-460)
    const float cy = ro[0] * az[2] + az[0], cx = ro[1] * az[3] + az[1];
    const float h = exp_cr(ro[2]) * az[2], w = exp_cr(ro[3]) * az[3];
    const float ay0 = cy - h / 2.f, ax0 = cx - w / 2.f, ay1 = cy + h / 2.f, ax1 = cx + w / 2.f;
    // gt corner (net_tools.py:463)
    const f32x4 gz = *(const f32x4*)(cbox + i * 4);
    const float gy0 = gz[0] - gz[2] / 2.f, gx0 = gz[1] - gz[3] / 2.f;
    const float gy1 = gz[0] + gz[2] / 2.f, gx1 = gz[1] + gz[3] / 2.f;
    // jaccard (net_tools.py:254-266)
    const float vol_a = (ax1 - ax0) * (ay1 - ay0);
    const float ih = fmaxf(fminf(ay1, gy1) - fmaxf(ay0, gy0), 0.f);
    const float iw = fmaxf(fminf(ax1, gx1) - fmaxf(ax0, gx0), 0.f);
    const float inter = ih * iw;
    const float uni = vol_a - inter + (gy1 - gy0) * (gx1 - gx0);
    const float iou = inter / uni;
    const int pos = (iou >= lv.thr[l] ? 1 : 0) * refine_pos[i];  // net_tools.py:468-469
    const float pm = (float)pos;
    const f32x4 rg = *(const f32x4*)(refine_gt + i * 4);
    f32x4 dg;
#pragma unroll
    for (int k = 0; k < 4; ++k) dg[k] = (rg[k] - ro[k]) * pm;  // (offset_gt - refine_out) * mask
    *(f32x4*)(det_gt + i * 4) = dg;
    det_pos[i] = pos;
    det_lbl[i] = label[i] * pos;
    iou_out[i] = iou;
  }
}

// Backward of det_targets wrt refine_out (train.py fix_refine=False; no stop-gradient in the
// reference): det_gt = (refine_gt - refine_out)*pos (net_tools.py:471) gives -g_det_gt*pos;
// iou = jaccard(corner(decode(anchor, refine_out)), corner(cbox)) (459-465) gives the chain
// below with TF's gradient rules (maximum -> the first argument when x >= y, minimum -> when
// x <= y, max(., 0) passes at >= 0).  The forward is recomputed with det_targets_kernel's
// exact operations.
template <typename T>
__global__ void det_targets_bwd_kernel(const float* __restrict__ anc_center, const T* __restrict__ refine_out,
                                       const float* __restrict__ cbox, const int* __restrict__ det_pos,
                                       const float* __restrict__ g_det_gt, const float* __restrict__ g_iou,
                                       T* __restrict__ g_ro, long BA, int A) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < BA; i += (long)gridDim.x * blockDim.x) {
    const int a = (int)(i % A);
    const f32x4 az = *(const f32x4*)(anc_center + (long)a * 4);
    float ro[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ro[k] = to_f32(refine_out[i * 4 + k]);
    const float cy = ro[0] * az[2] + az[0], cx = ro[1] * az[3] + az[1];
    const float h = exp_cr(ro[2]) * az[2], w = exp_cr(ro[3]) * az[3];
    const float ay0 = cy - h / 2.f, ax0 = cx - w / 2.f, ay1 = cy + h / 2.f, ax1 = cx + w / 2.f;
    const f32x4 gz = *(const f32x4*)(cbox + i * 4);
    const float gy0 = gz[0] - gz[2] / 2.f, gx0 = gz[1] - gz[3] / 2.f;
    const float gy1 = gz[0] + gz[2] / 2.f, gx1 = gz[1] + gz[3] / 2.f;
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    const float G = g_iou ? g_iou[i] : 0.f;
    if (G != 0.f) {
      const float vol_a = (ax1 - ax0) * (ay1 - ay0);
      const float ihr = fminf(ay1, gy1) - fmaxf(ay0, gy0);
      const float iwr = fminf(ax1, gx1) - fmaxf(ax0, gx0);
      const float ih = fmaxf(ihr, 0.f), iw = fmaxf(iwr, 0.f);
      const float inter = ih * iw;
      const float uni = vol_a - inter + (gy1 - gy0) * (gx1 - gx0);
      const float q = G * inter / (uni * uni);
      const float d_inter = G / uni + q;  // d iou/d inter, with union = vol_a - inter + vol_g
      const float d_vol = -q;
      const float d_ih = ihr >= 0.f ? d_inter * iw : 0.f;
      const float d_iw = iwr >= 0.f ? d_inter * ih : 0.f;
      float d_ay1 = ay1 <= gy1 ? d_ih : 0.f, d_ay0 = ay0 >= gy0 ? -d_ih : 0.f;
      float d_ax1 = ax1 <= gx1 ? d_iw : 0.f, d_ax0 = ax0 >= gx0 ? -d_iw : 0.f;
      d_ax1 += d_vol * (ay1 - ay0);
      d_ax0 -= d_vol * (ay1 - ay0);
      d_ay1 += d_vol * (ax1 - ax0);
      d_ay0 -= d_vol * (ax1 - ax0);
      const float d_cy = d_ay0 + d_ay1, d_h = (d_ay1 - d_ay0) / 2.f;
      const float d_cx = d_ax0 + d_ax1, d_w = (d_ax1 - d_ax0) / 2.f;
      g[0] = d_cy * az[2];
      g[1] = d_cx * az[3];
      g[2] = d_h * h;
      g[3] = d_w * w;
    }
    if (g_det_gt) {
      const float pm = (float)det_pos[i];
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] -= g_det_gt[i * 4 + k] * pm;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) g_ro[i * 4 + k] = from_f32<T>(g[k]);
  }
}

// ---------------------------------------------------------------- softmax over K classes
template <typename T>
__global__ void softmax_kernel(const T* __restrict__ logits, float* __restrict__ probs, long rows, int K) {
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (long)gridDim.x * blockDim.x) {
    const T* x = logits + r * K;
    float m = to_f32(x[0]);
    for (int k = 1; k < K; ++k) m = fmaxf(m, to_f32(x[k]));
    float e[16];
    float s = 0.f;
    for (int k = 0; k < K; ++k) {
      e[k] = exp_cr(to_f32(x[k]) - m);
      s += e[k];
    }
    for (int k = 0; k < K; ++k) probs[r * K + k] = e[k] / s;
  }
}

static int ew_grid(long n) { return (int)std::min<long>(cdivl(n, 256), 8192); }

static int fill_lv(Levels& lv, const int* off, const float* thr, int L, int A) {
  ROD_CHECK_ARG(L >= 1 && L <= MAXLV, "levels: L=%d out of range", L);
  lv.L = L;
  for (int i = 0; i <= MAXLV; ++i) lv.off[i] = i <= L ? off[i] : A;
  for (int i = 0; i < MAXLV; ++i) lv.thr[i] = (thr && i < L) ? thr[i] : 0.f;
  ROD_CHECK_ARG(lv.off[0] == 0 && lv.off[L] == A, "levels: offsets must span [0, A]");
  return 0;
}

}  // namespace rod

using namespace rod;

extern "C" {

int rod_resize_bilinear(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo, int dtype,
                        void* stream) {
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && Ho > 0 && Wo > 0, "rod_resize_bilinear: bad shape");
  const float sy = (float)H / (float)Ho, sx = (float)W / (float)Wo;  // CalculateResizeScale, no align_corners
  const long n = (long)N * Ho * Wo * C;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(resize_fwd_kernel<T>, dim3(ew_grid(n)), dim3(256), 0,
                                               ROD_STREAM(stream), (const T*)x, (T*)y, N, H, W, C, Ho, Wo, sy, sx));
  return check_launch("rod_resize_bilinear");
}

int rod_resize_bilinear_bwd(const void* dy, void* dx, int N, int H, int W, int C, int Ho, int Wo, int dtype,
                            void* stream) {
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && Ho > 0 && Wo > 0, "rod_resize_bilinear_bwd: bad shape");
  const float sy = (float)H / (float)Ho, sx = (float)W / (float)Wo;
  const long n = (long)N * H * W * C;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(resize_bwd_kernel<T>, dim3(ew_grid(n)), dim3(256), 0,
                                               ROD_STREAM(stream), (const T*)dy, (T*)dx, N, H, W, C, Ho, Wo, sy, sx));
  return check_launch("rod_resize_bilinear_bwd");
}

int rod_depth_to_space2(const void* z, void* out, int N, int h, int w, int F, int Ho, int Wo, int ldo, int dtype,
                        void* stream) {
  ROD_CHECK_ARG(N > 0 && h > 0 && w > 0 && F > 0, "rod_depth_to_space2: bad shape");
  ROD_CHECK_ARG(Ho <= 2 * h && Wo <= 2 * w && Ho > 2 * h - 2 && Wo > 2 * w - 2, "rod_depth_to_space2: bad crop");
  if (ldo == 0) ldo = F;
  const long n = (long)N * Ho * Wo * F;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(d2s_kernel<T>, dim3(ew_grid(n)), dim3(256), 0, ROD_STREAM(stream),
                                               (const T*)z, (T*)out, N, h, w, F, Ho, Wo, ldo));
  return check_launch("rod_depth_to_space2");
}

int rod_space_to_depth2(const void* dout, void* dz, int N, int h, int w, int F, int Ho, int Wo, int ldo, int dtype,
                        void* stream) {
  ROD_CHECK_ARG(N > 0 && h > 0 && w > 0 && F > 0, "rod_space_to_depth2: bad shape");
  ROD_CHECK_ARG(Ho <= 2 * h && Wo <= 2 * w, "rod_space_to_depth2: bad crop");
  if (ldo == 0) ldo = F;
  const long n = (long)N * h * w * 4 * F;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(s2d_kernel<T>, dim3(ew_grid(n)), dim3(256), 0, ROD_STREAM(stream),
                                               (const T*)dout, (T*)dz, N, h, w, F, Ho, Wo, ldo));
  return check_launch("rod_space_to_depth2");
}

int rod_add(const void* a, const void* b, void* c, long n, int dtype, void* stream) {
  ROD_CHECK_ARG(n >= 0, "rod_add: n < 0");
  if (n == 0) return 0;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(add_kernel<T>, dim3(ew_grid(n)), dim3(256), 0, ROD_STREAM(stream),
                                               (const T*)a, (const T*)b, (T*)c, n));
  return check_launch("rod_add");
}

int rod_decode(const float* anc_center, const void* off_a, const void* off_b, float* out, int B, int A, int to_corner,
               int dtype, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0, "rod_decode: bad shape");
  const long BA = (long)B * A;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(decode_kernel<T>, dim3(ew_grid(BA)), dim3(256), 0,
                                               ROD_STREAM(stream), anc_center, (const T*)off_a, (const T*)off_b, out,
                                               BA, A, to_corner));
  return check_launch("rod_decode");
}

int rod_det_targets(const float* anc_center, const void* refine_out, const float* refine_gt, const float* cbox,
                    const int* label, const int* refine_pos, const int* lvl_off, const float* thr, int L,
                    float* det_gt, int* det_pos, int* det_lbl, float* iou, int B, int A, int dtype, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0, "rod_det_targets: bad shape");
  ROD_CHECK_ARG(lvl_off && thr, "rod_det_targets: lvl_off/thr host arrays required");
  Levels lv;
  int e = fill_lv(lv, lvl_off, thr, L, A);
  if (e) return e;
  const long BA = (long)B * A;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(det_targets_kernel<T>, dim3(ew_grid(BA)), dim3(256), 0,
                                               ROD_STREAM(stream), anc_center, (const T*)refine_out, refine_gt, cbox,
                                               label, refine_pos, lv, det_gt, det_pos, det_lbl, iou, BA, A));
  return check_launch("rod_det_targets");
}

int rod_det_targets_bwd(const float* anc_center, const void* refine_out, const float* cbox, const int* det_pos,
                        const float* g_det_gt, const float* g_iou, void* g_refine_out, int B, int A, int dtype,
                        void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0 && g_refine_out, "rod_det_targets_bwd: bad arguments");
  const long BA = (long)B * A;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(det_targets_bwd_kernel<T>, dim3(ew_grid(BA)), dim3(256), 0,
                                               ROD_STREAM(stream), anc_center, (const T*)refine_out, cbox, det_pos,
                                               g_det_gt, g_iou, (T*)g_refine_out, BA, A));
  return check_launch("rod_det_targets_bwd");
}

int rod_softmax(const void* logits, float* probs, long rows, int K, int dtype, void* stream) {
  ROD_CHECK_ARG(rows >= 0 && K > 0 && K <= 16, "rod_softmax: bad shape (K <= 16)");
  if (rows == 0) return 0;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(softmax_kernel<T>, dim3(ew_grid(rows)), dim3(256), 0,
                                               ROD_STREAM(stream), (const T*)logits, probs, rows, K));
  return check_launch("rod_softmax");
}

}  // extern "C"
