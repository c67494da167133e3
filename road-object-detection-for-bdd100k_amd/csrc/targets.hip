// targets.hip — anchor matching (JACCARD_BIGGER) and the masked smooth-L1 loss.
//
// Bit-exactness: this file is compiled with -ffp-contract=off (Makefile), so every
// expression below rounds after each operation exactly like the reference's chain of
// separate TF float32 ops; transcendental functions are correctly rounded (exp_cr/log_cr)
// and the oracle uses the same definition.
#include <math.h>

#include "rod_common.h"

namespace rod {

constexpr int MAXL = 8;
struct LevelInfo {
  int off[MAXL + 1];
  float thr[MAXL];
  int L;
};

// One workgroup per (anchor block, image).  The image's centre-form GT boxes are staged
// in LDS together with their corner form and area.
// NN = false: JACCARD_BIGGER (net_tools.py:382-421): argmax IoU, positive if >= the level's
// threshold.  NN = true: NEAREST_NEIGHBOR (net_tools.py:354-380): argmin over the boxes of
// sum(encode(anchor, box)^2) (tf.argmin, first minimum), every anchor positive.
template <bool NN>
__global__ void __launch_bounds__(256) match_anchors_kernel(const float* __restrict__ anc_corner,
                                                            const float* __restrict__ anc_center, LevelInfo li,
                                                            const float* __restrict__ gt, const int* __restrict__ gt_lbl,
                                                            const int* __restrict__ gt_n, float* __restrict__ out_off,
                                                            float* __restrict__ out_cbox, int* __restrict__ out_lbl,
                                                            int* __restrict__ out_pos, int A, int G) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* gc = sm;              // [G][4] corner after round trip
  float* gz = sm + 4 * G;      // [G][4] centre (cy, cx, h, w)
  float* gv = sm + 8 * G;      // [G] volume
  int* gl = (int*)(sm + 9 * G);  // [G] label
  __shared__ int poison[8];    // per-channel count of non-finite encodings (0..3 offsets, 4..7 centre)

  const int b = blockIdx.y;
  int n = gt_n[b];
  if (n > G) n = G;
  if (threadIdx.x < 8) poison[threadIdx.x] = 0;
  __syncthreads();
  for (int g = threadIdx.x; g < n; g += blockDim.x) {
    // center_bboxes[i] = (cy, cx, h, w) (train.py:109 already converted them)
    const float* p = gt + ((long)b * G + g) * 4;
    const float cy = p[0], cx = p[1], h = p[2], w = p[3];
    // centerBboxes_2_cornerBboxes (common_tools.py:30-33), used by jaccard (net_tools.py:323, 398)
    const float y0 = cy - h / 2.f, x0 = cx - w / 2.f, y1 = cy + h / 2.f, x1 = cx + w / 2.f;
    gc[g * 4 + 0] = y0; gc[g * 4 + 1] = x0; gc[g * 4 + 2] = y1; gc[g * 4 + 3] = x1;
    gz[g * 4 + 0] = cy; gz[g * 4 + 1] = cx; gz[g * 4 + 2] = h; gz[g * 4 + 3] = w;
    gv[g] = (y1 - y0) * (x1 - x0);  // jaccard: (ymax-ymin)*(xmax-xmin) of the gt (net_tools.py:265)
    gl[g] = gt_lbl[(long)b * G + g];
    // every box contributes mask*encode(box) to every anchor (net_tools.py:340-342): a
    // non-finite encoding turns 0*x into NaN for all anchors (kept for parity).
    if (!isfinite(cy)) atomicAdd(&poison[0], 1);
    if (!isfinite(cx)) atomicAdd(&poison[1], 1);
    if (!(h > 0.f) || isinf(h)) atomicAdd(&poison[2], 1);
    if (!(w > 0.f) || isinf(w)) atomicAdd(&poison[3], 1);
    if (!isfinite(cy)) atomicAdd(&poison[4], 1);
    if (!isfinite(cx)) atomicAdd(&poison[5], 1);
    if (!isfinite(h)) atomicAdd(&poison[6], 1);
    if (!isfinite(w)) atomicAdd(&poison[7], 1);
  }
  __syncthreads();

  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A) return;
  int lvl = 0;
#pragma unroll
  for (int l = 1; l < MAXL; ++l)
    if (l < li.L && a >= li.off[l]) lvl = l;

  const f32x4 ac = *(const f32x4*)(anc_corner + (long)a * 4);
  const float aymin = ac[0], axmin = ac[1], aymax = ac[2], axmax = ac[3];
  const float vol_a = (axmax - axmin) * (aymax - aymin);  // net_tools.py:254

  float best = 0.f;
  int idx = 0;
  if constexpr (NN) {
    const f32x4 az = *(const f32x4*)(anc_center + (long)a * 4);
    for (int g = 0; g < n; ++g) {
      const float o0 = (gz[g * 4 + 0] - az[0]) / az[2], o1 = (gz[g * 4 + 1] - az[1]) / az[3];
      const float o2 = log_cr(gz[g * 4 + 2] / az[2]), o3 = log_cr(gz[g * 4 + 3] / az[3]);
      // reduce_sum over the 4 offsets, in index order (parity unpinned vs Eigen's order)
      const float d = ((o0 * o0 + o1 * o1) + o2 * o2) + o3 * o3;
      if (g == 0 || d < best) {
        best = d;
        idx = g;
      }
    }
  } else {
  for (int g = 0; g < n; ++g) {
    const float iy0 = fmaxf(aymin, gc[g * 4 + 0]);
    const float ix0 = fmaxf(axmin, gc[g * 4 + 1]);
    const float iy1 = fminf(aymax, gc[g * 4 + 2]);
    const float ix1 = fminf(axmax, gc[g * 4 + 3]);
    const float hh = fmaxf(iy1 - iy0, 0.f);
    const float ww = fmaxf(ix1 - ix0, 0.f);
    const float inter = hh * ww;
    const float uni = vol_a - inter + gv[g];  // (vol_anchors - inter_vol) + vol_gt
    const float iou = inter / uni;
    if (g == 0 || iou > best) {  // tf.argmax: first maximal index wins
      best = iou;
      idx = g;
    }
  }
  }
  // tf.greater_equal (net_tools.py:406); NEAREST_NEIGHBOR: pos_mask = ones (net_tools.py:375)
  const bool pos = n > 0 && (NN || best >= li.thr[lvl]);

  const long o = (long)b * A + a;
  float off[4] = {0.f, 0.f, 0.f, 0.f}, cb[4] = {0.f, 0.f, 0.f, 0.f};
  int lab = 0;
  if (pos) {
    const f32x4 az = *(const f32x4*)(anc_center + (long)a * 4);
    const float cy = gz[idx * 4 + 0], cx = gz[idx * 4 + 1], h = gz[idx * 4 + 2], w = gz[idx * 4 + 3];
    off[0] = (cy - az[0]) / az[2];          // encode_locations_one_layer (net_tools.py:174-177)
    off[1] = (cx - az[1]) / az[3];
    off[2] = log_cr(h / az[2]);
    off[3] = log_cr(w / az[3]);
    cb[0] = cy; cb[1] = cx; cb[2] = h; cb[3] = w;
    lab = gl[idx];
  }
  // NaN poisoning of the masked sum (see above): with P poisoned boxes on a channel, the
  // anchor's sum is NaN unless its own matched box is the single poisoned one.
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int P = poison[c];
    if (P > 0) {
      const bool mine = pos && !isfinite(off[c]);
      if (!(mine && P == 1)) off[c] = __builtin_nanf("");
    }
    const int Q = poison[4 + c];
    if (Q > 0) {
      const bool mine = pos && !isfinite(cb[c]);
      if (!(mine && Q == 1)) cb[c] = __builtin_nanf("");
    }
  }
  f32x4 vo = {off[0], off[1], off[2], off[3]};
  f32x4 vc = {cb[0], cb[1], cb[2], cb[3]};
  *(f32x4*)(out_off + o * 4) = vo;
  *(f32x4*)(out_cbox + o * 4) = vc;
  out_lbl[o] = lab;
  out_pos[o] = pos ? 1 : 0;
}

// ---------------------------------------------------------------- smooth L1
// grid: x over (image, anchor-in-level) pairs of one level, y = level.
template <typename T>
__global__ void __launch_bounds__(256) smoothl1_kernel(const T* __restrict__ pred, const float* __restrict__ target,
                                                       const int* __restrict__ mask, LevelInfo li, float inv_scale,
                                                       T* __restrict__ grad, float* __restrict__ grad_t,
                                                       float* __restrict__ slab, int B, int A, int nbx) {
  __shared__ float red[4];
  const int l = blockIdx.y;
  const int Al = li.off[l + 1] - li.off[l];
  const long total = (long)B * Al;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float s = 0.f;
  if (t < total) {
    const int b = (int)(t / Al);
    const int a = li.off[l] + (int)(t - (long)b * Al);
    const long o = (long)b * A + a;
    const float m = (float)mask[o];
    float gv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float x = to_f32(pred[o * 4 + c]);
      const float d = (target[o * 4 + c] - x) * m;       // (y - x) * mask
      const float ad = fabsf(d);
      const float mn = fminf(ad, 1.f);
      s += 0.5f * ((ad - 1.f) * mn + ad);                // smooth_l1 (net_tools.py:486-489)
      gv[c] = -m * fminf(fmaxf(d, -1.f), 1.f) * inv_scale;  // d/dx of the above / scale
    }
    if (grad) {
#pragma unroll
      for (int c = 0; c < 4; ++c) grad[o * 4 + c] = from_f32<T>(gv[c]);
    }
    if (grad_t) {  // d/d target = -d/d pred (the ODM target depends on refine_out, 471)
#pragma unroll
      for (int c = 0; c < 4; ++c) grad_t[o * 4 + c] = -gv[c];
    }
  }
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) slab[(long)l * nbx + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void level_sum_finalize_kernel(const float* __restrict__ slab, int nbx, int L, float scale,
                                          float* __restrict__ out) {
  // one 256-thread block: strided partial sums per level, fixed-order tree in LDS
  __shared__ double red[MAXL][256];
  for (int l = 0; l < L; ++l) {
    double s = 0.0;
    for (int i = threadIdx.x; i < nbx; i += 256) s += (double)slab[(long)l * nbx + i];
    red[l][threadIdx.x] = s;
  }
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int l = 0; l < L; ++l) red[l][threadIdx.x] += red[l][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  float total = 0.f;  // refine_loss = 0.; refine_loss += layer_loss (net_tools.py:505-515)
  for (int l = 0; l < L; ++l) {
    out[l] = (float)red[l][0] / scale;  // reduce_sum(...) / bs
    total = total + out[l];
  }
  out[L] = total;
}

// ---------------------------------------------------------------- box conversions
// common_tools.py:16-35 / 38-56 on [..., 4] fp32 tensors
__global__ void boxes_convert_kernel(const float* __restrict__ in, float* __restrict__ out, long n, int to_center) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const f32x4 v = *(const f32x4*)(in + i * 4);
  f32x4 o;
  if (to_center) {  // [ymin,xmin,ymax,xmax] -> [cy,cx,h,w]
    o[0] = (v[0] + v[2]) / 2.f;
    o[1] = (v[1] + v[3]) / 2.f;
    o[2] = v[2] - v[0];
    o[3] = v[3] - v[1];
  } else {          // [cy,cx,h,w] -> [ymin,xmin,ymax,xmax]
    o[0] = v[0] - v[2] / 2.f;
    o[1] = v[1] - v[3] / 2.f;
    o[2] = v[0] + v[2] / 2.f;
    o[3] = v[1] + v[3] / 2.f;
  }
  *(f32x4*)(out + i * 4) = o;
}

// dst[r, c] = src[r, c] for a rows x cols block with independent row strides (bytes)
template <int WB>
__global__ void copy2d_kernel(const char* __restrict__ src, long sld, char* __restrict__ dst, long dld, long rows,
                              long chunks) {
  // flattened (row, chunk) grid-stride: efficient for many short rows (channel concat)
  const long total = rows * chunks;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / chunks, c = (i - r * chunks) * WB;
    if constexpr (WB == 16) *(f32x4*)(dst + r * dld + c) = *(const f32x4*)(src + r * sld + c);
    else if constexpr (WB == 4) *(float*)(dst + r * dld + c) = *(const float*)(src + r * sld + c);
    else dst[r * dld + c] = src[r * sld + c];
  }
}

static int fill_levels(LevelInfo& li, const int* lvl_off, const float* thr, int L, int A) {
  ROD_CHECK_ARG(L >= 1 && L <= MAXL, "levels: L=%d out of range [1,%d]", L, MAXL);
  li.L = L;
  for (int i = 0; i <= MAXL; ++i) li.off[i] = i <= L ? lvl_off[i] : A;
  for (int i = 0; i < MAXL; ++i) li.thr[i] = (thr && i < L) ? thr[i] : 0.f;
  ROD_CHECK_ARG(li.off[0] == 0 && li.off[L] == A, "levels: offsets must span [0, A]");
  for (int i = 0; i < L; ++i) ROD_CHECK_ARG(li.off[i] <= li.off[i + 1], "levels: offsets must be monotone");
  return 0;
}

}  // namespace rod

using namespace rod;

extern "C" {

int rod_match_anchors(const float* anc_corner, const float* anc_center, const int* lvl_off, const float* thr, int L,
                      const float* gt, const int* gt_lbl, const int* gt_n, float* out_off, float* out_cbox,
                      int* out_lbl, int* out_pos, int B, int A, int G, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0 && G > 0, "rod_match_anchors: bad shape B=%d A=%d G=%d", B, A, G);
  ROD_CHECK_ARG(G <= 4096, "rod_match_anchors: G=%d exceeds 4096", G);
  ROD_CHECK_ARG(lvl_off && thr, "rod_match_anchors: lvl_off/thr are host arrays and must be given");
  LevelInfo li;
  int e = fill_levels(li, lvl_off, thr, L, A);
  if (e) return e;
  size_t lds = (size_t)G * 10 * sizeof(float);
  hipLaunchKernelGGL(match_anchors_kernel<false>, dim3(cdiv(A, 256), B), dim3(256), lds, ROD_STREAM(stream),
                     anc_corner, anc_center, li, gt, gt_lbl, gt_n, out_off, out_cbox, out_lbl, out_pos, A, G);
  return check_launch("rod_match_anchors");
}

int rod_match_anchors_nn(const float* anc_corner, const float* anc_center, const int* lvl_off, int L, const float* gt,
                         const int* gt_lbl, const int* gt_n, float* out_off, float* out_cbox, int* out_lbl,
                         int* out_pos, int B, int A, int G, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0 && G > 0, "rod_match_anchors_nn: bad shape B=%d A=%d G=%d", B, A, G);
  ROD_CHECK_ARG(G <= 4096, "rod_match_anchors_nn: G=%d exceeds 4096", G);
  ROD_CHECK_ARG(lvl_off, "rod_match_anchors_nn: lvl_off is a host array and must be given");
  LevelInfo li;
  int e = fill_levels(li, lvl_off, nullptr, L, A);
  if (e) return e;
  size_t lds = (size_t)G * 10 * sizeof(float);
  hipLaunchKernelGGL(match_anchors_kernel<true>, dim3(cdiv(A, 256), B), dim3(256), lds, ROD_STREAM(stream),
                     anc_corner, anc_center, li, gt, gt_lbl, gt_n, out_off, out_cbox, out_lbl, out_pos, A, G);
  return check_launch("rod_match_anchors_nn");
}

static int smoothl1_nbx(int B, const LevelInfo& li) {
  long mx = 1;
  for (int l = 0; l < li.L; ++l) mx = std::max<long>(mx, (long)B * (li.off[l + 1] - li.off[l]));
  return cdiv(mx, 256);
}

size_t rod_smoothl1_workspace(int B, int A) {
  // at most A*B/256 + MAXL blocks per level, MAXL levels
  return (size_t)(cdivl((long)B * A, 256) + 1) * MAXL * sizeof(float);
}

int rod_smoothl1_masked(const void* pred, const float* target, const int* mask, const int* lvl_off, int L,
                        float scale, float* loss_lvl, void* grad, float* grad_target, void* workspace, int B, int A,
                        int dtype, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0, "rod_smoothl1_masked: bad shape");
  ROD_CHECK_ARG(scale != 0.f, "rod_smoothl1_masked: scale must be non-zero");
  ROD_CHECK_ARG(workspace && loss_lvl, "rod_smoothl1_masked: workspace/loss_lvl NULL");
  LevelInfo li;
  int e = fill_levels(li, lvl_off, nullptr, L, A);
  if (e) return e;
  const int nbx = smoothl1_nbx(B, li);
  const float inv = 1.0f / scale;
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, {
    hipLaunchKernelGGL(smoothl1_kernel<T>, dim3(nbx, L), dim3(256), 0, s, (const T*)pred, target, mask, li, inv,
                       (T*)grad, grad_target, (float*)workspace, B, A, nbx);
  });
  hipLaunchKernelGGL(level_sum_finalize_kernel, dim3(1), dim3(256), 0, s, (const float*)workspace, nbx, L, scale,
                     loss_lvl);
  return check_launch("rod_smoothl1_masked");
}

int rod_boxes_convert(const float* in, float* out, long n_boxes, int to_center, void* stream) {
  ROD_CHECK_ARG(n_boxes >= 0, "rod_boxes_convert: n < 0");
  ROD_CHECK_ARG((((uintptr_t)in | (uintptr_t)out) & 15) == 0, "rod_boxes_convert: buffers must be 16B aligned");
  if (n_boxes == 0) return 0;
  hipLaunchKernelGGL(boxes_convert_kernel, dim3(cdivl(n_boxes, 256)), dim3(256), 0, ROD_STREAM(stream), in, out,
                     n_boxes, to_center);
  return check_launch("rod_boxes_convert");
}

int rod_copy2d(const void* src, long src_ld_bytes, void* dst, long dst_ld_bytes, long rows, long cols_bytes,
               void* stream) {
  ROD_CHECK_ARG(rows >= 0 && cols_bytes >= 0, "rod_copy2d: bad extent");
  if (rows == 0 || cols_bytes == 0) return 0;
  const uintptr_t al = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)src_ld_bytes | (uintptr_t)dst_ld_bytes |
                       (uintptr_t)cols_bytes;
  hipStream_t s = ROD_STREAM(stream);
  const int wb = (al & 15) == 0 ? 16 : ((al & 3) == 0 ? 4 : 1);
  const long chunks = cols_bytes / wb;
  const int grid = (int)std::min<long>(cdivl(rows * chunks, 256), 8192);
  if (wb == 16)
    hipLaunchKernelGGL(copy2d_kernel<16>, dim3(grid), dim3(256), 0, s, (const char*)src, src_ld_bytes, (char*)dst,
                       dst_ld_bytes, rows, chunks);
  else if (wb == 4)
    hipLaunchKernelGGL(copy2d_kernel<4>, dim3(grid), dim3(256), 0, s, (const char*)src, src_ld_bytes, (char*)dst,
                       dst_ld_bytes, rows, chunks);
  else
    hipLaunchKernelGGL(copy2d_kernel<1>, dim3(grid), dim3(256), 0, s, (const char*)src, src_ld_bytes, (char*)dst,
                       dst_ld_bytes, rows, chunks);
  return check_launch("rod_copy2d");
}

}  // extern "C"
