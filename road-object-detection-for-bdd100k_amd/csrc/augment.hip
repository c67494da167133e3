// augment.hip — the training data pipeline on the GPU.
//
// process_raw_data_train (utils/data_pileline_tools.py:76-108), per image of a batch:
//   tf.slice(crop window)             process.py:126-127 (window from sample_distorted_bounding_box,
//                                     sampled on the host: parity-free random part)
//   resize_image BILINEAR, legacy     tf_image.py:266-278 (uint8 in, float out, src = dst * in/out)
//   random_flip_left_right            tf_image.py:281-305 (reverse_v2 along the width)
//   distort_color(fast_mode=False)    process.py:27-80: brightness / saturation / contrast in one of
//                                     four orders picked by apply_with_random_selector (process.py:8-24);
//                                     values stay on the 0-255 scale and are never clamped
//   (2/255) x - 1, cast to DTYPE      train.py:126-127 (optional, fused)
// and on the boxes: bboxes_resize (bboxes.py:139-163), bboxes_filter_overlap(0.3)
// (bboxes.py:408-428 with bboxes_intersection 482-508), flip [ymin, 1-xmax, ymax, 1-xmin]
// (tf_image.py:284-289), clip to [0, 1] (data_pileline_tools.py:106-107).
//
// The image side is three launches: per-block channel sums of the image as it enters
// adjust_contrast (f64), a per-image mean, then one fused pass (crop-resize-flip-colour-
// normalise) that writes the network input.  Each output pixel re-reads its four uint8 taps;
// the sources are small (2.7 MB per 720p frame) and stay in L2/MALL between the two passes.
// Compiled with -ffp-contract=off: every float expression rounds per operation like the TF ops.
#include <math.h>

#include "rod_common.h"

namespace rod {

namespace {

struct AugParams {
  const uint8_t* src;
  const int64_t* src_off;   // [B] byte offset of image b in src
  const int32_t* src_hw;    // [B, 2] source height, width (row stride = 3 * width)
  const int32_t* crop;      // [B, 4] y0, x0, h, w  (tf.slice begin / size)
  const int32_t* mode;      // [B, 2] flip (0/1), colour ordering (-1 none, 0..3)
  const float* colour;      // [B, 3] brightness delta, saturation factor, contrast factor
  int Ho, Wo;
};

struct Lerp1 {
  int lo, hi;
  float f;
};
// LegacyScaler (resize_bilinear_op.cc, align_corners=False): in = out * (in_size / out_size)
__device__ __forceinline__ Lerp1 lerp1(int o, float scale, int n_in) {
  const float in = (float)o * scale;
  const float fl = floorf(in);
  Lerp1 r;
  r.lo = max((int)fl, 0);
  r.hi = min((int)ceilf(in), n_in - 1);
  r.f = in - fl;
  return r;
}

// adjust_saturation (TF AdjustSaturationOp, CPU): RGB -> HSV, s = clamp(s * scale, 0, 1), HSV -> RGB.
__device__ __forceinline__ void saturate(float& r, float& g, float& b, float scale) {
  const float vv = fmaxf(r, fmaxf(g, b));
  const float range = vv - fminf(r, fminf(g, b));
  float s = vv > 0.0f ? range / vv : 0.0f;
  const float norm = 1.0f / (6.0f * range);
  float h;
  if (r == vv) {
    h = norm * (g - b);
  } else if (g == vv) {
    h = (float)((double)(norm * (b - r)) + 2.0 / 6.0);  // float + double literal, as in the TF kernel
  } else {
    h = (float)((double)(norm * (r - g)) + 4.0 / 6.0);
  }
  if (range <= 0.0f) h = 0.0f;
  if (h < 0.0f) h = h + 1.0f;
  s = fminf(1.0f, fmaxf(0.0f, s * scale));
  const float c = s * vv;
  const float m = vv - c;
  const float dh = h * 6.0f;
  const int cat = (int)dh;
  float fm = dh;
  while (fm <= 0.0f) fm += 2.0f;
  while (fm >= 2.0f) fm -= 2.0f;
  const float x = c * (1.0f - fabsf(fm - 1.0f));
  float rr, gg, bb;
  switch (cat) {
    case 0: rr = c; gg = x; bb = 0.0f; break;
    case 1: rr = x; gg = c; bb = 0.0f; break;
    case 2: rr = 0.0f; gg = c; bb = x; break;
    case 3: rr = 0.0f; gg = x; bb = c; break;
    case 4: rr = x; gg = 0.0f; bb = c; break;
    case 5: rr = c; gg = 0.0f; bb = x; break;
    default: rr = 0.0f; gg = 0.0f; bb = 0.0f;
  }
  r = rr + m;
  g = gg + m;
  b = bb + m;
}

// op codes of the colour chain: 0 brightness, 1 saturation, 2 contrast (process.py:56-77)
__device__ __forceinline__ int chain_op(int ordering, int k) {
  // ordering 0: B S C   1: S B C   2: C B S   3: S C B
  const int table = ordering == 0 ? 0x210 : ordering == 1 ? 0x201 : ordering == 2 ? 0x102 : 0x021;
  return (table >> (4 * k)) & 0xF;
}

// Per-image parameters, loaded once per block (uniform: scalar registers).
struct ImgCtx {
  const uint8_t* base;
  int y0, x0, h, w, sw, flip, ordering;
  float sy, sx, delta, sat, con;
  float mean[3];
};

__device__ __forceinline__ ImgCtx load_ctx(const AugParams& p, int b, const float* mean) {
  ImgCtx c;
  c.base = p.src + p.src_off[b];
  c.y0 = p.crop[4 * b];
  c.x0 = p.crop[4 * b + 1];
  c.h = p.crop[4 * b + 2];
  c.w = p.crop[4 * b + 3];
  c.sw = p.src_hw[2 * b + 1];
  c.flip = p.mode[2 * b];
  c.ordering = p.mode[2 * b + 1];
  c.sy = (float)c.h / (float)p.Ho;  // CalculateResizeScale: in_size / out_size
  c.sx = (float)c.w / (float)p.Wo;
  c.delta = p.colour[3 * b];
  c.sat = p.colour[3 * b + 1];
  c.con = p.colour[3 * b + 2];
  for (int i = 0; i < 3; ++i) c.mean[i] = mean ? mean[3 * b + i] : 0.0f;
  return c;
}

// The resized (and flipped) pixel at output (yo, xo), as 0-255 floats.
__device__ __forceinline__ void resized_pixel(const ImgCtx& c, int Wo, int yo, int xo, float* v) {
  if (c.flip) xo = Wo - 1 - xo;  // reverse_v2 of the resized image
  const Lerp1 ly = lerp1(yo, c.sy, c.h), lx = lerp1(xo, c.sx, c.w);
  const uint8_t* r0 = c.base + ((c.y0 + ly.lo) * c.sw + c.x0) * 3;
  const uint8_t* r1 = c.base + ((c.y0 + ly.hi) * c.sw + c.x0) * 3;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float tl = (float)r0[lx.lo * 3 + ch], tr = (float)r0[lx.hi * 3 + ch];
    const float bl = (float)r1[lx.lo * 3 + ch], br = (float)r1[lx.hi * 3 + ch];
    const float top = tl + (tr - tl) * lx.f;
    const float bot = bl + (br - bl) * lx.f;
    v[ch] = top + (bot - top) * ly.f;
  }
}

// Colour ops k in [k0, k1) of the chain (contrast uses c.mean).
__device__ __forceinline__ void colour_ops(const ImgCtx& c, int k0, int k1, float* v) {
  for (int k = k0; k < k1; ++k) {
    const int op = chain_op(c.ordering, k);
    if (op == 0) {
      v[0] = v[0] + c.delta;
      v[1] = v[1] + c.delta;
      v[2] = v[2] + c.delta;
    } else if (op == 1) {
      saturate(v[0], v[1], v[2], c.sat);
    } else {
      // adjust_contrast: (x - mean) * factor + mean, per channel
      v[0] = (v[0] - c.mean[0]) * c.con + c.mean[0];
      v[1] = (v[1] - c.mean[1]) * c.con + c.mean[1];
      v[2] = (v[2] - c.mean[2]) * c.con + c.mean[2];
    }
  }
}

__device__ __forceinline__ int contrast_pos(int ordering) {
  return ordering == 0 || ordering == 1 ? 2 : ordering == 2 ? 0 : 1;
}

// Pass 1: per-block channel sums (f64) of the image entering adjust_contrast.
// grid (nblk, B); block 256; partial [B][nblk][3].
__global__ void __launch_bounds__(256) aug_contrast_sums_kernel(AugParams p, double* partial, int nblk) {
  const int b = blockIdx.y;
  const ImgCtx c = load_ctx(p, b, nullptr);
  const int npix = p.Ho * p.Wo;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  if (c.ordering >= 0) {
    const int kc = contrast_pos(c.ordering);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < npix; i += nblk * 256) {
      float v[3];
      const int yo = i / p.Wo;
      resized_pixel(c, p.Wo, yo, i - yo * p.Wo, v);
      colour_ops(c, 0, kc, v);
      s0 += v[0];
      s1 += v[1];
      s2 += v[2];
    }
  }
  __shared__ double red[3][256];
  red[0][threadIdx.x] = s0;
  red[1][threadIdx.x] = s1;
  red[2][threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
      red[2][threadIdx.x] += red[2][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x < 3) partial[((long)b * nblk + blockIdx.x) * 3 + threadIdx.x] = red[threadIdx.x][0];
}

// Pass 2: per-image channel means (one block per image, fixed order).
__global__ void __launch_bounds__(256) aug_contrast_mean_kernel(const double* partial, float* mean, int nblk, long npix) {
  const int b = blockIdx.x;
  __shared__ double red[3][4];
  for (int c = 0; c < 3; ++c) {
    double s = 0.0;
    for (int k = threadIdx.x; k < nblk; k += 256) s += partial[((long)b * nblk + k) * 3 + c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[c][threadIdx.x >> 6] = s;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const double s = (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
    mean[3 * b + threadIdx.x] = (float)(s / (double)npix);
  }
}

// Pass 3: the fused image chain; grid (blocks, B); each thread writes 4 consecutive pixels
// (12 values, three 16-/8-byte stores when the image's pixel count is a multiple of 4).
template <typename T>
__global__ void __launch_bounds__(256) aug_apply_kernel(AugParams p, const float* mean, T* out, int normalize) {
  const int b = blockIdx.y;
  const ImgCtx c = load_ctx(p, b, mean);
  const int npix = p.Ho * p.Wo;
  const bool vec = (npix & 3) == 0;
  const float k = 2.0f / 255.0f;
  T* img = out + (long)b * npix * 3;
  for (int g = (blockIdx.x * 256 + threadIdx.x) * 4; g < npix; g += gridDim.x * 256 * 4) {
    float o[12];
    const int n = min(4, npix - g);
    int yo = g / p.Wo, xo = g - yo * p.Wo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < n) {
        float v[3];
        resized_pixel(c, p.Wo, yo, xo, v);
        if (c.ordering >= 0) colour_ops(c, 0, 3, v);
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) o[3 * j + ch] = normalize ? k * v[ch] - 1.0f : v[ch];
        if (++xo == p.Wo) {
          xo = 0;
          ++yo;
        }
      }
    }
    T* dst = img + (long)g * 3;
    if (vec && n == 4) {
      if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          f32x4 w = {o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
          *(f32x4*)(dst + 4 * q) = w;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          bf16x4 w = {(bf16_t)o[4 * q], (bf16_t)o[4 * q + 1], (bf16_t)o[4 * q + 2], (bf16_t)o[4 * q + 3]};
          *(bf16x4*)(dst + 4 * q) = w;
        }
      }
    } else {
      for (int j = 0; j < 3 * n; ++j) dst[j] = from_f32<T>(o[j]);
    }
  }
}

// Boxes: one wave per image, 64 boxes per iteration, ballot + popcount for the stable
// compaction of tf.boolean_mask.
__global__ void __launch_bounds__(64) aug_boxes_kernel(const float* __restrict__ boxes, const int32_t* __restrict__ labels,
                                                       const int32_t* __restrict__ n_in, const float* __restrict__ ref,
                                                       const int32_t* __restrict__ mode, float* __restrict__ boxes_out,
                                                       int32_t* __restrict__ labels_out, int32_t* __restrict__ n_out,
                                                       int G, float threshold) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = min(n_in[b], G);
  const float* r = ref + 4 * b;
  const int flip = mode ? mode[2 * b] : 0;
  int kept = 0;
  for (int base = 0; base < G; base += 64) {
    const int i = base + lane;
    bool keep = false;
    float y0 = 0.f, x0 = 0.f, y1 = 0.f, x1 = 0.f;
    int lab = 0;
    if (i < n) {
      const float* bx = boxes + ((long)b * G + i) * 4;
      // bboxes_resize: (box - [r0, r1, r0, r1]) / [r2 - r0, r3 - r1, r2 - r0, r3 - r1]
      const float sh = r[2] - r[0], sw = r[3] - r[1];
      y0 = (bx[0] - r[0]) / sh;
      x0 = (bx[1] - r[1]) / sw;
      y1 = (bx[2] - r[0]) / sh;
      x1 = (bx[3] - r[1]) / sw;
      // bboxes_intersection with [0, 0, 1, 1] and safe_divide
      const float iy0 = fmaxf(y0, 0.f), ix0 = fmaxf(x0, 0.f), iy1 = fminf(y1, 1.f), ix1 = fminf(x1, 1.f);
      const float h = fmaxf(iy1 - iy0, 0.f), w = fmaxf(ix1 - ix0, 0.f);
      const float inter = h * w;
      const float vol = (y1 - y0) * (x1 - x0);
      const float score = vol > 0.f ? inter / vol : 0.f;
      keep = score > threshold;
      lab = labels[(long)b * G + i];
      if (flip) {  // [ymin, 1 - xmax, ymax, 1 - xmin]
        const float nx0 = 1.f - x1, nx1 = 1.f - x0;
        x0 = nx0;
        x1 = nx1;
      }
      y0 = fminf(fmaxf(y0, 0.f), 1.f);  // tf.maximum(., 0) then tf.minimum(., 1)
      x0 = fminf(fmaxf(x0, 0.f), 1.f);
      y1 = fminf(fmaxf(y1, 0.f), 1.f);
      x1 = fminf(fmaxf(x1, 0.f), 1.f);
    }
    const unsigned long long m = __ballot(keep);
    if (keep) {
      const int dst = kept + __popcll(m & ((1ull << lane) - 1ull));
      float* o = boxes_out + ((long)b * G + dst) * 4;
      o[0] = y0;
      o[1] = x0;
      o[2] = y1;
      o[3] = x1;
      labels_out[(long)b * G + dst] = lab;
    }
    kept += __popcll(m);
  }
  for (int i = kept + lane; i < G; i += 64) {
    float* o = boxes_out + ((long)b * G + i) * 4;
    o[0] = o[1] = o[2] = o[3] = 0.f;
    labels_out[(long)b * G + i] = 0;
  }
  if (lane == 0) n_out[b] = kept;
}

int aug_blocks_per_image(long npix) { return (int)min((long)1024, max((long)1, npix / 1024)); }

}  // namespace
}  // namespace rod

using namespace rod;

extern "C" {

size_t rod_augment_workspace(int B, int Ho, int Wo) {
  if (B <= 0 || Ho <= 0 || Wo <= 0) return 0;
  const int nblk = aug_blocks_per_image((long)Ho * Wo);
  return ((size_t)B * nblk * 3 * sizeof(double) + 255) / 256 * 256 + (size_t)B * 3 * sizeof(float);
}

int rod_augment_images(const void* src, const int64_t* src_off, const int32_t* src_hw, const int32_t* crop,
                       const int32_t* mode, const float* colour, void* workspace, void* out, int B, int Ho, int Wo,
                       int normalize, int dtype, void* stream) {
  ROD_CHECK_ARG(B > 0 && B <= 65535 && Ho > 0 && Wo > 0 && (long)Ho * Wo < (1L << 29),
                "rod_augment_images: bad shape");
  ROD_CHECK_ARG(src && src_off && src_hw && crop && mode && colour && workspace && out,
                "rod_augment_images: null argument");
  ROD_CHECK_ARG(((uintptr_t)out & 15) == 0, "rod_augment_images: out must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  AugParams p{(const uint8_t*)src, src_off, src_hw, crop, mode, colour, Ho, Wo};
  const long npix = (long)Ho * Wo;
  const int nblk = aug_blocks_per_image(npix);
  double* partial = (double*)workspace;
  float* mean = (float*)((char*)workspace + ((size_t)B * nblk * 3 * sizeof(double) + 255) / 256 * 256);
  hipLaunchKernelGGL(aug_contrast_sums_kernel, dim3(nblk, B), dim3(256), 0, s, p, partial, nblk);
  hipLaunchKernelGGL(aug_contrast_mean_kernel, dim3(B), dim3(256), 0, s, partial, mean, nblk, npix);
  const int per_img = (int)min((long)4096, (npix / 4 + 255) / 256 + 1);
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(aug_apply_kernel<T>, dim3(per_img, B), dim3(256), 0, s, p, mean,
                                               (T*)out, normalize));
  return check_launch("rod_augment_images");
}

int rod_augment_boxes(const float* boxes, const int32_t* labels, const int32_t* n, const float* ref,
                      const int32_t* mode, float* boxes_out, int32_t* labels_out, int32_t* n_out, int B, int G,
                      float threshold, void* stream) {
  ROD_CHECK_ARG(B > 0 && G > 0, "rod_augment_boxes: bad shape");
  ROD_CHECK_ARG(boxes && labels && n && ref && boxes_out && labels_out && n_out, "rod_augment_boxes: null argument");
  ROD_CHECK_ARG(boxes != boxes_out && labels != labels_out, "rod_augment_boxes: in-place not supported");
  hipLaunchKernelGGL(aug_boxes_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, boxes, labels, n, ref, mode,
                     boxes_out, labels_out, n_out, G, threshold);
  return check_launch("rod_augment_boxes");
}

}  // extern "C"
