// loss.hip — det_clf_loss classification part with global hard-negative mining
// (reference utils/net_tools.py:551-615), entirely on the device (no host sync):
//
//   p = softmax(logits) per row; nvalue = p[0] on negatives, 1 on positives      (571-575)
//   k = min(int32(3 * n_pos) + B, n_neg)                                          (578-581)
//   thr = k-th smallest nvalue  (exact 4 x 8-bit radix select on the f32 bits)   (583-584)
//   negatives kept: neg && nvalue < thr  (strict)                                  (587)
//   iou factor per (image, level): ((iou-mean)/sqrt(var+1e-8) - min) / (max+1e-8), ^4 (590-600)
//   pos_loss = sum CE(label) * pos * iouf / bs;  neg_loss = sum CE(0) * negmask / bs (605-613)
//   clf_loss = neg_loss / 2 + pos_loss                                             (615)
// plus d clf_loss / d logits.  Row layout: [B, A] anchors (levels concatenated per image).
#include <math.h>

#include "rod_common.h"

namespace rod {

constexpr int HNM_MAXL = 8;
constexpr int HNM_K = 16;  // max classes
struct HnmLevels {
  int off[HNM_MAXL + 1];
  int L;
};

// state words (int): [0] k  [1] prefix bits  [2] remaining rank  [3] n_pos  [4] n_neg  [5] n_neg_sel
// float outputs (8): pos_loss, neg_loss, clf_loss, max_hard_pred, n_pos, k, n_neg_selected, 0
struct HnmWs {
  float* nval;       // [R]
  float* gstat;      // [B*L][4]: mean, sd, zmin, den
  unsigned* hist;    // [256]
  int* state;        // [8]
  int* cnt_slab;     // [nb][2]
  double* loss_slab; // [nb][3]
};

template <typename T>
__device__ __forceinline__ void row_softmax(const T* __restrict__ x, int K, float* e, float& m, float& s) {
  m = to_f32(x[0]);
  for (int k = 1; k < K; ++k) m = fmaxf(m, to_f32(x[k]));
  s = 0.f;
  for (int k = 0; k < K; ++k) {
    e[k] = exp_cr(to_f32(x[k]) - m);
    s += e[k];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) hnm_rows_kernel(const T* __restrict__ logits, const int* __restrict__ pos,
                                                       long R, int K, float* __restrict__ nval,
                                                       int* __restrict__ cnt_slab) {
  __shared__ int red[2][4];
  int np = 0, nn = 0;
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (long)gridDim.x * blockDim.x) {
    float e[HNM_K], m, s;
    row_softmax(logits + r * K, K, e, m, s);
    const bool p = pos[r] != 0;
    nval[r] = p ? 1.f : e[0] / s;  // tf.where(nmask, predictions[:, 0], 1. - fnmask)
    np += p ? 1 : 0;
    nn += p ? 0 : 1;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    np += __shfl_xor(np, o, 64);
    nn += __shfl_xor(nn, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = np;
    red[1][threadIdx.x >> 6] = nn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    cnt_slab[blockIdx.x * 2 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    cnt_slab[blockIdx.x * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ void hnm_count_kernel(const int* __restrict__ cnt_slab, int nb, int B, int* __restrict__ state,
                                 unsigned* __restrict__ hist) {
  __shared__ int s[2][256];
  int np = 0, nn = 0;
  for (int i = threadIdx.x; i < nb; i += 256) {
    np += cnt_slab[2 * i];
    nn += cnt_slab[2 * i + 1];
  }
  s[0][threadIdx.x] = np;
  s[1][threadIdx.x] = nn;
  hist[threadIdx.x] = 0u;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      s[0][threadIdx.x] += s[0][threadIdx.x + w];
      s[1][threadIdx.x] += s[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float n_pos = (float)s[0][0];
    int k = (int)(3.0f * n_pos) + B;          // tf.cast(negative_ratio * n_positives, tf.int32) + bs
    k = min(k, s[1][0]);                       // tf.minimum(n_neg, max_neg_entries)
    state[0] = k;
    state[1] = 0;                              // prefix
    state[2] = k;                              // rank (1-based) still to locate
    state[3] = s[0][0];
    state[4] = s[1][0];
  }
}

// histogram of digit `shift` among values whose higher digits equal the prefix
__global__ void __launch_bounds__(256) radix_hist_kernel(const float* __restrict__ v, long R, int shift,
                                                         const int* __restrict__ state, unsigned* __restrict__ hist) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const unsigned prefix = (unsigned)state[1];
  const unsigned hmask = shift >= 24 ? 0u : (0xFFFFFFFFu << (shift + 8));
  if (state[0] > 0) {
    for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (long)gridDim.x * blockDim.x) {
      const unsigned b = __float_as_uint(v[r]);
      if ((b & hmask) == (prefix & hmask)) atomicAdd(&h[(b >> shift) & 255u], 1u);
    }
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// pick the bucket holding the remaining rank; fix the digit; clear the histogram
__global__ void radix_scan_kernel(int shift, int* __restrict__ state, unsigned* __restrict__ hist) {
  if (threadIdx.x == 0 && state[0] > 0) {
    unsigned rank = (unsigned)state[2];
    unsigned acc = 0;
    int d = 0;
    for (; d < 256; ++d) {
      if (acc + hist[d] >= rank) break;
      acc += hist[d];
    }
    if (d > 255) d = 255;
    state[1] = (int)((unsigned)state[1] | ((unsigned)d << shift));
    state[2] = (int)(rank - acc);
  }
  __syncthreads();
  hist[threadIdx.x] = 0u;
}

// per (image, level) group: mean, sd = sqrt(var + 1e-8), zmin, den = max(z') + 1e-8
__global__ void __launch_bounds__(256) iou_group_kernel(const float* __restrict__ iou, HnmLevels lv, int A,
                                                        float* __restrict__ gstat) {
  __shared__ double sd[256];
  __shared__ float smin[256], smax[256];
  const int g = blockIdx.x;
  const int b = g / lv.L, l = g - b * lv.L;
  const long r0 = (long)b * A + lv.off[l];
  const int n = lv.off[l + 1] - lv.off[l];
  double s = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float u = iou[r0 + i];
    s += (double)u;
    mn = fminf(mn, u);
    mx = fmaxf(mx, u);
  }
  sd[threadIdx.x] = s;
  smin[threadIdx.x] = mn;
  smax[threadIdx.x] = mx;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sd[threadIdx.x] += sd[threadIdx.x + w];
      smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + w]);
      smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + w]);
    }
    __syncthreads();
  }
  const float mean = (float)(sd[0] / (double)n);  // tf.nn.moments mean
  const float umin = smin[0], umax = smax[0];
  __syncthreads();
  double v = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float d = iou[r0 + i] - mean;
    v += (double)(d * d);                          // squared_difference(x, mean)
  }
  sd[threadIdx.x] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sd[threadIdx.x] += sd[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float var = (float)(sd[0] / (double)n);
    const float sdev = sqrtf(var + 1e-8f);
    const float zmin = (umin - mean) / sdev;       // reduce_min of the standardised values
    const float zmax = (umax - mean) / sdev + (0.f - zmin);
    gstat[g * 4 + 0] = mean;
    gstat[g * 4 + 1] = sdev;
    gstat[g * 4 + 2] = zmin;
    gstat[g * 4 + 3] = zmax + 1e-8f;
  }
}

__device__ __forceinline__ float iou_factor(float u, const float* gs) {
  const float z = (u - gs[0]) / gs[1];
  const float zz = z + (0.f - gs[2]);  // iou += 0. - reduce_min(iou)
  const float w = zz / gs[3];          // iou /= reduce_max(iou) + 1e-8
  return powf(w, 4.f);                 // tf.pow(iou, 4)
}

template <typename T>
__global__ void __launch_bounds__(256) hnm_loss_kernel(const T* __restrict__ logits, const int* __restrict__ lbl,
                                                       const int* __restrict__ pos, const float* __restrict__ iou,
                                                       const float* __restrict__ nval, const float* __restrict__ gstat,
                                                       const int* __restrict__ state, HnmLevels lv, long R, int A,
                                                       int K, float inv_bs, T* __restrict__ grad,
                                                       double* __restrict__ slab) {
  __shared__ double red[3][4];
  const float thr = state[0] > 0 ? __uint_as_float((unsigned)state[1]) : 0.f;  // max_hard_pred
  double sp = 0.0, sn = 0.0, cn = 0.0;
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (long)gridDim.x * blockDim.x) {
    float e[HNM_K], m, s;
    const T* x = logits + r * K;
    row_softmax(x, K, e, m, s);
    const bool p = pos[r] != 0;
    const bool ng = !p && nval[r] < thr;  // logical_and(nmask, nvalues < max_hard_pred)
    const int a = (int)(r % A);
    const int b = (int)(r / A);
    int l = 0;
#pragma unroll
    for (int q = 1; q < HNM_MAXL; ++q)
      if (q < lv.L && a >= lv.off[q]) l = q;
    const float lse = log_cr(s);
    const int lab = lbl[r];
    float wp = 0.f, wn = 0.f;
    if (p) {
      const float f = iou_factor(iou[r], gstat + (b * lv.L + l) * 4);
      const float ce = lse - (to_f32(x[lab]) - m);   // sparse softmax xent (label)
      sp += (double)(ce * f);                        // pos_loss * fpmask * iou_factor
      wp = f * inv_bs;
    } else {
      // iou factor is still multiplied in the reference (times fpmask = 0)
    }
    if (ng) {
      const float ce0 = lse - (to_f32(x[0]) - m);    // no_classes = 0 on negatives
      sn += (double)ce0;
      cn += 1.0;
      wn = 0.5f * inv_bs;                            // clf_loss = neg_loss / 2 + pos_loss
    }
    if (grad) {
      for (int k = 0; k < K; ++k) {
        const float pk = e[k] / s;
        float g = 0.f;
        if (p) g += wp * (pk - (k == lab ? 1.f : 0.f));
        if (ng) g += wn * (pk - (k == 0 ? 1.f : 0.f));
        grad[r * K + k] = from_f32<T>(g);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sp += __shfl_xor(sp, o, 64);
    sn += __shfl_xor(sn, o, 64);
    cn += __shfl_xor(cn, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sp;
    red[1][threadIdx.x >> 6] = sn;
    red[2][threadIdx.x >> 6] = cn;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int j = 0; j < 3; ++j) slab[blockIdx.x * 3 + j] = red[j][0] + red[j][1] + red[j][2] + red[j][3];
}

__global__ void hnm_finalize_kernel(const double* __restrict__ slab, int nb, const int* __restrict__ state,
                                    float bs, float* __restrict__ out) {
  __shared__ double s[3][256];
  double a = 0, b = 0, c = 0;
  for (int i = threadIdx.x; i < nb; i += 256) {
    a += slab[i * 3];
    b += slab[i * 3 + 1];
    c += slab[i * 3 + 2];
  }
  s[0][threadIdx.x] = a;
  s[1][threadIdx.x] = b;
  s[2][threadIdx.x] = c;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int j = 0; j < 3; ++j) s[j][threadIdx.x] += s[j][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float pos_loss = (float)s[0][0] / bs;  // tf.div(reduce_sum(...), bs)
    const float neg_loss = (float)s[1][0] / bs;
    out[0] = pos_loss;
    out[1] = neg_loss;
    out[2] = neg_loss / 2.f + pos_loss;
    out[3] = state[0] > 0 ? __uint_as_float((unsigned)state[1]) : 0.f;
    out[4] = (float)state[3];
    out[5] = (float)state[0];
    out[6] = (float)s[2][0];
    out[7] = 0.f;
  }
}

// data-parallel split (rod_hnm_*): the per-rank counts, then k from the all-reduced counts
__global__ void hnm_sum_counts_kernel(const int* __restrict__ cnt_slab, int nb, int* __restrict__ counts) {
  __shared__ int s[2][256];
  int np = 0, nn = 0;
  for (int i = threadIdx.x; i < nb; i += 256) {
    np += cnt_slab[2 * i];
    nn += cnt_slab[2 * i + 1];
  }
  s[0][threadIdx.x] = np;
  s[1][threadIdx.x] = nn;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      s[0][threadIdx.x] += s[0][threadIdx.x + w];
      s[1][threadIdx.x] += s[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    counts[0] = s[0][0];
    counts[1] = s[1][0];
  }
}
__global__ void hnm_begin_kernel(const int* __restrict__ counts, int B, int* __restrict__ state,
                                 unsigned* __restrict__ hist) {
  hist[threadIdx.x] = 0u;
  if (threadIdx.x == 0) {
    int k = (int)(3.0f * (float)counts[0]) + B;  // the same arithmetic as hnm_count_kernel
    k = min(k, counts[1]);
    state[0] = k;
    state[1] = 0;
    state[2] = k;
    state[3] = counts[0];
    state[4] = counts[1];
    state[5] = state[6] = state[7] = 0;
  }
}

// d clf_loss / d iou through the IoU focal factor (net_tools.py:590-607), the path that
// exists when refine_out is trained (train.py fix_refine=False; the reference applies no
// stop-gradient).  One block per (image, level) group, f64 sums, TF's gradient rules:
//   pos_loss = sum CE*pos*f / bs, f = w^4, w = zz/den, den = max(zz) + 1e-8, zz = z - min(z),
//   z = (u - mean)/sqrt(var + 1e-8) with tf.nn.moments (variance of stop_gradient(mean));
//   reduce_min / reduce_max split their gradient evenly over the tied elements.
// Recomputes the forward statistics with iou_group_kernel's exact float operations so the
// tie tests select the same elements.  g_iou [B*A] fp32 is written (0 for no gradient).
template <typename T>
__global__ void __launch_bounds__(256) iou_factor_bwd_kernel(const T* __restrict__ logits, const int* __restrict__ lbl,
                                                             const int* __restrict__ pos, const float* __restrict__ iou,
                                                             HnmLevels lv, int A, int K, float inv_bs,
                                                             float* __restrict__ g_iou) {
  __shared__ double sd[4][256];
  __shared__ float smin[256], smax[256];
  const int g = blockIdx.x;
  const int b = g / lv.L, l = g - b * lv.L;
  const long r0 = (long)b * A + lv.off[l];
  const int n = lv.off[l + 1] - lv.off[l];
  const int tid = threadIdx.x;
  auto block_sum = [&](double v0, double v1, double v2, double v3, double (&o)[4]) {
    __syncthreads();
    sd[0][tid] = v0;
    sd[1][tid] = v1;
    sd[2][tid] = v2;
    sd[3][tid] = v3;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (tid < w)
        for (int j = 0; j < 4; ++j) sd[j][tid] += sd[j][tid + w];
      __syncthreads();
    }
    for (int j = 0; j < 4; ++j) o[j] = sd[j][0];
  };
  // forward statistics (iou_group_kernel)
  double s = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = tid; i < n; i += 256) {
    const float u = iou[r0 + i];
    s += (double)u;
    mn = fminf(mn, u);
    mx = fmaxf(mx, u);
  }
  smin[tid] = mn;
  smax[tid] = mx;
  double o4[4];
  block_sum(s, 0.0, 0.0, 0.0, o4);
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) {
      smin[tid] = fminf(smin[tid], smin[tid + w]);
      smax[tid] = fmaxf(smax[tid], smax[tid + w]);
    }
    __syncthreads();
  }
  const float mean = (float)(o4[0] / (double)n);
  const float umin = smin[0], umax = smax[0];
  double v = 0.0;
  for (int i = tid; i < n; i += 256) {
    const float d = iou[r0 + i] - mean;
    v += (double)(d * d);
  }
  block_sum(v, 0.0, 0.0, 0.0, o4);
  const float var = (float)(o4[0] / (double)n);
  const float sdev = sqrtf(var + 1e-8f);
  const float zmin = (umin - mean) / sdev;
  const float zzmax = (umax - mean) / sdev + (0.f - zmin);
  const float den = zzmax + 1e-8f;
  // pass A: a_i = dL/dw_i = G_i * 4 w^3 (G_i = CE_i * pos_i / bs) -> g_iou (scratch);
  // sums a*zz (den), tie counts of max(zz) and min(z)
  double saz = 0.0, cmax = 0.0, cmin = 0.0;
  for (int i = tid; i < n; i += 256) {
    const long r = r0 + i;
    const float u = iou[r];
    const float z = (u - mean) / sdev;
    const float zz = z + (0.f - zmin);
    const float w = zz / den;
    float a = 0.f;
    if (pos[r] != 0) {
      const T* x = logits + r * K;
      float m = to_f32(x[0]);
      for (int k = 1; k < K; ++k) m = fmaxf(m, to_f32(x[k]));
      float se = 0.f;
      for (int k = 0; k < K; ++k) se += exp_cr(to_f32(x[k]) - m);
      const float ce = log_cr(se) - (to_f32(x[lbl[r]]) - m);
      a = ce * inv_bs * (4.f * powf(w, 3.f));
    }
    g_iou[r] = a;
    saz += (double)a * (double)zz;
    cmax += zz == zzmax ? 1.0 : 0.0;
    cmin += z == zmin ? 1.0 : 0.0;
  }
  block_sum(saz, cmax, cmin, 0.0, o4);
  const double dden = -o4[0] / ((double)den * (double)den);
  const double tmax = dden / o4[1];   // reduce_max: split over the ties
  const double ncmin = o4[2];
  // pass B: dzz_i = a_i/den + [zz_i max] tmax; sum dzz (-> d min(z))
  double sdzz = 0.0;
  for (int i = tid; i < n; i += 256) {
    const long r = r0 + i;
    const float u = iou[r];
    const float z = (u - mean) / sdev;
    const float zz = z + (0.f - zmin);
    double dzz = (double)g_iou[r] / (double)den + (zz == zzmax ? tmax : 0.0);
    g_iou[r] = (float)dzz;
    sdzz += dzz;
  }
  block_sum(sdzz, 0.0, 0.0, 0.0, o4);
  const double tmin = -o4[0] / ncmin;   // d min(z) = -sum dzz, split over the ties
  // pass C: g_i = dL/dz_i; sums g and g*(u - mean)
  double sg = 0.0, sgu = 0.0;
  for (int i = tid; i < n; i += 256) {
    const long r = r0 + i;
    const float u = iou[r];
    const float z = (u - mean) / sdev;
    const double gi = (double)g_iou[r] + (z == zmin ? tmin : 0.0);
    g_iou[r] = (float)gi;
    sg += gi;
    sgu += gi * (double)(u - mean);
  }
  block_sum(sg, sgu, 0.0, 0.0, o4);
  // z = (u - mean)/s, s = sqrt(var + 1e-8), var = mean((u - stop_gradient(mean))^2)
  const double sd_ = (double)sdev;
  const double dsdev = -o4[1] / (sd_ * sd_);
  const double cmean = -o4[0] / sd_ / (double)n;
  for (int i = tid; i < n; i += 256) {
    const long r = r0 + i;
    const double gi = (double)g_iou[r];
    const double du = gi / sd_ + cmean + dsdev * (double)(iou[r] - mean) / ((double)n * sd_);
    g_iou[r] = (float)du;
  }
}

static int hnm_blocks(long R) { return (int)std::min<long>(cdivl(R, 256), 2048); }

static HnmWs carve(void* ws, long R, int B, int L, int nb) {
  char* p = (char*)ws;
  auto take = [&](size_t n) {
    char* r = p;
    p += (n + 255) & ~(size_t)255;
    return r;
  };
  HnmWs w;
  w.nval = (float*)take(R * sizeof(float));
  w.gstat = (float*)take((size_t)B * L * 4 * sizeof(float));
  w.hist = (unsigned*)take(256 * sizeof(unsigned));
  w.state = (int*)take(8 * sizeof(int));
  w.cnt_slab = (int*)take((size_t)nb * 2 * sizeof(int));
  w.loss_slab = (double*)take((size_t)nb * 3 * sizeof(double));
  return w;
}

}  // namespace rod

using namespace rod;

extern "C" {

size_t rod_softmax_ce_hnm_workspace(int B, int A, int L) {
  const long R = (long)B * A;
  const int nb = hnm_blocks(R);
  return ((R * 4 + 255) & ~255L) + (((long)B * L * 16 + 255) & ~255L) + 1024 + 256 + (((long)nb * 8 + 255) & ~255L) +
         (((long)nb * 24 + 255) & ~255L) + 256;
}

int rod_softmax_ce_hnm(const void* logits, const int* det_lbl, const int* det_pos, const float* iou,
                       const int* lvl_off, int L, float bs, float* out, void* grad, void* workspace, int B, int A,
                       int K, int dtype, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0 && K > 1 && K <= HNM_K, "rod_softmax_ce_hnm: bad shape (K <= 16)");
  ROD_CHECK_ARG(L >= 1 && L <= HNM_MAXL && lvl_off, "rod_softmax_ce_hnm: bad levels");
  ROD_CHECK_ARG(lvl_off[0] == 0 && lvl_off[L] == A, "rod_softmax_ce_hnm: level offsets must span [0, A]");
  ROD_CHECK_ARG(workspace && out, "rod_softmax_ce_hnm: workspace/out NULL");
  HnmLevels lv;
  lv.L = L;
  for (int i = 0; i <= HNM_MAXL; ++i) lv.off[i] = i <= L ? lvl_off[i] : A;
  const long R = (long)B * A;
  const int nb = hnm_blocks(R);
  HnmWs w = carve(workspace, R, B, L, nb);
  hipStream_t s = ROD_STREAM(stream);
  const float inv_bs = 1.0f / bs;
  ROD_DISPATCH_DTYPE(dtype, {
    hipLaunchKernelGGL(hnm_rows_kernel<T>, dim3(nb), dim3(256), 0, s, (const T*)logits, det_pos, R, K, w.nval,
                       w.cnt_slab);
    hipLaunchKernelGGL(hnm_count_kernel, dim3(1), dim3(256), 0, s, w.cnt_slab, nb, B, w.state, w.hist);
    for (int shift = 24; shift >= 0; shift -= 8) {
      hipLaunchKernelGGL(radix_hist_kernel, dim3(nb), dim3(256), 0, s, w.nval, R, shift, w.state, w.hist);
      hipLaunchKernelGGL(radix_scan_kernel, dim3(1), dim3(256), 0, s, shift, w.state, w.hist);
    }
    hipLaunchKernelGGL(iou_group_kernel, dim3(B * L), dim3(256), 0, s, iou, lv, A, w.gstat);
    hipLaunchKernelGGL(hnm_loss_kernel<T>, dim3(nb), dim3(256), 0, s, (const T*)logits, det_lbl, det_pos, iou, w.nval,
                       w.gstat, w.state, lv, R, A, K, inv_bs, (T*)grad, w.loss_slab);
    hipLaunchKernelGGL(hnm_finalize_kernel, dim3(1), dim3(256), 0, s, w.loss_slab, nb, w.state, bs, out);
  });
  return check_launch("rod_softmax_ce_hnm");
}

int rod_iou_factor_bwd(const void* logits, const int* det_lbl, const int* det_pos, const float* iou,
                       const int* lvl_off, int L, float bs, float* g_iou, int B, int A, int K, int dtype,
                       void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0 && K > 1 && K <= HNM_K && g_iou, "rod_iou_factor_bwd: bad arguments");
  ROD_CHECK_ARG(L >= 1 && L <= HNM_MAXL && lvl_off && lvl_off[0] == 0 && lvl_off[L] == A,
                "rod_iou_factor_bwd: bad levels");
  HnmLevels lv;
  lv.L = L;
  for (int i = 0; i <= HNM_MAXL; ++i) lv.off[i] = i <= L ? lvl_off[i] : A;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(iou_factor_bwd_kernel<T>, dim3(B * L), dim3(256), 0,
                                               ROD_STREAM(stream), (const T*)logits, det_lbl, det_pos, iou, lv, A, K,
                                               1.0f / bs, g_iou));
  return check_launch("rod_iou_factor_bwd");
}

// ---- data-parallel split: per-rank rows, exchange points are counts[2] and hist[256] ----
size_t rod_hnm_workspace(int B, int A, int L) { return rod_softmax_ce_hnm_workspace(B, A, L); }

int rod_hnm_rows(const void* logits, const int* det_pos, void* workspace, int* counts, int B, int A, int K, int L,
                 int dtype, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0 && K > 1 && K <= HNM_K && workspace && counts, "rod_hnm_rows: bad arguments");
  const long R = (long)B * A;
  const int nb = hnm_blocks(R);
  HnmWs w = carve(workspace, R, B, L, nb);
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(hnm_rows_kernel<T>, dim3(nb), dim3(256), 0, s, (const T*)logits,
                                               det_pos, R, K, w.nval, w.cnt_slab));
  hipLaunchKernelGGL(hnm_sum_counts_kernel, dim3(1), dim3(256), 0, s, w.cnt_slab, nb, counts);
  return check_launch("rod_hnm_rows");
}

int rod_hnm_begin(const int* counts, int B_global, int* state, unsigned* hist, void* stream) {
  ROD_CHECK_ARG(counts && state && hist && B_global > 0, "rod_hnm_begin: bad arguments");
  hipLaunchKernelGGL(hnm_begin_kernel, dim3(1), dim3(256), 0, ROD_STREAM(stream), counts, B_global, state, hist);
  return check_launch("rod_hnm_begin");
}

int rod_hnm_radix_hist(const void* workspace, int B, int A, int L, int shift, const int* state, unsigned* hist,
                       void* stream) {
  ROD_CHECK_ARG(workspace && state && hist && (shift == 0 || shift == 8 || shift == 16 || shift == 24),
                "rod_hnm_radix_hist: bad arguments");
  const long R = (long)B * A;
  const int nb = hnm_blocks(R);
  HnmWs w = carve((void*)workspace, R, B, L, nb);
  hipLaunchKernelGGL(radix_hist_kernel, dim3(nb), dim3(256), 0, ROD_STREAM(stream), w.nval, R, shift, state, hist);
  return check_launch("rod_hnm_radix_hist");
}

int rod_hnm_radix_scan(int shift, int* state, unsigned* hist, void* stream) {
  ROD_CHECK_ARG(state && hist, "rod_hnm_radix_scan: bad arguments");
  hipLaunchKernelGGL(radix_scan_kernel, dim3(1), dim3(256), 0, ROD_STREAM(stream), shift, state, hist);
  return check_launch("rod_hnm_radix_scan");
}

int rod_hnm_loss(const void* logits, const int* det_lbl, const int* det_pos, const float* iou, const int* lvl_off,
                 int L, float bs, const int* state, float* out, void* grad, void* workspace, int B, int A, int K,
                 int dtype, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0 && K > 1 && K <= HNM_K, "rod_hnm_loss: bad shape (K <= 16)");
  ROD_CHECK_ARG(L >= 1 && L <= HNM_MAXL && lvl_off, "rod_hnm_loss: bad levels");
  ROD_CHECK_ARG(lvl_off[0] == 0 && lvl_off[L] == A, "rod_hnm_loss: level offsets must span [0, A]");
  ROD_CHECK_ARG(workspace && out && state, "rod_hnm_loss: workspace/out/state NULL");
  HnmLevels lv;
  lv.L = L;
  for (int i = 0; i <= HNM_MAXL; ++i) lv.off[i] = i <= L ? lvl_off[i] : A;
  const long R = (long)B * A;
  const int nb = hnm_blocks(R);
  HnmWs w = carve(workspace, R, B, L, nb);
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, {
    hipLaunchKernelGGL(iou_group_kernel, dim3(B * L), dim3(256), 0, s, iou, lv, A, w.gstat);
    hipLaunchKernelGGL(hnm_loss_kernel<T>, dim3(nb), dim3(256), 0, s, (const T*)logits, det_lbl, det_pos, iou, w.nval,
                       w.gstat, state, lv, R, A, K, 1.0f / bs, (T*)grad, w.loss_slab);
    hipLaunchKernelGGL(hnm_finalize_kernel, dim3(1), dim3(256), 0, s, w.loss_slab, nb, state, bs, out);
  });
  return check_launch("rod_hnm_loss");
}

}  // extern "C"
