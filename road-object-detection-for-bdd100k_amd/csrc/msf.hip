// msf.hip — process_backbone_method.PREORDER_MSF (reference nets/catch_net.py:115-152): the
// shallow endpoints are padded (tf.pad, top / left), compressed by a 1x1 conv + BatchNorm +
// leaky (the existing kernels), folded by tf.space_to_depth, concatenated with the tapped
// feature and recalibrated by a squeeze-and-excitation block (nets/attention_module.py:3-33).
// This file holds the data-movement ops and the SE block; all small maps (<= 1/8 resolution).
#include "rod_common.h"

namespace rod {

// V-element copies: one 16-byte vector (VEC) or one element (channel counts such as the 3- and
// 4-channel compressed endpoints, catch_net.py:121)
template <typename T, bool VEC>
struct Chunk {
  static constexpr int V = VEC ? Vec16<T>::N : 1;
  Vec16<T> v;
  T s;
  __device__ __forceinline__ void load(const T* p) {
    if constexpr (VEC) v.load(p); else s = *p;
  }
  __device__ __forceinline__ void store(T* p) const {
    if constexpr (VEC) v.store(p); else *p = s;
  }
  __device__ __forceinline__ void zero() {
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < V; ++i) v.set(i, 0.f);
    } else {
      s = from_f32<T>(0.f);
    }
  }
};

// ---------------------------------------------------------------- pad (top / left) and crop
// forward: y[n, h, w] = x[n, h - top, w - left] inside, 0 in the pad (tf.pad CONSTANT);
// inverse: y[n, h, w] = x[n, h + top, w + left] (the gradient: crop of the padded tensor).
template <typename T, bool VEC>
__global__ void pad2d_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int Hy, int Wy, int Hx, int Wx,
                             int C, int dh, int dw) {
  constexpr int V = Chunk<T, VEC>::V;
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)N * Hy * Wy * CV) return;
  const int cv = (int)(t % CV);
  const long p = t / CV;
  const int w = (int)(p % Wy);
  const long nh = p / Wy;
  const int h = (int)(nh % Hy);
  const int n = (int)(nh / Hy);
  const int hs = h - dh, ws = w - dw;
  Chunk<T, VEC> a;
  if (hs >= 0 && hs < Hx && ws >= 0 && ws < Wx) a.load(x + (((long)n * Hx + hs) * Wx + ws) * C + cv * V);
  else a.zero();
  a.store(y + p * C + cv * V);
}

// ---------------------------------------------------------------- space_to_depth (block r)
// TF NHWC order: out[n, i, j, (di*r + dj)*C + c] = in[n, i*r + di, j*r + dj, c]; one thread
// per output (pixel, tap, channel vector).  inverse: depth_to_space (its gradient).
template <typename T, bool VEC, bool INV>
__global__ void s2d_kernel(const T* __restrict__ src, T* __restrict__ dst, int N, int H, int W, int C, int r) {
  constexpr int V = Chunk<T, VEC>::V;
  const int CV = C / V, Ho = H / r, Wo = W / r;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)N * Ho * Wo * r * r * CV) return;
  const int cv = (int)(t % CV);
  const long q = t / CV;
  const int tap = (int)(q % (r * r));
  const long o = q / (r * r);
  const int j = (int)(o % Wo);
  const long ni = o / Wo;
  const int i = (int)(ni % Ho);
  const int n = (int)(ni / Ho);
  const long big = (((long)n * H + i * r + tap / r) * W + j * r + tap % r) * C + cv * V;
  const long small = (o * r * r + tap) * C + cv * V;
  Chunk<T, VEC> a;
  if constexpr (INV) {
    a.load(src + small);
    a.store(dst + big);
  } else {
    a.load(src + big);
    a.store(dst + small);
  }
}

// ---------------------------------------------------------------- squeeze-and-excitation
// per-(image, channel) sums over the HW rows of x (mean: squeeze) or of dy*x (the gradient
// of the excitation): block (channel group of 16 vectors, image) x 16 row lanes, fp32 lanes
// merged in f64 in a fixed order.
template <typename T, bool PROD>
__global__ void __launch_bounds__(256) se_rowsum_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                        float* __restrict__ out, long HW, int C, float scale) {
  constexpr int V = Vec16<T>::N;
  __shared__ float red[256 * V];
  const int CV = C / V;
  const int cvl = threadIdx.x % 16, pln = threadIdx.x / 16;
  const int cv = blockIdx.x * 16 + cvl;
  const int n = blockIdx.y;
  float acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = 0.f;
  if (cv < CV) {
    for (long r = pln; r < HW; r += 16) {
      Vec16<T> x;
      x.load(a + ((long)n * HW + r) * C + cv * V);
      if constexpr (PROD) {
        Vec16<T> y;
        y.load(b + ((long)n * HW + r) * C + cv * V);
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = fmaf(x.get(v), y.get(v), acc[v]);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += x.get(v);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) red[threadIdx.x * V + v] = acc[v];
  __syncthreads();
  if (threadIdx.x < 16 * V) {
    const int cb = threadIdx.x / V, v = threadIdx.x % V;
    const int c = (blockIdx.x * 16 + cb) * V + v;
    if (c < C) {
      double s = 0.0;
      for (int l = 0; l < 16; ++l) s += (double)red[(l * 16 + cb) * V + v];
      out[(long)n * C + c] = (float)(s * (double)scale);
    }
  }
}

__device__ __forceinline__ float sigmoid_f(float z) { return 1.f / (1.f + exp_cr(-z)); }

// tf.layers.dense(relu) then tf.layers.dense(sigmoid) on the squeezed [C] vector of one image
// (kernel [in][out], bias [out]); one block per image.
__global__ void __launch_bounds__(256) se_excite_kernel(const float* __restrict__ sq, const float* __restrict__ w1,
                                                        const float* __restrict__ b1, const float* __restrict__ w2,
                                                        const float* __restrict__ b2, float* __restrict__ hid,
                                                        float* __restrict__ e, int C, int C8) {
  extern __shared__ float sm[];   // [C] squeeze, [C8] hidden
  float* s = sm;
  float* h = sm + C;
  const int n = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) s[c] = sq[(long)n * C + c];
  __syncthreads();
  for (int k = threadIdx.x; k < C8; k += blockDim.x) {
    float a = 0.f;
    for (int c = 0; c < C; ++c) a = fmaf(s[c], w1[(long)c * C8 + k], a);
    a = fmaxf(a + b1[k], 0.f);
    h[k] = a;
    hid[(long)n * C8 + k] = a;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f;
    for (int k = 0; k < C8; ++k) a = fmaf(h[k], w2[(long)k * C + c], a);
    e[(long)n * C + c] = sigmoid_f(a + b2[c]);
  }
}

// y = x * e[n, c] (scale = input_feature * excitation)
template <typename T>
__global__ void se_scale_kernel(const T* __restrict__ x, const float* __restrict__ e, T* __restrict__ y, long HW,
                                int C, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const long n = i / ((long)HW * C);
  y[i] = from_f32<T>(to_f32(x[i]) * e[n * C + c]);
}

// Backward of the two dense layers for the whole batch in one block (parameter gradients
// summed over the images in a fixed order): de -> dpre2 = de*e*(1-e) (SigmoidGrad) ->
// dw2 / db2, dhid = dpre2 . w2^T -> dpre1 = dhid*(hid > 0) (ReluGrad) -> dw1 / db1,
// dsq = dpre1 . w1^T.  Scratch: [B][C] dpre2 + [B][C8] dpre1 in dynamic LDS.
__global__ void __launch_bounds__(256) se_excite_bwd_kernel(const float* __restrict__ de, const float* __restrict__ sq,
                                                            const float* __restrict__ w1, const float* __restrict__ w2,
                                                            const float* __restrict__ hid, const float* __restrict__ e,
                                                            float* __restrict__ dsq, float* __restrict__ dw1,
                                                            float* __restrict__ db1, float* __restrict__ dw2,
                                                            float* __restrict__ db2, int B, int C, int C8) {
  extern __shared__ float sm[];
  float* d2 = sm;              // [B][C]
  float* d1 = sm + B * C;      // [B][C8]
  for (int i = threadIdx.x; i < B * C; i += blockDim.x) {
    const float y = e[i];
    d2[i] = de[i] * y * (1.f - y);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B * C8; i += blockDim.x) {
    const int n = i / C8, k = i % C8;
    float a = 0.f;
    for (int c = 0; c < C; ++c) a = fmaf(d2[n * C + c], w2[(long)k * C + c], a);
    d1[i] = hid[i] > 0.f ? a : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C8 * C; i += blockDim.x) {   // dw2[k][c] = sum_n hid[n][k] * d2[n][c]
    const int k = i / C, c = i % C;
    float a = 0.f;
    for (int n = 0; n < B; ++n) a = fmaf(hid[n * C8 + k], d2[n * C + c], a);
    if (dw2) dw2[i] = a;
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f;
    for (int n = 0; n < B; ++n) a += d2[n * C + c];
    if (db2) db2[c] = a;
  }
  for (int i = threadIdx.x; i < C * C8; i += blockDim.x) {   // dw1[c][k] = sum_n sq[n][c] * d1[n][k]
    const int c = i / C8, k = i % C8;
    float a = 0.f;
    for (int n = 0; n < B; ++n) a = fmaf(sq[n * C + c], d1[n * C8 + k], a);
    if (dw1) dw1[i] = a;
  }
  for (int k = threadIdx.x; k < C8; k += blockDim.x) {
    float a = 0.f;
    for (int n = 0; n < B; ++n) a += d1[n * C8 + k];
    if (db1) db1[k] = a;
  }
  for (int i = threadIdx.x; i < B * C; i += blockDim.x) {    // dsq[n][c] = sum_k d1[n][k] * w1[c][k]
    const int n = i / C, c = i % C;
    float a = 0.f;
    for (int k = 0; k < C8; ++k) a = fmaf(d1[n * C8 + k], w1[(long)c * C8 + k], a);
    dsq[i] = a;
  }
}

// dx = dy * e[n, c] + dsq[n, c] / HW  (the product's and the mean's gradients)
template <typename T>
__global__ void se_input_grad_kernel(const T* __restrict__ dy, const float* __restrict__ e,
                                     const float* __restrict__ dsq, T* __restrict__ dx, long HW, int C, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const long n = i / ((long)HW * C);
  dx[i] = from_f32<T>(to_f32(dy[i]) * e[n * C + c] + dsq[n * C + c] / (float)HW);
}

static inline unsigned g256(long total) { return (unsigned)cdivl(total, 256); }

}  // namespace rod

using namespace rod;

extern "C" {

int rod_pad2d(const void* x, void* y, int N, int H, int W, int C, int top, int left, int Hp, int Wp, int inverse,
              int dtype, void* stream) {
  ROD_CHECK_ARG(x && y && N > 0 && H > 0 && W > 0 && C > 0 && top >= 0 && left >= 0 && Hp >= H + top &&
                    Wp >= W + left,
                "rod_pad2d: bad arguments");
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, {
    const bool vec = C % Vec16<T>::N == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0;
    const int V = vec ? Vec16<T>::N : 1;
    // inverse: [N, Hp, Wp] -> [N, H, W] (read shifted by +top / +left)
    const int Hy = inverse ? H : Hp, Wy = inverse ? W : Wp, Hx = inverse ? Hp : H, Wx = inverse ? Wp : W;
    const int dh = inverse ? -top : top, dw = inverse ? -left : left;
    const unsigned g = g256((long)N * Hy * Wy * (C / V));
    if (vec)
      hipLaunchKernelGGL((pad2d_kernel<T, true>), dim3(g), dim3(256), 0, s, (const T*)x, (T*)y, N, Hy, Wy, Hx, Wx, C,
                         dh, dw);
    else
      hipLaunchKernelGGL((pad2d_kernel<T, false>), dim3(g), dim3(256), 0, s, (const T*)x, (T*)y, N, Hy, Wy, Hx, Wx,
                         C, dh, dw);
  });
  return check_launch("rod_pad2d");
}

int rod_space_to_depth(const void* x, void* y, int N, int H, int W, int C, int block, int inverse, int dtype,
                       void* stream) {
  ROD_CHECK_ARG(x && y && N > 0 && C > 0 && block >= 2 && H % block == 0 && W % block == 0,
                "rod_space_to_depth: bad arguments (H, W must be multiples of the block)");
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, {
    const bool vec = C % Vec16<T>::N == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0;
    const unsigned g = g256((long)N * H * W * (C / (vec ? Vec16<T>::N : 1)));
if (vec && inverse)
      hipLaunchKernelGGL((s2d_kernel<T, true, true>), dim3(g), dim3(256), 0, s, (const T*)x, (T*)y, N, H, W, C, block);
    else if (vec)
      hipLaunchKernelGGL((s2d_kernel<T, true, false>), dim3(g), dim3(256), 0, s, (const T*)x, (T*)y, N, H, W, C, block);
    else if (inverse)
      hipLaunchKernelGGL((s2d_kernel<T, false, true>), dim3(g), dim3(256), 0, s, (const T*)x, (T*)y, N, H, W, C, block);
    else
      hipLaunchKernelGGL((s2d_kernel<T, false, false>), dim3(g), dim3(256), 0, s, (const T*)x, (T*)y, N, H, W, C,
                         block);
  });
  return check_launch("rod_space_to_depth");
}

int rod_se_fwd(const void* x, const float* w1, const float* b1, const float* w2, const float* b2, float* sq,
               float* hid, float* e, void* y, int N, long HW, int C, int C8, int dtype, void* stream) {
  ROD_CHECK_ARG(x && w1 && b1 && w2 && b2 && sq && hid && e && y && N > 0 && HW > 0 && C > 0 && C8 > 0,
                "rod_se_fwd: bad arguments");
  const int V = dtype == ROD_F32 ? 4 : 8;
  ROD_CHECK_ARG(C % V == 0 && (size_t)(C + C8) * 4 <= 64 * 1024, "rod_se_fwd: C=%d unsupported", C);
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, {
    hipLaunchKernelGGL((se_rowsum_kernel<T, false>), dim3(cdiv(C / V, 16), N), dim3(256), 0, s, (const T*)x,
                       (const T*)nullptr, sq, HW, C, (float)(1.0 / (double)HW));
    hipLaunchKernelGGL(se_excite_kernel, dim3(N), dim3(256), (C + C8) * sizeof(float), s, sq, w1, b1, w2, b2, hid, e,
                       C, C8);
    hipLaunchKernelGGL((se_scale_kernel<T>), dim3(g256((long)N * HW * C)), dim3(256), 0, s, (const T*)x, e, (T*)y,
                       HW, C, (long)N * HW * C);
  });
  return check_launch("rod_se_fwd");
}

int rod_se_bwd(const void* dy, const void* x, const float* w1, const float* w2, const float* sq, const float* hid,
               const float* e, float* de, float* dsq, float* dw1, float* db1, float* dw2, float* db2, void* dx, int N,
               long HW, int C, int C8, int dtype, void* stream) {
  ROD_CHECK_ARG(dy && x && w1 && w2 && sq && hid && e && de && dsq && dx && N > 0 && HW > 0 && C > 0 && C8 > 0,
                "rod_se_bwd: bad arguments");
  const int V = dtype == ROD_F32 ? 4 : 8;
  ROD_CHECK_ARG(C % V == 0 && (size_t)N * (C + C8) * 4 <= 64 * 1024, "rod_se_bwd: N=%d C=%d unsupported", N, C);
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, {
    hipLaunchKernelGGL((se_rowsum_kernel<T, true>), dim3(cdiv(C / V, 16), N), dim3(256), 0, s, (const T*)dy,
                       (const T*)x, de, HW, C, 1.f);
    hipLaunchKernelGGL(se_excite_bwd_kernel, dim3(1), dim3(256), (size_t)N * (C + C8) * sizeof(float), s, de, sq,
                       w1, w2, hid, e, dsq, dw1, db1, dw2, db2, N, C, C8);
    hipLaunchKernelGGL((se_input_grad_kernel<T>), dim3(g256((long)N * HW * C)), dim3(256), 0, s, (const T*)dy, e,
                       dsq, (T*)dx, HW, C, (long)N * HW * C);
  });
  return check_launch("rod_se_bwd");
}

}  // extern "C"
