// vgg.hip — the ops of the VGG-16 backbone that the MobileNet-v2 path does not have
// (reference nets/backbone/vgg.py:67-137, the second entry of config.supported_backbone_name):
//   * slim.max_pool2d([2, 2]) — stride 2, VALID — and its MaxPoolGrad;
//   * tf.layers.dropout (rate = dropout_keep_prob = 0.5 as the reference passes it, vgg.py:106,
//     111) with a counter-based hash RNG, and its gradient;
//   * 3x3 im2col / col2im for the convs the implicit-GEMM kernel does not cover: stride 2 after
//     custom_layers.pad2d (block8/9, VALID on a 1-padded map) and VALID stride 1 (block10).
//     The GEMM itself is rod_conv_fwd / rod_conv_wgrad with ksize 1 over the [M, 9*Cin]
//     column matrix (column order (i*3+j)*Cin + c = the [Cout][3][3][Cin] weight layout).
// Every kernel streams 16-byte channel vectors (C % 8 == 0 in bf16, C % 4 == 0 in fp32); the
// maps are small (<= 1/8 of the input resolution) except the first pools.
#include "rod_common.h"

namespace rod {

// ---------------------------------------------------------------- max pool 2x2 / 2, VALID
// One thread per (output pixel, channel vector).  TF's CPU kernel keeps the first maximum in
// row-major window order (strict >), recorded as argmax in 0..3 per channel.
template <typename T>
__global__ void maxpool2x2_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ am, int N, int H,
                                  int W, int C, int Ho, int Wo) {
  constexpr int V = Vec16<T>::N;
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * Ho * Wo * CV;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  const long o = t / CV;
  const int wo = (int)(o % Wo);
  const long nh = o / Wo;
  const int ho = (int)(nh % Ho);
  const int n = (int)(nh / Ho);
  float best[V];
  uint8_t arg[V];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int h = 2 * ho + (k >> 1), w = 2 * wo + (k & 1);
    Vec16<T> a;
    a.load(x + (((long)n * H + h) * W + w) * C + cv * V);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float f = a.get(v);
      if (k == 0 || f > best[v]) {
        best[v] = f;
        arg[v] = (uint8_t)k;
      }
    }
  }
  Vec16<T> r;
#pragma unroll
  for (int v = 0; v < V; ++v) r.set(v, best[v]);
  r.store(y + o * C + cv * V);
#pragma unroll
  for (int v = 0; v < V; ++v) am[o * C + cv * V + v] = arg[v];
}

// MaxPoolGrad as a gather over the INPUT: dx[h, w] = dy[h/2, w/2] where the window's argmax
// is this position, 0 elsewhere (rows / columns past the last VALID window included).
template <typename T>
__global__ void maxpool2x2_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ am, T* __restrict__ dx,
                                      int N, int H, int W, int C, int Ho, int Wo) {
  constexpr int V = Vec16<T>::N;
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * H * W * CV;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  const long p = t / CV;
  const int w = (int)(p % W);
  const long nh = p / W;
  const int h = (int)(nh % H);
  const int n = (int)(nh / H);
  const int ho = h >> 1, wo = w >> 1;
  Vec16<T> r;
  if (ho < Ho && wo < Wo) {
    const long o = ((long)n * Ho + ho) * Wo + wo;
    const uint8_t k = (uint8_t)(((h & 1) << 1) | (w & 1));
    Vec16<T> g;
    g.load(dy + o * C + cv * V);
#pragma unroll
    for (int v = 0; v < V; ++v) r.set(v, am[o * C + cv * V + v] == k ? g.get(v) : 0.f);
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) r.set(v, 0.f);
  }
  r.store(dx + p * C + cv * V);
}

// ---------------------------------------------------------------- dropout
// uniform in [0, 1) with 24 random bits from a splitmix64 of (seed, element index)
__device__ __forceinline__ float hash_uniform(unsigned long long seed, unsigned long long i) {
  unsigned long long z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// tf.nn.dropout: binary = floor(keep_prob + uniform); out = x / keep_prob * binary
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ mask, long n,
                               float keep, unsigned long long seed) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float b = floorf(keep + hash_uniform(seed, (unsigned long long)i));
  mask[i] = (uint8_t)(b != 0.f);
  y[i] = from_f32<T>(to_f32(x[i]) / keep * b);
}

// gradient of x / keep_prob * binary: (dy * binary) / keep_prob
template <typename T>
__global__ void dropout_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask, T* __restrict__ dx,
                                   long n, float keep) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dx[i] = from_f32<T>(to_f32(dy[i]) * (mask[i] ? 1.f : 0.f) / keep);
}

// ---------------------------------------------------------------- 3x3 im2col / col2im
// col[m = (n, ho, wo)][(i*3 + j)*C + c] = z(x[n, ho*s + i - pt, wo*s + j - pl, c]) or 0 outside,
// z = the BatchNorm-apply / activation prologue of the input when given (BnPro, as rod_conv_fwd).
template <typename T, bool PRO>
__global__ void im2col3x3_kernel(const T* __restrict__ x, BnPro pro, T* __restrict__ col, int N, int H, int W, int C,
                                 int s, int pt, int pl, int Ho, int Wo) {
  constexpr int V = Vec16<T>::N;
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * Ho * Wo * 9 * CV;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  const long q = t / CV;
  const int tap = (int)(q % 9);
  const long m = q / 9;
  const int wo = (int)(m % Wo);
  const long nh = m / Wo;
  const int ho = (int)(nh % Ho);
  const int n = (int)(nh / Ho);
  const int h = ho * s + tap / 3 - pt, w = wo * s + tap % 3 - pl;
  Vec16<T> a;
  if (h >= 0 && h < H && w >= 0 && w < W) {
    a.load(x + (((long)n * H + h) * W + w) * C + cv * V);
    if constexpr (PRO) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float sc, sh;
        bn_pro_affine(pro, cv * V + v, sc, sh);
        a.set(v, act_fwd(fmaf(a.get(v), sc, sh), pro.act));
      }
    }
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) a.set(v, 0.f);
  }
  a.store(col + m * 9 * C + tap * C + cv * V);
}

// dx[n, h, w, c] = sum over the taps (i, j) of the outputs (ho, wo) that read (h, w):
// h = ho*s + i - pt.  A gather with a fixed tap order (deterministic, no atomics).
template <typename T>
__global__ void col2im3x3_kernel(const T* __restrict__ col, T* __restrict__ dx, int N, int H, int W, int C, int s,
                                 int pt, int pl, int Ho, int Wo) {
  constexpr int V = Vec16<T>::N;
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * H * W * CV;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  const long p = t / CV;
  const int w = (int)(p % W);
  const long nh = p / W;
  const int h = (int)(nh % H);
  const int n = (int)(nh / H);
  float acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = 0.f;
  for (int i = 0; i < 3; ++i) {
    const int hh = h + pt - i;
    if (hh < 0 || hh % s) continue;
    const int ho = hh / s;
    if (ho >= Ho) continue;
    for (int j = 0; j < 3; ++j) {
      const int ww = w + pl - j;
      if (ww < 0 || ww % s) continue;
      const int wo = ww / s;
      if (wo >= Wo) continue;
      Vec16<T> g;
      g.load(col + ((((long)n * Ho + ho) * Wo + wo) * 9 + i * 3 + j) * C + cv * V);
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] += g.get(v);
    }
  }
  Vec16<T> r;
#pragma unroll
  for (int v = 0; v < V; ++v) r.set(v, acc[v]);
  r.store(dx + p * C + cv * V);
}

static inline unsigned grid1(long total) { return (unsigned)cdivl(total, 256); }

}  // namespace rod

using namespace rod;

extern "C" {

int rod_maxpool2x2(const void* x, void* y, uint8_t* argmax, int N, int H, int W, int C, int dtype, void* stream) {
  ROD_CHECK_ARG(x && y && argmax && N > 0 && H >= 2 && W >= 2 && C > 0, "rod_maxpool2x2: bad arguments");
  const int V = dtype == ROD_F32 ? 4 : 8;
  ROD_CHECK_ARG(C % V == 0, "rod_maxpool2x2: C %% %d != 0", V);
  const int Ho = H / 2, Wo = W / 2;
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL((maxpool2x2_kernel<T>), dim3(grid1((long)N * Ho * Wo * (C / V))),
                                               dim3(256), 0, s, (const T*)x, (T*)y, argmax, N, H, W, C, Ho, Wo));
  return check_launch("rod_maxpool2x2");
}

int rod_maxpool2x2_bwd(const void* dy, const uint8_t* argmax, void* dx, int N, int H, int W, int C, int dtype,
                       void* stream) {
  ROD_CHECK_ARG(dy && argmax && dx && N > 0 && H >= 2 && W >= 2 && C > 0, "rod_maxpool2x2_bwd: bad arguments");
  const int V = dtype == ROD_F32 ? 4 : 8;
  ROD_CHECK_ARG(C % V == 0, "rod_maxpool2x2_bwd: C %% %d != 0", V);
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL((maxpool2x2_bwd_kernel<T>), dim3(grid1((long)N * H * W * (C / V))),
                                               dim3(256), 0, s, (const T*)dy, argmax, (T*)dx, N, H, W, C, H / 2,
                                               W / 2));
  return check_launch("rod_maxpool2x2_bwd");
}

int rod_dropout(const void* x, void* y, uint8_t* mask, long n, float keep_prob, uint64_t seed, int dtype,
                void* stream) {
  ROD_CHECK_ARG(x && y && mask && n > 0 && keep_prob > 0.f && keep_prob <= 1.f, "rod_dropout: bad arguments");
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL((dropout_kernel<T>), dim3(grid1(n)), dim3(256), 0, s, (const T*)x,
                                               (T*)y, mask, n, keep_prob, seed));
  return check_launch("rod_dropout");
}

int rod_dropout_bwd(const void* dy, const uint8_t* mask, void* dx, long n, float keep_prob, int dtype, void* stream) {
  ROD_CHECK_ARG(dy && mask && dx && n > 0 && keep_prob > 0.f && keep_prob <= 1.f, "rod_dropout_bwd: bad arguments");
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL((dropout_bwd_kernel<T>), dim3(grid1(n)), dim3(256), 0, s,
                                               (const T*)dy, mask, (T*)dx, n, keep_prob));
  return check_launch("rod_dropout_bwd");
}

int rod_im2col3x3(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                  const float* pro_beta, int pro_act, void* col, int N, int H, int W, int C, int stride, int pad_t,
                  int pad_l, int Ho, int Wo, int dtype, void* stream) {
  ROD_CHECK_ARG(x && col && N > 0 && H > 0 && W > 0 && C > 0 && Ho > 0 && Wo > 0 && stride >= 1 && pad_t >= 0 &&
                    pad_l >= 0,
                "rod_im2col3x3: bad arguments");
  const int V = dtype == ROD_F32 ? 4 : 8;
  ROD_CHECK_ARG(C % V == 0, "rod_im2col3x3: C %% %d != 0", V);
  ROD_CHECK_ARG(!pro_mean || pro_rstd, "rod_im2col3x3: prologue needs mean and rstd");
  hipStream_t s = ROD_STREAM(stream);
  const BnPro pro{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  const unsigned g = grid1((long)N * Ho * Wo * 9 * (C / V));
  ROD_DISPATCH_DTYPE(dtype, {
    if (pro_mean)
      hipLaunchKernelGGL((im2col3x3_kernel<T, true>), dim3(g), dim3(256), 0, s, (const T*)x, pro, (T*)col, N, H, W,
                         C, stride, pad_t, pad_l, Ho, Wo);
    else
      hipLaunchKernelGGL((im2col3x3_kernel<T, false>), dim3(g), dim3(256), 0, s, (const T*)x, pro, (T*)col, N, H, W,
                         C, stride, pad_t, pad_l, Ho, Wo);
  });
  return check_launch("rod_im2col3x3");
}

int rod_col2im3x3(const void* col, void* dx, int N, int H, int W, int C, int stride, int pad_t, int pad_l, int Ho,
                  int Wo, int dtype, void* stream) {
  ROD_CHECK_ARG(col && dx && N > 0 && H > 0 && W > 0 && C > 0 && Ho > 0 && Wo > 0 && stride >= 1,
                "rod_col2im3x3: bad arguments");
  const int V = dtype == ROD_F32 ? 4 : 8;
  ROD_CHECK_ARG(C % V == 0, "rod_col2im3x3: C %% %d != 0", V);
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL((col2im3x3_kernel<T>), dim3(grid1((long)N * H * W * (C / V))),
                                               dim3(256), 0, s, (const T*)col, (T*)dx, N, H, W, C, stride, pad_t,
                                               pad_l, Ho, Wo));
  return check_launch("rod_col2im3x3");
}

}  // extern "C"
