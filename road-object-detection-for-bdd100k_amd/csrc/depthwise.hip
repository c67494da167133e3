// depthwise.hip — NHWC depthwise 3x3 (slim.separable_conv2d with num_outputs=None,
// depth_multiplier=1, padding SAME; reference nets/backbone/mobilenet/conv_blocks.py:238-247).
//
// Layout: x [N,H,W,C], y [N,Ho,Wo,C] in the storage dtype, w fp32 [3][3][C].
// Each thread owns one 16-byte channel vector (4 x f32 / 8 x bf16) of one output
// column and a strip of R output rows; the (R-1)*S+3 input rows of its three input
// columns are streamed once through registers, so vertical reuse is in VGPRs and the
// 3x horizontal reuse is served by L1 (neighbouring lanes share columns).
// Consecutive lanes walk the channel vectors of one pixel, so every wave-level load
// is a contiguous, 16-byte-per-lane coalesced segment.
#include "rod_common.h"

namespace rod {

// V contiguous elements of T held in registers (bf16 x4 = 8-byte, f32 x4 = 16-byte loads).
template <typename T, int V> struct PackV;
template <> struct PackV<float, 4> {
  f32x4 v;
  __device__ __forceinline__ void load(const float* p) { v = *(const f32x4*)p; }
  __device__ __forceinline__ void zero() { v = f32x4{0.f, 0.f, 0.f, 0.f}; }
  __device__ __forceinline__ float get(int i) const { return v[i]; }
  __device__ __forceinline__ void set(int i, float a) { v[i] = a; }
  __device__ __forceinline__ void store(float* p) const { *(f32x4*)p = v; }
};
template <> struct PackV<bf16_t, 4> {
  bf16x4 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *(const bf16x4*)p; }
  __device__ __forceinline__ void zero() { v = bf16x4{(bf16_t)0.f, (bf16_t)0.f, (bf16_t)0.f, (bf16_t)0.f}; }
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
  __device__ __forceinline__ void set(int i, float a) { v[i] = (bf16_t)a; }
  __device__ __forceinline__ void store(bf16_t* p) const { *(bf16x4*)p = v; }
};
template <typename T> struct PackV<T, 1> {
  T v;
  __device__ __forceinline__ void load(const T* p) { v = *p; }
  __device__ __forceinline__ void zero() { v = (T)0.f; }
  __device__ __forceinline__ float get(int) const { return to_f32(v); }
  __device__ __forceinline__ void set(int, float a) { v = from_f32<T>(a); }
  __device__ __forceinline__ void store(T* p) const { *p = v; }
};

constexpr int DW_RB = 8;  // output rows per thread (forward / backward-data strips)

// Forward: thread = (channel vector cv, output column wo), strip of DW_RB output rows; the
// 3x3 input window rolls down in registers (one new input row per output row for S=1, two
// for S=2) and lanes of a wave read consecutive channel vectors of neighbouring pixels.
template <typename T, int S, int V>
__global__ void __launch_bounds__(256) dw3x3_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                        T* __restrict__ y, int H, int W, int C, int pt, int pl,
                                                        int Ho, int Wo) {
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(t % CV);
  const int wo = (int)(t / CV);
  if (wo >= Wo) return;
  const int ho0 = blockIdx.y * DW_RB;
  const int ho1 = ho0 + DW_RB < Ho ? ho0 + DW_RB : Ho;
  const int n = blockIdx.z;
  const int c = cv * V;
  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = w[k * C + c + v];
  const T* xn = x + (long)n * H * W * C + c;
  T* yn = y + (long)n * Ho * Wo * C + c;
  PackV<T, V> xr[3][3];
  auto load_row = [&](PackV<T, V>(&row)[3], int hi) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int wi = wo * S - pl + j;
      if (hi >= 0 && hi < H && wi >= 0 && wi < W) row[j].load(xn + ((long)hi * W + wi) * C);
      else row[j].zero();
    }
  };
  load_row(xr[0], ho0 * S - pt);
  load_row(xr[1], ho0 * S - pt + 1);
  load_row(xr[2], ho0 * S - pt + 2);
  for (int ho = ho0; ho < ho1; ++ho) {
    if (ho > ho0) {
      if constexpr (S == 1) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          xr[0][j] = xr[1][j];
          xr[1][j] = xr[2][j];
        }
        load_row(xr[2], ho - pt + 2);
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) xr[0][j] = xr[2][j];
        load_row(xr[1], ho * 2 - pt + 1);
        load_row(xr[2], ho * 2 - pt + 2);
      }
    }
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = fmaf(xr[i][j].get(v), wr[i * 3 + j][v], acc[v]);
    PackV<T, V> o;
#pragma unroll
    for (int v = 0; v < V; ++v) o.set(v, acc[v]);
    o.store(yn + ((long)ho * Wo + wo) * C);
  }
}

// dx[n,h,w,c] = sum_{i,j} dy[n,(h+pt-i)/S,(w+pl-j)/S,c] * w[i,j,c] over exact divisions.
// S=1: the three dy rows h+pt-i roll down in registers; S=2: direct loads (each dx pixel
// sees 1, 2 or 4 dy pixels).
template <typename T, int S, int V>
__global__ void __launch_bounds__(256) dw3x3_bwd_data_kernel(const T* __restrict__ dy, const float* __restrict__ w,
                                                             T* __restrict__ dx, int H, int W, int C, int pt,
                                                             int pl, int Ho, int Wo) {
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(t % CV);
  const int wc = (int)(t / CV);
  if (wc >= W) return;
  const int h0 = blockIdx.y * DW_RB;
  const int h1 = h0 + DW_RB < H ? h0 + DW_RB : H;
  const int n = blockIdx.z;
  const int c = cv * V;
  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = w[k * C + c + v];
  const T* dn = dy + (long)n * Ho * Wo * C + c;
  T* xn = dx + (long)n * H * W * C + c;
  if constexpr (S == 1) {
    PackV<T, V> dr[3][3];  // dr[i][j] = dy[h+pt-i, wc+pl-j]
    auto load_row = [&](PackV<T, V>(&row)[3], int ho) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int wo = wc + pl - j;
        if (ho >= 0 && ho < Ho && wo >= 0 && wo < Wo) row[j].load(dn + ((long)ho * Wo + wo) * C);
        else row[j].zero();
      }
    };
    load_row(dr[0], h0 + pt);
    load_row(dr[1], h0 + pt - 1);
    load_row(dr[2], h0 + pt - 2);
    for (int h = h0; h < h1; ++h) {
      if (h > h0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          dr[2][j] = dr[1][j];
          dr[1][j] = dr[0][j];
        }
        load_row(dr[0], h + pt);
      }
      float acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] = fmaf(dr[i][j].get(v), wr[i * 3 + j][v], acc[v]);
      PackV<T, V> o;
#pragma unroll
      for (int v = 0; v < V; ++v) o.set(v, acc[v]);
      o.store(xn + ((long)h * W + wc) * C);
    }
  } else {
    for (int h = h0; h < h1; ++h) {
      float acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int hn = h + pt - i;
        if (hn < 0 || (hn & 1)) continue;
        const int ho = hn >> 1;
        if (ho >= Ho) continue;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int wn = wc + pl - j;
          if (wn < 0 || (wn & 1)) continue;
          const int wo = wn >> 1;
          if (wo >= Wo) continue;
          PackV<T, V> g;
          g.load(dn + ((long)ho * Wo + wo) * C);
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] = fmaf(g.get(v), wr[i * 3 + j][v], acc[v]);
        }
      }
      PackV<T, V> o;
#pragma unroll
      for (int v = 0; v < V; ++v) o.set(v, acc[v]);
      o.store(xn + ((long)h * W + wc) * C);
    }
  }
}

// Filter gradient: dw[i,j,c] = sum_{n,ho,wo} dy[n,ho,wo,c] * x[n, ho*S-pt+i, wo*S-pl+j, c].
// Thread = (channel vector cv, output column wo) exactly like the forward; it walks strips of
// RB output rows, keeping the 3x3 input window in registers (one new input row per output
// row for S=1, two for S=2), so each output pixel costs one dy load and three x loads and no
// index division.  blockIdx.y strides over the N*spi row strips; each block then sums its
// threads per channel in LDS (fixed order) and writes one [9][C] partial to the slab.
template <typename T, int S, int V>
__global__ void __launch_bounds__(256) dw3x3_bwd_filter_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                               float* __restrict__ slab, int N, int H, int W,
                                                               int C, int pt, int pl, int Ho, int Wo, int RB,
                                                               int spi) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [256][V]
  const int CV = C / V;
  const int tid = threadIdx.x;
  const long t = (long)blockIdx.x * 256 + tid;
  const int cv = (int)(t % CV);
  const int wo = (int)(t / CV);
  const int c = cv * V;
  float acc[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] = 0.f;

  if (wo < Wo) {
    const int nstrips = N * spi;
    for (int s = blockIdx.y; s < nstrips; s += gridDim.y) {
      const int n = s / spi;
      const int ho0 = (s - n * spi) * RB;
      const int ho1 = ho0 + RB < Ho ? ho0 + RB : Ho;
      const T* xn = x + (long)n * H * W * C + c;
      const T* dn = dy + (long)n * Ho * Wo * C + c;
      PackV<T, V> xr[3][3];
      auto load_row = [&](PackV<T, V>(&row)[3], int hi) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int wi = wo * S - pl + j;
          if (hi >= 0 && hi < H && wi >= 0 && wi < W) row[j].load(xn + ((long)hi * W + wi) * C);
          else row[j].zero();
        }
      };
      load_row(xr[0], ho0 * S - pt);
      load_row(xr[1], ho0 * S - pt + 1);
      load_row(xr[2], ho0 * S - pt + 2);
      for (int ho = ho0; ho < ho1; ++ho) {
        if (ho > ho0) {
          if constexpr (S == 1) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              xr[0][j] = xr[1][j];
              xr[1][j] = xr[2][j];
            }
            load_row(xr[2], ho - pt + 2);
          } else {
#pragma unroll
            for (int j = 0; j < 3; ++j) xr[0][j] = xr[2][j];
            load_row(xr[1], ho * 2 - pt + 1);
            load_row(xr[2], ho * 2 - pt + 2);
          }
        }
        PackV<T, V> g;
        g.load(dn + ((long)ho * Wo + wo) * C);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int v = 0; v < V; ++v) acc[i * 3 + j][v] = fmaf(g.get(v), xr[i][j].get(v), acc[i * 3 + j][v]);
      }
    }
  }
  // per-channel block sums: threads of this block holding channel vector cve sit at
  // tl = (cve - tb) mod CV, + CV, ... (threads past Wo hold zeros)
  const long tb = (long)blockIdx.x * 256;
  const int t0mod = (int)(tb % CV);
  float* out = slab + ((long)blockIdx.y * gridDim.x + blockIdx.x) * 9 * C;
  for (int k = 0; k < 9; ++k) {
#pragma unroll
    for (int v = 0; v < V; ++v) red[tid * V + v] = acc[k][v];
    __syncthreads();
    for (int e = tid; e < C; e += 256) {
      const int cve = e / V, v = e - cve * V;
      int tl = cve - t0mod;
      if (tl < 0) tl += CV;
      float s = 0.f;
      for (; tl < 256; tl += CV) s += red[tl * V + v];
      out[k * C + e] = s;
    }
    __syncthreads();
  }
}

struct DwFilterPlan {
  int gx, gy, RB, spi;
  long parts() const { return (long)gx * gy; }
};

// gx column tiles of 256 (cv, wo) threads; gy blocks stride over the N*spi row strips.
// ~2048 blocks, capped so the [parts][9][C] slab stays <= max(16 MB, dy bytes / 8).
static DwFilterPlan dw_filter_plan(int N, int Ho, int Wo, int C, int V, int es) {
  DwFilterPlan p;
  p.gx = cdiv((long)(C / V) * Wo, 256);
  // strips of RB rows; short maps get shorter strips so that there are enough of them
  p.RB = std::max(2, std::min(16, Ho / 4));
  p.spi = cdiv(Ho, p.RB);
  const long strips = (long)N * p.spi;
  const long cap_bytes = std::max<long>(16L << 20, (long)N * Ho * Wo * C * es / 8);
  long gy = std::min<long>(strips, std::max<long>(1, 2048 / p.gx));
  gy = std::min<long>(gy, std::max<long>(1, cap_bytes / ((long)p.gx * 36 * C)));
  p.gy = (int)std::max<long>(1, gy);
  return p;
}

template <typename T>
static bool dw_pack4_ok(const void* a, const void* b, int C) {
  const uintptr_t al = 4 * sizeof(T) - 1;
  return (C % 4 == 0) && (((uintptr_t)a & al) == 0) && (((uintptr_t)b & al) == 0);
}

}  // namespace rod

using namespace rod;

#define DW_ARGS_OK(fn)                                                                                  \
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && Ho > 0 && Wo > 0, fn ": bad shape");                \
  ROD_CHECK_ARG(stride == 1 || stride == 2, fn ": stride must be 1 or 2");                              \
  ROD_CHECK_ARG(pad_t >= 0 && pad_t <= 2 && pad_l >= 0 && pad_l <= 2, fn ": bad padding");              \
  ROD_CHECK_ARG((Ho - 1) * stride + 3 - pad_t > 0 && (Wo - 1) * stride + 3 - pad_l > 0, fn ": bad output")

namespace rod {

template <typename T, int S, bool VK>
static void dw_fwd_launch(const void* x, const float* w, void* y, int N, int H, int W, int C, int pt, int pl, int Ho,
                          int Wo, hipStream_t s) {
  constexpr int V = VK ? 4 : 1;
  dim3 grid(cdiv((long)(C / V) * Wo, 256), cdiv(Ho, DW_RB), N);
  hipLaunchKernelGGL((dw3x3_fwd_kernel<T, S, V>), grid, dim3(256), 0, s, (const T*)x, w, (T*)y, H, W, C, pt, pl, Ho,
                     Wo);
}
template <typename T, int S, bool VK>
static void dw_bwd_data_launch(const void* dy, const float* w, void* dx, int N, int H, int W, int C, int pt, int pl,
                               int Ho, int Wo, hipStream_t s) {
  constexpr int V = VK ? 4 : 1;
  dim3 grid(cdiv((long)(C / V) * W, 256), cdiv(H, DW_RB), N);
  hipLaunchKernelGGL((dw3x3_bwd_data_kernel<T, S, V>), grid, dim3(256), 0, s, (const T*)dy, w, (T*)dx, H, W, C, pt,
                     pl, Ho, Wo);
}
template <typename T, int S, bool VK>
static void dw_bwd_filter_launch(const void* x, const void* dy, float* dw, float* slab, int N, int H, int W, int C,
                                 int pt, int pl, int Ho, int Wo, hipStream_t s) {
  constexpr int V = VK ? 4 : 1;
  DwFilterPlan p = dw_filter_plan(N, Ho, Wo, C, V, (int)sizeof(T));
  hipLaunchKernelGGL((dw3x3_bwd_filter_kernel<T, S, V>), dim3(p.gx, p.gy), dim3(256), 256 * V * sizeof(float), s,
                     (const T*)x, (const T*)dy, slab, N, H, W, C, pt, pl, Ho, Wo, p.RB, p.spi);
  slab_sum(slab, dw, (int)p.parts(), 9L * C, s);
}

}  // namespace rod

using namespace rod;

#define DW_SELECT(FN, T_, ...)                                         \
  do {                                                                 \
    if (stride == 1) {                                                 \
      if (vec) FN<T_, 1, true>(__VA_ARGS__); else FN<T_, 1, false>(__VA_ARGS__); \
    } else {                                                           \
      if (vec) FN<T_, 2, true>(__VA_ARGS__); else FN<T_, 2, false>(__VA_ARGS__); \
    }                                                                  \
  } while (0)

extern "C" {

int rod_dw3x3_fwd(const void* x, const float* w, void* y, int N, int H, int W, int C, int stride, int pad_t,
                  int pad_l, int Ho, int Wo, int dtype, void* stream) {
  DW_ARGS_OK("rod_dw3x3_fwd");
  hipStream_t s = ROD_STREAM(stream);
  if (dtype == ROD_F32) {
    const bool vec = dw_pack4_ok<float>(x, y, C);
    DW_SELECT(dw_fwd_launch, float, x, w, y, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else if (dtype == ROD_BF16) {
    const bool vec = dw_pack4_ok<bf16_t>(x, y, C);
    DW_SELECT(dw_fwd_launch, bf16_t, x, w, y, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else {
    set_error("rod_dw3x3_fwd: bad dtype %d", dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_dw3x3_fwd");
}

int rod_dw3x3_bwd_data(const void* dy, const float* w, void* dx, int N, int H, int W, int C, int stride,
                       int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream) {
  DW_ARGS_OK("rod_dw3x3_bwd_data");
  hipStream_t s = ROD_STREAM(stream);
  if (dtype == ROD_F32) {
    const bool vec = dw_pack4_ok<float>(dy, dx, C);
    DW_SELECT(dw_bwd_data_launch, float, dy, w, dx, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else if (dtype == ROD_BF16) {
    const bool vec = dw_pack4_ok<bf16_t>(dy, dx, C);
    DW_SELECT(dw_bwd_data_launch, bf16_t, dy, w, dx, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else {
    set_error("rod_dw3x3_bwd_data: bad dtype %d", dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_dw3x3_bwd_data");
}

size_t rod_dw3x3_bwd_filter_workspace(int N, int Ho, int Wo, int C) {
  long parts = 0;
  for (int V : {1, 4})
    for (int es : {2, 4}) parts = std::max(parts, dw_filter_plan(N, Ho, Wo, C, V, es).parts());
  return (size_t)parts * 9 * C * sizeof(float);
}

int rod_dw3x3_bwd_filter(const void* x, const void* dy, float* dw, void* workspace, int N, int H, int W, int C,
                         int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream) {
  DW_ARGS_OK("rod_dw3x3_bwd_filter");
  ROD_CHECK_ARG(workspace != nullptr, "rod_dw3x3_bwd_filter: workspace is NULL");
  hipStream_t s = ROD_STREAM(stream);
  float* slab = (float*)workspace;
  if (dtype == ROD_F32) {
    const bool vec = dw_pack4_ok<float>(x, dy, C);
    DW_SELECT(dw_bwd_filter_launch, float, x, dy, dw, slab, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else if (dtype == ROD_BF16) {
    const bool vec = dw_pack4_ok<bf16_t>(x, dy, C);
    DW_SELECT(dw_bwd_filter_launch, bf16_t, x, dy, dw, slab, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else {
    set_error("rod_dw3x3_bwd_filter: bad dtype %d", dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_dw3x3_bwd_filter");
}

}  // extern "C"
