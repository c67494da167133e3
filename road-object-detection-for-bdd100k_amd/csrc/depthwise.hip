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

constexpr int DW_R = 4;  // output rows per thread

template <typename T, int S, bool VECOK>
__global__ void __launch_bounds__(256) dw3x3_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                        T* __restrict__ y, int H, int W, int C, int pt, int pl,
                                                        int Ho, int Wo) {
  constexpr int V = VECOK ? Vec16<T>::N : 1;
  const int CV = C / V;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = t % CV;
  const int wo = t / CV;
  if (wo >= Wo) return;
  const int ho0 = blockIdx.y * DW_R;
  const int n = blockIdx.z;
  const int c = cv * V;

  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = w[k * C + c + v];

  float acc[DW_R][V];
#pragma unroll
  for (int q = 0; q < DW_R; ++q)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[q][v] = 0.f;

  const long img = (long)n * H * W;
  constexpr int NR = (DW_R - 1) * S + 3;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int hi = ho0 * S - pt + r;
    if (hi < 0 || hi >= H) continue;
    float xv[3][V];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int wi = wo * S - pl + j;
      if (wi >= 0 && wi < W) {
        const T* p = x + (img + (long)hi * W + wi) * C + c;
        if constexpr (VECOK) {
          Vec16<T> vv;
          vv.load(p);
#pragma unroll
          for (int v = 0; v < V; ++v) xv[j][v] = vv.get(v);
        } else {
          xv[j][0] = to_f32(p[0]);
        }
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) xv[j][v] = 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < DW_R; ++q) {
      const int i = r - q * S;  // tap row of output row ho0+q fed by input row r
      if (i < 0 || i > 2) continue;
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[q][v] = fmaf(xv[j][v], wr[i * 3 + j][v], acc[q][v]);
    }
  }
#pragma unroll
  for (int q = 0; q < DW_R; ++q) {
    const int ho = ho0 + q;
    if (ho >= Ho) break;
    T* p = y + (((long)n * Ho + ho) * Wo + wo) * C + c;
    if constexpr (VECOK) {
      Vec16<T> vv;
#pragma unroll
      for (int v = 0; v < V; ++v) vv.set(v, acc[q][v]);
      vv.store(p);
    } else {
      p[0] = from_f32<T>(acc[q][0]);
    }
  }
}

// dx[n,h,w,c] = sum_{i,j} dy[n,(h+pt-i)/S,(w+pl-j)/S,c] * w[i,j,c] over exact divisions.
template <typename T, int S, bool VECOK>
__global__ void __launch_bounds__(256) dw3x3_bwd_data_kernel(const T* __restrict__ dy, const float* __restrict__ w,
                                                             T* __restrict__ dx, int H, int W, int C, int pt,
                                                             int pl, int Ho, int Wo) {
  constexpr int V = VECOK ? Vec16<T>::N : 1;
  const int CV = C / V;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = t % CV;
  const int wc = t / CV;
  if (wc >= W) return;
  const int h0 = blockIdx.y * DW_R;
  const int n = blockIdx.z;
  const int c = cv * V;

  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = w[k * C + c + v];

  const long img = (long)n * Ho * Wo;
#pragma unroll
  for (int q = 0; q < DW_R; ++q) {
    const int h = h0 + q;
    if (h >= H) break;
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int hn = h + pt - i;
      if (hn < 0 || (S == 2 && (hn & 1))) continue;
      const int ho = hn / S;
      if (ho >= Ho) continue;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int wn = wc + pl - j;
        if (wn < 0 || (S == 2 && (wn & 1))) continue;
        const int wo = wn / S;
        if (wo >= Wo) continue;
        const T* p = dy + (img + (long)ho * Wo + wo) * C + c;
        if constexpr (VECOK) {
          Vec16<T> vv;
          vv.load(p);
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] = fmaf(vv.get(v), wr[i * 3 + j][v], acc[v]);
        } else {
          acc[0] = fmaf(to_f32(p[0]), wr[i * 3 + j][0], acc[0]);
        }
      }
    }
    T* p = dx + (((long)n * H + h) * W + wc) * C + c;
    if constexpr (VECOK) {
      Vec16<T> vv;
#pragma unroll
      for (int v = 0; v < V; ++v) vv.set(v, acc[v]);
      vv.store(p);
    } else {
      p[0] = from_f32<T>(acc[0]);
    }
  }
}

// Filter gradient, stage 1: block (bx, by) reduces output pixels [bx*chunk, ...)
// for channel-vector group by; partial sums [9][C] per bx go to the slab.
// Thread layout: lane t -> (pixel lane t / CVp, channel vector t % CVp).
template <typename T, int S, bool VECOK>
__global__ void __launch_bounds__(256) dw3x3_bwd_filter_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                               float* __restrict__ slab, int N, int H, int W,
                                                               int C, int pt, int pl, int Ho, int Wo,
                                                               int CVp, long chunk) {
  constexpr int V = VECOK ? Vec16<T>::N : 1;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [256][V]
  const int CV = C / V;
  const int lanes = 256 / CVp;  // >= 1
  const int tid = threadIdx.x;
  const int cvl = tid % CVp;
  const int pln = tid / CVp;
  const int cv = blockIdx.y * CVp + cvl;
  const bool active = (cvl < CVp) && (cv < CV);
  const int c = cv * V;
  const long P = (long)N * Ho * Wo;
  const long p0 = (long)blockIdx.x * chunk;
  const long p1 = p0 + chunk < P ? p0 + chunk : P;

  float acc[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] = 0.f;

  if (active) {
    for (long p = p0 + pln; p < p1; p += lanes) {
      const int wo = (int)(p % Wo);
      const long t2 = p / Wo;
      const int ho = (int)(t2 % Ho);
      const int n = (int)(t2 / Ho);
      float g[V];
      const T* pg = dy + p * C + c;
      if constexpr (VECOK) {
        Vec16<T> vv;
        vv.load(pg);
#pragma unroll
        for (int v = 0; v < V; ++v) g[v] = vv.get(v);
      } else {
        g[0] = to_f32(pg[0]);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int hi = ho * S - pt + i;
        if (hi < 0 || hi >= H) continue;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int wi = wo * S - pl + j;
          if (wi < 0 || wi >= W) continue;
          const T* px = x + (((long)n * H + hi) * W + wi) * C + c;
          if constexpr (VECOK) {
            Vec16<T> vv;
            vv.load(px);
#pragma unroll
            for (int v = 0; v < V; ++v) acc[i * 3 + j][v] = fmaf(g[v], vv.get(v), acc[i * 3 + j][v]);
          } else {
            acc[i * 3 + j][0] = fmaf(g[0], to_f32(px[0]), acc[i * 3 + j][0]);
          }
        }
      }
    }
  }
  // deterministic tree reduction over pixel lanes, one tap at a time
  for (int k = 0; k < 9; ++k) {
#pragma unroll
    for (int v = 0; v < V; ++v) red[tid * V + v] = acc[k][v];
    __syncthreads();
    for (int s = lanes >> 1; s > 0; s >>= 1) {
      if (pln < s) {
#pragma unroll
        for (int v = 0; v < V; ++v) red[tid * V + v] += red[(tid + s * CVp) * V + v];
      }
      __syncthreads();
    }
    if (pln == 0 && active) {
#pragma unroll
      for (int v = 0; v < V; ++v) slab[((long)blockIdx.x * 9 + k) * C + c + v] = red[tid * V + v];
    }
    __syncthreads();
  }
}

__global__ void slab_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out, int nslab, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int b = 0; b < nslab; ++b) s += slab[(long)b * n + i];
  out[i] = s;
}

static int pow2_at_least(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

struct DwFilterPlan {
  int CVp, cgroups, nbx;
  long chunk;
};

template <typename T>
static DwFilterPlan dw_filter_plan(int N, int Ho, int Wo, int C, bool vecok) {
  const int V = vecok ? Vec16<T>::N : 1;
  const int CV = C / V;
  DwFilterPlan pl;
  pl.CVp = std::min(pow2_at_least(CV), 256);
  pl.cgroups = cdiv(CV, pl.CVp);
  const long P = (long)N * Ho * Wo;
  // aim for ~2048 blocks in total, each covering >= 64 pixels per lane-row
  long want = std::max<long>(1, 2048 / pl.cgroups);
  long minchunk = (long)(256 / pl.CVp) * 8;
  long chunk = std::max<long>(cdivl(P, want), minchunk);
  pl.chunk = chunk;
  pl.nbx = (int)cdivl(P, chunk);
  return pl;
}

template <typename T>
static bool dw_vec_ok(const void* a, const void* b, int C) {
  const int V = Vec16<T>::N;
  return (C % V == 0) && (((uintptr_t)a & 15) == 0) && (((uintptr_t)b & 15) == 0);
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
  const int V = VK ? Vec16<T>::N : 1;
  dim3 grid(cdiv((long)(C / V) * Wo, 256), cdiv(Ho, DW_R), N);
  hipLaunchKernelGGL((dw3x3_fwd_kernel<T, S, VK>), grid, dim3(256), 0, s, (const T*)x, w, (T*)y, H, W, C, pt, pl, Ho,
                     Wo);
}
template <typename T, int S, bool VK>
static void dw_bwd_data_launch(const void* dy, const float* w, void* dx, int N, int H, int W, int C, int pt, int pl,
                               int Ho, int Wo, hipStream_t s) {
  const int V = VK ? Vec16<T>::N : 1;
  dim3 grid(cdiv((long)(C / V) * W, 256), cdiv(H, DW_R), N);
  hipLaunchKernelGGL((dw3x3_bwd_data_kernel<T, S, VK>), grid, dim3(256), 0, s, (const T*)dy, w, (T*)dx, H, W, C, pt,
                     pl, Ho, Wo);
}
template <typename T, int S, bool VK>
static void dw_bwd_filter_launch(const void* x, const void* dy, float* dw, float* slab, int N, int H, int W, int C,
                                 int pt, int pl, int Ho, int Wo, hipStream_t s) {
  const int V = VK ? Vec16<T>::N : 1;
  DwFilterPlan pl_ = dw_filter_plan<T>(N, Ho, Wo, C, VK);
  dim3 grid(pl_.nbx, pl_.cgroups);
  size_t lds = 256 * V * sizeof(float);
  hipLaunchKernelGGL((dw3x3_bwd_filter_kernel<T, S, VK>), grid, dim3(256), lds, s, (const T*)x, (const T*)dy, slab, N,
                     H, W, C, pt, pl, Ho, Wo, pl_.CVp, pl_.chunk);
  slab_sum(slab, dw, pl_.nbx, 9L * C, s);
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
    const bool vec = dw_vec_ok<float>(x, y, C);
    DW_SELECT(dw_fwd_launch, float, x, w, y, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else if (dtype == ROD_BF16) {
    const bool vec = dw_vec_ok<bf16_t>(x, y, C);
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
    const bool vec = dw_vec_ok<float>(dy, dx, C);
    DW_SELECT(dw_bwd_data_launch, float, dy, w, dx, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else if (dtype == ROD_BF16) {
    const bool vec = dw_vec_ok<bf16_t>(dy, dx, C);
    DW_SELECT(dw_bwd_data_launch, bf16_t, dy, w, dx, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else {
    set_error("rod_dw3x3_bwd_data: bad dtype %d", dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_dw3x3_bwd_data");
}

size_t rod_dw3x3_bwd_filter_workspace(int N, int Ho, int Wo, int C) {
  DwFilterPlan a = dw_filter_plan<float>(N, Ho, Wo, C, false);
  DwFilterPlan b = dw_filter_plan<float>(N, Ho, Wo, C, C % 4 == 0);
  DwFilterPlan c = dw_filter_plan<bf16_t>(N, Ho, Wo, C, C % 8 == 0);
  int nbx = std::max(a.nbx, std::max(b.nbx, c.nbx));
  return (size_t)nbx * 9 * C * sizeof(float);
}

int rod_dw3x3_bwd_filter(const void* x, const void* dy, float* dw, void* workspace, int N, int H, int W, int C,
                         int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream) {
  DW_ARGS_OK("rod_dw3x3_bwd_filter");
  ROD_CHECK_ARG(workspace != nullptr, "rod_dw3x3_bwd_filter: workspace is NULL");
  hipStream_t s = ROD_STREAM(stream);
  float* slab = (float*)workspace;
  if (dtype == ROD_F32) {
    const bool vec = dw_vec_ok<float>(x, dy, C);
    DW_SELECT(dw_bwd_filter_launch, float, x, dy, dw, slab, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else if (dtype == ROD_BF16) {
    const bool vec = dw_vec_ok<bf16_t>(x, dy, C);
    DW_SELECT(dw_bwd_filter_launch, bf16_t, x, dy, dw, slab, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else {
    set_error("rod_dw3x3_bwd_filter: bad dtype %d", dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_dw3x3_bwd_filter");
}

}  // extern "C"
