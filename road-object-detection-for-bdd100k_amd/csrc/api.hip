// api.hip — error reporting, version, and small elementwise entry points.
#include <stdarg.h>
#include <stdio.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "rod_common.h"

namespace rod {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

// ---------------------------------------------------------------- slab reduction
// block = CB columns x (256/CB) slab lanes; each lane keeps 4 independent f64 partials
// (4 loads in flight), then a fixed-order LDS combine.  CB is chosen so that short rows
// with many slabs (filter gradients: n = 9*C, thousands of parts) still fill the chip.
template <int CB>
__global__ void __launch_bounds__(256) slab_sum_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                       int nslab, long n) {
  constexpr int L = 256 / CB;
  __shared__ double red[L][CB + 1];
  const int tx = threadIdx.x % CB, ty = threadIdx.x / CB;
  const long i = (long)blockIdx.x * CB + tx;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (i < n) {
    int b = ty;
    for (; b + 3 * L < nslab; b += 4 * L) {
      s0 += (double)slab[(long)b * n + i];
      s1 += (double)slab[(long)(b + L) * n + i];
      s2 += (double)slab[(long)(b + 2 * L) * n + i];
      s3 += (double)slab[(long)(b + 3 * L) * n + i];
    }
    for (; b < nslab; b += L) s0 += (double)slab[(long)b * n + i];
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && i < n) {
    double t = 0.0;
    for (int k = 0; k < L; ++k) t += red[k][tx];
    out[i] = (float)t;
  }
}

// Deferred slab sums (rod_slab_defer / rod_slab_flush).  A training step's parameter-gradient
// entries (conv / depthwise / fused-pointwise weight gradients, bias column sums) each end in a
// slab_sum of a few microseconds, ~115 launches per step whose only consumers are the optimizer
// and the data-parallel reducer.  While deferral is on, those sums are queued on the host and
// rod_slab_flush runs them as ONE batched launch per SLAB_BATCH jobs, each job with the exact
// block geometry and summation order of its own launch (bit-identical outputs).  The jobs are
// passed by value in the kernel arguments, so a flush is capturable in a HIP graph.
struct SlabJob {
  const float* slab;
  float* out;
  long n;
  int nslab;
  int cb;   // columns per block (4, 8 or 32): as slab_sum would have launched it
  int vec;  // 4: each thread sums 4 adjacent columns with 16-byte loads (n % 4 == 0, aligned slab)
};
constexpr int SLAB_BATCH = 32;
struct SlabBatch {
  SlabJob job[SLAB_BATCH];
  int first[SLAB_BATCH + 1];  // first block of each job; first[cnt] = grid size
  int cnt;
};

// vec == 4: a thread owns 4 adjacent columns (one 16-byte load per slab row instead of four
// 4-byte ones: 4x the bytes in flight per load instruction); every column keeps the thread row
// ty, the four chains and the block's ty-order combine of the scalar form (bit-identical sums)
__global__ void __launch_bounds__(256) slab_sum_batch_kernel(SlabBatch b) {
  __shared__ double red[1088];  // [L][VW * CB + 1] for L = 256 / CB, CB in {4, 8, 32}, VW in {1, 4}
  int e = 0;
  while (e + 1 < b.cnt && (int)blockIdx.x >= b.first[e + 1]) ++e;
  const SlabJob j = b.job[e];
  const int CB = j.cb, L = 256 / CB;
  const int tx = threadIdx.x % CB, ty = threadIdx.x / CB;
  if (j.vec == 4) {
    const int RW = 4 * CB + 1;
    const long i0 = (long)(blockIdx.x - b.first[e]) * CB * 4 + tx * 4;
    const long n = j.n;
    double s[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int v = 0; v < 4; ++v) s[c][v] = 0.0;
    if (i0 < n) {
      int k = ty;
      for (; k + 3 * L < j.nslab; k += 4 * L) {
        f32x4 a[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] = *(const f32x4*)(j.slab + (long)(k + c * L) * n + i0);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int v = 0; v < 4; ++v) s[c][v] += (double)a[c][v];
      }
      for (; k < j.nslab; k += L) {
        const f32x4 a = *(const f32x4*)(j.slab + (long)k * n + i0);
#pragma unroll
        for (int v = 0; v < 4; ++v) s[0][v] += (double)a[v];
      }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) red[ty * RW + tx * 4 + v] = (s[0][v] + s[1][v]) + (s[2][v] + s[3][v]);
    __syncthreads();
    if (ty == 0 && i0 < n) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        double t = 0.0;
        for (int k = 0; k < L; ++k) t += red[k * RW + tx * 4 + v];
        j.out[i0 + v] = (float)t;
      }
    }
    return;
  }
  const long i = (long)(blockIdx.x - b.first[e]) * CB + tx;
  const long n = j.n;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (i < n) {
    int k = ty;
    for (; k + 3 * L < j.nslab; k += 4 * L) {
      s0 += (double)j.slab[(long)k * n + i];
      s1 += (double)j.slab[(long)(k + L) * n + i];
      s2 += (double)j.slab[(long)(k + 2 * L) * n + i];
      s3 += (double)j.slab[(long)(k + 3 * L) * n + i];
    }
    for (; k < j.nslab; k += L) s0 += (double)j.slab[(long)k * n + i];
  }
  red[ty * (CB + 1) + tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && i < n) {
    double t = 0.0;
    for (int k = 0; k < L; ++k) t += red[k * (CB + 1) + tx];
    j.out[i] = (float)t;
  }
}

// process-wide, not thread-local: PyTorch runs the backward of custom autograd Functions on its
// per-device worker thread, not on the thread that calls rod_slab_defer / rod_slab_flush
static std::atomic<bool> g_slab_defer{false};
static std::mutex g_slab_mu;
static std::vector<SlabJob>* g_slab_jobs = nullptr;

int slab_cb(int nslab, long n) {
  if (n >= 256L * 32 || nslab <= 64) return 32;
  if (n >= 256L * 8) return 8;
  return 4;
}

void slab_sum(const float* slab, float* out, int nslab, long n, hipStream_t s, bool deferrable) {
  if (n <= 0) return;
  const int cb = slab_cb(nslab, n);
  if (deferrable && g_slab_defer.load()) {
    std::lock_guard<std::mutex> lk(g_slab_mu);
    if (!g_slab_jobs) g_slab_jobs = new std::vector<SlabJob>();
    static const bool vec_off = getenv("ROD_SLAB_VEC") && atoi(getenv("ROD_SLAB_VEC")) == 0;  // A/B switch
    const int vec = !vec_off && n % 4 == 0 && ((uintptr_t)slab & 15) == 0 ? 4 : 1;
    g_slab_jobs->push_back(SlabJob{slab, out, n, nslab, cb, vec});
    return;
  }
  if (cb == 32)
    hipLaunchKernelGGL(slab_sum_kernel<32>, dim3(cdivl(n, 32)), dim3(256), 0, s, slab, out, nslab, n);
  else if (cb == 8)
    hipLaunchKernelGGL(slab_sum_kernel<8>, dim3(cdivl(n, 8)), dim3(256), 0, s, slab, out, nslab, n);
  else
    hipLaunchKernelGGL(slab_sum_kernel<4>, dim3(cdivl(n, 4)), dim3(256), 0, s, slab, out, nslab, n);
}

int const_channel_blocks(int CV, long total, int target) {
  // smallest block count step s with (s*256) % CV == 0
  int g = CV, b = 256;
  while (b) { int t = g % b; g = b; b = t; }  // gcd(CV, 256)
  const int step = CV / g;
  long want = std::min<long>(target, cdivl(total, 256));
  long blocks = std::max<long>(1, cdivl(want, step)) * step;
  return (int)blocks;
}

// ---------------------------------------------------------------- kernels
template <typename T>
__global__ void normalize_image_kernel(const uint8_t* __restrict__ img, T* __restrict__ out, long n) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const float k = 2.0f / 255.0f;  // (2.0 / 255.0) * imgs - 1.0, train.py:126 (f32 graph)
  if (i + 3 < n) {
    uchar4 v = *(const uchar4*)(img + i);
    out[i + 0] = from_f32<T>(k * (float)v.x - 1.0f);
    out[i + 1] = from_f32<T>(k * (float)v.y - 1.0f);
    out[i + 2] = from_f32<T>(k * (float)v.z - 1.0f);
    out[i + 3] = from_f32<T>(k * (float)v.w - 1.0f);
  } else {
    for (; i < n; ++i) out[i] = from_f32<T>(k * (float)img[i] - 1.0f);
  }
}

template <typename S, typename D>
__global__ void cast_kernel(const S* __restrict__ src, D* __restrict__ dst, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) dst[i] = from_f32<D>(to_f32(src[i]));
}

// tf.clip_by_value = minimum(maximum(g, -clip), clip) with Eigen's scalar max/min
// (a < b ? b : a / b < a ? b : a): a NaN gradient stays NaN and poisons the variable, as in TF.
__device__ __forceinline__ float clip_tf(float g, float clip) {
  return g != g ? g : fminf(fmaxf(g, -clip), clip);
}

__global__ void sgd_clip_kernel(float* __restrict__ p, const float* __restrict__ g, long n, float lr,
                                float clip) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  long stride = (long)gridDim.x * blockDim.x * 4;
  for (; i < n; i += stride) {
    if (i + 3 < n) {
      f32x4 pv = *(f32x4*)(p + i);
      f32x4 gv = *(const f32x4*)(g + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float c = clip_tf(gv[j], clip);               // tf.clip_by_value
        pv[j] = pv[j] - lr * c;                       // ApplyGradientDescent: var -= alpha * delta
      }
      *(f32x4*)(p + i) = pv;
    } else {
      for (long k = i; k < n; ++k) p[k] = p[k] - lr * clip_tf(g[k], clip);
    }
  }
}

}  // namespace rod

using namespace rod;

extern "C" {

int rod_abi_version(void) { return ROD_ABI_VERSION; }
const char* rod_last_error(void) { return rod::g_err; }

int rod_normalize_image(const void* img_u8, void* out, long n, int out_dtype, void* stream) {
  ROD_CHECK_ARG(n >= 0, "rod_normalize_image: n < 0");
  if (n == 0) return 0;
  ROD_CHECK_ARG(((uintptr_t)img_u8 & 3) == 0, "rod_normalize_image: input must be 4-byte aligned");
  int blocks = cdiv(cdivl(n, 4), 256);
  ROD_DISPATCH_DTYPE(out_dtype, hipLaunchKernelGGL(normalize_image_kernel<T>, dim3(blocks), dim3(256),
                                                   0, ROD_STREAM(stream), (const uint8_t*)img_u8,
                                                   (T*)out, n));
  return check_launch("rod_normalize_image");
}

int rod_cast(const void* src, int src_dtype, void* dst, int dst_dtype, long n, void* stream) {
  ROD_CHECK_ARG(n >= 0, "rod_cast: n < 0");
  if (n == 0) return 0;
  int blocks = (int)std::min<long>(cdivl(n, 256), 8192);
  hipStream_t s = ROD_STREAM(stream);
  if (src_dtype == ROD_F32 && dst_dtype == ROD_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16_t>), dim3(blocks), dim3(256), 0, s, (const float*)src,
                       (bf16_t*)dst, n);
  else if (src_dtype == ROD_BF16 && dst_dtype == ROD_F32)
    hipLaunchKernelGGL((cast_kernel<bf16_t, float>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)src,
                       (float*)dst, n);
  else if (src_dtype == ROD_F32 && dst_dtype == ROD_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(blocks), dim3(256), 0, s, (const float*)src,
                       (float*)dst, n);
  else if (src_dtype == ROD_BF16 && dst_dtype == ROD_BF16)
    hipLaunchKernelGGL((cast_kernel<bf16_t, bf16_t>), dim3(blocks), dim3(256), 0, s,
                       (const bf16_t*)src, (bf16_t*)dst, n);
  else {
    set_error("rod_cast: bad dtype pair %d -> %d", src_dtype, dst_dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_cast");
}

int rod_slab_defer(int on) { return g_slab_defer.exchange(on != 0) ? 1 : 0; }

int rod_slab_pending(void) {
  std::lock_guard<std::mutex> lk(g_slab_mu);
  return g_slab_jobs ? (int)g_slab_jobs->size() : 0;
}

static int slab_launch(std::vector<SlabJob>& jobs, hipStream_t s) {
  for (size_t k0 = 0; k0 < jobs.size(); k0 += SLAB_BATCH) {
    SlabBatch b{};
    b.cnt = (int)std::min<size_t>(SLAB_BATCH, jobs.size() - k0);
    long blocks = 0;
    for (int e = 0; e < b.cnt; ++e) {
      b.job[e] = jobs[k0 + e];
      b.first[e] = (int)blocks;
      blocks += cdivl(b.job[e].n, (long)b.job[e].cb * b.job[e].vec);
    }
    b.first[b.cnt] = (int)blocks;
    ROD_CHECK_ARG(blocks < (1L << 31), "rod_slab_flush: batch too large");
    hipLaunchKernelGGL(slab_sum_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, s, b);
    const int rc = check_launch("rod_slab_flush");
    if (rc) return rc;
  }
  return 0;
}

int rod_slab_flush(void* stream) {
  hipStream_t s = ROD_STREAM(stream);
  std::vector<SlabJob> jobs;
  {
    std::lock_guard<std::mutex> lk(g_slab_mu);
    if (!g_slab_jobs || g_slab_jobs->empty()) return 0;
    jobs.swap(*g_slab_jobs);
  }
  return slab_launch(jobs, s);
}

int rod_slab_flush_range(const void* lo, const void* hi, void* stream) {
  hipStream_t s = ROD_STREAM(stream);
  ROD_CHECK_ARG((const char*)lo <= (const char*)hi, "rod_slab_flush_range: lo > hi");
  std::vector<SlabJob> jobs;
  {
    std::lock_guard<std::mutex> lk(g_slab_mu);
    if (!g_slab_jobs || g_slab_jobs->empty()) return 0;
    std::vector<SlabJob> keep;
    for (const SlabJob& j : *g_slab_jobs) {
      const char* o = (const char*)j.out;
      const bool in = o >= (const char*)lo && o + j.n * sizeof(float) <= (const char*)hi;
      (in ? jobs : keep).push_back(j);
    }
    g_slab_jobs->swap(keep);
  }
  return jobs.empty() ? 0 : slab_launch(jobs, s);
}

int rod_sgd_clip(float* param, const float* grad, long n, float lr, float clip, void* stream) {
  ROD_CHECK_ARG(n >= 0, "rod_sgd_clip: n < 0");
  ROD_CHECK_ARG(((uintptr_t)param & 15) == 0 && ((uintptr_t)grad & 15) == 0,
                "rod_sgd_clip: buffers must be 16-byte aligned");
  if (n == 0) return 0;
  int blocks = (int)std::min<long>(cdivl(cdivl(n, 4), 256), 4096);
  hipLaunchKernelGGL(sgd_clip_kernel, dim3(blocks), dim3(256), 0, ROD_STREAM(stream), param, grad, n,
                     lr, clip);
  return check_launch("rod_sgd_clip");
}

}  // extern "C"
