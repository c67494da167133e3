// batchnorm.hip — slim.batch_norm (fused, NHWC) forward statistics, apply(+activation
// +residual) and backward.  Reference semantics: nets/backbone/mobilenet/mobilenet.py:417-420
// (decay 0.997, center+scale in the backbone) and slim defaults in the heads
// (nets/catch_net.py:302: decay 0.999, center, no scale); epsilon 1e-3.
//
// Statistics are computed on x - k where k = x[row 0, c] (a per-channel pivot taken
// from the data), so E[(x-k)^2] - E[x-k]^2 does not cancel catastrophically; per-block
// partial sums go to a slab [nblk][2][C] and are combined in f64 by a finalize kernel
// (deterministic, no atomics).
//
// Elementwise passes (apply, backward-apply) are HBM streams: each thread keeps ONE
// 16-byte channel vector for the whole grid-stride loop (grid*256 is a multiple of the
// channel-vector count), so the per-channel parameters live in registers and each
// iteration is one 16-byte load per operand and one 16-byte store.
#include <mutex>

#include "rod_common.h"

namespace rod {


// Row-chunk reduction plan shared by the statistics and backward-reduce kernels.
// CV channel vectors are split into cgroups of CVb <= 256 (blockIdx.y); the 256 threads of a
// block are `lanes` row lanes x CVb channel vectors (no power-of-two padding, so at most
// CVb-1 threads idle); blockIdx.x owns `chunk` consecutive rows.  ~1024 blocks keep >= 16 MB
// of loads in flight (4 unrolled 16-byte loads per thread), which HBM needs to stream.
struct RedPlan {
  int V, CV, CVb, cgroups, lanes, nbx;
  long chunk;
};

template <typename T>
static RedPlan red_plan(long M, int C, bool vec, long want_blocks = 1024) {
  RedPlan r;
  r.V = vec ? Vec16<T>::N : 1;
  r.CV = C / r.V;
  r.cgroups = cdiv(r.CV, 256);
  r.CVb = cdiv(r.CV, r.cgroups);
  r.lanes = 256 / r.CVb;
  const long want = std::max<long>(1, want_blocks / r.cgroups);
  // >= 16 rows per lane; 4 on small narrow tensors (C <= 256, M*C <= 4M), whose launches are
  // latency-bound (measured, tools/bn_bench.py)
  const long minchunk = (long)r.lanes * (C <= 256 && M * C <= (4L << 20) ? 4 : 16);
  r.chunk = std::max<long>(cdivl(M, want), minchunk);
  r.nbx = (int)cdivl(M, r.chunk);
  return r;
}

template <typename T, bool VEC>
__device__ __forceinline__ void load_v(const T* p, float (&out)[VEC ? Vec16<T>::N : 1]) {
  if constexpr (VEC) {
    Vec16<T> a;
    a.load(p);
#pragma unroll
    for (int v = 0; v < Vec16<T>::N; ++v) out[v] = a.get(v);
  } else {
    out[0] = to_f32(p[0]);
  }
}
// Non-temporal (streaming) store for the backward-apply output: measured 2.7 % faster over
// the step's BatchNorm-backward shapes (tools/bn_bench.py), outputs bit-identical.
template <typename T, bool VEC>
__device__ __forceinline__ void store_nt(T* p, const float (&in)[VEC ? Vec16<T>::N : 1]) {
  if constexpr (VEC) {
    Vec16<T> a;
#pragma unroll
    for (int v = 0; v < Vec16<T>::N; ++v) a.set(v, in[v]);
    __builtin_nontemporal_store(a.v, (decltype(a.v)*)p);
  } else {
    p[0] = from_f32<T>(in[0]);
  }
}
template <typename T, bool VEC>
__device__ __forceinline__ void store_v(T* p, const float (&in)[VEC ? Vec16<T>::N : 1]) {
  if constexpr (VEC) {
    Vec16<T> a;
#pragma unroll
    for (int v = 0; v < Vec16<T>::N; ++v) a.set(v, in[v]);
    a.store(p);
  } else {
    p[0] = from_f32<T>(in[0]);
  }
}

// ---------------------------------------------------------------- statistics
// Per block: pivot k = x[first row of the chunk, c]; s1 = sum(x-k), s2 = sum((x-k)^2) per
// thread (fp32), lane partials combined in f64 in fixed order; the block emits its exact
// (mean_b, M2_b) pair so the finalize is Chan's parallel merge (no global cancellation).
template <typename T, bool VEC>
__global__ void __launch_bounds__(256) bn_stats_kernel(const T* __restrict__ x, long M, int C, int ldx, int CVb,
                                                       int lanes, long chunk, float* __restrict__ slab) {
  constexpr int V = VEC ? Vec16<T>::N : 1;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][256][V]
  const int tid = threadIdx.x;
  const int cvl = tid % CVb, pln = tid / CVb;
  const int CV = C / V;
  const int cv = blockIdx.y * CVb + cvl;
  const bool active = pln < lanes && cv < CV;
  const int c = cv * V;
  const long r0 = (long)blockIdx.x * chunk;
  const long r1 = r0 + chunk < M ? r0 + chunk : M;
  if (r0 >= M) {  // a part past the end (grid sized to a producer's part count): count 0
    for (int e = tid; e < CVb * V; e += 256) {
      const int cg = blockIdx.y * CVb + e / V;
      if (cg < CV) store_stat_part(slab, C, blockIdx.x, cg * V + e % V, 0.f, 0.f, 0.f);
    }
    return;
  }
  float s1[V], s2[V], k[V];
#pragma unroll
  for (int v = 0; v < V; ++v) s1[v] = s2[v] = 0.f;
  if (active) {
    load_v<T, VEC>(x + r0 * ldx + c, k);
    long r = r0 + pln;
    for (; r + 3L * lanes < r1; r += 4L * lanes) {
      float a[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_v<T, VEC>(x + (r + (long)u * lanes) * ldx + c, a[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float d = a[u][v] - k[v];
          s1[v] += d;
          s2[v] = fmaf(d, d, s2[v]);
        }
    }
    for (; r < r1; r += lanes) {
      float a[V];
      load_v<T, VEC>(x + r * ldx + c, a);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float d = a[v] - k[v];
        s1[v] += d;
        s2[v] = fmaf(d, d, s2[v]);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    red[tid * V + v] = s1[v];
    red[(256 + tid) * V + v] = s2[v];
  }
  __syncthreads();
  const double nb = (double)(r1 - r0);
  for (int e = tid; e < CVb * V; e += 256) {
    const int cb = e / V, v = e - cb * V;
    const int cg = blockIdx.y * CVb + cb;
    if (cg >= CV) continue;
    double a = 0.0, b = 0.0;
    for (int l = 0; l < lanes; ++l) {
      a += (double)red[(l * CVb + cb) * V + v];
      b += (double)red[(256 + l * CVb + cb) * V + v];
    }
    const int ch = cg * V + v;
    const double kk = (double)to_f32(x[r0 * ldx + ch]);
    const double m2 = b - a * a / nb;
    store_stat_part(slab, C, blockIdx.x, ch, (float)nb, (float)(kk + a / nb), (float)(m2 > 0.0 ? m2 : 0.0));
  }
}

// Partial slabs are laid out [2][C][nparts] (quantity, channel, part) so that the finalize
// reads each channel's parts contiguously: one wave per channel, 64 lanes striding over the
// parts (4 independent loads in flight per lane), f64 accumulation, fixed-order wave tree.
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Merge of part-major partial statistics, one level: block (s, g) merges parts
// [s*slice, (s+1)*slice) of channels [g*CB, (g+1)*CB) — PL = 256/CB part lanes per channel,
// <= 16 serial part loads per thread (1024-thread blocks) on coalesced rows, then a fixed-order LDS tree
// over the lanes — into part s of `out`.  When a single part remains (gridDim.x == 1) the
// same block finishes: mean, rstd and the moving-average update.
__device__ __forceinline__ void chan_merge_d(double& n, double& mean, double& m2, double nb, double meanb, double m2b) {
  if (nb == 0.0) return;
  if (n == 0.0) {
    n = nb;
    mean = meanb;
    m2 = m2b;
    return;
  }
  const double nt = n + nb;
  const double d = meanb - mean;
  mean += d * (nb / nt);
  m2 += m2b + d * d * (n * nb / nt);
  n = nt;
}

constexpr int MERGE_T = 1024;  // threads per merge block

struct MergePlan {
  int CB, PL, slice;
};
static MergePlan merge_plan(int C, int nparts) {
  // ROD_MERGE_LANE_PARTS (diagnosis switch): parts per lane per level (default 16) — a different
  // slice grouping of the same fixed-order f64 merge
  static const int lane_parts = getenv("ROD_MERGE_LANE_PARTS") ? atoi(getenv("ROD_MERGE_LANE_PARTS")) : 16;
  const int lp = lane_parts > 0 ? lane_parts : 16;
  MergePlan p;
  p.CB = C < 64 ? C : 64;   // 64 channels x 16+ part lanes per block
  // ROD_MERGE_ONE_LEVEL=1 (opt-in): one level wherever it can — fewer channels per block (more
  // part lanes) until one slice of <= 16 parts a lane holds every part, down to 2 channels (512
  // lanes, 8192 parts): a 720p step's merges 124 -> 100 launches.  Its grouping differs from the
  // fixed 64-channel plan (a rounding-level change of the merged statistics): the ALL-mode step
  // tests accept it (the fp64 truth's own input-noise sensitivity covers the head-kink flip it
  // causes), the 720p b8 fp32 step test (test_gpu_fullsize, no such probe: the fp64 truth takes
  // minutes there) does not — refine/block_1 0.011 against a 0.0041 bar
  static const bool one_level = getenv("ROD_MERGE_ONE_LEVEL") && atoi(getenv("ROD_MERGE_ONE_LEVEL")) == 1;
  while (one_level && p.CB > 2 && (long)lp * (MERGE_T / p.CB) < nparts) p.CB = (p.CB + 1) / 2;
  p.PL = MERGE_T / p.CB;
  p.slice = lp * p.PL;   // <= 16 parts per lane per level: short load chains
  return p;
}

// Parts are merged in shifted-sum form (no divisions in the loop): with a pivot k per
// channel (the mean of the slice's first non-empty part), every part contributes
// n, S1 = n*(mean-k), S2 = M2 + n*(mean-k)^2 in f64; lanes and then the block's part lanes
// are added in a fixed order, and the slice's (n, mean, M2) = (n, k + S1/n, S2 - S1^2/n).
// One block's work: slice bx of the parts, channels [by*CB, (by+1)*CB); its part goes to part
// bx of `out`, or (last) mean, rstd and the moving averages.  Slice parts are stored with
// agent-scope (L2-coherent across the XCDs) stores, and COH reads them the same way: the
// single-launch second level reads parts other blocks of the same launch wrote, with no
// whole-cache write-back / invalidate (an agent-scope fence per block cost more than the launch
// it saves: 93 launches at 13.5 us against 124 at 5.7 us).
__device__ __forceinline__ float merge_ld(const float* p, bool coh) {
  return coh ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}
template <bool COH>
__device__ __forceinline__ void merge_slice(const float* parts, int nparts, int C, int CB, int slice, int bx, int by,
                                            bool last, float* out, long M, float eps, float decay, float* mean,
                                            float* rstd, float* mmean, float* mvar, double* sn, double* s1,
                                            double* s2, float* piv) {
  const int tid = threadIdx.x;
  const int PL = MERGE_T / CB;
  const int cl = tid % CB, pl = tid / CB;
  const int c = by * CB + cl;
  const bool ok = pl < PL && c < C;
  const int b0 = bx * slice;
  const int b1 = b0 + slice < nparts ? b0 + slice : nparts;
  if (pl == 0 && c < C) {  // pivot: mean of the first non-empty part of the slice
    float k = 0.f;
    for (int b = b0; b < b1; ++b) {
      if (merge_ld(parts + (long)b * 3 * C + c, COH) != 0.f) {
        k = merge_ld(parts + (long)b * 3 * C + C + c, COH);
        break;
      }
    }
    piv[cl] = k;
  }
  __syncthreads();
  double n = 0.0, a1 = 0.0, a2 = 0.0;
  if (ok) {
    const double k = (double)piv[cl];
#pragma unroll 4
    for (int b = b0 + pl; b < b1; b += PL) {
      const float* p = parts + (long)b * 3 * C + c;
      const double nb = (double)merge_ld(p, COH);
      const double d = (double)merge_ld(p + C, COH) - k;
      const double q = nb * d;
      n += nb;
      a1 += q;
      a2 += (double)merge_ld(p + 2 * C, COH) + q * d;
    }
  }
  sn[tid] = n;
  s1[tid] = a1;
  s2[tid] = a2;
  __syncthreads();
  if (PL > 32) {
    // many part lanes (narrow channel blocks): lanes [g*LG, (g+1)*LG) added in order by lane g of
    // 16 groups, then the 16 group sums by lane 0 — a fixed order with short serial chains
    const int LG = (PL + 15) / 16;
    double gn = 0.0, g1 = 0.0, g2 = 0.0;
    if (ok && pl < 16) {
      for (int l = pl * LG; l < (pl + 1) * LG && l < PL; ++l) {
        gn += sn[l * CB + cl];
        g1 += s1[l * CB + cl];
        g2 += s2[l * CB + cl];
      }
    }
    __syncthreads();
    if (ok && pl < 16) {
      sn[tid] = gn;
      s1[tid] = g1;
      s2[tid] = g2;
    }
    __syncthreads();
    if (ok && pl == 0) {
      n = gn;
      a1 = g1;
      a2 = g2;
      for (int l = 1; l < 16; ++l) {
        n += sn[l * CB + cl];
        a1 += s1[l * CB + cl];
        a2 += s2[l * CB + cl];
      }
    }
  } else if (ok && pl == 0) {
    for (int l = 1; l < PL; ++l) {
      n += sn[l * CB + cl];
      a1 += s1[l * CB + cl];
      a2 += s2[l * CB + cl];
    }
  }
  if (ok && pl == 0) {
    const double k = (double)piv[cl];
    const double mu = n > 0.0 ? k + a1 / n : 0.0;
    const double m2 = n > 0.0 ? fmax(a2 - a1 * a1 / n, 0.0) : 0.0;
    if (!last) {
      float* o = out + (long)bx * 3 * C + c;
      __hip_atomic_store(o, (float)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + C, (float)mu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 2 * C, (float)m2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    const double var = m2 / (double)M;
    const float mu_f = (float)mu;
    const float vf = (float)var;
    mean[c] = mu_f;
    rstd[c] = (float)(1.0 / sqrt((double)vf + (double)eps));
    if (mmean != nullptr) {
      // slim: assign_moving_average(zero_debias=False): v -= (v - value) * (1 - decay)
      const float one_m = 1.0f - decay;
      const float unbiased = M > 1 ? (float)(m2 / (double)(M - 1)) : vf;
      mmean[c] = mmean[c] - (mmean[c] - mu_f) * one_m;
      mvar[c] = mvar[c] - (mvar[c] - unbiased) * one_m;
    }
  }
}

__global__ void __launch_bounds__(MERGE_T) bn_parts_merge_kernel(const float* parts, int nparts, int C, int CB,
                                                             int slice, float* out, long M, float eps,
                                                             float decay, float* __restrict__ mean,
                                                             float* __restrict__ rstd, float* __restrict__ mmean,
                                                             float* __restrict__ mvar, unsigned* cnt, int slice2) {
  __shared__ double sn[MERGE_T], s1[MERGE_T], s2[MERGE_T];
  __shared__ float piv[64];
  __shared__ int is_last;
  const bool one = gridDim.x == 1;
  merge_slice<false>(parts, nparts, C, CB, slice, blockIdx.x, blockIdx.y, one, out, M, eps, decay, mean, rstd, mmean, mvar,
              sn, s1, s2, piv);
  if (cnt == nullptr || one) return;
  // Second level in the same launch: the last block of channel group blockIdx.y to finish merges
  // the gridDim.x slice parts as one slice of the next level's plan — the grouping and order of a
  // second launch (bit-identical to it), without the launch.  The part's agent-scope stores have
  // completed (vmcnt 0, before the barrier) when the block counts itself; the last block reads the
  // parts with agent-scope loads issued after it has seen the count.
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(cnt + blockIdx.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = prev == gridDim.x - 1;
    // self-cleaning: the counter is zero again for the next call (and every graph replay)
    if (is_last) __hip_atomic_store(cnt + blockIdx.y, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!is_last) return;
  // The release side: every block's parts went out as agent-scope (sc1, L2-coherent across the
  // XCDs) stores, completed (vmcnt 0) before its thread 0 counted the block.  The acquire side,
  // here: an agent-scope acquire fence in the last block (only one block per channel group pays
  // for it) before its agent-scope loads of the parts, so the hand-off holds by the memory model,
  // not only by how gfx950 compiles the relaxed accesses.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  merge_slice<true>(out, gridDim.x, C, CB, slice2, 0, blockIdx.y, true, nullptr, M, eps, decay, mean, rstd, mmean, mvar, sn,
              s1, s2, piv);
}

// merge levels until one part remains; ws holds two ping-pong part buffers
static size_t finalize_ws_bytes(int nparts, int C) {
  const MergePlan p = merge_plan(C, nparts);
  const int s1 = cdiv(nparts, p.slice);
  return s1 > 1 ? 2 * (size_t)s1 * 3 * C * sizeof(float) : 0;
}
// Zero-initialised per-device arrival counters of the single-launch two-level merge; each counter
// is zero again when its launch ends.  Two ranges: eager calls take counters round-robin from the
// first 65,536 (a 720p training step takes ~1,300, so calls that may run at the same time on the
// head-chain streams never share one); a call being captured into a HIP graph takes counters of
// its own from the second range, which are never handed out again — a graph's replays can then
// overlap eager merges or another graph's replays without sharing a counter.  When the graph
// range is used up (~800 captured training steps in one process) captured calls fall back to two
// launches (bit-identical).  The pool is allocated on first use outside a stream capture; a call
// captured before that also falls back.  ROD_MERGE_TWO_LAUNCH=1 (read per call): always two launches.
static unsigned* merge_counters(int n, hipStream_t s) {
  const char* e = getenv("ROD_MERGE_TWO_LAUNCH");
  if (e != nullptr && atoi(e) == 1) return nullptr;
  constexpr int POOL = 1 << 16, GPOOL = 1 << 20, MAXDEV = 64;
  static unsigned* base[MAXDEV] = {};
  static int next[MAXDEV] = {};
  static int gnext[MAXDEV] = {};
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV || n > POOL) return nullptr;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) return nullptr;
  const bool capturing = st != hipStreamCaptureStatusNone;
  std::lock_guard<std::mutex> g(mu);
  if (base[dev] == nullptr) {
    if (capturing) return nullptr;
    void* p = nullptr;
    const size_t bytes = (size_t)(POOL + GPOOL) * sizeof(unsigned);
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    if (hipMemsetAsync(p, 0, bytes, s) != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    (void)hipStreamSynchronize(s);   // zeroed before any other stream takes a counter
    base[dev] = (unsigned*)p;
  }
  if (capturing) {
    if (gnext[dev] + n > GPOOL) return nullptr;
    unsigned* r = base[dev] + POOL + gnext[dev];
    gnext[dev] += n;
    return r;
  }
  if (next[dev] + n > POOL) next[dev] = 0;
  unsigned* r = base[dev] + next[dev];
  next[dev] += n;
  return r;
}

static void finalize_launch(const float* parts, int nparts, long M, int C, float eps, float decay, float* mean,
                            float* rstd, float* mm, float* mv, float* ws, hipStream_t s) {
  const MergePlan p0 = merge_plan(C, nparts);
  const int s1 = cdiv(nparts, p0.slice);
  float* buf[2] = {ws, ws ? ws + (size_t)s1 * 3 * C : nullptr};
  unsigned* cnt = nullptr;
  int slice2 = 0;
  if (s1 > 1) {
    // two levels in one launch when the second is one slice with the same channel blocks
    const MergePlan p1 = merge_plan(C, s1);
    if (p1.CB == p0.CB && s1 <= p1.slice && (cnt = merge_counters(cdiv(C, p0.CB), s)) != nullptr) slice2 = p1.slice;
  }
  static const bool dbg = getenv("ROD_DEBUG_MERGE") != nullptr;
  if (dbg)
    fprintf(stderr, "rod merge: nparts %d C %d M %ld levels %d launches %d\n", nparts, C, M, s1 > 1 ? 2 : 1,
            s1 > 1 && cnt == nullptr ? 2 : 1);
  if (cnt != nullptr) {
    hipLaunchKernelGGL(bn_parts_merge_kernel, dim3(s1, cdiv(C, p0.CB)), dim3(MERGE_T), 0, s, parts, nparts, C, p0.CB,
                       p0.slice, buf[0], M, eps, decay, mean, rstd, mm, mv, cnt, slice2);
    return;
  }
  int k = 0;
  while (true) {
    const MergePlan p = merge_plan(C, nparts);
    const int S = cdiv(nparts, p.slice);
    hipLaunchKernelGGL(bn_parts_merge_kernel, dim3(S, cdiv(C, p.CB)), dim3(MERGE_T), 0, s, parts, nparts, C, p.CB, p.slice,
                       S > 1 ? buf[k] : nullptr, M, eps, decay, mean, rstd, mm, mv, (unsigned*)nullptr, 0);
    if (S == 1) break;
    parts = buf[k];
    nparts = S;
    k ^= 1;
  }
}

__global__ void bn_eval_stats_kernel(const float* __restrict__ mm, const float* __restrict__ mv, float eps,
                                     float* __restrict__ mean, float* __restrict__ rstd, int C) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = mm[c];
  rstd[c] = (float)(1.0 / sqrt((double)mv[c] + (double)eps));
}

// ---------------------------------------------------------------- apply
template <typename T, bool VEC, bool RES>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, const T* __restrict__ res,
                                                       T* __restrict__ y, long M, int C, int ldx, int ldr, int ldy,
                                                       int act) {
  constexpr int V = VEC ? Vec16<T>::N : 1;
  const int CV = C / V;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;  // multiple of CV
  const int c = (int)(t0 % CV) * V;
  const long rstep = stride / CV;
  float sc[V], sh[V];
#pragma unroll
  for (int v = 0; v < V; ++v) bn_affine(mean, rstd, gamma, beta, c + v, sc[v], sh[v]);
  auto row = [&](float (&xv)[V], const float (&rv)[V]) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float z = act_fwd(fmaf(xv[v], sc[v], sh[v]), act);
      if constexpr (RES) z = z + rv[v];
      xv[v] = z;
    }
  };
  long r = t0 / CV;
  for (; r + 3 * rstep < M; r += 4 * rstep) {  // four rows in flight per thread
    float xa[4][V], ra[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      load_v<T, VEC>(x + (r + u * rstep) * ldx + c, xa[u]);
      if constexpr (RES) load_v<T, VEC>(res + (r + u * rstep) * ldr + c, ra[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      row(xa[u], ra[u]);
      store_v<T, VEC>(y + (r + u * rstep) * ldy + c, xa[u]);
    }
  }
  for (; r < M; r += rstep) {
    float xv[V], rv[V];
    load_v<T, VEC>(x + r * ldx + c, xv);
    if constexpr (RES) load_v<T, VEC>(res + r * ldr + c, rv);
    row(xv, rv);
    store_v<T, VEC>(y + r * ldy + c, xv);
  }
}

// ---------------------------------------------------------------- backward
// PIPE: the row batches are software-pipelined (batch k+1's loads issued before batch k's
// arithmetic, ping-pong registers), so a wave keeps loads in flight while it computes; same
// rows in the same order as the plain loop (sums bit-identical)
template <typename T, bool VEC, bool PM = false, int U = 4, bool PIPE = false>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, long M, int C, int lddy,
                                                            int ldx, int act, int CVb, int lanes, long chunk,
                                                            float* __restrict__ slab) {
  constexpr int V = VEC ? Vec16<T>::N : 1;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][256][V]
  const int tid = threadIdx.x;
  const int cvl = tid % CVb, pln = tid / CVb;
  const int CV = C / V;
  const int cv = blockIdx.y * CVb + cvl;
  const bool active = pln < lanes && cv < CV;
  const int c = cv * V;
  const long r0 = (long)blockIdx.x * chunk;
  const long r1 = r0 + chunk < M ? r0 + chunk : M;
  float sg[V], sgx[V], mu[V], rs[V], sc[V], sh[V];
#pragma unroll
  for (int v = 0; v < V; ++v) sg[v] = sgx[v] = 0.f;
  if (active) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      mu[v] = mean[c + v];
      rs[v] = rstd[c + v];
      bn_affine(mean, rstd, gamma, beta, c + v, sc[v], sh[v]);
    }
    auto acc = [&](const float (&xv)[V], const float (&gv)[V]) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float d = xv[v] - mu[v];
        const float z = fmaf(xv[v], sc[v], sh[v]);
        const float g = gv[v] * act_grad(z, act);
        sg[v] += g;
        sgx[v] = fmaf(g, d * rs[v], sgx[v]);
      }
    };
    long r = r0 + pln;
    if constexpr (PIPE) {
      const long step = (long)U * lanes;
      auto full = [&](long rr) { return rr + (U - 1L) * lanes < r1; };
      static_assert(VEC, "the pipelined form holds raw 16-byte vectors");
      Vec16<T> xa[2][U], ga[2][U];  // raw (bf16: 4 VGPRs per 8 values), widened at use
      auto ld = [&](int b, long rr) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          xa[b][u].load(x + (rr + (long)u * lanes) * ldx + c);
          ga[b][u].load(dy + (rr + (long)u * lanes) * lddy + c);
        }
      };
      auto use = [&](int b) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float xv[V], gv[V];
#pragma unroll
          for (int v = 0; v < V; ++v) {
            xv[v] = xa[b][u].get(v);
            gv[v] = ga[b][u].get(v);
          }
          acc(xv, gv);
        }
      };
      if (full(r)) ld(0, r);
      while (full(r)) {
        if (full(r + step)) ld(1, r + step);
        use(0);
        r += step;
        if (!full(r)) break;
        if (full(r + step)) ld(0, r + step);
        use(1);
        r += step;
      }
    } else {
      for (; r + (U - 1L) * lanes < r1; r += (long)U * lanes) {
        float xa[U][V], ga[U][V];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          load_v<T, VEC>(x + (r + (long)u * lanes) * ldx + c, xa[u]);
          load_v<T, VEC>(dy + (r + (long)u * lanes) * lddy + c, ga[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc(xa[u], ga[u]);
      }
    }
    for (; r < r1; r += lanes) {
      float xv[V], gv[V];
      load_v<T, VEC>(x + r * ldx + c, xv);
      load_v<T, VEC>(dy + r * lddy + c, gv);
      acc(xv, gv);
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    red[tid * V + v] = sg[v];
    red[(256 + tid) * V + v] = sgx[v];
  }
  __syncthreads();
  for (int e = tid; e < CVb * V; e += 256) {
    const int cb = e / V, v = e - cb * V;
    const int cg = blockIdx.y * CVb + cb;
    if (cg >= CV) continue;
    float a = 0.f, b = 0.f;
    for (int l = 0; l < lanes; ++l) {
      a += red[(l * CVb + cb) * V + v];
      b += red[(256 + l * CVb + cb) * V + v];
    }
    if constexpr (PM) {  // part-major [nparts][2][C] (rod_bn_bwd_finalize)
      slab[(long)blockIdx.x * 2 * C + cg * V + v] = a;
      slab[(long)blockIdx.x * 2 * C + C + cg * V + v] = b;
    } else {
      const long nblk = gridDim.x;
      slab[(long)(cg * V + v) * nblk + blockIdx.x] = a;
      slab[((long)C + cg * V + v) * nblk + blockIdx.x] = b;
    }
  }
}

__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(const float* __restrict__ slab, int nblk, long M, int C,
                                                              const float* __restrict__ rstd,
                                                              const float* __restrict__ gamma,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ coef) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  const float* pa = slab + (long)c * nblk;
  const float* pb = slab + ((long)C + c) * nblk;
  // four independent chains per lane: the slab loads of a wave are issued 8 at a time
  // instead of one dependent f64 add per load round trip
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, b0 = 0.0, b1 = 0.0, b2 = 0.0, b3 = 0.0;
  int k = lane;
  for (; k + 192 < nblk; k += 256) {
    a0 += (double)pa[k];
    a1 += (double)pa[k + 64];
    a2 += (double)pa[k + 128];
    a3 += (double)pa[k + 192];
    b0 += (double)pb[k];
    b1 += (double)pb[k + 64];
    b2 += (double)pb[k + 128];
    b3 += (double)pb[k + 192];
  }
  for (; k < nblk; k += 64) {
    a0 += (double)pa[k];
    b0 += (double)pb[k];
  }
  const double sg = wave_sum_f64((a0 + a1) + (a2 + a3));
  const double sgx = wave_sum_f64((b0 + b1) + (b2 + b3));
  if (lane != 0) return;
  if (dbeta) dbeta[c] = (float)sg;
  if (dgamma) dgamma[c] = (float)sgx;
  coef[c] = gamma ? rstd[c] * gamma[c] : rstd[c];
  coef[C + c] = (float)(sg / (double)M);
  coef[2 * C + c] = (float)(sgx / (double)M);
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ coef, T* __restrict__ dx,
                                                           long M, int C, int lddy, int ldx, int lddx, int act) {
  constexpr int V = VEC ? Vec16<T>::N : 1;
  const int CV = C / V;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  const int c = (int)(t0 % CV) * V;
  const long rstep = stride / CV;
  float sc[V], sh[V], a[V], k1[V], k0[V], km[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    bn_affine(mean, rstd, gamma, beta, c + v, sc[v], sh[v]);
    a[v] = coef[c + v];
    bn_bwd_k<T>(a[v], mean[c + v], rstd[c + v], coef[C + c + v], coef[2 * C + c + v], k1[v], k0[v], km[v]);
  }
  auto row = [&](float (&xv)[V], const float (&gv)[V]) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float z = fmaf(xv[v], sc[v], sh[v]);
      const float g = gv[v] * act_grad(z, act);
      xv[v] = bn_bwd_apply1<T>(a[v], g, k1[v], k0[v], km[v], xv[v]);
    }
  };
  long r = t0 / CV;
  // four rows per iteration, loads first: the small-M launches give each thread only a few
  // rows, so memory-level parallelism per thread decides their speed
  for (; r + 3 * rstep < M; r += 4 * rstep) {
    float xa[4][V], ga[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      load_v<T, VEC>(x + (r + u * rstep) * ldx + c, xa[u]);
      load_v<T, VEC>(dy + (r + u * rstep) * lddy + c, ga[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      row(xa[u], ga[u]);
      store_nt<T, VEC>(dx + (r + u * rstep) * lddx + c, xa[u]);
    }
  }
  for (; r < M; r += rstep) {
    float xv[V], gv[V];
    load_v<T, VEC>(x + r * ldx + c, xv);
    load_v<T, VEC>(dy + r * lddy + c, gv);
    row(xv, gv);
    store_nt<T, VEC>(dx + r * lddx + c, xv);
  }
}

// Small tensors (M <= SMALL_M rows) in ONE launch: each 1024-thread block owns CVb channel
// vectors over ALL rows — reduce (fp32 per lane; lanes merged in f64 by wave shuffles, then the
// 16 wave partials in LDS, fixed order), the coefficients, then (dx != NULL) the apply pass
// over the same rows, which the block has just read (L2-hot).  The three-launch reduce ->
// finalize -> apply chain costs 15-45 us on such tensors, mostly launch boundaries and the
// finalize's dependent loads.
constexpr int SMALL_T = 1024;
constexpr long SMALL_M = 4096;
constexpr int SMALL_CVB = 4;   // channel vectors per block (measured: 4 < 8 < 16 on the step's shapes)
// the one-launch path needs >= 8 channel groups to spread over CUs (C >= 256 bf16 / 128 fp32);
// narrower small tensors keep the three-launch chain (measured faster for 4096 x 64)
static bool small_ok(long M, int CV) { return M <= SMALL_M && CV >= 8 * SMALL_CVB; }

__device__ __forceinline__ double shfl_xor_f64(double v, int o) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __shfl_xor(lo, o, 64);
  hi = __shfl_xor(hi, o, 64);
  return __hiloint2double(hi, lo);
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(SMALL_T) bn_bwd_small_kernel(const T* __restrict__ dz, const T* __restrict__ y,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, long M, int C,
                                                               int act, int CVb, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta, float* __restrict__ coef,
                                                               T* __restrict__ dx) {
  constexpr int V = VEC ? Vec16<T>::N : 1;
  constexpr int NW = SMALL_T / 64;
  __shared__ double red[2][NW][16 * V];
  __shared__ float cf[3][16 * V];
  const int tid = threadIdx.x;
  const int lanes = SMALL_T / CVb;       // CVb a power of two <= 16
  const int cvl = tid % CVb, pln = tid / CVb;
  const int CV = C / V;
  const int cv = blockIdx.x * CVb + cvl;
  const bool active = cv < CV;
  const int c = cv * V;
  float sg[V], sgx[V], mu[V], rs[V], sc[V], sh[V];
#pragma unroll
  for (int v = 0; v < V; ++v) sg[v] = sgx[v] = 0.f;
  if (active) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      mu[v] = mean[c + v];
      rs[v] = rstd[c + v];
      bn_affine(mean, rstd, gamma, beta, c + v, sc[v], sh[v]);
    }
    long r = pln;
    for (; r + 3L * lanes < M; r += 4L * lanes) {
      float xa[4][V], ga[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        load_v<T, VEC>(y + (r + (long)u * lanes) * C + c, xa[u]);
        load_v<T, VEC>(dz + (r + (long)u * lanes) * C + c, ga[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float g = ga[u][v] * act_grad(fmaf(xa[u][v], sc[v], sh[v]), act);
          sg[v] += g;
          sgx[v] = fmaf(g, (xa[u][v] - mu[v]) * rs[v], sgx[v]);
        }
    }
    for (; r < M; r += lanes) {
      float xv[V], gv[V];
      load_v<T, VEC>(y + r * C + c, xv);
      load_v<T, VEC>(dz + r * C + c, gv);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float g = gv[v] * act_grad(fmaf(xv[v], sc[v], sh[v]), act);
        sg[v] += g;
        sgx[v] = fmaf(g, (xv[v] - mu[v]) * rs[v], sgx[v]);
      }
    }
  }
  // the lanes of one channel vector inside a wave sit CVb apart: xor-shuffle tree in f64
  const int wave = tid >> 6;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    double a = (double)sg[v], b = (double)sgx[v];
    for (int o = CVb; o < 64; o <<= 1) {
      a += shfl_xor_f64(a, o);
      b += shfl_xor_f64(b, o);
    }
    if ((tid & 63) < CVb) {
      red[0][wave][cvl * V + v] = a;
      red[1][wave][cvl * V + v] = b;
    }
  }
  __syncthreads();
  if (tid < CVb * V) {
    const int cb = tid / V, v = tid - cb * V;
    const int cg = blockIdx.x * CVb + cb;
    if (cg < CV) {
      double a = 0.0, b = 0.0;
      for (int w = 0; w < NW; ++w) {
        a += red[0][w][cb * V + v];
        b += red[1][w][cb * V + v];
      }
      const int ch = cg * V + v;
      const float c0 = gamma ? rstd[ch] * gamma[ch] : rstd[ch];
      const float c1 = (float)(a / (double)M), c2 = (float)(b / (double)M);
      if (dbeta) dbeta[ch] = (float)a;
      if (dgamma) dgamma[ch] = (float)b;
      if (coef) {
        coef[ch] = c0;
        coef[C + ch] = c1;
        coef[2 * C + ch] = c2;
      }
      cf[0][cb * V + v] = c0;
      cf[1][cb * V + v] = c1;
      cf[2][cb * V + v] = c2;
    }
  }
  if (dx == nullptr) return;
  __syncthreads();
  if (!active) return;
  float a[V], k1[V], k0[V], km[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    a[v] = cf[0][cvl * V + v];
    bn_bwd_k<T>(a[v], mu[v], rs[v], cf[1][cvl * V + v], cf[2][cvl * V + v], k1[v], k0[v], km[v]);
  }
  auto row = [&](float (&xv)[V], const float (&gv)[V]) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float g = gv[v] * act_grad(fmaf(xv[v], sc[v], sh[v]), act);
      xv[v] = bn_bwd_apply1<T>(a[v], g, k1[v], k0[v], km[v], xv[v]);
    }
  };
  long r = pln;
  for (; r + 3L * lanes < M; r += 4L * lanes) {
    float xa[4][V], ga[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      load_v<T, VEC>(y + (r + (long)u * lanes) * C + c, xa[u]);
      load_v<T, VEC>(dz + (r + (long)u * lanes) * C + c, ga[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      row(xa[u], ga[u]);
      store_v<T, VEC>(dx + (r + (long)u * lanes) * C + c, xa[u]);
    }
  }
  for (; r < M; r += lanes) {
    float xv[V], gv[V];
    load_v<T, VEC>(y + r * C + c, xv);
    load_v<T, VEC>(dz + r * C + c, gv);
    row(xv, gv);
    store_v<T, VEC>(dx + r * C + c, xv);
  }
}

// Small path launch: SMALL_CVB channel vectors per 1024-thread block (256 row lanes).
template <typename T>
static void small_launch(bool vec, const void* dz, const void* y, const float* mean, const float* rstd,
                         const float* gamma, const float* beta, long M, int C, int act, float* dgamma, float* dbeta,
                         float* coef, void* dx, hipStream_t s) {
  const int V = vec ? Vec16<T>::N : 1;
  const int CV = C / V;
  const int CVb = SMALL_CVB;
  if (vec)
    hipLaunchKernelGGL((bn_bwd_small_kernel<T, true>), dim3(cdiv(CV, CVb)), dim3(SMALL_T), 0, s, (const T*)dz,
                       (const T*)y, mean, rstd, gamma, beta, M, C, act, CVb, dgamma, dbeta, coef, (T*)dx);
  else
    hipLaunchKernelGGL((bn_bwd_small_kernel<T, false>), dim3(cdiv(CV, CVb)), dim3(SMALL_T), 0, s, (const T*)dz,
                       (const T*)y, mean, rstd, gamma, beta, M, C, act, CVb, dgamma, dbeta, coef, (T*)dx);
}

template <typename T>
static bool vec_ok(int C, std::initializer_list<std::pair<const void*, int>> bufs) {
  const int V = Vec16<T>::N;
  if (C % V) return false;
  for (auto& b : bufs) {
    if (b.first == nullptr) continue;
    if (((uintptr_t)b.first & 15) != 0) return false;
    if (b.second % V) return false;
  }
  return true;
}

// Threads for the row-streaming apply kernels: >= ~8 rows per thread on large tensors (the
// per-thread coefficient loads amortised), but at least 256 blocks' worth on small ones.
static long apply_threads(long total) { return std::max(total / 8, std::min(total, 256L * 256)); }
// grid cap of the apply kernels: ROD_TUNE_APPLY_CAP = 0 -> 2048 blocks, -1 -> one resident wave
// Grid cap of the apply kernels (68-84 VGPRs: 6-7 blocks of 256 per CU resident): one partial
// wave of 768 blocks with more rows per thread for mid-size tensors (<= 12M thread-rows:
// 115200 x 384 147 -> 120 us, 460800 x 192 231 -> 209 us), 1792 (7 per CU) for the large ones
// (tools/bn_bench.py sweep).
static int apply_target(long thread_rows) { return thread_rows <= (12L << 20) ? 768 : 1792; }

static int max_nbx(long M, int C) {
  int a = red_plan<float>(M, C, false).nbx;
  int b = red_plan<float>(M, C, C % 4 == 0).nbx;
  int c = red_plan<bf16_t>(M, C, C % 8 == 0).nbx;
  return std::max(a, std::max(b, c));
}

template <typename T>
static void apply_launch(bool vec, const void* x, const float* mean, const float* rstd, const float* gamma,
                         const float* beta, const void* res, void* y, long M, int C, int ldx, int ldr, int ldy,
                         int act, hipStream_t s) {
  const int V = vec ? Vec16<T>::N : 1;
  const int blocks = const_channel_blocks(C / V, apply_threads(M * (C / V)), apply_target(M * (C / V)));
#define LA(VE, RE)                                                                                            \
  hipLaunchKernelGGL((bn_apply_kernel<T, VE, RE>), dim3(blocks), dim3(256), 0, s, (const T*)x, mean, rstd, gamma, \
                     beta, (const T*)res, (T*)y, M, C, ldx, ldr, ldy, act)
  if (vec) {
    if (res) LA(true, true); else LA(true, false);
  } else {
    if (res) LA(false, true); else LA(false, false);
  }
#undef LA
}

template <typename T>
static void stats_launch(bool vec, const void* x, long M, int C, int ldx, float eps, float decay, float* mean,
                         float* rstd, float* mm, float* mv, float* slab, hipStream_t s) {
  RedPlan pl = red_plan<T>(M, C, vec);
  dim3 grid(pl.nbx, pl.cgroups);
  size_t lds = 2 * 256 * pl.V * sizeof(float);
  if (vec)
    hipLaunchKernelGGL((bn_stats_kernel<T, true>), grid, dim3(256), lds, s, (const T*)x, M, C, ldx, pl.CVb, pl.lanes,
                       pl.chunk, slab);
  else
    hipLaunchKernelGGL((bn_stats_kernel<T, false>), grid, dim3(256), lds, s, (const T*)x, M, C, ldx, pl.CVb,
                       pl.lanes, pl.chunk, slab);
  finalize_launch(slab, pl.nbx, M, C, eps, decay, mean, rstd, mm, mv, slab + (size_t)pl.nbx * 3 * C, s);
}

// Partial statistics of y[M, C] (row stride ld) as exactly `nparts` parts of
// ceil(M / nparts) rows: the fallback for producers that cannot fuse the statistics.
template <typename T>
static void stat_parts_typed(const void* y, long M, int C, int ld, float* parts, int nparts, hipStream_t s) {
  const bool vec = vec_ok<T>(C, {{y, ld}});
  RedPlan pl = red_plan<T>(M, C, vec);
  pl.chunk = cdivl(M, nparts);
  dim3 grid(nparts, pl.cgroups);
  size_t lds = 2 * 256 * pl.V * sizeof(float);
  if (vec)
    hipLaunchKernelGGL((bn_stats_kernel<T, true>), grid, dim3(256), lds, s, (const T*)y, M, C, ld, pl.CVb, pl.lanes,
                       pl.chunk, parts);
  else
    hipLaunchKernelGGL((bn_stats_kernel<T, false>), grid, dim3(256), lds, s, (const T*)y, M, C, ld, pl.CVb,
                       pl.lanes, pl.chunk, parts);
}

void stat_parts(int dtype, const void* y, long M, int C, int ld, float* parts, int nparts, hipStream_t s) {
  if (dtype == ROD_F32) stat_parts_typed<float>(y, M, C, ld, parts, nparts, s);
  else stat_parts_typed<bf16_t>(y, M, C, ld, parts, nparts, s);
}

template <typename T>
static void bwd_launch(bool vec, const void* dy, const void* x, const float* mean, const float* rstd,
                       const float* gamma, const float* beta, void* dx, float* dgamma, float* dbeta, float* slab,
                       float* coef, long M, int C, int lddy, int ldx, int lddx, int act, hipStream_t s) {
  RedPlan pl = red_plan<T>(M, C, vec);
  dim3 grid(pl.nbx, pl.cgroups);
  size_t lds = 2 * 256 * pl.V * sizeof(float);
  if (vec)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true>), grid, dim3(256), lds, s, (const T*)dy, (const T*)x, mean,
                       rstd, gamma, beta, M, C, lddy, ldx, act, pl.CVb, pl.lanes, pl.chunk, slab);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, false>), grid, dim3(256), lds, s, (const T*)dy, (const T*)x, mean,
                       rstd, gamma, beta, M, C, lddy, ldx, act, pl.CVb, pl.lanes, pl.chunk, slab);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(cdiv(C, 4)), dim3(256), 0, s, slab, pl.nbx, M, C, rstd, gamma,
                     dgamma, dbeta, coef);
  const int V = pl.V;
  // >= ~8 rows per thread so the per-thread coefficient loads (7 x V floats) are amortised
  const int blocks = const_channel_blocks(
      C / V, apply_threads(M * (C / V)),
      apply_target(M * (C / V)));
  if (vec)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true>), dim3(blocks), dim3(256), 0, s, (const T*)dy, (const T*)x, mean,
                       rstd, gamma, beta, coef, (T*)dx, M, C, lddy, ldx, lddx, act);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, false>), dim3(blocks), dim3(256), 0, s, (const T*)dy, (const T*)x,
                       mean, rstd, gamma, beta, coef, (T*)dx, M, C, lddy, ldx, lddx, act);
}

// rod_bn_bwd_finalize in one launch: block b owns channels [b*CB/2, (b+1)*CB/2) and both of their
// columns (sum g at c, sum g*yhat at C + c) of the part-major [nparts][2][C] slab.  Every column
// is summed exactly as slab_sum_kernel<CB> sums it — part rows ty, ty + L, ... over L = 256/CB
// lanes, four chains per lane, the lanes added in ty order, rounded to float — so the sums, and
// dbeta, dgamma and the coefficients bn_bwd_apply_kernel uses, (rstd*gamma, mean g, mean g*yhat),
// formed from those rounded sums, are bit-identical to the round-4 two-launch form.
template <int CB>
__global__ void __launch_bounds__(256) bn_bwd_finalize1_kernel(const float* __restrict__ parts, int nparts, long M,
                                                               int C, const float* __restrict__ rstd,
                                                               const float* __restrict__ gamma,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                               float* __restrict__ coef) {
  constexpr int L = 256 / CB, H = CB / 2;
  __shared__ double red[L][CB + 1];
  __shared__ float tot[CB];
  const int tx = threadIdx.x % CB, ty = threadIdx.x / CB;
  const int c = blockIdx.x * H + tx % H;
  const bool ok = c < C;
  const long n = 2L * C;
  const long i = (long)(tx / H) * C + c;   // the column slab_sum would give this sum
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (ok) {
    int b = ty;
    for (; b + 3 * L < nparts; b += 4 * L) {
      s0 += (double)parts[(long)b * n + i];
      s1 += (double)parts[(long)(b + L) * n + i];
      s2 += (double)parts[(long)(b + 2 * L) * n + i];
      s3 += (double)parts[(long)(b + 3 * L) * n + i];
    }
    for (; b < nparts; b += L) s0 += (double)parts[(long)b * n + i];
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0) {
    double t = 0.0;
    for (int k = 0; k < L; ++k) t += red[k][tx];
    tot[tx] = (float)t;
  }
  __syncthreads();
  if (ty == 0 && tx < H && ok) {
    const float sg = tot[tx], sgx = tot[tx + H];
    if (dbeta) dbeta[c] = sg;
    if (dgamma) dgamma[c] = sgx;
    coef[c] = gamma ? rstd[c] * gamma[c] : rstd[c];
    coef[C + c] = (float)((double)sg / (double)M);
    coef[2 * C + c] = (float)((double)sgx / (double)M);
  }
}

// Backward partial sums [nparts][2][C] of g = dz*act'(u), g*yhat over exactly nparts row
// chunks: the fallback for producers of dz that cannot fuse the reduction.
template <typename T>
static void gred_pass_typed(const void* dz, const void* y, const BnPro& p, long M, int C, float* parts, int nparts,
                            hipStream_t s) {
  const bool vec = vec_ok<T>(C, {{dz, C}, {y, C}});
  RedPlan pl = red_plan<T>(M, C, vec);
  pl.chunk = cdivl(M, nparts);
  dim3 grid(nparts, pl.cgroups);
  size_t lds = 2 * 256 * pl.V * sizeof(float);
  if (vec)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true, true>), grid, dim3(256), lds, s, (const T*)dz, (const T*)y,
                       p.mean, p.rstd, p.gamma, p.beta, M, C, C, C, p.act, pl.CVb, pl.lanes, pl.chunk, parts);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, false, true>), grid, dim3(256), lds, s, (const T*)dz, (const T*)y,
                       p.mean, p.rstd, p.gamma, p.beta, M, C, C, C, p.act, pl.CVb, pl.lanes, pl.chunk, parts);
}
void gred_parts(int dtype, const void* dz, const void* y, const BnPro& p, long M, int C, float* parts, int nparts,
                hipStream_t s) {
  if (dtype == ROD_F32) gred_pass_typed<float>(dz, y, p, M, C, parts, nparts, s);
  else gred_pass_typed<bf16_t>(dz, y, p, M, C, parts, nparts, s);
}

}  // namespace rod

using namespace rod;

extern "C" {

int rod_bn_bwd_finalize(const float* parts, int nparts, long M, int C, const float* rstd, const float* gamma,
                        float* dgamma, float* dbeta, float* coef, void* stream) {
  ROD_CHECK_ARG(parts != nullptr && nparts > 0 && M > 0 && C > 0 && coef != nullptr && rstd != nullptr,
                "rod_bn_bwd_finalize: bad arguments");
  hipStream_t s = ROD_STREAM(stream);
  // one launch: slab_sum's f64 fixed-order column sums and the coefficients
  const int cb = slab_cb(nparts, 2L * C);
  const dim3 grid(cdiv(C, cb / 2));
  if (cb == 32)
    hipLaunchKernelGGL(bn_bwd_finalize1_kernel<32>, grid, dim3(256), 0, s, parts, nparts, M, C, rstd, gamma, dgamma,
                       dbeta, coef);
  else if (cb == 8)
    hipLaunchKernelGGL(bn_bwd_finalize1_kernel<8>, grid, dim3(256), 0, s, parts, nparts, M, C, rstd, gamma, dgamma,
                       dbeta, coef);
  else
    hipLaunchKernelGGL(bn_bwd_finalize1_kernel<4>, grid, dim3(256), 0, s, parts, nparts, M, C, rstd, gamma, dgamma,
                       dbeta, coef);
  return check_launch("rod_bn_bwd_finalize");
}

int rod_bn_bwd_apply(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                     const float* beta, const float* coef, void* dy, long M, int C, int act, int dtype, void* stream) {
  ROD_CHECK_ARG(M > 0 && C > 0 && coef != nullptr, "rod_bn_bwd_apply: bad arguments");
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, {
    const bool vec = vec_ok<T>(C, {{dz, C}, {y, C}, {dy, C}});
    const int V = vec ? Vec16<T>::N : 1;
    const int blocks = const_channel_blocks(
        C / V, apply_threads(M * (C / V)),
        apply_target(M * (C / V)));
    if (vec)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true>), dim3(blocks), dim3(256), 0, s, (const T*)dz, (const T*)y,
                         mean, rstd, gamma, beta, coef, (T*)dy, M, C, C, C, C, act);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, false>), dim3(blocks), dim3(256), 0, s, (const T*)dz, (const T*)y,
                         mean, rstd, gamma, beta, coef, (T*)dy, M, C, C, C, C, act);
  });
  return check_launch("rod_bn_bwd_apply");
}

// Partial statistics only (ABI 8), for a BatchNorm whose statistics are merged over more
// rows than this process holds (SyncBN over data-parallel ranks).
int rod_bn_stat_parts(const void* x, long M, int C, float* parts, int nparts, int dtype, void* stream) {
  ROD_CHECK_ARG(x != nullptr && parts != nullptr && M > 0 && C > 0 && nparts > 0 && nparts <= M,
                "rod_bn_stat_parts: bad arguments M=%ld C=%d nparts=%d", M, C, nparts);
  stat_parts(dtype, x, M, C, C, parts, nparts, ROD_STREAM(stream));
  return check_launch("rod_bn_stat_parts");
}

int rod_bn_bwd_parts(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                     const float* beta, int act, float* parts, int nparts, long M, int C, int dtype, void* stream) {
  ROD_CHECK_ARG(dz != nullptr && y != nullptr && mean != nullptr && rstd != nullptr && parts != nullptr && M > 0 &&
                    C > 0 && nparts > 0 && nparts <= M,
                "rod_bn_bwd_parts: bad arguments M=%ld C=%d nparts=%d", M, C, nparts);
  ROD_CHECK_ARG(act >= ROD_ACT_NONE && act <= ROD_ACT_RELU, "rod_bn_bwd_parts: bad act %d", act);
  BnPro p;
  p.mean = mean;
  p.rstd = rstd;
  p.gamma = gamma;
  p.beta = beta;
  p.act = act;
  gred_parts(dtype, dz, y, p, M, C, parts, nparts, ROD_STREAM(stream));
  return check_launch("rod_bn_bwd_parts");
}

size_t rod_bn_stats_workspace(long M, int C) {
  const int nbx = max_nbx(M, C);
  return (size_t)nbx * 3 * C * sizeof(float) + finalize_ws_bytes(nbx, C);
}

size_t rod_bn_finalize_workspace(int nparts, int C) { return finalize_ws_bytes(nparts, C); }

int rod_bn_finalize(const float* parts, int nparts, long M, int C, float eps, float decay, float* mean, float* rstd,
                    float* moving_mean, float* moving_var, void* workspace, void* stream) {
  ROD_CHECK_ARG(parts != nullptr && nparts > 0 && M > 0 && C > 0, "rod_bn_finalize: bad arguments");
  ROD_CHECK_ARG((moving_mean == nullptr) == (moving_var == nullptr), "rod_bn_finalize: moving stats mismatch");
  ROD_CHECK_ARG(workspace != nullptr || finalize_ws_bytes(nparts, C) == 0, "rod_bn_finalize: workspace is NULL");
  finalize_launch(parts, nparts, M, C, eps, decay, mean, rstd, moving_mean, moving_var, (float*)workspace,
                  ROD_STREAM(stream));
  return check_launch("rod_bn_finalize");
}

int rod_bn_stats(const void* x, long M, int C, int ldx, float eps, float decay, float* mean, float* rstd,
                 float* moving_mean, float* moving_var, void* workspace, int dtype, void* stream) {
  ROD_CHECK_ARG(M > 0 && C > 0, "rod_bn_stats: bad shape M=%ld C=%d", M, C);
  if (ldx == 0) ldx = C;
  ROD_CHECK_ARG(ldx >= C, "rod_bn_stats: ldx < C");
  ROD_CHECK_ARG((moving_mean == nullptr) == (moving_var == nullptr), "rod_bn_stats: moving stats mismatch");
  ROD_CHECK_ARG(workspace != nullptr, "rod_bn_stats: workspace is NULL");
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, stats_launch<T>(vec_ok<T>(C, {{x, ldx}}), x, M, C, ldx, eps, decay, mean, rstd,
                                            moving_mean, moving_var, (float*)workspace, s));
  return check_launch("rod_bn_stats");
}

int rod_bn_eval_stats(const float* moving_mean, const float* moving_var, float eps, float* mean, float* rstd, int C,
                      void* stream) {
  ROD_CHECK_ARG(C > 0, "rod_bn_eval_stats: C <= 0");
  hipLaunchKernelGGL(bn_eval_stats_kernel, dim3(cdiv(C, 256)), dim3(256), 0, ROD_STREAM(stream), moving_mean,
                     moving_var, eps, mean, rstd, C);
  return check_launch("rod_bn_eval_stats");
}

int rod_bn_apply(const void* x, const float* mean, const float* rstd, const float* gamma, const float* beta,
                 const void* residual, void* y, long M, int C, int ldx, int ldr, int ldy, int act, int dtype,
                 void* stream) {
  ROD_CHECK_ARG(M > 0 && C > 0, "rod_bn_apply: bad shape");
  ROD_CHECK_ARG(act >= ROD_ACT_NONE && act <= ROD_ACT_RELU, "rod_bn_apply: bad act %d", act);
  if (ldx == 0) ldx = C;
  if (ldy == 0) ldy = C;
  if (ldr == 0) ldr = C;
  ROD_CHECK_ARG(ldx >= C && ldy >= C && ldr >= C, "rod_bn_apply: leading dim < C");
  hipStream_t s = ROD_STREAM(stream);
  ROD_DISPATCH_DTYPE(dtype, apply_launch<T>(vec_ok<T>(C, {{x, ldx}, {y, ldy}, {residual, ldr}}), x, mean, rstd,
                                            gamma, beta, residual, y, M, C, ldx, ldr, ldy, act, s));
  return check_launch("rod_bn_apply");
}

size_t rod_bn_bwd_workspace(long M, int C) {
  return (size_t)max_nbx(M, C) * 2 * C * sizeof(float) + (size_t)3 * C * sizeof(float) + 16;
}

// reduce + finalize only: (dgamma, dbeta, coef[3][C]) for a consumer that applies the
// BatchNorm backward itself (rod_pw_bwd; the apply pass is never written out)
int rod_bn_bwd_reduce(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                      const float* beta, float* dgamma, float* dbeta, float* coef, void* workspace, long M, int C,
                      int act, int dtype, void* stream) {
  ROD_CHECK_ARG(M > 0 && C > 0 && coef != nullptr, "rod_bn_bwd_reduce: bad arguments");
  ROD_CHECK_ARG(workspace != nullptr, "rod_bn_bwd_reduce: workspace is NULL");
  hipStream_t s = ROD_STREAM(stream);
  float* slab = (float*)workspace;
  ROD_DISPATCH_DTYPE(dtype, {
    const bool vec = vec_ok<T>(C, {{dz, C}, {y, C}});
    if (small_ok(M, C / (vec ? Vec16<T>::N : 1))) {
      small_launch<T>(vec, dz, y, mean, rstd, gamma, beta, M, C, act, dgamma, dbeta, coef, nullptr, s);
      return check_launch("rod_bn_bwd_reduce");
    }
    // the backward reduce aims at 512 blocks (fewer, longer row chunks per block than the
    // statistics' 1024: tools/bn_bench.py total 3558 -> 3455 us, 460800 x 192 208 -> 182 us);
    // ROD_BN_RED_WANT overrides (A/B switch).  <= the 1024 plan's blocks, so the workspace
    // bound (max_nbx) holds
    static const long red_want = getenv("ROD_BN_RED_WANT") ? atol(getenv("ROD_BN_RED_WANT")) : 512;
    RedPlan pl = red_plan<T>(M, C, vec, std::min<long>(red_want, 1024));
    dim3 grid(pl.nbx, pl.cgroups);
    size_t lds = 2 * 256 * pl.V * sizeof(float);
    // eight rows (16 loads) in flight per lane instead of four on the large tensors (>= 64 M
    // elements: 1471 -> 1401 us at 7372800 x 96, 567 -> 541 us at 1843200 x 144 for reduce + apply,
    // bit-identical; the mid-size ones lose, e.g. 28800 x 576 77 -> 85 us; tools/bn_bench.py).
    // ROD_BN_RED_U=4 / 8 forces one form
    static const int red_u = getenv("ROD_BN_RED_U") ? atoi(getenv("ROD_BN_RED_U")) : 0;
    const bool u8 = red_u == 8 || (red_u == 0 && (long)M * C >= (64L << 20));
    // the large tensors take the software-pipelined form (4-row batches, ping-pong): the step's
    // shapes in tools/bn_bench.py 7372800 x 96 1459 -> 1369 us, x 32 480 -> 448, x 16 248 -> 231,
    // 1843200 x 144 571 -> 528, 460800 x 192 203 -> 187 (reduce + apply, bit-identical); the
    // mid-size ones are neutral to +3 us.  ROD_BN_RED_PIPE=0 keeps the 8-row form
    static const bool red_pipe = !(getenv("ROD_BN_RED_PIPE") && atoi(getenv("ROD_BN_RED_PIPE")) == 0);
    if (vec && u8 && red_pipe)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true, false, 4, true>), grid, dim3(256), lds, s, (const T*)dz,
                         (const T*)y, mean, rstd, gamma, beta, M, C, C, C, act, pl.CVb, pl.lanes, pl.chunk, slab);
    else if (vec && u8)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true, false, 8>), grid, dim3(256), lds, s, (const T*)dz,
                         (const T*)y, mean, rstd, gamma, beta, M, C, C, C, act, pl.CVb, pl.lanes, pl.chunk, slab);
    else if (vec)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true>), grid, dim3(256), lds, s, (const T*)dz, (const T*)y, mean,
                         rstd, gamma, beta, M, C, C, C, act, pl.CVb, pl.lanes, pl.chunk, slab);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, false>), grid, dim3(256), lds, s, (const T*)dz, (const T*)y, mean,
                         rstd, gamma, beta, M, C, C, C, act, pl.CVb, pl.lanes, pl.chunk, slab);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(cdiv(C, 4)), dim3(256), 0, s, slab, pl.nbx, M, C, rstd, gamma,
                       dgamma, dbeta, coef);
  });
  return check_launch("rod_bn_bwd_reduce");
}

int rod_bn_bwd(const void* dy, const void* x, const float* mean, const float* rstd, const float* gamma,
               const float* beta, void* dx, float* dgamma, float* dbeta, void* workspace, long M, int C, int lddy,
               int ldx, int lddx, int act, int dtype, void* stream) {
  ROD_CHECK_ARG(M > 0 && C > 0, "rod_bn_bwd: bad shape");
  ROD_CHECK_ARG(workspace != nullptr, "rod_bn_bwd: workspace is NULL");
  if (lddy == 0) lddy = C;
  if (ldx == 0) ldx = C;
  if (lddx == 0) lddx = C;
  ROD_CHECK_ARG(lddy >= C && ldx >= C && lddx >= C, "rod_bn_bwd: leading dim < C");
  hipStream_t s = ROD_STREAM(stream);
  float* slab = (float*)workspace;
  float* coef = slab + (size_t)max_nbx(M, C) * 2 * C;  // after the largest slab
  if (M <= SMALL_M && lddy == C && ldx == C && lddx == C) {
    ROD_DISPATCH_DTYPE(dtype, {
      const bool vec = vec_ok<T>(C, {{dy, C}, {x, C}, {dx, C}});
      if (small_ok(M, C / (vec ? Vec16<T>::N : 1))) {
        small_launch<T>(vec, dy, x, mean, rstd, gamma, beta, M, C, act, dgamma, dbeta, coef, dx, s);
        return check_launch("rod_bn_bwd");
      }
    });
  }
  ROD_DISPATCH_DTYPE(dtype, bwd_launch<T>(vec_ok<T>(C, {{dy, lddy}, {x, ldx}, {dx, lddx}}), dy, x, mean, rstd, gamma,
                                          beta, dx, dgamma, dbeta, slab, coef, M, C, lddy, ldx, lddx, act, s));
  return check_launch("rod_bn_bwd");
}

}  // extern "C"
