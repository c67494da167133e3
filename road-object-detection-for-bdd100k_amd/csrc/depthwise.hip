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
#include "dw_common.h"

namespace rod {

// template value of the prologue activation meaning "any, chosen at run time" (act_fwd);
// RELU6 gets its own instantiation, -1 = no prologue
constexpr int DW_ACT_RT = 99;


constexpr int DW_RB = 8;  // output rows per thread (forward / backward-data strips)

// Forward: thread = (channel vector cv, output column wo), strip of DW_RB output rows; the
// 3x3 input window rolls down in fp32 registers (one new input row per output row for S=1,
// two for S=2) and lanes of a wave read consecutive channel vectors of neighbouring pixels.
// The row(s) the NEXT output row adds are prefetched raw before this row's FMAs and only
// converted when they enter the window, so one row of arithmetic covers the load latency.
// PACT: BatchNorm-apply prologue on the input (rod_common.h): -1 none, ROD_ACT_RELU6 the
// fixed ReLU6 form, 3 any activation (runtime); padding stays 0.
template <typename T, int V, int PACT>
struct DwIn {
  float sc[PACT >= 0 ? V : 1], sh[PACT >= 0 ? V : 1];
  int act;
  __device__ __forceinline__ void init(const BnPro& p, int c) {
    if constexpr (PACT >= 0) {
#pragma unroll
      for (int v = 0; v < V; ++v) bn_pro_affine(p, c + v, sc[v], sh[v]);
      act = p.act;
    }
  }
  // raw pack -> fp32 window entry (the activation the reference convolves, rounded to T)
  __device__ __forceinline__ void cvt(const PackV<T, V>& p, bool ok, float (&o)[V]) const {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float a = p.get(v);
      if constexpr (PACT >= 0) {
        float z = fmaf(a, sc[v], sh[v]);
        z = PACT == ROD_ACT_RELU6 ? act_t<ROD_ACT_RELU6>(z) : act_fwd(z, act);
        a = ok ? to_f32(from_f32<T>(z)) : 0.f;
      }
      o[v] = a;
    }
  }
};

template <typename T, int S, int V, bool STATS, int PACT = -1>
__global__ void __launch_bounds__(256) dw3x3_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                        T* __restrict__ y, int H, int W, int C, int pt, int pl,
                                                        int Ho, int Wo, float* __restrict__ parts,
                                                        BnPro pro = BnPro{}) {
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(t % CV);
  const int wo = (int)(t / CV);
  const bool active = wo < Wo;
  const int ho0 = blockIdx.y * DW_RB;
  const int ho1 = ho0 + DW_RB < Ho ? ho0 + DW_RB : Ho;
  const int n = blockIdx.z;
  const int c = cv * V;
  // STATS: shifted sums of this thread's rounded outputs (pivot = its first output), for
  // its (n, mean, M2) per channel
  float piv[V], s1[V], s2[V];
#pragma unroll
  for (int v = 0; v < V; ++v) piv[v] = s1[v] = s2[v] = 0.f;
  if (active) {
    float wr[9][V];
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int v = 0; v < V; ++v) wr[k][v] = w[k * C + c + v];
    DwIn<T, V, PACT> in;
    in.init(pro, c);
    const T* xn = x + (long)n * H * W * C + c;
    T* yn = y + (long)n * Ho * Wo * C + c;
    float xr[3][3][V];
    PackV<T, V> nx[S][3];
    bool nok[S][3];
    auto load_row = [&](PackV<T, V>(&row)[3], bool (&ok)[3], int hi) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int wi = wo * S - pl + j;
        ok[j] = hi >= 0 && hi < H && wi >= 0 && wi < W;
        if (ok[j]) row[j].load(xn + ((long)hi * W + wi) * C);
        else row[j].zero();
      }
    };
    auto prefetch = [&](int ho) {
#pragma unroll
      for (int q = 0; q < S; ++q) load_row(nx[q], nok[q], ho * S - pt + 3 - S + q);
    };
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      PackV<T, V> r0[3];
      bool k0[3];
      load_row(r0, k0, ho0 * S - pt + i);
#pragma unroll
      for (int j = 0; j < 3; ++j) in.cvt(r0[j], k0[j], xr[i][j]);
    }
    if (ho0 + 1 < ho1) prefetch(ho0 + 1);
#pragma unroll
    for (int q = 0; q < DW_RB; ++q) {
      const int ho = ho0 + q;
      if (ho >= ho1) break;
      float acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] = fmaf(xr[i][j][v], wr[i * 3 + j][v], acc[v]);
      PackV<T, V> o;
#pragma unroll
      for (int v = 0; v < V; ++v) o.set(v, acc[v]);
      o.store_out(yn + ((long)ho * Wo + wo) * C);
      if constexpr (STATS) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float ov = o.get(v);
          if (q == 0) piv[v] = ov;
          const float d = ov - piv[v];
          s1[v] += d;
          s2[v] = fmaf(d, d, s2[v]);
        }
      }
      if (ho + 1 < ho1) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          if constexpr (S == 1) {
#pragma unroll
            for (int v = 0; v < V; ++v) {
              xr[0][j][v] = xr[1][j][v];
              xr[1][j][v] = xr[2][j][v];
            }
            in.cvt(nx[0][j], nok[0][j], xr[2][j]);
          } else {
#pragma unroll
            for (int v = 0; v < V; ++v) xr[0][j][v] = xr[2][j][v];
            in.cvt(nx[0][j], nok[0][j], xr[1][j]);
            in.cvt(nx[1][j], nok[1][j], xr[2][j]);
          }
        }
        if (ho + 2 < ho1) prefetch(ho + 2);
      }
    }
  }
  if constexpr (STATS) {
    // per thread: (mean, M2) of its <= DW_RB rows from the pivot-shifted sums; per block:
    // Chan merge of the threads holding each channel vector, in thread order, into part
    // (z*gy + y)*gx + x of the [nparts][3][C] slab
    __shared__ float sn[256], sm[256 * V], sq[256 * V];
    const int tid = threadIdx.x;
    const int nr = active ? ho1 - ho0 : 0;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float inv = nr > 0 ? 1.f / (float)nr : 0.f;
      const float dm = s1[v] * inv;
      sm[tid * V + v] = piv[v] + dm;
      sq[tid * V + v] = nr > 0 ? fmaxf(s2[v] - s1[v] * dm, 0.f) : 0.f;
    }
    sn[tid] = (float)nr;
    __syncthreads();
    const long tb = (long)blockIdx.x * 256;
    const int t0mod = (int)(tb % CV);
    const long part = ((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    for (int e = tid; e < C; e += 256) {
      const int cve = e / V, v = e - cve * V;
      int tl = cve - t0mod;
      if (tl < 0) tl += CV;
      float pn = 0.f, pm = 0.f, pq = 0.f;
      for (; tl < 256; tl += CV) chan_merge(pn, pm, pq, sn[tl], sm[tl * V + v], sq[tl * V + v]);
      store_stat_part(parts, C, part, e, pn, pm, pq);
    }
  }
}

// GRED (backward-data kernels): BatchNorm-backward partial sums of the rounded dx against the
// pre-BatchNorm y of the layer below (rod_common.h gred_acc), per thread, then per block into
// part (z*gy + y)*gx + x of [nparts][2][C].
template <int V>
struct DwGred {
  float sc[V], sh[V], mu[V], rs[V], sg[V], sgx[V];
  __device__ __forceinline__ void init(const BnGred& g, int c, bool ok) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      sg[v] = sgx[v] = 0.f;
      sc[v] = sh[v] = mu[v] = rs[v] = 0.f;
      if (ok) gred_coef(g.p, c + v, sc[v], sh[v], mu[v], rs[v]);
    }
  }
  template <typename T>
  __device__ __forceinline__ void acc(const PackV<T, V>& dz, const T* yp, int act) {
    PackV<T, V> yv;
    yv.load(yp);
#pragma unroll
    for (int v = 0; v < V; ++v) gred_acc(dz.get(v), yv.get(v), sc[v], sh[v], mu[v], rs[v], act, sg[v], sgx[v]);
  }
  // block sums: threads holding channel vector cve sit at tl = (cve - tb) mod CV + k*CV
  __device__ __forceinline__ void flush(float* red, int C, int CV, float* parts) {
    const int tid = threadIdx.x;
    const long tb = (long)blockIdx.x * 256;
    const int t0mod = (int)(tb % CV);
    const long part = ((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int v = 0; v < V; ++v) red[tid * V + v] = q == 0 ? sg[v] : sgx[v];
      __syncthreads();
      for (int e = tid; e < C; e += 256) {
        const int cve = e / V, v = e - cve * V;
        int tl = cve - t0mod;
        if (tl < 0) tl += CV;
        float a = 0.f;
        for (; tl < 256; tl += CV) a += red[tl * V + v];
        parts[part * 2 * C + q * C + e] = a;
      }
      __syncthreads();
    }
  }
};

// =====================================================================================
// LDS neighbour-exchange engine (forward).
//
// A block owns a tile of P input columns x CVb 16-byte channel vectors (Cc = CVb*V channels)
// and a strip of RB output rows.  Thread (p, cvb) loads ONE 16-byte vector per input row
// (S=2: two, its column pair) — each input byte crosses the memory system once, in full
// CVb*16-byte pixel segments — applies the BatchNorm prologue to it in registers, and
// publishes it in an LDS row slot; its left / right taps come back from the neighbouring
// threads' slots.  Rows stream through a 3-deep (S=2: 4-deep) register prefetch ring, the
// three output rows in progress are rolling fp32 accumulators, and the LDS slot is double
// buffered so each input row costs one barrier.  Halo columns (S=1: one each side, S=2: one
// on the right) load but do not compute.  Accumulation order per output is tap (0,0) ..
// (2,2), the order of dw3x3_fwd_kernel, so both kernels round identically.
// =====================================================================================
// One 16-byte LDS-DMA (global_load_lds_dwordx4) per lane: lane l of the wave lands at
// lds_wave + 16*l.  Issued from inline asm so that hipcc's wait-count bookkeeping does not
// drain it (it would put vmcnt(0) before every LDS read); completion is counted by hand
// with s_waitcnt vmcnt(N) — loads retire in issue order, so N = DMAs issued later.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_wave) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"((unsigned)__builtin_amdgcn_readfirstlane((int)lds_wave))
               : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// FLIP (S=1 only): the correlation with the flipped taps w[2-i][2-j] — the stride-1
// backward-data (DepthwiseConv2dNativeBackpropInput) is this kernel on dy with pads
// (2-pt, 2-pl).  GRED: the BatchNorm-backward partial sums of the rounded outputs against the
// pre-BatchNorm y of the layer below (rod_common.h), y prefetched two rows ahead.
template <typename T, int S, int PACT, bool STATS, bool FLIP, bool GRED, int V = Vec16<T>::N>
__device__ __forceinline__ void dw_lx_body(const T* __restrict__ x, const float* __restrict__ w, T* __restrict__ y,
                                           int H, int W, int C, int pt, int pl, int Ho, int Wo, const DwTile& tl,
                                           float* __restrict__ parts, const BnPro& pro, const BnGred& gr) {
  static_assert(S == 1 || !(FLIP || GRED), "the backward-data form is stride 1");
  typedef PackV<T, V> PK;  // 16-byte packs, or 8-byte (bf16 x 4: half the per-thread state)
  // LDS: prefetch ring of D input rows (S=2: column pairs) + the double-buffered exchange
  // slot; the statistics merge reuses the front after the row loop
  constexpr int XS = 2 * 256 * 16;            // double-buffered exchange slot
  constexpr int SS = STATS ? (256 * (2 * V + 1) + 3 * 512) * 4 : (GRED ? 256 * 2 * V * 4 : 0);
  __shared__ __attribute__((aligned(16))) char smem[XS > SS ? XS : SS];
  T* xs = (T*)smem;
  const int tid = threadIdx.x;
  const int CVb = tl.CVb, P = tl.P;
  const int p = tid / CVb, cvb = tid - (tid / CVb) * CVb;
  int bx, strip, n;
  xcd_block(bx, strip, n);
  const int cg = bx % tl.cgroups, ct = bx / tl.cgroups;
  const int c = (cg * CVb + cvb) * V;
  const int wo0 = ct * tl.TWo;
  const int ho0 = strip * tl.RB;
  const int ho1 = ho0 + tl.RB < Ho ? ho0 + tl.RB : Ho;
  constexpr int HL = S == 1 ? 1 : 0;
  const int wo = wo0 + p - HL;
  const bool comp = p >= HL && p <= P - 2 && wo < Wo;
  // input columns of this thread
  const int ci0 = S == 1 ? wo0 + p - pl : 2 * (wo0 + p) - pl;
  const bool cok0 = p < P && ci0 >= 0 && ci0 < W;
  const bool cok1 = S == 2 && p < P && ci0 + 1 >= 0 && ci0 + 1 < W;

  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = w[(FLIP ? 8 - k : k) * C + c + v];
  DwIn<T, V, PACT> in;
  in.init(pro, c);
  const T* xn = x + (long)n * H * W * C + c;
  T* yn = y + (long)n * Ho * Wo * C + c;

  float piv[V], s1[V], s2[V];
#pragma unroll
  for (int v = 0; v < V; ++v) piv[v] = s1[v] = s2[v] = 0.f;
  DwGred<GRED ? V : 1> gd;
  if constexpr (GRED) gd.init(gr, c, comp);
  const T* gyn = GRED ? (const T*)gr.y + (long)n * Ho * Wo * C + c : nullptr;
  PackV<T, V> gring[GRED ? 3 : 1];

  auto cvt = [&](const PK& r, bool ok, float (&o)[V]) {
    in.cvt(r, ok, o);
    if constexpr (PACT < 0) {
#pragma unroll
      for (int v = 0; v < V; ++v) o[v] = ok ? o[v] : 0.f;
    }
  };
  auto publish = [&](const float (&o)[V], int buf) {
    PK st;
#pragma unroll
    for (int v = 0; v < V; ++v) st.set(v, o[v]);
    st.store(xs + (buf * 256 + tid) * V);
  };
  // Buffer I/O (rod_common.h): every load is issued (rows / columns clamped into the map, uses
  // masked by rok), every output store too (lane offset ROD_OOB off the strip and on halo lanes),
  // and every lane runs the row arithmetic (neighbours from clamped slots; halo results are
  // dropped), so no memory operation sits under a branch and the prefetch ring's wait counts
  // stay exact.  The GRED form (opt-in) keeps its conditional y loads.
  const unsigned es = sizeof(T);
  const rsrc_t rxs = rod_rsrc(xn - c, (unsigned)((long)H * W * C * es));
  const rsrc_t rys = rod_rsrc(yn - c, (unsigned)((long)Ho * Wo * C * es));
  const rsrc_t rnull = rod_rsrc(yn - c, 0u);   // rows off the strip: every store dropped
  const int cc0 = ci0 < 0 ? 0 : (ci0 >= W ? W - 1 : ci0);
  const int cc1 = ci0 + 1 < 0 ? 0 : (ci0 + 1 >= W ? W - 1 : ci0 + 1);
  const unsigned vx0 = (unsigned)(((long)cc0 * C + c) * es), vx1 = (unsigned)(((long)cc1 * C + c) * es);
  const unsigned vy = comp ? (unsigned)(((long)wo * C + c) * es) : ROD_OOB;
  const unsigned rsx = (unsigned)(W * C * es), rsy = (unsigned)(Wo * C * es);
  const int li = tid >= CVb ? tid - CVb : tid, ri = tid + CVb < 256 ? tid + CVb : tid;
  auto emit = [&](const float (&a)[V], int ho, bool valid, bool first) {
    PK o;
#pragma unroll
    for (int v = 0; v < V; ++v) o.set(v, a[v]);
    // statistics of the rounded outputs, then the store (fenced: rod_common.h buf_st)
    if constexpr (STATS) {
      if (valid) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float ov = o.get(v);
          if (first) piv[v] = ov;
          const float d = ov - piv[v];
          s1[v] += d;
          s2[v] = fmaf(d, d, s2[v]);
        }
      }
    }
    o.bstore(valid ? rys : rnull, vy, (unsigned)(valid ? ho : 0) * rsy);
  };
  auto emit_g = [&](const float (&a)[V], int ho, int gslot) {  // GRED: y of row ho is in gring[gslot]
    PackV<T, V> o;
#pragma unroll
    for (int v = 0; v < V; ++v) o.set(v, a[v]);
    o.store_out(yn + ((long)ho * Wo + wo) * C);
    if constexpr (GRED) {
#pragma unroll
      for (int v = 0; v < V; ++v)
        gred_acc(o.get(v), gring[gslot].get(v), gd.sc[v], gd.sh[v], gd.mu[v], gd.rs[v], gr.p.act, gd.sg[v], gd.sgx[v]);
    }
  };

  if constexpr (S == 1) {
    const int hi0 = ho0 - pt;
    const int nin = ho1 - ho0 + 2;
    PK ring[3];
    bool rok[3];
    auto issue = [&](int k, int q) {
      const int hi = hi0 + q;
      rok[k] = cok0 && q < nin && hi >= 0 && hi < H;
      const int hc = hi < 0 ? 0 : (hi >= H ? H - 1 : hi);
      ring[k].bload(rxs, vx0, (unsigned)hc * rsx);
    };
#pragma unroll
    for (int k = 0; k < 3; ++k) {   // slot order, so the loop header's wait is the same on entry
      issue(k, k);
      __builtin_amdgcn_sched_barrier(0);
    }
    // GRED: y of output row m is loaded at input row q = m into slot m % 3 (two rows ahead)
    auto gissue = [&](int k, int m) {
      if constexpr (GRED) {
        if (comp && ho0 + m < ho1) gring[k].load(gyn + ((long)(ho0 + m) * Wo + wo) * C);
      }
    };
    float acc[3][V];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[a][v] = 0.f;
    for (int q0 = 0; q0 < nin; q0 += 3) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int q = q0 + k;
        const int buf = q & 1;
        float cen[V];
        cvt(ring[k], rok[k], cen);
        __builtin_amdgcn_sched_barrier(0);   // the slot's reload stays after its last read
        issue(k, q + 3);
        gissue(k, q);
        publish(cen, buf);
        __syncthreads();
        PK L, R;
        L.load(xs + (buf * 256 + li) * V);
        R.load(xs + (buf * 256 + ri) * V);
        // row q feeds output m = q - i with weight row i: slot (k - i) mod 3
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int sl = (k - i + 3) % 3;
#pragma unroll
          for (int v = 0; v < V; ++v) {
            float a = acc[sl][v];
            a = fmaf(L.get(v), wr[i * 3][v], a);
            a = fmaf(cen[v], wr[i * 3 + 1][v], a);
            a = fmaf(R.get(v), wr[i * 3 + 2][v], a);
            acc[sl][v] = a;
          }
        }
        const int sd = (k + 1) % 3;  // output m = q - 2 is complete
        const int m = q - 2;
        if constexpr (GRED) {
          if (comp && m >= 0 && ho0 + m < ho1) emit_g(acc[sd], ho0 + m, sd);
        } else {
          emit(acc[sd], ho0 + m, m >= 0 && ho0 + m < ho1, m == 0);
        }
#pragma unroll
        for (int v = 0; v < V; ++v) acc[sd][v] = 0.f;
      }
    }
  } else {
    const int hi0 = 2 * ho0 - pt;
    const int nin = 2 * (ho1 - ho0) + 1;
    PK ring[4][2];
    bool rok[4][2];
    auto issue = [&](int k, int q) {
      const int hi = hi0 + q;
      const bool rowok = q < nin && hi >= 0 && hi < H;
      rok[k][0] = rowok && cok0;
      rok[k][1] = rowok && cok1;
      const int hc = hi < 0 ? 0 : (hi >= H ? H - 1 : hi);
      ring[k][0].bload(rxs, vx0, (unsigned)hc * rsx);
      ring[k][1].bload(rxs, vx1, (unsigned)hc * rsx);
    };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      issue(k, k);
      __builtin_amdgcn_sched_barrier(0);
    }
    float acc[2][V];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[a][v] = 0.f;
    for (int q0 = 0; q0 < nin; q0 += 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = q0 + k;
        const int buf = q & 1;
        float c0[V], c1[V];
        cvt(ring[k][0], rok[k][0], c0);
        cvt(ring[k][1], rok[k][1], c1);
        __builtin_amdgcn_sched_barrier(0);
        issue(k, q + 4);
        publish(c0, buf);
        __syncthreads();
        PK R;
        R.load(xs + (buf * 256 + ri) * V);
        // q = q0 + k, q0 % 4 == 0: k even -> weight row 0 into output q/2 (slot k/2) and
        // row 2 into output q/2 - 1 (slot 1 - k/2, then complete); k odd -> row 1 into
        // output (q-1)/2 (slot k/2)
        auto addrow = [&](int i, int sl) {
#pragma unroll
          for (int v = 0; v < V; ++v) {
            float a = acc[sl][v];
            a = fmaf(c0[v], wr[i * 3][v], a);
            a = fmaf(c1[v], wr[i * 3 + 1][v], a);
            a = fmaf(R.get(v), wr[i * 3 + 2][v], a);
            acc[sl][v] = a;
          }
        };
        if ((k & 1) == 0) {
          const int sn = k >> 1, sd = 1 - (k >> 1);
          addrow(2, sd);
          const int m = (q >> 1) - 1;
          emit(acc[sd], ho0 + m, m >= 0 && ho0 + m < ho1, m == 0);
#pragma unroll
          for (int v = 0; v < V; ++v) acc[sd][v] = 0.f;
          addrow(0, sn);
        } else {
          addrow(1, k >> 1);
        }
      }
    }
  }

  if constexpr (GRED) {
    // per channel: sum over the computing columns in column order -> part
    // (n*strips + strip)*coltiles + ct, channels of cgroup cg
    __syncthreads();
    float* ga = (float*)smem;
    float* gb = ga + 256 * V;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      ga[tid * V + v] = gd.sg[v];
      gb[tid * V + v] = gd.sgx[v];
    }
    __syncthreads();
    const int Cc = CVb * V;
    const long part = ((long)n * tl.strips + strip) * tl.coltiles + ct;
    for (int e = tid; e < Cc; e += 256) {
      const int cve = e / V, v = e - cve * V;
      float a = 0.f, b = 0.f;
      for (int pp = HL; pp <= P - 2; ++pp) {
        a += ga[(pp * CVb + cve) * V + v];
        b += gb[(pp * CVb + cve) * V + v];
      }
      gr.parts[part * 2 * C + cg * Cc + e] = a;
      gr.parts[part * 2 * C + C + cg * Cc + e] = b;
    }
  }
  if constexpr (STATS) {
    // per thread (n, mean, M2) of its rows; per channel, Chan merge over the computing
    // columns in column order -> part (n*strips + strip)*coltiles + ct, channels of cgroup cg
    __syncthreads();
    float* sm = (float*)smem;
    float* sq = sm + 256 * V;
    float* sn = sq + 256 * V;
    const int nr = comp ? ho1 - ho0 : 0;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float inv = nr > 0 ? 1.f / (float)nr : 0.f;
      const float dm = s1[v] * inv;
      sm[tid * V + v] = piv[v] + dm;
      sq[tid * V + v] = nr > 0 ? fmaxf(s2[v] - s1[v] * dm, 0.f) : 0.f;
    }
    sn[tid] = (float)nr;
    __syncthreads();
    // two levels (runs of 8 columns, then the runs, each in column order) so the serial
    // merge depth is ~8 + P/8 rather than P
    const int Cc = CVb * V;
    const int nrun = (P + 7) / 8;
    float* l1n = sn + 256;
    float* l1m = l1n + 512;
    float* l1q = l1m + 512;
    for (int e = tid; e < Cc * nrun; e += 256) {
      const int ch = e % Cc, run = e / Cc;
      const int cve = ch / V, v = ch - cve * V;
      float pn = 0.f, pm = 0.f, pq = 0.f;
      for (int pp = run * 8; pp < run * 8 + 8 && pp < P; ++pp) {
        const int t2 = pp * CVb + cve;
        chan_merge(pn, pm, pq, sn[t2], sm[t2 * V + v], sq[t2 * V + v]);
      }
      l1n[e] = pn;
      l1m[e] = pm;
      l1q[e] = pq;
    }
    __syncthreads();
    const long part = ((long)n * tl.strips + strip) * tl.coltiles + ct;
    for (int ch = tid; ch < Cc; ch += 256) {
      float pn = 0.f, pm = 0.f, pq = 0.f;
      for (int run = 0; run < nrun; ++run) chan_merge(pn, pm, pq, l1n[run * Cc + ch], l1m[run * Cc + ch], l1q[run * Cc + ch]);
      store_stat_part(parts, C, part, cg * Cc + ch, pn, pm, pq);
    }
  }
}

template <typename T, int S, int PACT, bool STATS, int V = Vec16<T>::N>
__global__ void __launch_bounds__(256) dw3x3_fwd_lx_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                           T* __restrict__ y, int H, int W, int C, int pt, int pl,
                                                           int Ho, int Wo, DwTile tl, float* __restrict__ parts,
                                                           BnPro pro) {
  dw_lx_body<T, S, PACT, STATS, false, false, V>(x, w, y, H, W, C, pt, pl, Ho, Wo, tl, parts, pro, BnGred{});
}
// stride-1 backward-data (DepthwiseConv2dNativeBackpropInput): the body with flipped taps
template <typename T, bool GRED>
__global__ void __launch_bounds__(256) dw3x3_bwd_data_lx_kernel(const T* __restrict__ dy, const float* __restrict__ w,
                                                                T* __restrict__ dx, int Ho, int Wo, int C, int pt,
                                                                int pl, int H, int W, DwTile tl, BnGred gr) {
  dw_lx_body<T, 1, -1, false, true, GRED>(dy, w, dx, Ho, Wo, C, pt, pl, H, W, tl, nullptr, BnPro{}, gr);
}

// Filter gradient on the LDS-exchange engine: dw[i][j][c] = sum dy[n,ho,wo,c] *
// z[n, ho*S-pt+i, wo*S-pl+j, c], z = the forward's input (BatchNorm prologue applied when
// PACT >= 0).  Input rows stream exactly as in dw3x3_fwd_lx_kernel (register ring, one LDS
// exchange per row); dy of the thread's own output column rides a register queue loaded three
// (S=2: five) input rows ahead; the 9 taps accumulate in fp32 registers; per block the
// computing columns are summed per channel in column order into part (n*strips + strip)*
// coltiles + ct of the [parts][9][C] slab (channels of cgroup cg).
// GP (rod_dw3x3_bwd_filter_bn): `dy` holds dz, the gradient at this depthwise's BatchNorm +
// activation output; the dy queue loads dz and the pre-BatchNorm y of the same pixel and forms
// the BatchNorm-backward apply in registers (rod_bn_bwd_apply's arithmetic, rounded to T) when
// the row enters the queue, contracts that value and stores it once to gd.dy (every output
// pixel belongs to exactly one thread's computing column / strip / channel group).
struct DwGrad {
  const void* y;
  const float *mean, *rstd, *gamma, *beta, *coef;
  int act;
  void* dy;
};
template <typename T, int S, int PACT, bool GP = false>
__global__ void __launch_bounds__(256) dw3x3_bwdw_lx_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                            float* __restrict__ slab, int H, int W, int C, int pt,
                                                            int pl, int Ho, int Wo, DwTile tl, BnPro pro,
                                                            DwGrad gd = DwGrad{}) {
  constexpr int V = Vec16<T>::N;
  constexpr int XS = 2 * 256 * 16;
  constexpr int SS = 256 * V * 4;
  __shared__ __attribute__((aligned(16))) char smem[XS > SS ? XS : SS];
  T* xs = (T*)smem;
  const int tid = threadIdx.x;
  const int CVb = tl.CVb, P = tl.P;
  const int p = tid / CVb, cvb = tid - (tid / CVb) * CVb;
  int bx, strip, n;
  xcd_block(bx, strip, n);
  const int cg = bx % tl.cgroups, ct = bx / tl.cgroups;
  const int c = (cg * CVb + cvb) * V;
  const int wo0 = ct * tl.TWo;
  const int ho0 = strip * tl.RB;
  const int ho1 = ho0 + tl.RB < Ho ? ho0 + tl.RB : Ho;
  constexpr int HL = S == 1 ? 1 : 0;
  const int wo = wo0 + p - HL;
  const bool comp = p >= HL && p <= P - 2 && wo < Wo;
  const int ci0 = S == 1 ? wo0 + p - pl : 2 * (wo0 + p) - pl;
  const bool cok0 = p < P && ci0 >= 0 && ci0 < W;
  const bool cok1 = S == 2 && p < P && ci0 + 1 >= 0 && ci0 + 1 < W;
  DwIn<T, V, PACT> in;
  in.init(pro, c);
  const T* xn = x + (long)n * H * W * C + c;
  const T* dn = dy + (long)n * Ho * Wo * C + c;
  const int nout = ho1 - ho0;

  float acc[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] = 0.f;

  auto cvt = [&](const Vec16<T>& r, bool ok, float (&o)[V]) {
    PackV<T, V> pk;
    pk.v = r.v;
    in.cvt(pk, ok, o);
    if constexpr (PACT < 0) {
#pragma unroll
      for (int v = 0; v < V; ++v) o[v] = ok ? o[v] : 0.f;
    }
  };
  auto publish = [&](const float (&o)[V], int buf) {
    Vec16<T> st;
#pragma unroll
    for (int v = 0; v < V; ++v) st.set(v, o[v]);
    st.store(xs + (buf * 256 + tid) * V);
  };
  // dy of output row m (own column), zero outside the strip
  auto dload = [&](Vec16<T>& d, int m) {
    if (comp && m >= 0 && m < nout) d.load(dn + ((long)(ho0 + m) * Wo + wo) * C);
    else {
#pragma unroll
      for (int v = 0; v < V; ++v) d.set(v, 0.f);
    }
  };
  // GP: per-channel constants of the BatchNorm-backward apply, and the raw (dz, y) loads of
  // the rows still in flight (their apply runs when they enter the contraction queue)
  constexpr int GV = GP ? V : 1;
  float gsc[GV], gsh[GV], ga[GV], gmg[GV], gmx[GV], gmm[GV];
  const T* yn = nullptr;
  T* dyo = nullptr;
  if constexpr (GP) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      bn_affine(gd.mean, gd.rstd, gd.gamma, gd.beta, c + v, gsc[v], gsh[v]);
      ga[v] = gd.coef[c + v];
      bn_bwd_k<T>(ga[v], gd.mean[c + v], gd.rstd[c + v], gd.coef[C + c + v], gd.coef[2 * C + c + v], gmg[v], gmx[v],
                  gmm[v]);
    }
    yn = (const T*)gd.y + (long)n * Ho * Wo * C + c;
    dyo = (T*)gd.dy + (long)n * Ho * Wo * C + c;
  }
  auto gload = [&](Vec16<T>& d, Vec16<T>& yv, int m) {
    if (comp && m >= 0 && m < nout) {
      const long o = ((long)(ho0 + m) * Wo + wo) * C;
      d.load(dn + o);
      yv.load(yn + o);
    }
  };
  // (dz, y) of row m -> the applied gradient in d (zero outside the strip), stored to gd.dy
  auto gapply = [&](Vec16<T>& d, const Vec16<T>& yv, int m) {
    if (comp && m >= 0 && m < nout) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float xv = yv.get(v);
        const float z = fmaf(xv, gsc[v], gsh[v]);
        const float g = d.get(v) * act_grad(z, gd.act);
        d.set(v, bn_bwd_apply1<T>(ga[v], g, gmg[v], gmx[v], gmm[v], xv));   // gmg / gmx hold k1 / k0
      }
      d.store(dyo + ((long)(ho0 + m) * Wo + wo) * C);
    } else {
#pragma unroll
      for (int v = 0; v < V; ++v) d.set(v, 0.f);
    }
  };
  auto addrow = [&](int i, const Vec16<T>& d, const float (&t0)[V], const float (&t1)[V], const float (&t2)[V]) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float g = d.get(v);
      acc[i * 3][v] = fmaf(g, t0[v], acc[i * 3][v]);
      acc[i * 3 + 1][v] = fmaf(g, t1[v], acc[i * 3 + 1][v]);
      acc[i * 3 + 2][v] = fmaf(g, t2[v], acc[i * 3 + 2][v]);
    }
  };

  if constexpr (S == 1) {
    const int hi0 = ho0 - pt;
    const int nin = nout + 2;
    Vec16<T> ring[3];
    bool rok[3];
    auto issue = [&](int k, int q) {
      const int hi = hi0 + q;
      rok[k] = cok0 && q < nin && hi >= 0 && hi < H;
      if (rok[k]) ring[k].load(xn + ((long)hi * W + ci0) * C);
    };
    issue(0, 0);
    issue(1, 1);
    issue(2, 2);
    // dy queue: d0 = output q, d1 = q-1, d2 = q-2 at input row q; f1, f2 = q+1, q+2 in flight
    Vec16<T> d0, d1, d2, f1, f2;
    Vec16<T> y1, y2;  // GP: y of the rows in flight in f1, f2
    if constexpr (GP) {
      Vec16<T> y0;
      gload(d0, y0, 0);
      gapply(d0, y0, 0);
      dload(d1, -1);
      dload(d2, -2);
      gload(f1, y1, 1);
      gload(f2, y2, 2);
    } else {
      dload(d0, 0);
      dload(d1, -1);
      dload(d2, -2);
      dload(f1, 1);
      dload(f2, 2);
    }
    for (int q0 = 0; q0 < nin; q0 += 3) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int q = q0 + k;
        const int buf = q & 1;
        float cen[V];
        cvt(ring[k], rok[k], cen);
        issue(k, q + 3);
        publish(cen, buf);
        __syncthreads();
        if (comp) {
          Vec16<T> L, R;
          L.load(xs + (buf * 256 + tid - CVb) * V);
          R.load(xs + (buf * 256 + tid + CVb) * V);
          float l[V], r[V];
#pragma unroll
          for (int v = 0; v < V; ++v) {
            l[v] = L.get(v);
            r[v] = R.get(v);
          }
          // row q is tap row i of output q - i
          addrow(0, d0, l, cen, r);
          addrow(1, d1, l, cen, r);
          addrow(2, d2, l, cen, r);
        }
        d2 = d1;
        d1 = d0;
        d0 = f1;
        f1 = f2;
        if constexpr (GP) {
          gapply(d0, y1, q + 1);
          y1 = y2;
          gload(f2, y2, q + 3);
        } else {
          dload(f2, q + 3);
        }
      }
    }
  } else {
    const int hi0 = 2 * ho0 - pt;
    const int nin = 2 * nout + 1;
    Vec16<T> ring[4][2];
    bool rok[4][2];
    auto issue = [&](int k, int q) {
      const int hi = hi0 + q;
      const bool rowok = q < nin && hi >= 0 && hi < H;
      rok[k][0] = rowok && cok0;
      rok[k][1] = rowok && cok1;
      if (rok[k][0]) ring[k][0].load(xn + ((long)hi * W + ci0) * C);
      if (rok[k][1]) ring[k][1].load(xn + ((long)hi * W + ci0 + 1) * C);
    };
#pragma unroll
    for (int k = 0; k < 4; ++k) issue(k, k);
    // dy queue at input row q = 2m (+1): dm1 = output m-1, dm = m; f1, f2 = m+1, m+2 in flight
    Vec16<T> dm1, dm, f1, f2;
    Vec16<T> y1, y2;  // GP: y of the rows in flight in f1, f2
    if constexpr (GP) {
      Vec16<T> y0;
      dload(dm1, -1);
      gload(dm, y0, 0);
      gapply(dm, y0, 0);
      gload(f1, y1, 1);
      gload(f2, y2, 2);
    } else {
      dload(dm1, -1);
      dload(dm, 0);
      dload(f1, 1);
      dload(f2, 2);
    }
    for (int q0 = 0; q0 < nin; q0 += 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = q0 + k;
        const int buf = q & 1;
        float c0[V], c1[V];
        cvt(ring[k][0], rok[k][0], c0);
        cvt(ring[k][1], rok[k][1], c1);
        issue(k, q + 4);
        publish(c0, buf);
        __syncthreads();
        if (comp) {
          Vec16<T> R;
          R.load(xs + (buf * 256 + tid + CVb) * V);
          float r[V];
#pragma unroll
          for (int v = 0; v < V; ++v) r[v] = R.get(v);
          if ((k & 1) == 0) {   // q = 2m: tap row 0 of output m, tap row 2 of output m-1
            addrow(0, dm, c0, c1, r);
            addrow(2, dm1, c0, c1, r);
          } else {              // q = 2m+1: tap row 1 of output m
            addrow(1, dm, c0, c1, r);
          }
        }
        if (k & 1) {  // next input row starts output m+1
          dm1 = dm;
          dm = f1;
          f1 = f2;
          if constexpr (GP) {
            gapply(dm, y1, (q >> 1) + 1);
            y1 = y2;
            gload(f2, y2, (q >> 1) + 3);
          } else {
            dload(f2, (q >> 1) + 3);
          }
        }
      }
    }
  }

  // per channel: sum over the computing columns (column order), tap by tap
  __syncthreads();
  float* red = (float*)smem;
  const int Cc = CVb * V;
  const long part = ((long)n * tl.strips + strip) * tl.coltiles + ct;
  for (int k = 0; k < 9; ++k) {
#pragma unroll
    for (int v = 0; v < V; ++v) red[tid * V + v] = acc[k][v];
    __syncthreads();
    for (int e = tid; e < Cc; e += 256) {
      const int cve = e / V, v = e - cve * V;
      float a = 0.f;
      for (int pp = HL; pp <= P - 2; ++pp) a += red[(pp * CVb + cve) * V + v];
      slab[(part * 9 + k) * C + cg * Cc + e] = a;
    }
    __syncthreads();
  }
}

// dx[n,h,w,c] = sum_{i,j} dy[n,(h+pt-i)/S,(w+pl-j)/S,c] * w[i,j,c] over exact divisions.
// S=1: the three dy rows h+pt-i roll down in registers; S=2: direct loads (each dx pixel
// sees 1, 2 or 4 dy pixels).
template <typename T, int S, int V, bool GRED = false>
__global__ void __launch_bounds__(256) dw3x3_bwd_data_kernel(const T* __restrict__ dy, const float* __restrict__ w,
                                                             T* __restrict__ dx, int H, int W, int C, int pt,
                                                             int pl, int Ho, int Wo, BnGred gr = BnGred{}) {
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(t % CV);
  const int wc = (int)(t / CV);
  __shared__ __attribute__((aligned(16))) float gred_red[GRED ? 256 * V : 1];
  DwGred<GRED ? V : 1> gd;
  if constexpr (GRED) gd.init(gr, cv * V, wc < W);
  const T* gy = GRED ? (const T*)gr.y + (long)blockIdx.z * H * W * C + cv * V : nullptr;
  // (no early return: the GRED flush barriers must be reached by every lane of every wave)
  if (wc < W) {
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
    PackV<T, V> nx[3];
    load_row(dr[0], h0 + pt);
    load_row(dr[1], h0 + pt - 1);
    load_row(dr[2], h0 + pt - 2);
    if (h0 + 1 < h1) load_row(nx, h0 + 1 + pt);
    for (int h = h0; h < h1; ++h) {
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
      o.store_out(xn + ((long)h * W + wc) * C);
      if constexpr (GRED) gd.template acc<T>(o, gy + ((long)h * W + wc) * C, gr.p.act);
      if (h + 1 < h1) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          dr[2][j] = dr[1][j];
          dr[1][j] = dr[0][j];
          dr[0][j] = nx[j];
        }
        if (h + 2 < h1) load_row(nx, h + 2 + pt);
      }
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
      o.store_out(xn + ((long)h * W + wc) * C);
      if constexpr (GRED) gd.template acc<T>(o, gy + ((long)h * W + wc) * C, gr.p.act);
    }
  }
  }  // wc < W
  if constexpr (GRED) gd.flush(gred_red, C, CV, gr.parts);
}

// Stride-2 backward data, phase-split: with u = h + pt and v = w + pl, dx row u=2a takes dy
// rows a (tap 0) and a-1 (tap 2), row u=2a+1 takes dy row a (tap 1); columns likewise.  A
// thread owns the 2x2 dx block u in {2a, 2a+1}, v in {2b, 2b+1} for a strip of a; it needs
// dy[a-1..a][b-1..b], of which row a-1 is carried from the previous step, so each step
// loads two dy pixels (one shared with the left neighbour via L1) and stores four.
constexpr int DW_S2_RP = 4;  // row pairs per thread
template <typename T, int V, bool GRED = false>
__global__ void __launch_bounds__(256) dw3x3_bwd_data_s2_kernel(const T* __restrict__ dy, const float* __restrict__ w,
                                                                T* __restrict__ dx, int H, int W, int C, int pt,
                                                                int pl, int Ho, int Wo, int Bc,
                                                                BnGred gr = BnGred{}) {
  const int CV = C / V;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(t % CV);
  const int b = (int)(t / CV);
  __shared__ __attribute__((aligned(16))) float gred_red[GRED ? 256 * V : 1];
  DwGred<GRED ? V : 1> gd;
  if constexpr (GRED) gd.init(gr, cv * V, b < Bc);
  const T* gy = GRED ? (const T*)gr.y + (long)blockIdx.z * H * W * C + cv * V : nullptr;
  if (b < Bc) {  // (no early return: see dw3x3_bwd_data_kernel)
  const int a0 = blockIdx.y * DW_S2_RP;
  const int amax = (H - 1 + pt) >> 1;  // last a with a dx row
  const int a1 = a0 + DW_S2_RP - 1 < amax ? a0 + DW_S2_RP - 1 : amax;
  const int n = blockIdx.z;
  const int c = cv * V;
  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = w[k * C + c + v];
  const T* dn = dy + (long)n * Ho * Wo * C + c;
  T* xn = dx + (long)n * H * W * C + c;
  auto load2 = [&](PackV<T, V>(&p)[2], int a) {  // p[0] = dy[a][b-1], p[1] = dy[a][b]
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int bb = b - 1 + q;
      if (a >= 0 && a < Ho && bb >= 0 && bb < Wo) p[q].load(dn + ((long)a * Wo + bb) * C);
      else p[q].zero();
    }
  };
  const int w0 = 2 * b - pl, w1 = 2 * b + 1 - pl;  // dx columns of this thread
  PackV<T, V> prev[2], cur[2], nxt[2];
  // GRED: y of the 2x2 dx block of step a (rows 2a-pt, 2a+1-pt x columns w0, w1), one step ahead
  PackV<T, V> yq[GRED ? 4 : 1], yn[GRED ? 4 : 1];
  auto yload = [&](PackV<T, V>(&q)[GRED ? 4 : 1], int a) {
    if constexpr (GRED) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int h = 2 * a + (i >> 1) - pt, ww = (i & 1) ? w1 : w0;
        if (h >= 0 && h < H && ww >= 0 && ww < W) q[i].load(gy + ((long)h * W + ww) * C);
      }
    }
  };
  yload(yq, a0);
  load2(prev, a0 - 1);
  load2(cur, a0);
  if (a0 + 1 <= a1) load2(nxt, a0 + 1);
  for (int a = a0; a <= a1; ++a) {
    if (a + 1 <= a1) yload(yn, a + 1);
    float o00[V], o01[V], o10[V], o11[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float c1 = cur[1].get(v), c0 = cur[0].get(v), p1 = prev[1].get(v), p0 = prev[0].get(v);
      // (u=2a, v=2b) taps (0,0),(0,2),(2,0),(2,2); (2a,2b+1) taps (0,1),(2,1);
      // (2a+1,2b) taps (1,0),(1,2); (2a+1,2b+1) tap (1,1)
      o00[v] = fmaf(p0, wr[8][v], fmaf(p1, wr[6][v], fmaf(c0, wr[2][v], c1 * wr[0][v])));
      o01[v] = fmaf(p1, wr[7][v], c1 * wr[1][v]);
      o10[v] = fmaf(c0, wr[5][v], c1 * wr[3][v]);
      o11[v] = c1 * wr[4][v];
    }
    auto put = [&](int h, int ww, const float (&o)[V], int i) {
      if (h < 0 || h >= H || ww < 0 || ww >= W) return;
      PackV<T, V> pk;
#pragma unroll
      for (int v = 0; v < V; ++v) pk.set(v, o[v]);
      pk.store_out(xn + ((long)h * W + ww) * C);
      if constexpr (GRED) {
#pragma unroll
        for (int v = 0; v < V; ++v)
          gred_acc(pk.get(v), yq[i].get(v), gd.sc[v], gd.sh[v], gd.mu[v], gd.rs[v], gr.p.act, gd.sg[v], gd.sgx[v]);
      }
    };
    put(2 * a - pt, w0, o00, 0);
    put(2 * a - pt, w1, o01, 1);
    put(2 * a + 1 - pt, w0, o10, 2);
    put(2 * a + 1 - pt, w1, o11, 3);
    if constexpr (GRED) {
#pragma unroll
      for (int i = 0; i < 4; ++i) yq[i] = yn[i];
    }
    if (a + 1 <= a1) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        prev[q] = cur[q];
        cur[q] = nxt[q];
      }
      if (a + 2 <= a1) load2(nxt, a + 2);
    }
  }
  }  // b < Bc
  if constexpr (GRED) gd.flush(gred_red, C, CV, gr.parts);
}

// Filter gradient: dw[i,j,c] = sum_{n,ho,wo} dy[n,ho,wo,c] * x[n, ho*S-pt+i, wo*S-pl+j, c].
// Thread = (channel vector cv, output column wo) exactly like the forward; it walks strips of
// RB output rows, keeping the 3x3 input window in registers (one new input row per output
// row for S=1, two for S=2), so each output pixel costs one dy load and three x loads and no
// index division.  blockIdx.y strides over the N*spi row strips; each block then sums its
// threads per channel in LDS (fixed order) and writes one [9][C] partial to the slab.
template <typename T, int S, int V, int PACT = -1>
__global__ void __launch_bounds__(256) dw3x3_bwd_filter_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                               float* __restrict__ slab, int N, int H, int W,
                                                               int C, int pt, int pl, int Ho, int Wo, int RB,
                                                               int spi, BnPro pro = BnPro{}) {
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
    DwIn<T, V, PACT> in;  // the forward's input (BatchNorm prologue when PACT >= 0)
    in.init(pro, c);
    const int nstrips = N * spi;
    for (int s = blockIdx.y; s < nstrips; s += gridDim.y) {
      const int n = s / spi;
      const int ho0 = (s - n * spi) * RB;
      const int ho1 = ho0 + RB < Ho ? ho0 + RB : Ho;
      const T* xn = x + (long)n * H * W * C + c;
      const T* dn = dy + (long)n * Ho * Wo * C + c;
      float xr[3][3][V];
      auto load_row = [&](PackV<T, V>(&row)[3], bool (&ok)[3], int hi) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int wi = wo * S - pl + j;
          ok[j] = hi >= 0 && hi < H && wi >= 0 && wi < W;
          if (ok[j]) row[j].load(xn + ((long)hi * W + wi) * C);
          else row[j].zero();
        }
      };
      PackV<T, V> nx[S][3], g, ng;
      bool nok[S][3];
      auto prefetch = [&](int ho) {
#pragma unroll
        for (int q = 0; q < S; ++q) load_row(nx[q], nok[q], ho * S - pt + 3 - S + q);
        ng.load(dn + ((long)ho * Wo + wo) * C);
      };
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        PackV<T, V> r0[3];
        bool k0[3];
        load_row(r0, k0, ho0 * S - pt + i);
#pragma unroll
        for (int j = 0; j < 3; ++j) in.cvt(r0[j], k0[j], xr[i][j]);
      }
      g.load(dn + ((long)ho0 * Wo + wo) * C);
      if (ho0 + 1 < ho1) prefetch(ho0 + 1);
      for (int ho = ho0; ho < ho1; ++ho) {
        float gv[V];
#pragma unroll
        for (int v = 0; v < V; ++v) gv[v] = g.get(v);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int v = 0; v < V; ++v) acc[i * 3 + j][v] = fmaf(gv[v], xr[i][j][v], acc[i * 3 + j][v]);
        if (ho + 1 < ho1) {
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            if constexpr (S == 1) {
#pragma unroll
              for (int v = 0; v < V; ++v) {
                xr[0][j][v] = xr[1][j][v];
                xr[1][j][v] = xr[2][j][v];
              }
              in.cvt(nx[0][j], nok[0][j], xr[2][j]);
            } else {
#pragma unroll
              for (int v = 0; v < V; ++v) xr[0][j][v] = xr[2][j][v];
              in.cvt(nx[0][j], nok[0][j], xr[1][j]);
              in.cvt(nx[1][j], nok[1][j], xr[2][j]);
            }
          }
          g = ng;
          if (ho + 2 < ho1) prefetch(ho + 2);
        }
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


}  // namespace rod

using namespace rod;

#define DW_ARGS_OK(fn)                                                                                  \
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && Ho > 0 && Wo > 0, fn ": bad shape");                \
  ROD_CHECK_ARG(stride == 1 || stride == 2, fn ": stride must be 1 or 2");                              \
  ROD_CHECK_ARG(pad_t >= 0 && pad_t <= 2 && pad_l >= 0 && pad_l <= 2, fn ": bad padding");              \
  ROD_CHECK_ARG((Ho - 1) * stride + 3 - pad_t > 0 && (Wo - 1) * stride + 3 - pad_l > 0, fn ": bad output")

namespace rod {

static dim3 dw_fwd_grid(int N, int Ho, int Wo, int C, int V) {
  return dim3(cdiv((long)(C / V) * Wo, 256), cdiv(Ho, DW_RB), N);
}

// channel pack per thread: 16-byte (bf16 x8 / f32 x4) when C and the pointers allow it,
// bf16 x4 (8-byte) when only C % 4 == 0, else scalar
// `cap`: the forward and the filter gradient keep an fp32 3x3 window per channel, so they
// use 4-channel packs; the data gradient 16-byte packs (ROD_DW_PACK overrides, A/B only)
template <typename T>
static int dw_pack(const void* a, const void* b, int C, int cap) {
  auto al = [&](uintptr_t n) { return (((uintptr_t)a | (uintptr_t)b) & (n - 1)) == 0; };
  static const int force = getenv("ROD_DW_PACK") ? atoi(getenv("ROD_DW_PACK")) : 0;
  if (force) cap = force;
  if (sizeof(T) == 2 && C % 8 == 0 && al(16) && cap >= 8) return 8;
  if (C % 4 == 0 && al(4 * sizeof(T))) return 4;
  return 1;
}

template <typename T, int S, int V>
static void dw_fwd_launch(const void* x, const BnPro* pro, const float* w, void* y, float* parts, int N, int H, int W,
                          int C, int pt, int pl, int Ho, int Wo, hipStream_t s) {
  const dim3 grid = dw_fwd_grid(N, Ho, Wo, C, V);
  const BnPro pv = pro ? *pro : BnPro{};
#define DWF(ST, PA)                                                                                              \
  hipLaunchKernelGGL((dw3x3_fwd_kernel<T, S, V, ST, PA>), grid, dim3(256), 0, s, (const T*)x, w, (T*)y, H, W, C, pt, \
                     pl, Ho, Wo, parts, pv)
  const int pa = !pro ? -1 : (pro->act == ROD_ACT_RELU6 ? ROD_ACT_RELU6 : DW_ACT_RT);
  if (parts) {
    if (pa == ROD_ACT_RELU6) DWF(true, ROD_ACT_RELU6); else if (pa == DW_ACT_RT) DWF(true, DW_ACT_RT); else DWF(true, -1);
  } else {
    if (pa == ROD_ACT_RELU6) DWF(false, ROD_ACT_RELU6); else if (pa == DW_ACT_RT) DWF(false, DW_ACT_RT); else DWF(false, -1);
  }
#undef DWF
}
// LDS-exchange forward: needs 16-byte packs (C % V == 0, 16-byte aligned x and y).
template <typename T>
static bool dw_lx_ok(const void* x, const void* y, int C) {
  static const bool legacy = getenv("ROD_DW_LEGACY") != nullptr;  // A/B timing switch
  return !legacy && C % Vec16<T>::N == 0 && ((((uintptr_t)x) | ((uintptr_t)y)) & 15) == 0;
}
static long dw_lx_parts(int N, int Ho, int Wo, int C, int S, int V) {
  const DwTile t = dw_tile(N, Ho, Wo, C, S, V);
  return (long)N * t.strips * t.coltiles;
}
template <typename T>
static long dw_fwd_lx_launch(const void* x, const BnPro* pro, const float* w, void* y, float* parts, int N, int H,
                             int W, int C, int S, int pt, int pl, int Ho, int Wo, hipStream_t s) {
  // input pixels as N*Ho*Wo*S*S: the same function of the output shape as rod_dw3x3_fwd_stat_parts
  const int V = dw_fwd_v(sizeof(T) == 2 ? ROD_BF16 : ROD_F32, (long)N * Ho * Wo * S * S, C);
  const DwTile t = dw_tile(N, Ho, Wo, C, S, V);
  const dim3 grid(t.coltiles * t.cgroups, t.strips, N);
  const BnPro pv = pro ? *pro : BnPro{};
  const int pa = !pro ? -1 : (pro->act == ROD_ACT_RELU6 ? ROD_ACT_RELU6 : DW_ACT_RT);
#define DWL(S_, PA, ST)                                                                                           \
  do {                                                                                                            \
    if (sizeof(T) == 2 && V == 4)                                                                                 \
      hipLaunchKernelGGL((dw3x3_fwd_lx_kernel<T, S_, PA, ST, 4>), grid, dim3(256), 0, s, (const T*)x, w, (T*)y, H, W, \
                         C, pt, pl, Ho, Wo, t, parts, pv);                                                        \
    else                                                                                                          \
      hipLaunchKernelGGL((dw3x3_fwd_lx_kernel<T, S_, PA, ST>), grid, dim3(256), 0, s, (const T*)x, w, (T*)y, H, W,  \
                         C, pt, pl, Ho, Wo, t, parts, pv);                                                        \
  } while (0)
#define DWL_PA(S_, ST)                    \
  if (pa == ROD_ACT_RELU6) DWL(S_, ROD_ACT_RELU6, ST); \
  else if (pa == DW_ACT_RT) DWL(S_, DW_ACT_RT, ST); \
  else DWL(S_, -1, ST)
  if (S == 1) {
    if (parts) { DWL_PA(1, true); } else { DWL_PA(1, false); }
  } else {
    if (parts) { DWL_PA(2, true); } else { DWL_PA(2, false); }
  }
#undef DWL_PA
#undef DWL
  return (long)N * t.strips * t.coltiles;
}

// the grid of the backward-data launch (phase-split kernel for stride 2): its block count is
// the gred part count
static dim3 dw_bwd_data_grid(int N, int H, int W, int C, int S, int pt, int pl, int V, bool* s2k) {
  static const bool no_s2 = getenv("ROD_DEBUG_NOS2") != nullptr;  // debug bisection
  *s2k = S == 2 && pt <= 1 && pl <= 1 && !no_s2;
  if (*s2k) {
    const int Bc = (W - 1 + pl) / 2 + 1;
    const int Ar = (H - 1 + pt) / 2 + 1;
    return dim3(cdiv((long)(C / V) * Bc, 256), cdiv(Ar, DW_S2_RP), N);
  }
  return dim3(cdiv((long)(C / V) * W, 256), cdiv(H, DW_RB), N);
}
// stride-1 backward-data on the LDS-exchange kernel: correlation of dy [N,Ho,Wo,C] with the
// flipped taps, pads (2-pt, 2-pl), output dx [N,H,W,C]; returns the gred part count
template <typename T>
static long dw_bwd_data_lx_launch(const void* dy, const float* w, void* dx, const BnGred* gr, int N, int H, int W,
                                  int C, int pt, int pl, int Ho, int Wo, hipStream_t s) {
  const DwTile t = dw_tile(N, H, W, C, 1, Vec16<T>::N);
  const dim3 grid(t.coltiles * t.cgroups, t.strips, N);
  const BnGred g = gr ? *gr : BnGred{};
  if (gr)
    hipLaunchKernelGGL((dw3x3_bwd_data_lx_kernel<T, true>), grid, dim3(256), 0, s, (const T*)dy, w, (T*)dx, Ho, Wo,
                       C, 2 - pt, 2 - pl, H, W, t, g);
  else
    hipLaunchKernelGGL((dw3x3_bwd_data_lx_kernel<T, false>), grid, dim3(256), 0, s, (const T*)dy, w, (T*)dx, Ho, Wo,
                       C, 2 - pt, 2 - pl, H, W, t, g);
  return (long)N * t.strips * t.coltiles;
}

template <typename T, int S, int V>
static void dw_bwd_data_launch(const void* dy, const float* w, void* dx, int N, int H, int W, int C, int pt, int pl,
                               int Ho, int Wo, const BnGred* gr, hipStream_t s) {
  bool s2k;
  const dim3 grid = dw_bwd_data_grid(N, H, W, C, S, pt, pl, V, &s2k);
  const BnGred g = gr ? *gr : BnGred{};
  if (s2k) {
    const int Bc = (W - 1 + pl) / 2 + 1;
    if (gr)
      hipLaunchKernelGGL((dw3x3_bwd_data_s2_kernel<T, V, true>), grid, dim3(256), 0, s, (const T*)dy, w, (T*)dx, H, W,
                         C, pt, pl, Ho, Wo, Bc, g);
    else
      hipLaunchKernelGGL((dw3x3_bwd_data_s2_kernel<T, V, false>), grid, dim3(256), 0, s, (const T*)dy, w, (T*)dx, H,
                         W, C, pt, pl, Ho, Wo, Bc, g);
    return;
  }
  if (gr)
    hipLaunchKernelGGL((dw3x3_bwd_data_kernel<T, S, V, true>), grid, dim3(256), 0, s, (const T*)dy, w, (T*)dx, H, W,
                       C, pt, pl, Ho, Wo, g);
  else
    hipLaunchKernelGGL((dw3x3_bwd_data_kernel<T, S, V, false>), grid, dim3(256), 0, s, (const T*)dy, w, (T*)dx, H, W,
                       C, pt, pl, Ho, Wo, g);
}
template <typename T, int S, int V>
static void dw_bwd_filter_launch(const void* x, const BnPro* pro, const void* dy, float* dw, float* slab, int N, int H,
                                 int W, int C, int pt, int pl, int Ho, int Wo, hipStream_t s) {
  DwFilterPlan p = dw_filter_plan(N, Ho, Wo, C, V, (int)sizeof(T));
  const BnPro pv = pro ? *pro : BnPro{};
#define DWW(PA)                                                                                                   \
  hipLaunchKernelGGL((dw3x3_bwd_filter_kernel<T, S, V, PA>), dim3(p.gx, p.gy), dim3(256), 256 * V * sizeof(float), \
                     s, (const T*)x, (const T*)dy, slab, N, H, W, C, pt, pl, Ho, Wo, p.RB, p.spi, pv)
  const int pa = !pro ? -1 : (pro->act == ROD_ACT_RELU6 ? ROD_ACT_RELU6 : DW_ACT_RT);
  if (pa == ROD_ACT_RELU6) DWW(ROD_ACT_RELU6); else if (pa == DW_ACT_RT) DWW(DW_ACT_RT); else DWW(-1);
#undef DWW
  slab_sum(slab, dw, (int)p.parts(), 9L * C, s);
}

}  // namespace rod

using namespace rod;

// dispatch on stride and channel pack; defines the launch for T_ (pack from the pointers)
#define DW_SELECT(FN, T_, PK, ...)                                            \
  do {                                                                        \
    if (stride == 1) {                                                        \
      if ((PK) == 8) FN<T_, 1, (sizeof(T_) == 2 ? 8 : 4)>(__VA_ARGS__);      \
      else if ((PK) == 4) FN<T_, 1, 4>(__VA_ARGS__);                          \
      else FN<T_, 1, 1>(__VA_ARGS__);                                         \
    } else {                                                                  \
      if ((PK) == 8) FN<T_, 2, (sizeof(T_) == 2 ? 8 : 4)>(__VA_ARGS__);      \
      else if ((PK) == 4) FN<T_, 2, 4>(__VA_ARGS__);                          \
      else FN<T_, 2, 1>(__VA_ARGS__);                                         \
    }                                                                         \
  } while (0)

extern "C" {

int rod_dw3x3_fwd_stat_parts(int N, int Ho, int Wo, int C, int stride, int dtype) {
  // exactly the parts the launch for 16-byte-aligned x / y writes: the LDS-exchange kernel
  // when C fills 16-byte packs, else the register-strip kernel's grid
  const int V16 = dtype == ROD_F32 ? 4 : 8;
  if (C % V16 == 0)
    return (int)dw_lx_parts(N, Ho, Wo, C, stride == 2 ? 2 : 1, dw_fwd_v(dtype, (long)N * Ho * Wo * stride * stride, C));
  const int V = dtype == ROD_F32 ? (C % 4 == 0 ? 4 : 1) : (C % 4 == 0 ? 4 : 1);
  const dim3 g = dw_fwd_grid(N, Ho, Wo, C, V);
  return (int)(g.x * g.y * g.z);
}

int rod_dw3x3_fwd(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                  const float* pro_beta, int pro_act, const float* w, void* y, float* stat_parts, int N, int H, int W,
                  int C, int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream) {
  DW_ARGS_OK("rod_dw3x3_fwd");
  ROD_CHECK_ARG(!pro_mean || pro_rstd, "rod_dw3x3_fwd: BatchNorm prologue needs mean and rstd");
  hipStream_t s = ROD_STREAM(stream);
  const BnPro pro{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  const BnPro* pp = pro_mean ? &pro : nullptr;
  const int nparts = rod_dw3x3_fwd_stat_parts(N, Ho, Wo, C, stride, dtype);
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    if (dw_lx_ok<T>(x, y, C)) {
      dw_fwd_lx_launch<T>(x, pp, w, y, stat_parts, N, H, W, C, stride, pad_t, pad_l, Ho, Wo, s);
      return;
    }
    const int pk = dw_pack<T>(x, y, C, 4);
    const int V = pk == 8 ? (sizeof(T) == 2 ? 8 : 4) : pk;
    const dim3 g = dw_fwd_grid(N, Ho, Wo, C, V);
    // the fused statistics write one part per block; when that is not the count the caller
    // sized the slab for (misaligned pointers, legacy switch), a separate pass writes them
    const bool fuse = stat_parts && (long)g.x * g.y * g.z == nparts;
    DW_SELECT(dw_fwd_launch, T, pk, x, pp, w, y, fuse ? stat_parts : nullptr, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
    if (stat_parts && !fuse)
      ::rod::stat_parts(sizeof(T) == 4 ? ROD_F32 : ROD_BF16, y, (long)N * Ho * Wo, C, C, stat_parts, nparts, s);
  };
  if (dtype == ROD_F32) run(float{});
  else if (dtype == ROD_BF16) run(bf16_t{});
  else {
    set_error("rod_dw3x3_fwd: bad dtype %d", dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_dw3x3_fwd");
}

static int dw_bwd_data_pack(int C, int dtype) {  // the pack dw_pack picks for 16-byte-aligned pointers
  if (dtype == ROD_BF16 && C % 8 == 0) return 8;
  return C % 4 == 0 ? 4 : 1;
}

int rod_dw3x3_bwd_data_gred_parts(int N, int H, int W, int C, int stride, int dtype) {
  const int V16 = dtype == ROD_F32 ? 4 : 8;
  if (stride == 1 && C % V16 == 0) return (int)dw_lx_parts(N, H, W, C, 1, V16);  // LDS-exchange kernel
  const int pt = stride == 2 ? std::max((cdiv(H, 2) - 1) * 2 + 3 - H, 0) / 2 : 1;
  const int pl = stride == 2 ? std::max((cdiv(W, 2) - 1) * 2 + 3 - W, 0) / 2 : 1;
  const int pk = dw_bwd_data_pack(C, dtype);
  const int V = pk == 8 ? (dtype == ROD_BF16 ? 8 : 4) : pk;
  bool s2k;
  const dim3 g = dw_bwd_data_grid(N, H, W, C, stride, pt, pl, V, &s2k);
  return (int)(g.x * g.y * g.z);
}

int rod_dw3x3_bwd_data(const void* dy, const float* w, void* dx, const void* gred_y, const float* gred_mean,
                       const float* gred_rstd, const float* gred_gamma, const float* gred_beta, int gred_act,
                       float* gred_parts, int N, int H, int W, int C, int stride, int pad_t, int pad_l, int Ho, int Wo,
                       int dtype, void* stream) {
  DW_ARGS_OK("rod_dw3x3_bwd_data");
  ROD_CHECK_ARG(!gred_parts || (gred_y && gred_mean && gred_rstd), "rod_dw3x3_bwd_data: gred needs y, mean, rstd");
  hipStream_t s = ROD_STREAM(stream);
  const BnGred gr{gred_y, BnPro{gred_mean, gred_rstd, gred_gamma, gred_beta, gred_act}, gred_parts};
  auto run = [&](auto tag) {
    typedef decltype(tag) T;
    const int nparts = gred_parts ? rod_dw3x3_bwd_data_gred_parts(N, H, W, C, stride, dtype) : 0;
    if (stride == 1 && dw_lx_ok<T>(dy, dx, C) && (!gred_parts || ((((uintptr_t)gred_y) & 15) == 0))) {
      dw_bwd_data_lx_launch<T>(dy, w, dx, gred_parts ? &gr : nullptr, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
      return;
    }
    const int pk = dw_pack<T>(dy, dx, C, 8);
    const int V = pk == 8 ? (sizeof(T) == 2 ? 8 : 4) : pk;
    bool s2k;
    const dim3 g = dw_bwd_data_grid(N, H, W, C, stride, pad_t, pad_l, V, &s2k);
    // fused when this launch's blocks are the parts the caller sized (aligned pointers,
    // 16-byte-aligned y too); otherwise a separate pass
    const bool fuse = gred_parts && (long)g.x * g.y * g.z == nparts && (((uintptr_t)gred_y) & 15) == 0;
    const BnGred* gp = fuse ? &gr : nullptr;
    DW_SELECT(dw_bwd_data_launch, T, pk, dy, w, dx, N, H, W, C, pad_t, pad_l, Ho, Wo, gp, s);
    if (gred_parts && !fuse) ::rod::gred_parts(dtype, dx, gred_y, gr.p, (long)N * H * W, C, gred_parts, nparts, s);
  };
  if (dtype == ROD_F32) run(float{});
  else if (dtype == ROD_BF16) run(bf16_t{});
  else {
    set_error("rod_dw3x3_bwd_data: bad dtype %d", dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_dw3x3_bwd_data");
}

size_t rod_dw3x3_bwd_filter_workspace(int N, int Ho, int Wo, int C) {
  long parts = 0;
  for (int V : {1, 4, 8}) {
    if (C % V) continue;
    for (int es : {2, 4}) parts = std::max(parts, dw_filter_plan(N, Ho, Wo, C, V, es).parts());
    if (V >= 4)
      for (int S : {1, 2}) parts = std::max(parts, dw_lx_parts(N, Ho, Wo, C, S, V));
  }
  return (size_t)parts * 9 * C * sizeof(float);
}

int rod_dw3x3_bwd_filter(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                         const float* pro_beta, int pro_act, const void* dy, float* dw, void* workspace, int N, int H,
                         int W, int C, int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream) {
  DW_ARGS_OK("rod_dw3x3_bwd_filter");
  ROD_CHECK_ARG(workspace != nullptr, "rod_dw3x3_bwd_filter: workspace is NULL");
  ROD_CHECK_ARG(!pro_mean || pro_rstd, "rod_dw3x3_bwd_filter: BatchNorm prologue needs mean and rstd");
  hipStream_t s = ROD_STREAM(stream);
  float* slab = (float*)workspace;
  const BnPro pro{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  const BnPro* pp = pro_mean ? &pro : nullptr;
  auto lx = [&](auto tag) {  // LDS-exchange kernel (16-byte packs)
    typedef decltype(tag) T;
    const DwTile t = dw_tile(N, Ho, Wo, C, stride, Vec16<T>::N);
    const dim3 grid(t.coltiles * t.cgroups, t.strips, N);
    const BnPro pv = pp ? *pp : BnPro{};
    const int pa = !pp ? -1 : (pp->act == ROD_ACT_RELU6 ? ROD_ACT_RELU6 : DW_ACT_RT);
#define DWW(S_, PA)                                                                                               \
  hipLaunchKernelGGL((dw3x3_bwdw_lx_kernel<T, S_, PA>), grid, dim3(256), 0, s, (const T*)x, (const T*)dy, slab, H, W, \
                     C, pad_t, pad_l, Ho, Wo, t, pv)
    if (stride == 1) {
      if (pa == ROD_ACT_RELU6) DWW(1, ROD_ACT_RELU6); else if (pa == DW_ACT_RT) DWW(1, DW_ACT_RT); else DWW(1, -1);
    } else {
      if (pa == ROD_ACT_RELU6) DWW(2, ROD_ACT_RELU6); else if (pa == DW_ACT_RT) DWW(2, DW_ACT_RT); else DWW(2, -1);
    }
#undef DWW
    slab_sum(slab, dw, (int)((long)N * t.strips * t.coltiles), 9L * C, s);
  };
  if (dtype == ROD_F32 && dw_lx_ok<float>(x, dy, C)) {
    lx(float{});
  } else if (dtype == ROD_BF16 && dw_lx_ok<bf16_t>(x, dy, C)) {
    lx(bf16_t{});
  } else if (dtype == ROD_F32) {
    const int pk = dw_pack<float>(x, dy, C, 4);
    DW_SELECT(dw_bwd_filter_launch, float, pk, x, pp, dy, dw, slab, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else if (dtype == ROD_BF16) {
    const int pk = dw_pack<bf16_t>(x, dy, C, 4);
    DW_SELECT(dw_bwd_filter_launch, bf16_t, pk, x, pp, dy, dw, slab, N, H, W, C, pad_t, pad_l, Ho, Wo, s);
  } else {
    set_error("rod_dw3x3_bwd_filter: bad dtype %d", dtype);
    return ROD_EINVAL;
  }
  return check_launch("rod_dw3x3_bwd_filter");
}

int rod_bn_bwd_apply(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                     const float* beta, const float* coef, void* dy, long M, int C, int act, int dtype, void* stream);

int rod_dw3x3_bwd_filter_bn(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                            const float* pro_beta, int pro_act, const void* dz, const void* y, const float* bn_mean,
                            const float* bn_rstd, const float* bn_gamma, const float* bn_beta, int bn_act,
                            const float* coef, void* dy, float* dw, void* workspace, int N, int H, int W, int C,
                            int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype, void* stream) {
  DW_ARGS_OK("rod_dw3x3_bwd_filter_bn");
  ROD_CHECK_ARG(workspace != nullptr && dz != nullptr && y != nullptr && dy != nullptr && coef != nullptr &&
                    bn_mean != nullptr && bn_rstd != nullptr,
                "rod_dw3x3_bwd_filter_bn: NULL tensor argument");
  ROD_CHECK_ARG(!pro_mean || pro_rstd, "rod_dw3x3_bwd_filter_bn: BatchNorm prologue needs mean and rstd");
  ROD_CHECK_ARG(bn_act >= ROD_ACT_NONE && bn_act <= ROD_ACT_RELU, "rod_dw3x3_bwd_filter_bn: bad act %d", bn_act);
  hipStream_t s = ROD_STREAM(stream);
  const BnPro pro{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  const BnPro* pp = pro_mean ? &pro : nullptr;
  const DwGrad gd{y, bn_mean, bn_rstd, bn_gamma, bn_beta, coef, bn_act, dy};
  auto gp = [&](auto tag) {  // the fused kernel (LDS-exchange engine, 16-byte packs)
    typedef decltype(tag) T;
    const DwTile t = dw_tile(N, Ho, Wo, C, stride, Vec16<T>::N);
    const dim3 grid(t.coltiles * t.cgroups, t.strips, N);
    const BnPro pv = pp ? *pp : BnPro{};
    const int pa = !pp ? -1 : (pp->act == ROD_ACT_RELU6 ? ROD_ACT_RELU6 : DW_ACT_RT);
    float* slab = (float*)workspace;
#define DWG(S_, PA)                                                                                                \
  hipLaunchKernelGGL((dw3x3_bwdw_lx_kernel<T, S_, PA, true>), grid, dim3(256), 0, s, (const T*)x, (const T*)dz, slab, \
                     H, W, C, pad_t, pad_l, Ho, Wo, t, pv, gd)
    if (stride == 1) {
      if (pa == ROD_ACT_RELU6) DWG(1, ROD_ACT_RELU6); else if (pa == DW_ACT_RT) DWG(1, DW_ACT_RT); else DWG(1, -1);
    } else {
      if (pa == ROD_ACT_RELU6) DWG(2, ROD_ACT_RELU6); else if (pa == DW_ACT_RT) DWG(2, DW_ACT_RT); else DWG(2, -1);
    }
#undef DWG
    slab_sum(slab, dw, (int)((long)N * t.strips * t.coltiles), 9L * C, s);
  };
  const bool al = ((((uintptr_t)y) | ((uintptr_t)dy)) & 15) == 0;
  if (dtype == ROD_BF16 && al && dw_lx_ok<bf16_t>(x, dz, C)) {
    gp(bf16_t{});
  } else if (dtype == ROD_F32 && al && dw_lx_ok<float>(x, dz, C)) {
    gp(float{});
  } else {  // no fused kernel for this layout: apply pass, then the plain filter gradient
    int rc = rod_bn_bwd_apply(dz, y, bn_mean, bn_rstd, bn_gamma, bn_beta, coef, dy, (long)N * Ho * Wo, C, bn_act,
                              dtype, stream);
    if (rc) return rc;
    return rod_dw3x3_bwd_filter(x, pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act, dy, dw, workspace, N, H, W, C,
                                stride, pad_t, pad_l, Ho, Wo, dtype, stream);
  }
  return check_launch("rod_dw3x3_bwd_filter_bn");
}

}  // extern "C"

// =====================================================================================
// Fused stride-1 depthwise backward (ABI 12): the backward of
//   x = act_e(BN_e(ye))  ->  yd = dw3x3(x, w) (stride 1, TF-SAME)  ->  act_d(BN_d(yd))
// from dz (the gradient at act_d(BN_d(yd))) in ONE pass over the rows, for a depthwise whose
// input is the BatchNorm-prologue form of its producer (the expand conv, or the stem):
//   dy  = the BatchNorm-backward apply of BN_d (rod_bn_bwd_apply's arithmetic, rounded to T;
//         coef from rod_bn_bwd_reduce over (dz, yd));
//   dx  = DepthwiseConv2dNativeBackpropInput(dy, w)        (rounded to T: dz of BN_e)
//   dw  = DepthwiseConv2dNativeBackpropFilter(x, dy)       (fp32 partials, fixed-order sum)
//   and, with gparts, the BatchNorm-backward sums of BN_e over (dx, ye): per part and channel
//   (sum g, sum g*yhat), g = dx*act_e'(BN_e(ye)), yhat = (ye - mean_e)*rstd_e — what
//   rod_bn_bwd_reduce would compute next, in rod_bn_bwd_finalize's [parts][2][C] format.
// Unfused, these are rod_bn_bwd_apply (read dz, yd; write dy), rod_dw3x3_bwd_data (read dy;
// write dx), rod_dw3x3_bwd_filter (read ye, dy) and the producer's rod_bn_bwd_reduce (read
// dx, ye): 9 passes over C-wide tensors.  Fused: read ye, dz, yd, write dx — 4 passes; dy never
// exists in memory.
//
// Engine: the LDS neighbour exchange of dw_lx_body (stride 1), 4 channels per thread (bf16:
// 8-byte packs) to hold the weights, both BatchNorms' constants and the nine filter
// accumulators in registers.  Step q handles x row rho = ho0 - 2 + q and dy row rho + 1: each
// thread converts its column's ye (prologue) and (dz, yd) (apply), publishes both, and takes
// its left / right neighbours from LDS.  dy row rho + 1 is the last dy row dx row rho needs
// (taps (0, *)), so dx row rho is emitted at step q; the filter pairs x row rho with the dy rows
// rho + 1, rho, rho - 1 of the thread's own column (a two-row queue).  dx accumulates in the
// order of the stride-1 rod_dw3x3_bwd_data kernel (dy rows ascending, taps L, C, R), so dx is
// bit-identical to the unfused chain; dw and the BN_e sums are reassociated (column tiles).
// =====================================================================================

template <typename T, int PACT, bool RED, int D = 3>
__global__ void __launch_bounds__(256) dw3x3_bwd_fused_kernel(const T* __restrict__ ye, const T* __restrict__ dz,
                                                              const T* __restrict__ yd, const float* __restrict__ w,
                                                              T* __restrict__ dx, float* __restrict__ slab,
                                                              float* __restrict__ gparts, int H, int W, int C,
                                                              DwTile tl, BnPro pro, DwBwdBn bd) {
  constexpr int V = 4;
  typedef PackV<T, V> PK;
  constexpr int XS = 2 * 2 * 256 * (int)sizeof(PK);  // x and dy slots, double buffered
  constexpr int SS = 256 * V * 4;                     // per-tap column reduction
  __shared__ __attribute__((aligned(16))) char smem[XS > SS ? XS : SS];
  PK* xs = (PK*)smem;              // [2][256]
  PK* dsl = xs + 2 * 256;          // [2][256]
  const int tid = threadIdx.x;
  const int CVb = tl.CVb, P = tl.P;
  const int p = tid / CVb, cvb = tid - (tid / CVb) * CVb;
  int bx, strip, n;
  xcd_block(bx, strip, n);
  const int cg = bx % tl.cgroups, ct = bx / tl.cgroups;
  const int c = (cg * CVb + cvb) * V;
  const int col = ct * tl.TWo + p - 1;                  // pads (1, 1): input column = output column
  const bool comp = p >= 1 && p <= P - 2 && col < W;
  const bool cok = p < P && col >= 0 && col < W;
  const int ho0 = strip * tl.RB;
  const int ho1 = ho0 + tl.RB < H ? ho0 + tl.RB : H;
  const int xlo = ho0 - 1 > 0 ? ho0 - 1 : 0, xhi = ho1 < H - 1 ? ho1 : H - 1;  // rows of x / dy needed

  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = w[k * C + c + v];
  DwIn<T, V, PACT> in;
  in.init(pro, c);
  float dsc[V], dsh[V], da[V], dmg[V], dmx[V], dmm[V];   // dmg / dmx / dmm: the apply's k1 / k0 / m
#pragma unroll
  for (int v = 0; v < V; ++v) {
    bn_affine(bd.mean, bd.rstd, bd.gamma, bd.beta, c + v, dsc[v], dsh[v]);
    da[v] = bd.coef[c + v];
    bn_bwd_k<T>(da[v], bd.mean[c + v], bd.rstd[c + v], bd.coef[C + c + v], bd.coef[2 * C + c + v], dmg[v], dmx[v],
                dmm[v]);
  }
  constexpr int RV = RED ? V : 1;
  float emu[RV], ers[RV], sg[RV], sgx[RV];
  if constexpr (RED) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      emu[v] = pro.mean[c + v];
      ers[v] = pro.rstd[c + v];
      sg[v] = sgx[v] = 0.f;
    }
  }
  const long nb = (long)n * H * W * C + c;
  const T* yen = ye + nb;
  const T* dzn = dz + nb;
  const T* ydn = yd + nb;
  T* dxn = dx + nb;

  // prefetch ring of D steps: step q loads x row ho0-2+q and (dz, yd) of row ho0-1+q
  PK rx[D], rz[D], ry[D];
  bool okx[D], okd[D];
  auto issue = [&](int k, int q) {
    const int rho = ho0 - 2 + q;
    okx[k] = cok && rho >= xlo && rho <= xhi;
    okd[k] = cok && rho + 1 >= xlo && rho + 1 <= xhi;
    if (okx[k]) rx[k].load(yen + ((long)rho * W + col) * C);
    if (okd[k]) {
      rz[k].load(dzn + ((long)(rho + 1) * W + col) * C);
      ry[k].load(ydn + ((long)(rho + 1) * W + col) * C);
    }
  };
  const int nst = ho1 - ho0 + 3;
#pragma unroll
  for (int k = 0; k < D; ++k) issue(k, k);
  float acc[3][V], fa[9][V], q1[V], q2[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    acc[0][v] = acc[1][v] = acc[2][v] = 0.f;
    q1[v] = q2[v] = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) fa[k][v] = 0.f;
  }
  // D is a multiple of 3: the ring slot (q mod D) and the dx accumulator slot (q mod 3) are
  // both compile-time under the unroll
  static_assert(D % 3 == 0, "ring depth must be a multiple of 3");
  for (int q0 = 0; q0 < nst; q0 += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int q = q0 + k;
      const int rho = ho0 - 2 + q;
      const int buf = q & 1;
      const int k3 = k % 3;
      // x row rho: the forward's input (prologue, rounded to T), 0 outside the rows needed
      float xv[V], yraw[V];
      {
        in.cvt(rx[k], okx[k], xv);
        if constexpr (PACT < 0) {
#pragma unroll
          for (int v = 0; v < V; ++v) xv[v] = okx[k] ? xv[v] : 0.f;
        }
#pragma unroll
        for (int v = 0; v < V; ++v) yraw[v] = rx[k].get(v);
      }
      // dy row rho + 1: the BatchNorm-backward apply of BN_d, rounded to T
      float dv[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float yv = ry[k].get(v);
        const float z = fmaf(yv, dsc[v], dsh[v]);
        const float g = rz[k].get(v) * act_grad(z, bd.act);
        const float o = bn_bwd_apply1<T>(da[v], g, dmg[v], dmx[v], dmm[v], yv);
        dv[v] = okd[k] ? to_f32(from_f32<T>(o)) : 0.f;
      }
      PK px, pd;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        px.set(v, xv[v]);
        pd.set(v, dv[v]);
      }
      issue(k, q + D);
      xs[buf * 256 + tid] = px;
      dsl[buf * 256 + tid] = pd;
      __syncthreads();
      if (comp) {
        const PK xl = xs[buf * 256 + tid - CVb], xr = xs[buf * 256 + tid + CVb];
        const PK dl = dsl[buf * 256 + tid - CVb], dr = dsl[buf * 256 + tid + CVb];
        // backward-data: dy row rho+1 is tap row 0 of dx row rho, 1 of rho+1, 2 of rho+2
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int sl = (k3 + i) % 3;
#pragma unroll
          for (int v = 0; v < V; ++v) {
            float a = acc[sl][v];
            a = fmaf(dl.get(v), wr[i * 3 + 2][v], a);
            a = fmaf(dv[v], wr[i * 3 + 1][v], a);
            a = fmaf(dr.get(v), wr[i * 3][v], a);
            acc[sl][v] = a;
          }
        }
        // filter: x row rho with the strip's dy rows rho+1 (tap row 0), rho (1), rho-1 (2)
        const bool own = rho + 1 >= ho0 && rho + 1 < ho1;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float f0 = own ? dv[v] : 0.f;
          const float t0 = xl.get(v), t2 = xr.get(v);
          fa[0][v] = fmaf(f0, t0, fa[0][v]);
          fa[1][v] = fmaf(f0, xv[v], fa[1][v]);
          fa[2][v] = fmaf(f0, t2, fa[2][v]);
          fa[3][v] = fmaf(q1[v], t0, fa[3][v]);
          fa[4][v] = fmaf(q1[v], xv[v], fa[4][v]);
          fa[5][v] = fmaf(q1[v], t2, fa[5][v]);
          fa[6][v] = fmaf(q2[v], t0, fa[6][v]);
          fa[7][v] = fmaf(q2[v], xv[v], fa[7][v]);
          fa[8][v] = fmaf(q2[v], t2, fa[8][v]);
          q2[v] = q1[v];
          q1[v] = f0;
        }
        // dx row rho is complete
        if (rho >= ho0 && rho < ho1) {
          PK o;
#pragma unroll
          for (int v = 0; v < V; ++v) o.set(v, acc[k3][v]);
          o.store_out(dxn + ((long)rho * W + col) * C);
          if constexpr (RED) {
#pragma unroll
            for (int v = 0; v < V; ++v) {
              const float z = fmaf(yraw[v], in.sc[v], in.sh[v]);
              const float g = o.get(v) * act_grad(z, pro.act);
              sg[v] += g;
              sgx[v] = fmaf(g, (yraw[v] - emu[v]) * ers[v], sgx[v]);
            }
          }
        }
#pragma unroll
        for (int v = 0; v < V; ++v) acc[k3][v] = 0.f;
      }
    }
  }

  // per channel: sum over the computing columns (column order), tap by tap, then the BN_e sums
  __syncthreads();
  float* red = (float*)smem;
  const int Cc = CVb * V;
  const long part = ((long)n * tl.strips + strip) * tl.coltiles + ct;
  auto colsum = [&](const float (&a)[V], float* dst) {
#pragma unroll
    for (int v = 0; v < V; ++v) red[tid * V + v] = comp ? a[v] : 0.f;
    __syncthreads();
    for (int e = tid; e < Cc; e += 256) {
      const int cve = e / V, v = e - cve * V;
      float s = 0.f;
      for (int pp = 1; pp <= P - 2; ++pp) s += red[(pp * CVb + cve) * V + v];
      dst[cg * Cc + e] = s;
    }
    __syncthreads();
  };
#pragma unroll
  for (int k = 0; k < 9; ++k) colsum(fa[k], slab + (part * 9 + k) * C);
  if constexpr (RED) {
    colsum(sg, gparts + part * 2 * C);
    colsum(sgx, gparts + part * 2 * C + C);
  }
}

// Issue-lean form of dw3x3_bwd_fused_kernel (the default; ROD_DWF_V1=1 selects the one above).
// Same engine, same per-element arithmetic and accumulation order (dx bit-identical), cut for
// the instruction stream (tools/dwfused_bench.py PMC: the step was ~230 VALU + ~90 SALU per
// barrier interval, 2 waves / SIMD, VALU-issue and latency bound):
//   * per-lane conditions leave the loop body: every thread (halo columns included) loads a
//     clamped, always-valid column, computes dx / filter / BN_e sums, and only the dx store is
//     predicated on `comp`; halo sums are dropped by the column reduction as before.  Row
//     conditions are block-uniform (scalar branches);
//   * channel pairs run as packed f32 ops (v_pk_fma / v_pk_mul / v_pk_add, per element the same
//     operation in the same order);
//   * the activation gradients are specialised (ReLU6: one compare pair + select), and the
//     BN_e gradient mask comes from the prologue's own z (the x element of the same row);
//   * yhat_e = fma(ye, rstd, -mean * rstd) (the stride-2 kernel's form).

// Project-gradient recompute (PW, ABI 20: rod_dw3x3_bwd_fused_pw).  In an inverted-residual block
// dz — the gradient at act_d(BN_d(yd)), i.e. at the project conv's input — is dy_p . W_p with dy_p
// the project BatchNorm's backward output [M][cout] (cout = 16..32) and W_p^T [C][cout].  Instead of
// reading a materialised C-wide dz, the kernel reads the cout-wide dy_p (rod_pw_bwd_gred_dyp writes
// it in place of dz) and forms each row step's dz tile [<=32 pixels][the block's channels] with the
// MFMA rod_pw_bwd_gred uses for it — v_mfma_f32_16x16x32_bf16, k zero-padded to 32, one instruction
// (cout <= 32) — rounded to bf16 once: bit-identical to the dz it would have written.  The tile is
// computed one step ahead by waves 0 .. 2*ceil(Cc/16)-1 (one 16x16 tile each, A fragments from a
// 3-step register ring like the other loads, B = W_p^T rows in registers) into a 3-slot LDS ring,
// which the step's existing barrier publishes; the dz read and write of 2*es*M*C bytes disappear.
struct DwPw {
  const bf16_t* dyp;   // [N*H*W][cout] (rows = the depthwise output pixels)
  const bf16_t* wt1;   // [C][cout]: W_p^T, the project conv's mode-1 GEMM layout
  int cout;
};
constexpr int DWPW_LD = 52;
#ifndef DW_QG_PW
#define DW_QG_PW 6
#endif   // LDS row stride (bf16) of the recomputed dz tile: <= 48 channels + pad

// V = 2: the same tile with twice the threads (512 per block), each holding 2 channels — half the
// per-thread weights, accumulators and BatchNorm constants, twice the waves in flight
template <typename T, int PACT, bool RED, int BACT, int V = 4, int D = 3, bool PW = false>
__global__ void __launch_bounds__(1024 / V, PW ? 4 : 1) dw3x3_bwd_fused2_kernel(const T* __restrict__ ye, const T* __restrict__ dz,
                                                               const T* __restrict__ yd, const float* __restrict__ w,
                                                               T* __restrict__ dx, float* __restrict__ slab,
                                                               float* __restrict__ gparts, int H, int W, int C,
                                                               DwTile tl, BnPro pro, DwBwdBn bd, DwPw pw = DwPw{}) {
  static_assert(D % 3 == 0, "the ring steps a multiple of the 3 accumulator rows");
  static_assert(!PW || (V == 2 && D == 3 && sizeof(T) == 2), "PW: the bf16 2-channel form, 3-step ring");
  constexpr int VP = V / 2;  // V channels per thread = VP packed pairs
  constexpr int TB = 1024 / V;      // threads per block (the tile of the 4-channel plan)
  typedef PackV<T, V> PK;
  // the row exchange holds the rounded fp32 pairs (no pack / unpack around the LDS trip); three
  // slots, one per step of the 3-step body, so every LDS address is the thread's base plus a
  // compile-time offset
  constexpr int XS = 3 * 2 * TB * VP * (int)sizeof(dw_f2);
  // the epilogue's staged column sums: all at once (dw_colsum_emit), or — PW, whose main loop
  // is at the 128-VGPR bound and spills with the one-barrier epilogue — DW_QG_PW at a time
  constexpr int SS = (PW ? DW_QG_PW : (RED ? 11 : 9)) * TB * V * 4;
  __shared__ __attribute__((aligned(16))) char smem[XS > SS ? XS : SS];
  dw_f2* xs = (dw_f2*)smem;
  dw_f2* dsl = xs + 3 * TB * VP;
  const int tid = threadIdx.x;
  const int CVb = tl.CVb * (4 / V), P = tl.P;
  const int p = tid / CVb, cvb = tid - (tid / CVb) * CVb;
  int bx, strip, n;
  xcd_block(bx, strip, n);
  const int cg = bx % tl.cgroups, ct = bx / tl.cgroups;
  const int c = (cg * CVb + cvb) * V;
  const int col = ct * tl.TWo + p - 1;
  const bool comp = p >= 1 && p <= P - 2 && col < W;
  const bool cok = p < P && col >= 0 && col < W;
  const int colc = col < 0 ? 0 : (col >= W ? W - 1 : col);         // always a valid address
  const int li = tid >= CVb ? tid - CVb : tid, ri = tid + CVb < TB ? tid + CVb : tid;
  const int ho0 = strip * tl.RB;
  const int ho1 = ho0 + tl.RB < H ? ho0 + tl.RB : H;
  const int xlo = ho0 - 1 > 0 ? ho0 - 1 : 0, xhi = ho1 < H - 1 ? ho1 : H - 1;

  dw_f2 wr[9][VP];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int h = 0; h < VP; ++h) wr[k][h] = dw_f2{w[k * C + c + 2 * h], w[k * C + c + 2 * h + 1]};
  dw_f2 psc[VP], psh[VP], ers[VP], enb[VP];
  int pact = 0;
  if constexpr (PACT >= 0) {
    pact = pro.act;
#pragma unroll
    for (int h = 0; h < VP; ++h) {
      float a0, b0, a1, b1;
      bn_pro_affine(pro, c + 2 * h, a0, b0);
      bn_pro_affine(pro, c + 2 * h + 1, a1, b1);
      psc[h] = dw_f2{a0, a1};
      psh[h] = dw_f2{b0, b1};
      if constexpr (RED) {
        ers[h] = dw_f2{pro.rstd[c + 2 * h], pro.rstd[c + 2 * h + 1]};
        enb[h] = dw_f2{-pro.mean[c + 2 * h] * ers[h].x, -pro.mean[c + 2 * h + 1] * ers[h].y};
      }
    }
  }
  dw_f2 dsc[VP], dsh[VP], da[VP], dmg[VP], dmx[VP], dmm[VP];
#pragma unroll
  for (int h = 0; h < VP; ++h) {
    const int c0 = c + 2 * h;
    float s0, t0, s1, t1, k10, k00, k11, k01, m0, m1;
    bn_affine(bd.mean, bd.rstd, bd.gamma, bd.beta, c0, s0, t0);
    bn_affine(bd.mean, bd.rstd, bd.gamma, bd.beta, c0 + 1, s1, t1);
    dsc[h] = dw_f2{s0, s1};
    dsh[h] = dw_f2{t0, t1};
    da[h] = dw_f2{bd.coef[c0], bd.coef[c0 + 1]};
    bn_bwd_k<T>(da[h].x, bd.mean[c0], bd.rstd[c0], bd.coef[C + c0], bd.coef[2 * C + c0], k10, k00, m0);
    bn_bwd_k<T>(da[h].y, bd.mean[c0 + 1], bd.rstd[c0 + 1], bd.coef[C + c0 + 1], bd.coef[2 * C + c0 + 1], k11, k01, m1);
    dmg[h] = dw_f2{k10, k11};   // the apply's k1 / k0 / centring shift (bn_bwd_k)
    dmx[h] = dw_f2{k00, k01};
    dmm[h] = dw_f2{m0, m1};
  }
  dw_f2 sg[VP], sgx[VP];
#pragma unroll
  for (int h = 0; h < VP; ++h) sg[h] = sgx[h] = dw_f2{0.f, 0.f};
  // buffer resources over this image (wave-uniform base); lane offset = its (clamped) column and
  // channels, the row goes in the scalar offset
  const long img = (long)n * H * W * C;
  const unsigned ib = (unsigned)((long)H * W * C * sizeof(T));
  const rsrc_t rye = rod_rsrc(ye + img, ib), rdz = rod_rsrc(dz + img, ib), ryd = rod_rsrc(yd + img, ib);
  const rsrc_t rdx = rod_rsrc(dx + img, ib), rnull = rod_rsrc(dx + img, 0u);
  const unsigned vo = (unsigned)(((long)colc * C + c) * sizeof(T));
  const unsigned vox = comp ? vo : ROD_OOB;   // halo lanes store nothing
  const unsigned rstrb = (unsigned)(W * C * sizeof(T));

  // PW: the dz-tile MFMA roles.  Wave wv < 2*NTN owns tile (mt, nt): pixels mt*16 + l16 of the
  // block's P columns (A: their dy_p rows, k = 8*g4 .. +7), channels nt*16 + l16 of the group
  // (B: W_p^T rows); lanes past P / the group's Cc / cout load zeros (out-of-range buffer loads)
  __shared__ __attribute__((aligned(16))) bf16_t dzs[PW ? 3 * 32 * DWPW_LD : 1];
  const int Ccg = CVb * V;
  const int lane = tid & 63, wv = tid >> 6, g4 = lane >> 4, l16 = lane & 15;
  const int NTN = (Ccg + 15) >> 4;
  const int mt = wv / NTN, nt = wv - (wv / NTN) * NTN;
  const bool mfw = PW && mt < 2;                      // wave-uniform
  bf16x8 fbw;
  rsrc_t rdp = rnull;
  unsigned voa = ROD_OOB, rstp = 0;
  if constexpr (PW) {
    const int pm = mt * 16 + l16, cm = nt * 16 + l16;
    const int colm = ct * tl.TWo + pm - 1;
    const int colmc = colm < 0 ? 0 : (colm >= W ? W - 1 : colm);
    const bool kin = 8 * g4 < pw.cout;
    voa = mfw && pm < P && kin ? (unsigned)(((long)colmc * pw.cout + 8 * g4) * 2) : ROD_OOB;
    rdp = rod_rsrc(pw.dyp + (long)n * H * W * pw.cout, (unsigned)((long)H * W * pw.cout * 2));
    rstp = (unsigned)(W * pw.cout * 2);
#pragma unroll
    for (int e = 0; e < 8; ++e) fbw[e] = (bf16_t)0.f;
    if (mfw && cm < Ccg && kin) fbw = *(const bf16x8*)(pw.wt1 + (long)(cg * Ccg + cm) * pw.cout + 8 * g4);
  }
  typedef unsigned dwpw_u4 __attribute__((ext_vector_type(4)));
  dwpw_u4 ra[PW ? D : 1];
  // the dz tile of the row whose dy_p fragment is `a` -> LDS slot `dst` (rounded to bf16 once)
  auto dz_tile = [&](const dwpw_u4& a, int dst) {
    if (mfw) {
      f32x4 t4 = {0.f, 0.f, 0.f, 0.f};
      t4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), fbw, t4, 0, 0, 0);
      if (nt * 16 + l16 < Ccg) {
        bf16_t* d = dzs + (dst * 32 + mt * 16 + 4 * g4) * DWPW_LD + nt * 16 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r * DWPW_LD] = (bf16_t)t4[r];
      }
    }
  };

  PK rx[D], rz[PW ? 1 : D], ry[D];
  // every step loads all three rows unconditionally, rows clamped into [xlo, xhi] (a clamped row
  // re-reads one the block just read: a cache hit; the xok / dok masks zero its use), and the dx
  // store is a buffer store every step (dropped by the range check off the strip / on halo
  // lanes): with no memory operation under a branch the compiler counts the ring exactly
  // (s_waitcnt vmcnt(N) for the step being consumed) instead of draining every load in flight
  // (vmcnt(0)) at each step.
  auto issue = [&](int k, int q) {
    const int rho = ho0 - 2 + q;
    const int rx_ = rho < xlo ? xlo : (rho > xhi ? xhi : rho);
    const int rd_ = rho + 1 < xlo ? xlo : (rho + 1 > xhi ? xhi : rho + 1);
    rx[k].bload(rye, vo, (unsigned)rx_ * rstrb);
    if constexpr (PW) ra[k] = buf_ld<dwpw_u4>(rdp, voa, (unsigned)rd_ * rstp);
    else rz[k].bload(rdz, vo, (unsigned)rd_ * rstrb);
    ry[k].bload(ryd, vo, (unsigned)rd_ * rstrb);
  };
  const int nst = ho1 - ho0 + 3;
  // the prologue issues the slots in order (slot 0 first), so that the loop header's wait for
  // slot 0 is the same count on entry as around the back-edge
#pragma unroll
  for (int k = 0; k < D; ++k) {
    issue(k, k);
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (PW) {   // step 0's dz tile, published before the loop
    dz_tile(ra[0], 0);
    __syncthreads();
  }
  dw_f2 acc[3][VP], fa[9][VP], q1[VP], q2[VP];
#pragma unroll
  for (int h = 0; h < VP; ++h) {
    acc[0][h] = acc[1][h] = acc[2][h] = q1[h] = q2[h] = dw_f2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 9; ++k) fa[k][h] = dw_f2{0.f, 0.f};
  }
  for (int q0 = 0; q0 < nst; q0 += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int q = q0 + k;
      if constexpr (D > 3) {  // the deep ring's tail: whole 3-step groups only (block-uniform), so
        if (k % 3 == 0 && q >= nst) break;   // every path to the back-edge issued the same loads
      }
      const int rho = ho0 - 2 + q;
      const int k3 = k % 3;
      const int buf = k3;
      const bool xok = cok && rho >= xlo && rho <= xhi;
      const bool dok = cok && rho + 1 >= xlo && rho + 1 <= xhi;
      // x row rho (prologue, rounded to T) and, with RED, BN_e's gradient mask at the same element
      dw_f2 xv[VP], yr[VP], em[VP];
      unpackv(rx[k], yr);
#pragma unroll
      for (int h = 0; h < VP; ++h) {
        dw_f2 a = yr[h];
        if constexpr (PACT >= 0) {
          const dw_f2 z = f2fma(a, psc[h], psh[h]);
          dw_f2 t;
          if constexpr (PACT == ROD_ACT_RELU6) {
            t = dw_f2{act_t<ROD_ACT_RELU6>(z.x), act_t<ROD_ACT_RELU6>(z.y)};
          } else {
            t = dw_f2{act_fwd(z.x, pact), act_fwd(z.y, pact)};
          }
          a = round2(t, T{});
          if constexpr (RED) em[h] = z;   // BN_e's pre-activation: the gradient gate of this element
        }
        xv[h] = xok ? a : dw_f2{0.f, 0.f};
      }
      // dy row rho + 1: BN_d backward apply (rod_bn_bwd_apply's arithmetic), rounded to T
      dw_f2 dv[VP];
      {
        dw_f2 yv[VP], zv[VP];
        unpackv(ry[k], yv);
        if constexpr (PW) {   // this step's dz pair from the recomputed tile (slot k % 3)
          const unsigned u = *(const unsigned*)(dzs + ((k % 3) * 32 + (p < 32 ? p : 31)) * DWPW_LD + cvb * 2);
          zv[0] = dw_f2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
        } else {
          unpackv(rz[k], zv);
        }
#pragma unroll
        for (int h = 0; h < VP; ++h) {
          const dw_f2 z = f2fma(yv[h], dsc[h], dsh[h]);
          const dw_f2 g = gate2<BACT>(z, zv[h], bd.act);
          // bn_bwd_apply1<T>, pairwise
          const dw_f2 yc = sizeof(T) == 4 ? yv[h] - dmm[h] : yv[h];
          const dw_f2 o = f2fma(da[h], g, f2fma(dmg[h], yc, dmx[h]));
          dv[h] = dok ? round2(o, T{}) : dw_f2{0.f, 0.f};
        }
      }
      // keep the ring slot's reload after its last read: the scheduler hoisting it would make the
      // slot's old and new values overlap, and the copy that resolves that at the loop back-edge
      // has to wait for the load in flight (s_waitcnt vmcnt(0))
      __builtin_amdgcn_sched_barrier(0);
      issue(k, q + D);
      if constexpr (PW) dz_tile(ra[(k + 1) % D], (k + 1) % 3);   // the next step's dz, published below
#pragma unroll
      for (int h = 0; h < VP; ++h) {
        xs[(buf * TB + tid) * VP + h] = xv[h];
        dsl[(buf * TB + tid) * VP + h] = dv[h];
      }
      __syncthreads();
      dw_f2 xl[VP], xr[VP], dl[VP], dr[VP];
#pragma unroll
      for (int h = 0; h < VP; ++h) {
        xl[h] = xs[(buf * TB + li) * VP + h];
        xr[h] = xs[(buf * TB + ri) * VP + h];
        dl[h] = dsl[(buf * TB + li) * VP + h];
        dr[h] = dsl[(buf * TB + ri) * VP + h];
      }
      // backward-data: dy row rho+1 is tap row 0 of dx row rho, 1 of rho+1, 2 of rho+2
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int sl = (k3 + i) % 3;
#pragma unroll
        for (int h = 0; h < VP; ++h) {
          dw_f2 a = acc[sl][h];
          a = f2fma(dl[h], wr[i * 3 + 2][h], a);
          a = f2fma(dv[h], wr[i * 3 + 1][h], a);
          a = f2fma(dr[h], wr[i * 3][h], a);
          acc[sl][h] = a;
        }
      }
      // filter: x row rho with the strip's dy rows rho+1 (tap row 0), rho (1), rho-1 (2)
      const bool own = rho + 1 >= ho0 && rho + 1 < ho1;
#pragma unroll
      for (int h = 0; h < VP; ++h) {
        const dw_f2 f0 = own ? dv[h] : dw_f2{0.f, 0.f};
        fa[0][h] = f2fma(f0, xl[h], fa[0][h]);
        fa[1][h] = f2fma(f0, xv[h], fa[1][h]);
        fa[2][h] = f2fma(f0, xr[h], fa[2][h]);
        fa[3][h] = f2fma(q1[h], xl[h], fa[3][h]);
        fa[4][h] = f2fma(q1[h], xv[h], fa[4][h]);
        fa[5][h] = f2fma(q1[h], xr[h], fa[5][h]);
        fa[6][h] = f2fma(q2[h], xl[h], fa[6][h]);
        fa[7][h] = f2fma(q2[h], xv[h], fa[7][h]);
        fa[8][h] = f2fma(q2[h], xr[h], fa[8][h]);
        q2[h] = q1[h];
        q1[h] = f0;
      }
      // dx row rho is complete
      const bool rowout = rho >= ho0 && rho < ho1;
      PK o;
#pragma unroll
      for (int h = 0; h < VP; ++h) {
        if constexpr (sizeof(T) == 2) {   // one v_cvt_pk_bf16_f32 per pair
          const dw_b2 b = __builtin_convertvector(acc[k3][h], dw_b2);
          o.v[2 * h] = b.x;
          o.v[2 * h + 1] = b.y;
        } else {
          o.set(2 * h, acc[k3][h].x);
          o.set(2 * h + 1, acc[k3][h].y);
        }
      }
      if (rowout) {   // BN_e sums from the rounded dx, before the store (its last use)
        if constexpr (RED) {
#pragma unroll
          for (int h = 0; h < VP; ++h) {
            const dw_f2 ov = dw_f2{o.get(2 * h), o.get(2 * h + 1)};
            const dw_f2 g = gate2<PACT>(em[h], ov, pact);
            sg[h] += g;
            sgx[h] = f2fma(g, f2fma(yr[h], ers[h], enb[h]), sgx[h]);
          }
        }
      }
      o.bstore(rowout ? rdx : rnull, vox, (unsigned)(rho < 0 ? 0 : rho) * rstrb);
#pragma unroll
      for (int h = 0; h < VP; ++h) acc[k3][h] = dw_f2{0.f, 0.f};
    }
  }

  __syncthreads();
  float* red = (float*)smem;
  const int Cc = CVb * V;
  const long part = ((long)n * tl.strips + strip) * tl.coltiles + ct;
  constexpr int NQ = RED ? 11 : 9;
  // quantities per staging round: all at once, or (PW, whose row loop runs at the 128-VGPR
  // bound and spills with an all-at-once epilogue) QG_PW at a time
  constexpr int QG = PW ? DW_QG_PW : NQ;
  auto stage = [&](const dw_f2 (&a)[VP], int slot) {
#pragma unroll
    for (int h = 0; h < VP; ++h) {
      red[(slot * TB + tid) * V + 2 * h] = comp ? a[h].x : 0.f;
      red[(slot * TB + tid) * V + 2 * h + 1] = comp ? a[h].y : 0.f;
    }
  };
#pragma unroll
  for (int q0 = 0; q0 < NQ; q0 += QG) {
#pragma unroll
    for (int qk = q0; qk < q0 + QG && qk < NQ; ++qk) {
      if (qk < 9) stage(fa[qk], qk - q0);
      else if constexpr (RED) stage(qk == 9 ? sg : sgx, qk - q0);
    }
    __syncthreads();
    dw_colsum_emit<V>(red, q0, (q0 + QG < NQ ? q0 + QG : NQ) - q0, TB, Cc, CVb, P, slab, gparts, part, C, cg);
    if (q0 + QG < NQ) __syncthreads();
  }
}

// Stride-2 form.  Thread (p, cvb) owns output column b = wo0 + p - 1 (one halo column each
// side) and the dx / x column pair (2b - pl, 2b - pl + 1); step q handles dy row a = a0 - 1 + q
// and the x / dx rows 2a - pt, 2a + 1 - pt.  dx's 2x2 block (rows 2a-pt, 2a+1-pt x its column
// pair) takes dy[a][b], dy[a][b-1] (left neighbour, LDS) and the previous step's dy[a-1][b],
// dy[a-1][b-1], in the order of dw3x3_bwd_data_s2_kernel (bit-identical dx); the filter pairs
// dy[a] with x rows 2a-pt (tap row 0), 2a+1-pt (1) and dy[a-1] with 2a-pt (2), the third tap
// column coming from the right neighbour's first column (LDS).
template <typename T, int PACT, bool RED, int D = 3>
__global__ void __launch_bounds__(256, 2) dw3x3_bwd_fused_s2_kernel(const T* __restrict__ ye, const T* __restrict__ dz,
                                                                 const T* __restrict__ yd, const float* __restrict__ w,
                                                                 T* __restrict__ dx, float* __restrict__ slab,
                                                                 float* __restrict__ gparts, int H, int W, int C,
                                                                 int pt, int pl, int Ho, int Wo, DwTile tl, BnPro pro,
                                                                 DwBwdBn bd) {
  constexpr int V = 4;
  typedef PackV<T, V> PK;
  constexpr int XS = 3 * 2 * 256 * (int)sizeof(PK);  // dy, x row 0, x row 1 slots, double buffered
  constexpr int SS = 256 * V * 4;
  __shared__ __attribute__((aligned(16))) char smem[XS > SS ? XS : SS];
  PK* dsl = (PK*)smem;         // [2][256]
  PK* x0s = dsl + 2 * 256;     // [2][256]
  PK* x1s = x0s + 2 * 256;     // [2][256]
  const int tid = threadIdx.x;
  const int CVb = tl.CVb, P = tl.P;
  const int p = tid / CVb, cvb = tid - (tid / CVb) * CVb;
  int bx, strip, n;
  xcd_block(bx, strip, n);
  const int cg = bx % tl.cgroups, ct = bx / tl.cgroups;
  const int c = (cg * CVb + cvb) * V;
  const int b = ct * tl.TWo + p - 1;
  const int ci0 = 2 * b - pl;
  // the tiled map is (A, B): every a / b with a dx row / column (dy rows >= Ho read as zero)
  const int A = ((H - 1 + pt) >> 1) + 1, B = ((W - 1 + pl) >> 1) + 1;
  const bool comp = p >= 1 && p <= P - 2 && b < B;
  const bool cokd = p < P && b >= 0 && b < Wo;
  const bool cok0 = p < P && ci0 >= 0 && ci0 < W;
  const bool cok1 = p < P && ci0 + 1 >= 0 && ci0 + 1 < W;
  const int a0 = strip * tl.RB;
  const int a1 = a0 + tl.RB < A ? a0 + tl.RB : A;

  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = w[k * C + c + v];
  DwIn<T, V, PACT> in;
  in.init(pro, c);
  float dsc[V], dsh[V], da[V], dmg[V], dmx[V], dmm[V];   // dmg / dmx / dmm: the apply's k1 / k0 / m
#pragma unroll
  for (int v = 0; v < V; ++v) {
    bn_affine(bd.mean, bd.rstd, bd.gamma, bd.beta, c + v, dsc[v], dsh[v]);
    da[v] = bd.coef[c + v];
    bn_bwd_k<T>(da[v], bd.mean[c + v], bd.rstd[c + v], bd.coef[C + c + v], bd.coef[2 * C + c + v], dmg[v], dmx[v],
                dmm[v]);
  }
  constexpr int RV = RED ? V : 1;
  float enb[RV], ers[RV], sg[RV], sgx[RV];  // xhat_e = fma(y_e, rstd, -mean * rstd)
  if constexpr (RED) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      ers[v] = pro.rstd[c + v];
      enb[v] = -pro.mean[c + v] * ers[v];
      sg[v] = sgx[v] = 0.f;
    }
  }
  // buffer resources over this image; every load is issued (rows / columns clamped into the
  // map, uses masked by okd / okx) and every dx store too (vo = ROD_OOB where nothing is to be
  // written), so the wait counts of the prefetch ring stay exact (see rod_common.h)
  const unsigned es = sizeof(T);
  const rsrc_t rye = rod_rsrc(ye + (long)n * H * W * C, (unsigned)((long)H * W * C * es));
  const rsrc_t rdx = rod_rsrc(dx + (long)n * H * W * C, (unsigned)((long)H * W * C * es));
  const rsrc_t rnull = rod_rsrc(dx + (long)n * H * W * C, 0u);
  const rsrc_t rdz = rod_rsrc(dz + (long)n * Ho * Wo * C, (unsigned)((long)Ho * Wo * C * es));
  const rsrc_t ryd = rod_rsrc(yd + (long)n * Ho * Wo * C, (unsigned)((long)Ho * Wo * C * es));
  const int bc = b < 0 ? 0 : (b >= Wo ? Wo - 1 : b);
  const int x0c = ci0 < 0 ? 0 : (ci0 >= W ? W - 1 : ci0), x1c = ci0 + 1 < 0 ? 0 : (ci0 + 1 >= W ? W - 1 : ci0 + 1);
  const unsigned vod = (unsigned)(((long)bc * C + c) * es);
  const unsigned vox0 = (unsigned)(((long)x0c * C + c) * es), vox1 = (unsigned)(((long)x1c * C + c) * es);
  const unsigned vst0 = comp && cok0 ? vox0 : ROD_OOB, vst1 = comp && cok1 ? vox1 : ROD_OOB;
  const unsigned rsx = (unsigned)(W * C * es), rsd = (unsigned)(Wo * C * es);

  // ring slot: dy (dz, yd) of row a, x (ye) at rows 2a-pt, 2a+1-pt x columns ci0, ci0+1
  PK rz[D], ry[D], rx[D][4];
  bool okd[D], okx[D][4];
  const int dlo = a0 - 1 > 0 ? a0 - 1 : 0;
  const int dhi = a1 - 1 < Ho - 1 ? a1 - 1 : Ho - 1;
  auto issue = [&](int k, int q) {
    const int a = a0 - 1 + q;
    okd[k] = cokd && a >= dlo && a <= dhi;
    const int ac = a < dlo ? dlo : (a > dhi ? dhi : a);
    rz[k].bload(rdz, vod, (unsigned)ac * rsd);
    ry[k].bload(ryd, vod, (unsigned)ac * rsd);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = 2 * a - pt + (i >> 1);
      const bool rowok = a >= a0 && (i < 2 ? a <= a1 : a < a1) && h >= 0 && h < H;
      okx[k][i] = rowok && ((i & 1) ? cok1 : cok0);
      const int hc = h < 0 ? 0 : (h >= H ? H - 1 : h);
      rx[k][i].bload(rye, (i & 1) ? vox1 : vox0, (unsigned)hc * rsx);
    }
  };
  const int nst = a1 - a0 + 2;
#pragma unroll
  for (int k = 0; k < D; ++k) {   // slot order (the loop header's wait is then the same on entry)
    issue(k, k);
    __builtin_amdgcn_sched_barrier(0);
  }
  float fa[9][V], pv[V], pL[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    pv[v] = pL[v] = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) fa[k][v] = 0.f;
  }
  for (int q0 = 0; q0 < nst; q0 += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int q = q0 + k;
      const int a = a0 - 1 + q;
      const int buf = q & 1;
      float dv[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float yv = ry[k].get(v);
        const float z = fmaf(yv, dsc[v], dsh[v]);
        const float g = rz[k].get(v) * act_grad(z, bd.act);
        const float o = bn_bwd_apply1<T>(da[v], g, dmg[v], dmx[v], dmm[v], yv);
        dv[v] = okd[k] ? to_f32(from_f32<T>(o)) : 0.f;
      }
      float xv[4][V], yr[4][V];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        in.cvt(rx[k][i], okx[k][i], xv[i]);
#pragma unroll
        for (int v = 0; v < V; ++v) {
          if constexpr (PACT < 0) xv[i][v] = okx[k][i] ? xv[i][v] : 0.f;
          yr[i][v] = rx[k][i].get(v);
        }
      }
      PK pd, p0, p1;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        pd.set(v, dv[v]);
        p0.set(v, xv[0][v]);
        p1.set(v, xv[2][v]);
      }
      __builtin_amdgcn_sched_barrier(0);   // the slots' reloads stay after their last reads
      issue(k, q + D);
      dsl[buf * 256 + tid] = pd;
      x0s[buf * 256 + tid] = p0;
      x1s[buf * 256 + tid] = p1;
      __syncthreads();
      {
        // every lane computes (halo lanes' results are dropped: stores out of range, column sums
        // masked by comp), so no memory operation sits under a branch
        const int li = tid >= CVb ? tid - CVb : tid, ri = tid + CVb < 256 ? tid + CVb : tid;
        const PK dlp = dsl[buf * 256 + li];
        const PK r0 = x0s[buf * 256 + ri], r1 = x1s[buf * 256 + ri];
        float dL[V];
#pragma unroll
        for (int v = 0; v < V; ++v) dL[v] = dlp.get(v);
        const bool own = a >= a0 && a < a1, ownp = a - 1 >= a0 && a - 1 < a1;
        // dx block: taps as dw3x3_bwd_data_s2_kernel (c1 = dy[a][b], c0 = dy[a][b-1], p1, p0 = row a-1)
        float o[4][V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float c1 = dv[v], c0 = dL[v], p1v = pv[v], p0v = pL[v];
          o[0][v] = fmaf(p0v, wr[8][v], fmaf(p1v, wr[6][v], fmaf(c0, wr[2][v], c1 * wr[0][v])));
          o[1][v] = fmaf(p1v, wr[7][v], c1 * wr[1][v]);
          o[2][v] = fmaf(c0, wr[5][v], c1 * wr[3][v]);
          o[3][v] = c1 * wr[4][v];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int h = 2 * a - pt + (i >> 1);
          const bool hok = own && h >= 0 && h < H;
          PK pk;
#pragma unroll
          for (int v = 0; v < V; ++v) pk.set(v, o[i][v]);
          if constexpr (RED) {   // BN_e sums from the rounded dx, before the store (its last use)
            if (hok) {
              const bool cc = (i & 1) ? cok1 : cok0;
#pragma unroll
              for (int v = 0; v < V; ++v) {
                const float z = fmaf(yr[i][v], in.sc[v], in.sh[v]);
                const float g = cc ? pk.get(v) * act_grad(z, pro.act) : 0.f;
                sg[v] += g;
                sgx[v] = fmaf(g, fmaf(yr[i][v], ers[v], enb[v]), sgx[v]);
              }
            }
          }
          pk.bstore(hok ? rdx : rnull, (i & 1) ? vst1 : vst0, (unsigned)(hok ? h : 0) * rsx);
        }
        // filter: dy[a] with x rows 2a-pt (tap row 0) and 2a+1-pt (1), dy[a-1] with 2a-pt (2)
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float f0 = own ? dv[v] : 0.f, f2 = ownp ? pv[v] : 0.f;
          const float t02 = r0.get(v), t12 = r1.get(v);
          fa[0][v] = fmaf(f0, xv[0][v], fa[0][v]);
          fa[1][v] = fmaf(f0, xv[1][v], fa[1][v]);
          fa[2][v] = fmaf(f0, t02, fa[2][v]);
          fa[3][v] = fmaf(f0, xv[2][v], fa[3][v]);
          fa[4][v] = fmaf(f0, xv[3][v], fa[4][v]);
          fa[5][v] = fmaf(f0, t12, fa[5][v]);
          fa[6][v] = fmaf(f2, xv[0][v], fa[6][v]);
          fa[7][v] = fmaf(f2, xv[1][v], fa[7][v]);
          fa[8][v] = fmaf(f2, t02, fa[8][v]);
          pv[v] = dv[v];
          pL[v] = dL[v];
        }
      }
    }
  }

  __syncthreads();
  float* red = (float*)smem;
  const int Cc = CVb * V;
  const long part = ((long)n * tl.strips + strip) * tl.coltiles + ct;
  auto colsum = [&](const float (&acc)[V], float* dst) {
#pragma unroll
    for (int v = 0; v < V; ++v) red[tid * V + v] = comp ? acc[v] : 0.f;
    __syncthreads();
    for (int e = tid; e < Cc; e += 256) {
      const int cve = e / V, v = e - cve * V;
      float s = 0.f;
      for (int pp = 1; pp <= P - 2; ++pp) s += red[(pp * CVb + cve) * V + v];
      dst[cg * Cc + e] = s;
    }
    __syncthreads();
  };
#pragma unroll
  for (int k = 0; k < 9; ++k) colsum(fa[k], slab + (part * 9 + k) * C);
  if constexpr (RED) {
    colsum(sg, gparts + part * 2 * C);
    colsum(sgx, gparts + part * 2 * C + C);
  }
}

// Packed stride-2 form (bf16, the default): the same tile, step order, dx accumulation order
// (bit-identical dx) and filter / BN_e sums as dw3x3_bwd_fused_s2_kernel, with the four channels
// of a thread as two packed fp32 pairs (v_pk_fma / v_pk_mul: one instruction per pair), the
// BatchNorm-backward apply in its two-FMA form, one v_cvt_pk_bf16_f32 per rounded pair, the
// ReLU6 gates as selects, the row exchange in fp32 pairs (no pack / unpack around the LDS trip)
// with one LDS slot per step of the 2-step body (compile-time addresses), and the BN_e gate
// taken from the prologue's own pre-activation.
template <int PACT, bool RED, int BACT, int D = 2, int V = 4>
__global__ void __launch_bounds__(1024 / V, V == 4 ? 2 : 1) dw3x3_bwd_fused_s2p_kernel(
    const bf16_t* __restrict__ ye, const bf16_t* __restrict__ dz, const bf16_t* __restrict__ yd,
    const float* __restrict__ w, bf16_t* __restrict__ dx, float* __restrict__ slab, float* __restrict__ gparts, int H,
    int W, int C, int pt, int pl, int Ho, int Wo, DwTile tl, BnPro pro, DwBwdBn bd) {
  typedef bf16_t T;
  constexpr int VP = V / 2;
  constexpr int TB = 1024 / V;   // threads per block: the 4-channel tile with V channels a thread
  typedef PackV<T, V> PK;
  static_assert(D >= 2, "one LDS slot per step of the D-step body");
  // slots [D][3][256][VP] fp32 pairs: dy, x row 0, x row 1 (column ci0)
  constexpr int XS = D * 3 * TB * VP * (int)sizeof(dw_f2);
  constexpr int SS = (RED ? 11 : 9) * TB * V * 4;   // the epilogue's staged column sums
  __shared__ __attribute__((aligned(16))) char smem[XS > SS ? XS : SS];
  dw_f2* sl = (dw_f2*)smem;
  const int tid = threadIdx.x;
  const int CVb = tl.CVb * (4 / V), P = tl.P;
  const int p = tid / CVb, cvb = tid - (tid / CVb) * CVb;
  int bx, strip, n;
  xcd_block(bx, strip, n);
  const int cg = bx % tl.cgroups, ct = bx / tl.cgroups;
  const int c = (cg * CVb + cvb) * V;
  const int b = ct * tl.TWo + p - 1;
  const int ci0 = 2 * b - pl;
  const int A = ((H - 1 + pt) >> 1) + 1, B = ((W - 1 + pl) >> 1) + 1;
  const bool comp = p >= 1 && p <= P - 2 && b < B;
  const bool cokd = p < P && b >= 0 && b < Wo;
  const bool cok0 = p < P && ci0 >= 0 && ci0 < W;
  const bool cok1 = p < P && ci0 + 1 >= 0 && ci0 + 1 < W;
  const int a0 = strip * tl.RB;
  const int a1 = a0 + tl.RB < A ? a0 + tl.RB : A;
  const int li = tid >= CVb ? tid - CVb : tid, ri = tid + CVb < TB ? tid + CVb : tid;

  dw_f2 wr[9][VP];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int h = 0; h < VP; ++h) wr[k][h] = dw_f2{w[k * C + c + 2 * h], w[k * C + c + 2 * h + 1]};
  dw_f2 psc[VP], psh[VP], ers[VP], enb[VP];
  int pact = 0;
  if constexpr (PACT >= 0) {
    pact = pro.act;
#pragma unroll
    for (int h = 0; h < VP; ++h) {
      float a0_, b0_, a1_, b1_;
      bn_pro_affine(pro, c + 2 * h, a0_, b0_);
      bn_pro_affine(pro, c + 2 * h + 1, a1_, b1_);
      psc[h] = dw_f2{a0_, a1_};
      psh[h] = dw_f2{b0_, b1_};
      if constexpr (RED) {
        ers[h] = dw_f2{pro.rstd[c + 2 * h], pro.rstd[c + 2 * h + 1]};
        enb[h] = dw_f2{-pro.mean[c + 2 * h] * ers[h].x, -pro.mean[c + 2 * h + 1] * ers[h].y};
      }
    }
  }
  dw_f2 dsc[VP], dsh[VP], da[VP], dk1[VP], dk0[VP];
#pragma unroll
  for (int h = 0; h < VP; ++h) {
    const int c0 = c + 2 * h;
    float s0, t0, s1, t1, k10, k00, k11, k01;
    bn_affine(bd.mean, bd.rstd, bd.gamma, bd.beta, c0, s0, t0);
    bn_affine(bd.mean, bd.rstd, bd.gamma, bd.beta, c0 + 1, s1, t1);
    dsc[h] = dw_f2{s0, s1};
    dsh[h] = dw_f2{t0, t1};
    da[h] = dw_f2{bd.coef[c0], bd.coef[c0 + 1]};
    float m0, m1;   // bf16 storage: the folded form (m unused)
    bn_bwd_k<bf16_t>(da[h].x, bd.mean[c0], bd.rstd[c0], bd.coef[C + c0], bd.coef[2 * C + c0], k10, k00, m0);
    bn_bwd_k<bf16_t>(da[h].y, bd.mean[c0 + 1], bd.rstd[c0 + 1], bd.coef[C + c0 + 1], bd.coef[2 * C + c0 + 1], k11, k01,
                     m1);
    dk1[h] = dw_f2{k10, k11};
    dk0[h] = dw_f2{k00, k01};
  }
  dw_f2 sg[VP], sgx[VP];
#pragma unroll
  for (int h = 0; h < VP; ++h) sg[h] = sgx[h] = dw_f2{0.f, 0.f};

  const unsigned es = sizeof(T);
  const rsrc_t rye = rod_rsrc(ye + (long)n * H * W * C, (unsigned)((long)H * W * C * es));
  const rsrc_t rdx = rod_rsrc(dx + (long)n * H * W * C, (unsigned)((long)H * W * C * es));
  const rsrc_t rnull = rod_rsrc(dx + (long)n * H * W * C, 0u);
  const rsrc_t rdz = rod_rsrc(dz + (long)n * Ho * Wo * C, (unsigned)((long)Ho * Wo * C * es));
  const rsrc_t ryd = rod_rsrc(yd + (long)n * Ho * Wo * C, (unsigned)((long)Ho * Wo * C * es));
  const int bc = b < 0 ? 0 : (b >= Wo ? Wo - 1 : b);
  const int x0c = ci0 < 0 ? 0 : (ci0 >= W ? W - 1 : ci0), x1c = ci0 + 1 < 0 ? 0 : (ci0 + 1 >= W ? W - 1 : ci0 + 1);
  const unsigned vod = (unsigned)(((long)bc * C + c) * es);
  const unsigned vox0 = (unsigned)(((long)x0c * C + c) * es), vox1 = (unsigned)(((long)x1c * C + c) * es);
  const unsigned vst0 = comp && cok0 ? vox0 : ROD_OOB, vst1 = comp && cok1 ? vox1 : ROD_OOB;
  const unsigned rsx = (unsigned)(W * C * es), rsd = (unsigned)(Wo * C * es);

  PK rz[D], ry[D], rx[D][4];
  bool okd[D], okx[D][4];
  const int dlo = a0 - 1 > 0 ? a0 - 1 : 0;
  const int dhi = a1 - 1 < Ho - 1 ? a1 - 1 : Ho - 1;
  auto issue = [&](int k, int q) {
    const int a = a0 - 1 + q;
    okd[k] = cokd && a >= dlo && a <= dhi;
    const int ac = a < dlo ? dlo : (a > dhi ? dhi : a);
    rz[k].bload(rdz, vod, (unsigned)ac * rsd);
    ry[k].bload(ryd, vod, (unsigned)ac * rsd);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hh = 2 * a - pt + (i >> 1);
      const bool rowok = a >= a0 && (i < 2 ? a <= a1 : a < a1) && hh >= 0 && hh < H;
      okx[k][i] = rowok && ((i & 1) ? cok1 : cok0);
      const int hc = hh < 0 ? 0 : (hh >= H ? H - 1 : hh);
      rx[k][i].bload(rye, (i & 1) ? vox1 : vox0, (unsigned)hc * rsx);
    }
  };
  const int nst = a1 - a0 + 2;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    issue(k, k);
    __builtin_amdgcn_sched_barrier(0);
  }
  dw_f2 fa[9][VP], pv[VP], pL[VP];
#pragma unroll
  for (int h = 0; h < VP; ++h) {
    pv[h] = pL[h] = dw_f2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 9; ++k) fa[k][h] = dw_f2{0.f, 0.f};
  }
  const dw_f2 zero2 = dw_f2{0.f, 0.f};
  for (int q0 = 0; q0 < nst; q0 += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const int q = q0 + k;
      const int a = a0 - 1 + q;
      // dy[a][b]: BN_d backward apply (two-FMA form), rounded to bf16
      dw_f2 dv[VP];
      {
        dw_f2 yv[VP], zv[VP];
        unpackv(ry[k], yv);
        unpackv(rz[k], zv);
#pragma unroll
        for (int h = 0; h < VP; ++h) {
          const dw_f2 z = f2fma(yv[h], dsc[h], dsh[h]);
          const dw_f2 g = gate2<BACT>(z, zv[h], bd.act);
          const dw_f2 o = f2fma(da[h], g, f2fma(dk1[h], yv[h], dk0[h]));
          dv[h] = okd[k] ? round2(o, T{}) : zero2;
        }
      }
      // x at the 4 positions (prologue, rounded) and, with RED, BN_e's pre-activation (the gate)
      dw_f2 xv[4][VP], yr[4][VP], ez[4][VP];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        unpackv(rx[k][i], yr[i]);
#pragma unroll
        for (int h = 0; h < VP; ++h) {
          dw_f2 av = yr[i][h];
          if constexpr (PACT >= 0) {
            const dw_f2 z = f2fma(av, psc[h], psh[h]);
            dw_f2 t;
            if constexpr (PACT == ROD_ACT_RELU6) t = dw_f2{act_t<ROD_ACT_RELU6>(z.x), act_t<ROD_ACT_RELU6>(z.y)};
            else t = dw_f2{act_fwd(z.x, pact), act_fwd(z.y, pact)};
            av = round2(t, T{});
            if constexpr (RED) ez[i][h] = z;
          }
          xv[i][h] = okx[k][i] ? av : zero2;
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // the slots' reloads stay after their last reads
      issue(k, q + D);
      dw_f2* S = sl + k * 3 * TB * VP;
#pragma unroll
      for (int h = 0; h < VP; ++h) {
        S[tid * VP + h] = dv[h];
        S[(TB + tid) * VP + h] = xv[0][h];
        S[(2 * TB + tid) * VP + h] = xv[2][h];
      }
      __syncthreads();
      dw_f2 dL[VP], r0[VP], r1[VP];
#pragma unroll
      for (int h = 0; h < VP; ++h) {
        dL[h] = S[li * VP + h];
        r0[h] = S[(TB + ri) * VP + h];
        r1[h] = S[(2 * TB + ri) * VP + h];
      }
      const bool own = a >= a0 && a < a1, ownp = a - 1 >= a0 && a - 1 < a1;
      // dx 2x2 block in the order of dw3x3_bwd_data_s2_kernel (bit-identical)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hh = 2 * a - pt + (i >> 1);
        const bool hok = own && hh >= 0 && hh < H;
        dw_f2 o[VP];
#pragma unroll
        for (int h = 0; h < VP; ++h) {
          const dw_f2 c1 = dv[h], c0 = dL[h], p1v = pv[h], p0v = pL[h];
          if (i == 0) o[h] = f2fma(p0v, wr[8][h], f2fma(p1v, wr[6][h], f2fma(c0, wr[2][h], c1 * wr[0][h])));
          else if (i == 1) o[h] = f2fma(p1v, wr[7][h], c1 * wr[1][h]);
          else if (i == 2) o[h] = f2fma(c0, wr[5][h], c1 * wr[3][h]);
          else o[h] = c1 * wr[4][h];
        }
        PK pk;
        dw_f2 orr[VP];
#pragma unroll
        for (int h = 0; h < VP; ++h) {
          const dw_b2 bb = __builtin_convertvector(o[h], dw_b2);
          pk.v[2 * h] = bb.x;
          pk.v[2 * h + 1] = bb.y;
          const unsigned u = __builtin_bit_cast(unsigned, bb);
          orr[h] = dw_f2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
        }
        if constexpr (RED) {   // BN_e sums from the rounded dx, before the store (its last use)
          if (hok) {
            const bool cc = (i & 1) ? cok1 : cok0;
#pragma unroll
            for (int h = 0; h < VP; ++h) {
              const dw_f2 g = cc ? gate2<PACT>(ez[i][h], orr[h], pact) : zero2;
              sg[h] += g;
              sgx[h] = f2fma(g, f2fma(yr[i][h], ers[h], enb[h]), sgx[h]);
            }
          }
        }
        pk.bstore(hok ? rdx : rnull, (i & 1) ? vst1 : vst0, (unsigned)(hok ? hh : 0) * rsx);
      }
      // filter: dy[a] with x rows 2a-pt (tap row 0) and 2a+1-pt (1), dy[a-1] with 2a-pt (2)
      if (own) {
#pragma unroll
        for (int h = 0; h < VP; ++h) {
          fa[0][h] = f2fma(dv[h], xv[0][h], fa[0][h]);
          fa[1][h] = f2fma(dv[h], xv[1][h], fa[1][h]);
          fa[2][h] = f2fma(dv[h], r0[h], fa[2][h]);
          fa[3][h] = f2fma(dv[h], xv[2][h], fa[3][h]);
          fa[4][h] = f2fma(dv[h], xv[3][h], fa[4][h]);
          fa[5][h] = f2fma(dv[h], r1[h], fa[5][h]);
        }
      }
      if (ownp) {
#pragma unroll
        for (int h = 0; h < VP; ++h) {
          fa[6][h] = f2fma(pv[h], xv[0][h], fa[6][h]);
          fa[7][h] = f2fma(pv[h], xv[1][h], fa[7][h]);
          fa[8][h] = f2fma(pv[h], r0[h], fa[8][h]);
        }
      }
#pragma unroll
      for (int h = 0; h < VP; ++h) {
        pv[h] = dv[h];
        pL[h] = dL[h];
      }
    }
  }

  __syncthreads();
  float* red = (float*)smem;
  const int Cc = CVb * V;
  const long part = ((long)n * tl.strips + strip) * tl.coltiles + ct;
  auto stage = [&](const dw_f2 (&a)[VP], int qk) {
#pragma unroll
    for (int h = 0; h < VP; ++h) {
      red[(qk * TB + tid) * V + 2 * h] = comp ? a[h].x : 0.f;
      red[(qk * TB + tid) * V + 2 * h + 1] = comp ? a[h].y : 0.f;
    }
  };
#pragma unroll
  for (int k = 0; k < 9; ++k) stage(fa[k], k);
  if constexpr (RED) {
    stage(sg, 9);
    stage(sgx, 10);
  }
  __syncthreads();
  dw_colsum_emit<V>(red, 0, RED ? 11 : 9, TB, Cc, CVb, P, slab, gparts, part, C, cg);
}

extern "C" {

int rod_dw3x3_bwd_fused_parts(int N, int H, int W, int C, int stride, int pad_t, int pad_l) {
  int A, B;
  if (!dw_fused_geom(N, H, W, C, stride, pad_t, pad_l, A, B)) return 0;
  const DwTile t = dw_tile(N, A, B, C, 1, 4);
  return (int)((long)N * t.strips * t.coltiles);
}

size_t rod_dw3x3_bwd_fused_workspace(int N, int H, int W, int C, int stride, int pad_t, int pad_l) {
  return (size_t)rod_dw3x3_bwd_fused_parts(N, H, W, C, stride, pad_t, pad_l) * 9 * C * sizeof(float);
}

int rod_dw3x3_bwd_fused(const void* ye, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                        const float* pro_beta, int pro_act, const void* dz, const void* yd, const float* bn_mean,
                        const float* bn_rstd, const float* bn_gamma, const float* bn_beta, int bn_act,
                        const float* coef, const float* w, void* dx, float* dw, float* gparts, void* workspace, int N,
                        int H, int W, int C, int stride, int pad_t, int pad_l, int Ho, int Wo, int dtype,
                        void* stream) {
  int A = 0, B = 0;
  ROD_CHECK_ARG(dw_fused_geom(N, H, W, C, stride, pad_t, pad_l, A, B),
                "rod_dw3x3_bwd_fused: bad shape / stride / padding (C %% 4 != 0? stride 1 needs pad 1, stride 2 pad 0|1)");
  ROD_CHECK_ARG(Ho > 0 && Wo > 0 && (stride == 1 ? Ho == H && Wo == W : Ho <= A + 1 && Wo <= B + 1),
                "rod_dw3x3_bwd_fused: output map %dx%d does not match the input", Ho, Wo);
  ROD_CHECK_ARG(ye && dz && yd && bn_mean && bn_rstd && coef && w && dx && dw && workspace,
                "rod_dw3x3_bwd_fused: NULL tensor argument");
  ROD_CHECK_ARG(!pro_mean || pro_rstd, "rod_dw3x3_bwd_fused: BatchNorm prologue needs mean and rstd");
  ROD_CHECK_ARG(!gparts || pro_mean, "rod_dw3x3_bwd_fused: the BN_e sums need the input's BatchNorm prologue");
  ROD_CHECK_ARG(bn_act >= ROD_ACT_NONE && bn_act <= ROD_ACT_RELU, "rod_dw3x3_bwd_fused: bad act %d", bn_act);
  ROD_CHECK_ARG(dtype == ROD_F32 || dtype == ROD_BF16, "rod_dw3x3_bwd_fused: bad dtype %d", dtype);
  const int al = dtype == ROD_BF16 ? 7 : 15;
  ROD_CHECK_ARG(((((uintptr_t)ye) | ((uintptr_t)dz) | ((uintptr_t)yd) | ((uintptr_t)dx)) & al) == 0,
                "rod_dw3x3_bwd_fused: tensors must be %d-byte aligned", al + 1);
  hipStream_t s = ROD_STREAM(stream);
  const DwTile t = dw_tile(N, A, B, C, 1, 4);
  const dim3 grid(t.coltiles * t.cgroups, t.strips, N);
  const BnPro pv{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  const DwBwdBn bd{bn_mean, bn_rstd, bn_gamma, bn_beta, coef, bn_act};
  const int pa = !pro_mean ? -1 : (pro_act == ROD_ACT_RELU6 ? ROD_ACT_RELU6 : DW_ACT_RT);
  float* slab = (float*)workspace;
  auto go = [&](auto tag) {
    typedef decltype(tag) T;
    // 4-channel stride-1 forms: prefetch ring depth 3; ROD_DWF_RING=6 (measurement switch)
    // measured 3.27 ms (3) vs 3.34 ms (6) for the first form over the step's bf16 shapes
    static const int ring_env = getenv("ROD_DWF_RING") ? atoi(getenv("ROD_DWF_RING")) : 0;
    const int ring = ring_env == 6 ? 6 : 3;
    // stride 1: the issue-lean kernel; ROD_DWF_V1=1 (A/B switch) the first form
    static const bool v1 = getenv("ROD_DWF_V1") && atoi(getenv("ROD_DWF_V1")) == 1;
    // bf16 default: 2 channels per thread in 512-thread blocks (122 VGPRs, 4 waves/SIMD) with a
    // 3-step ring: with branch-free buffer loads / stores the ring's wait counts are exact, and a
    // 6-step ring needs 131 VGPRs (3 waves/SIMD; capped at 128 it spills).  ROD_DWF_C2=0 the
    // 4-channel form, ROD_DWF_RING=6 the 6-step ring
    static const bool v2 = !(getenv("ROD_DWF_C2") && atoi(getenv("ROD_DWF_C2")) == 0);
    const int vring = ring_env == 6 ? 6 : 3;
#define DWF1(PA, R, D)                                                                                               \
  hipLaunchKernelGGL((dw3x3_bwd_fused_kernel<T, PA, R, D>), grid, dim3(256), 0, s, (const T*)ye, (const T*)dz,      \
                     (const T*)yd, w, (T*)dx, slab, gparts, H, W, C, t, pv, bd)
    // stride 2 ring (branch-free buffer I/O, exact wait counts): 2 steps for bf16 (238 VGPRs;
    // 3 steps spill), 1 for fp32 (16-byte slots: 2 steps spill)
    constexpr int D2 = sizeof(T) == 2 ? 2 : 1;
    // bf16: the packed form (ROD_DWF_S2P=0: the scalar one)
    static const bool s2p = !(getenv("ROD_DWF_S2P") && atoi(getenv("ROD_DWF_S2P")) == 0);
    // packed stride-2 form with 2 channels a thread in 512-thread blocks (116 VGPRs: 4 waves /
    // SIMD instead of 2 at 204): tools/dwfused_bench.py stride-2 shapes 1686 -> 1604 us, dx
    // bit-identical.  ROD_DWF_S2P_V=4: the 4-channel form; ROD_DWF_S2P_D=3: a 3-step ring (A/B)
    static const bool s2p2 = !(getenv("ROD_DWF_S2P_V") && atoi(getenv("ROD_DWF_S2P_V")) == 4);
    static const bool s2pd3 = getenv("ROD_DWF_S2P_D") && atoi(getenv("ROD_DWF_S2P_D")) == 3;
#define DWS2(PA, R)                                                                                                  \
  do {                                                                                                              \
    if constexpr (sizeof(T) == 2) {                                                                                 \
      if (s2p && s2p2 && s2pd3 && bn_act == ROD_ACT_RELU6) {                                                        \
        hipLaunchKernelGGL((dw3x3_bwd_fused_s2p_kernel<PA, R, ROD_ACT_RELU6, 3, 2>), grid, dim3(512), 0, s,         \
                           (const bf16_t*)ye, (const bf16_t*)dz, (const bf16_t*)yd, w, (bf16_t*)dx, slab, gparts, H,  \
                           W, C, pad_t, pad_l, Ho, Wo, t, pv, bd);                                                  \
        break;                                                                                                      \
      }                                                                                                             \
      if (s2p && s2p2 && bn_act == ROD_ACT_RELU6) {                                                                 \
        hipLaunchKernelGGL((dw3x3_bwd_fused_s2p_kernel<PA, R, ROD_ACT_RELU6, 2, 2>), grid, dim3(512), 0, s,         \
                           (const bf16_t*)ye, (const bf16_t*)dz, (const bf16_t*)yd, w, (bf16_t*)dx, slab, gparts, H,  \
                           W, C, pad_t, pad_l, Ho, Wo, t, pv, bd);                                                  \
        break;                                                                                                      \
      }                                                                                                             \
      if (s2p && bn_act == ROD_ACT_RELU6) {                                                                         \
        hipLaunchKernelGGL((dw3x3_bwd_fused_s2p_kernel<PA, R, ROD_ACT_RELU6>), grid, dim3(256), 0, s,               \
                           (const bf16_t*)ye, (const bf16_t*)dz, (const bf16_t*)yd, w, (bf16_t*)dx, slab, gparts, H,  \
                           W, C, pad_t, pad_l, Ho, Wo, t, pv, bd);                                                  \
        break;                                                                                                      \
      }                                                                                                             \
      if (s2p) {                                                                                                    \
        hipLaunchKernelGGL((dw3x3_bwd_fused_s2p_kernel<PA, R, DW_ACT_RT>), grid, dim3(256), 0, s, (const bf16_t*)ye,  \
                           (const bf16_t*)dz, (const bf16_t*)yd, w, (bf16_t*)dx, slab, gparts, H, W, C, pad_t, pad_l, \
                           Ho, Wo, t, pv, bd);                                                                      \
        break;                                                                                                      \
      }                                                                                                             \
    }                                                                                                               \
    hipLaunchKernelGGL((dw3x3_bwd_fused_s2_kernel<T, PA, R, D2>), grid, dim3(256), 0, s, (const T*)ye, (const T*)dz, \
                       (const T*)yd, w, (T*)dx, slab, gparts, H, W, C, pad_t, pad_l, Ho, Wo, t, pv, bd);             \
  } while (0)
#define DWV2(PA, R, BA)                                                                                              \
  do {                                                                                                              \
    if constexpr (sizeof(T) == 2) {                                                                                 \
      if (v2 && vring == 6)                                                                                         \
        hipLaunchKernelGGL((dw3x3_bwd_fused2_kernel<T, PA, R, BA, 2, 6>), grid, dim3(512), 0, s, (const T*)ye,      \
                           (const T*)dz, (const T*)yd, w, (T*)dx, slab, gparts, H, W, C, t, pv, bd);                \
      else if (v2)                                                                                                  \
        hipLaunchKernelGGL((dw3x3_bwd_fused2_kernel<T, PA, R, BA, 2>), grid, dim3(512), 0, s, (const T*)ye,         \
                           (const T*)dz, (const T*)yd, w, (T*)dx, slab, gparts, H, W, C, t, pv, bd);                \
      if (v2) break;                                                                                                \
    }                                                                                                               \
    if (ring == 6)                                                                                                  \
      hipLaunchKernelGGL((dw3x3_bwd_fused2_kernel<T, PA, R, BA, 4, 6>), grid, dim3(256), 0, s, (const T*)ye,        \
                         (const T*)dz, (const T*)yd, w, (T*)dx, slab, gparts, H, W, C, t, pv, bd);                  \
    else                                                                                                            \
      hipLaunchKernelGGL((dw3x3_bwd_fused2_kernel<T, PA, R, BA>), grid, dim3(256), 0, s, (const T*)ye, (const T*)dz, \
                         (const T*)yd, w, (T*)dx, slab, gparts, H, W, C, t, pv, bd);                                \
  } while (0)
#define DWF2(PA, R)                                                                                                  \
  do {                                                                                                              \
    if (stride == 2) DWS2(PA, R);                                                                                   \
    else if (!v1 && bn_act == ROD_ACT_RELU6) DWV2(PA, R, ROD_ACT_RELU6);                                            \
    else if (!v1) DWV2(PA, R, DW_ACT_RT);                                                                           \
    else if (ring == 3) DWF1(PA, R, 3);                                                                             \
    else DWF1(PA, R, 6);                                                                                            \
  } while (0)
    if (pa == ROD_ACT_RELU6) {
      if (gparts) DWF2(ROD_ACT_RELU6, true); else DWF2(ROD_ACT_RELU6, false);
    } else if (pa == DW_ACT_RT) {
      if (gparts) DWF2(DW_ACT_RT, true); else DWF2(DW_ACT_RT, false);
    } else {
      DWF2(-1, false);
    }
#undef DWF2
#undef DWV2
#undef DWS2
#undef DWF1
  };
  if (dtype == ROD_BF16) go(bf16_t{}); else go(float{});
  const int rc = check_launch("rod_dw3x3_bwd_fused");
  if (rc) return rc;
  slab_sum(slab, dw, (int)((long)N * t.strips * t.coltiles), 9L * C, s);
  return check_launch("rod_dw3x3_bwd_fused");
}

// PW (ABI 20): the plan the recompute kernel supports — bf16, stride 1, both BatchNorms ReLU6 (the
// inverted-residual block), cout a multiple of 8 up to 32 (one MFMA k step), and a tile of at most
// 32 columns x 48 channels (2 x 3 MFMA tiles on the block's 8 waves)
int rod_dw3x3_bwd_fused_pw_supported(int N, int H, int W, int C, int cout, int pro_act, int bn_act, int dtype) {
  int A = 0, B = 0;
  if (dtype != ROD_BF16 || cout <= 0 || cout > 32 || cout % 8 || pro_act != ROD_ACT_RELU6 ||
      bn_act != ROD_ACT_RELU6 || !dw_fused_geom(N, H, W, C, 1, 1, 1, A, B))
    return 0;
  const DwTile t = dw_tile(N, A, B, C, 1, 4);
  return t.P <= 32 && t.CVb * 4 <= 48 ? 1 : 0;
}

int rod_dw3x3_bwd_fused_pw(const void* ye, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                           const float* pro_beta, int pro_act, const void* dyp, const void* wt1, int cout,
                           const void* yd, const float* bn_mean, const float* bn_rstd, const float* bn_gamma,
                           const float* bn_beta, int bn_act, const float* coef, const float* w, void* dx, float* dw,
                           float* gparts, void* workspace, int N, int H, int W, int C, int dtype, void* stream) {
  ROD_CHECK_ARG(rod_dw3x3_bwd_fused_pw_supported(N, H, W, C, cout, pro_act, bn_act, dtype),
                "rod_dw3x3_bwd_fused_pw: unsupported plan (N=%d H=%d W=%d C=%d cout=%d acts %d/%d dtype %d)", N, H, W,
                C, cout, pro_act, bn_act, dtype);
  ROD_CHECK_ARG(ye && pro_mean && pro_rstd && dyp && wt1 && yd && bn_mean && bn_rstd && coef && w && dx && dw &&
                    workspace,
                "rod_dw3x3_bwd_fused_pw: NULL tensor argument");
  ROD_CHECK_ARG(((((uintptr_t)ye) | ((uintptr_t)yd) | ((uintptr_t)dx)) & 7) == 0 &&
                    ((((uintptr_t)dyp) | ((uintptr_t)wt1)) & 15) == 0,
                "rod_dw3x3_bwd_fused_pw: ye / yd / dx must be 8-byte, dyp / wt1 16-byte aligned");
  hipStream_t s = ROD_STREAM(stream);
  const DwTile t = dw_tile(N, H, W, C, 1, 4);
  const dim3 grid(t.coltiles * t.cgroups, t.strips, N);
  const BnPro pv{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  const DwBwdBn bd{bn_mean, bn_rstd, bn_gamma, bn_beta, coef, bn_act};
  const DwPw pw{(const bf16_t*)dyp, (const bf16_t*)wt1, cout};
  float* slab = (float*)workspace;
#define DWPW(R)                                                                                                     \
  hipLaunchKernelGGL((dw3x3_bwd_fused2_kernel<bf16_t, ROD_ACT_RELU6, R, ROD_ACT_RELU6, 2, 3, true>), grid, dim3(512), \
                     0, s, (const bf16_t*)ye, (const bf16_t*)nullptr, (const bf16_t*)yd, w, (bf16_t*)dx, slab, gparts,  \
                     H, W, C, t, pv, bd, pw)
  if (gparts) DWPW(true); else DWPW(false);
#undef DWPW
  const int rc = check_launch("rod_dw3x3_bwd_fused_pw");
  if (rc) return rc;
  slab_sum(slab, dw, (int)((long)N * t.strips * t.coltiles), 9L * C, s);
  return check_launch("rod_dw3x3_bwd_fused_pw");
}

}  // extern "C"
