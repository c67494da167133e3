// dwrc.hip — depthwise 3x3 forward of an inverted-residual block whose expanded input is
// recomputed from the narrow block input instead of read (ABI 23, rod_dw3x3_fwd_rc; reference
// conv_blocks.py:263-270 expand + mobilenet.py:417-420 BatchNorm + conv_blocks.py:238-247
// depthwise, in training).
//
// The depthwise input is xe = ReLU6(BN_e(ye)), ye = bf16(x_act . We^T) the expand conv's output
// (x_act the block input x through its own pending BatchNorm).  rod_dw3x3_fwd reads ye (the
// C-wide expanded tensor: 1.42 GB at 720p b8 for block 1's 16 -> 96) and applies BN_e + ReLU6 in
// its load prologue.  Here a block reads its x rows instead (Cin = 16..32 channels: 6x fewer
// bytes) and forms each input row of its tile with MFMA:
//   * x rows go through a two-slot LDS ring (the input prologue applied, k zero-padded to 32);
//   * ye^T tile by tile — A = We rows (16 channels x k, in registers), B = the row's x
//     (k x 16 pixels) — v_mfma_f32_16x16x32_bf16, the expand forward's instruction with the
//     operands swapped, so every ye value is the stored one bit for bit; BN_e + ReLU6 and the
//     rounding in the epilogue, one 8-byte LDS write of 4 channels per lane and tile, into a
//     two-slot [pixel][channel] tile (pixels outside the map / rows outside the strip: 0, the
//     padding the reference convolves);
//   * the depthwise part is rod_dw3x3_fwd's LDS-exchange engine with its exchange slot replaced
//     by that tile: thread (p, cvb) reads its column (pair) and right neighbour from it, the same
//     tap order, rounding, statistics and tile plan (dw_tile: the same part structure), so y and
//     the BatchNorm parts are bit-identical to rod_dw3x3_fwd over the stored ye.
// One barrier per input row: row q's tile is read, row q+1's formed, row q+2's x staged.
#include "rod_common.h"
#include "dw_common.h"

namespace rod {

typedef float rc_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 rc_b2 __attribute__((ext_vector_type(2)));

struct DwRcArgs {
  const bf16_t* x;      // [N, H, W, Cin] block input
  BnPro xp;             // its pending BatchNorm (mean NULL: none)
  const bf16_t* wt0;    // [C][Cin] expand forward operand
  BnPro ep;             // the expand BatchNorm + ReLU6: the depthwise input
  const float* w;       // [3][3][C]
  bf16_t* y;            // [N, Ho, Wo, C]
  float* parts;         // statistics parts or NULL
  int H, W, C, pt, pl, Ho, Wo;
};

constexpr int RC_XLD = 40;   // x slot row: k 0..31 (zero past Cin) + 8 pad (bf16 elements)

// LDS plan of one block (bytes): two x slots, two ye tiles, the two prologue tables
struct DwRcLds {
  int npt, nct, ldy;
  size_t xs, ys, tabs, total;
};
inline DwRcLds dw_rc_lds(const DwTile& t, int S, int V, int Cin) {
  DwRcLds l;
  const int npix = S == 2 ? 2 * t.P : t.P;
  const int Cc = t.CVb * V;
  l.npt = std::max(2, (npix + 15) / 16);   // the kernel instantiates 2, 3 or 4 pixel tiles
  l.nct = (Cc + 15) / 16;
  l.ldy = l.nct * 16 + 8;
  l.xs = (size_t)2 * l.npt * 16 * RC_XLD * 2;
  l.ys = (size_t)2 * l.npt * 16 * l.ldy * 2;
  l.tabs = (size_t)(2 * Cin + 2 * l.nct * 16) * 4;
  const size_t stats = (size_t)(256 * (2 * V + 1) + 3 * 512) * 4;   // the epilogue merge (reuses the front)
  l.total = std::max(l.xs + l.ys + l.tabs, stats);
  return l;
}

template <int S, int V, int CIN, bool STATS, int NPT>
__global__ void __launch_bounds__(256) dw3x3_fwd_rc_kernel(DwRcArgs a, DwTile tl, int nct, int ldy) {
  constexpr int npt = NPT;
  typedef bf16_t T;
  typedef PackV<T, V> PK;
  static_assert(CIN % 8 == 0 && CIN <= 32, "one k step");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int CVb = tl.CVb, P = tl.P;
  const int p = tid / CVb, cvb = tid - (tid / CVb) * CVb;
  int bx, strip, n;
  xcd_block(bx, strip, n);
  const int cg = bx % tl.cgroups, ct = bx / tl.cgroups;
  const int Cc = CVb * V, cb = cg * Cc;
  const int c = cb + cvb * V;
  const int H = a.H, W = a.W, C = a.C, Ho = a.Ho, Wo = a.Wo;
  const int wo0 = ct * tl.TWo;
  const int ho0 = strip * tl.RB;
  const int ho1 = ho0 + tl.RB < Ho ? ho0 + tl.RB : Ho;
  constexpr int HL = S == 1 ? 1 : 0;
  const int wo = wo0 + p - HL;
  const bool comp = p >= HL && p <= P - 2 && wo < Wo;
  const int npix = S == 2 ? 2 * P : P;                 // tile pixels (input columns) of the block
  const int cbase = S == 2 ? 2 * wo0 - a.pl : wo0 - a.pl;   // input column of tile pixel 0
  const int NPX = npt * 16;

  bf16_t* xs = (bf16_t*)smem;                          // [2][NPX][RC_XLD]
  bf16_t* ys = xs + 2 * NPX * RC_XLD;                  // [2][NPX][ldy]
  float* xt = (float*)(ys + 2 * NPX * ldy);            // [CIN][2]: x prologue (scale, shift)
  float* et = xt + 2 * CIN;                            // [nct*16][2]: BN_e (scale, shift)

  // ---- set-up: tables, weights, zero k padding of the x slots --------------------------------
  const bool xpro = a.xp.mean != nullptr;
  if (tid < CIN) {
    float sc = 1.f, sh = 0.f;
    if (xpro) bn_pro_affine(a.xp, tid, sc, sh);
    xt[2 * tid] = sc;
    xt[2 * tid + 1] = sh;
  }
  for (int i = tid; i < nct * 16; i += 256) {
    float sc = 0.f, sh = 0.f;
    if (cb + i < C) bn_pro_affine(a.ep, cb + i, sc, sh);
    et[2 * i] = sc;
    et[2 * i + 1] = sh;
  }
  for (int i = tid; i < 2 * NPX * (RC_XLD - CIN) / 8; i += 256) {
    const int row = i / ((RC_XLD - CIN) / 8), k8 = i - row * ((RC_XLD - CIN) / 8);
    *(bf16x8*)(xs + row * RC_XLD + CIN + k8 * 8) = bf16x8{};
  }
  __syncthreads();   // the tables are read by every thread's first x staging below
  // this wave's channel tiles (wave, wave + 4) and their We fragments
  bf16x8 wf[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ctile = wave + 4 * j;
    const int ch = cb + ctile * 16 + li;
    wf[j] = bf16x8{};
    if (ctile < nct && ch < C && 8 * g < CIN) wf[j] = *(const bf16x8*)(a.wt0 + (long)ch * CIN + 8 * g);
  }
  float wr[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) wr[k][v] = a.w[k * C + c + v];

  // ---- x staging: thread u < NPX*CIN/8 owns chunk (pixel u / (CIN/8), k8 = u % (CIN/8)) -------
  constexpr int KC = CIN / 8;
  const int xpx = tid / KC, xk8 = tid - (tid / KC) * KC;
  const bool xown = xpx < NPX;
  const int xci = cbase + xpx;
  const bool xcol = xown && xpx < npix && xci >= 0 && xci < W;
  const T* xn = a.x + (long)n * H * W * CIN;
  const int hi0 = S == 2 ? 2 * ho0 - a.pt : ho0 - a.pt;
  const int nin = S == 2 ? 2 * (ho1 - ho0) + 1 : ho1 - ho0 + 2;
  // buffer loads, issued unconditionally (rod_common.h: a load under a branch makes the compiler
  // drain the ring every step): the row clamped into the map (rows outside it are zeroed when the
  // tile is formed), columns outside it at the out-of-range offset (they return 0)
  const rsrc_t rx = rod_rsrc(xn, (unsigned)((long)H * W * CIN * 2));
  const unsigned vx = xcol ? (unsigned)((xci * CIN + xk8 * 8) * 2) : ROD_OOB;
  auto xload = [&](int q) -> bf16x8 {
    const int hi = hi0 + q;
    const int hc = hi < 0 ? 0 : (hi >= H ? H - 1 : hi);
    return buf_ld<bf16x8>(rx, vx, (unsigned)hc * (unsigned)(W * CIN * 2));
  };
  auto xstage = [&](bf16x8 v, int slot) {   // the input prologue, rounded once (the forward's values)
    if (!xown) return;
    if (xpro) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = xk8 * 8 + e;
        v[e] = (bf16_t)act_fwd(fmaf((float)v[e], xt[2 * k], xt[2 * k + 1]), a.xp.act);
      }
    }
    *(bf16x8*)(xs + (slot * NPX + xpx) * RC_XLD + xk8 * 8) = v;
  };
  // ---- ye tile of input row q into slot q & 1 ------------------------------------------------
  auto form = [&](int q) {
    const int slot = q & 1;
    const int hi = hi0 + q;
    const bool rowok = q < nin && hi >= 0 && hi < H;
    const bf16_t* xsl = xs + slot * NPX * RC_XLD;
    bf16_t* ysl = ys + slot * NPX * ldy;
    // wave w forms channel tiles w and w + 4 for every pixel tile: the B fragments (x) read once
    // per row, the A fragments (We) in registers.  (Dealing the units round-robin over the waves
    // measured slower: 570 -> 703 us at 720p b8 block 1, a runtime unit loop and A from LDS.)
    bf16x8 fb[npt];
#pragma unroll
    for (int pt_ = 0; pt_ < npt; ++pt_) fb[pt_] = *(const bf16x8*)(xsl + (pt_ * 16 + li) * RC_XLD + 8 * g);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ctile = wave + 4 * j;
      if (ctile >= nct) break;
      const int c0 = ctile * 16 + 4 * g;                // local channel of this lane's first value
      const f32x4 t0 = *(const f32x4*)(et + 2 * c0), t1 = *(const f32x4*)(et + 2 * c0 + 4);
#pragma unroll
      for (int pt_ = 0; pt_ < npt; ++pt_) {
        const int px = pt_ * 16 + li;
        const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], fb[pt_], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        const int ci = cbase + px;
        const bool ok = rowok && px < npix && ci >= 0 && ci < W;
        // ye rounded to bf16 (the stored value), then BN_e + ReLU6 rounded (rod_dw3x3_fwd's prologue)
        const rc_f2 y01 = __builtin_convertvector(__builtin_convertvector(rc_f2{acc[0], acc[1]}, rc_b2), rc_f2);
        const rc_f2 y23 = __builtin_convertvector(__builtin_convertvector(rc_f2{acc[2], acc[3]}, rc_b2), rc_f2);
        rc_f2 z01 = __builtin_elementwise_fma(y01, rc_f2{t0[0], t0[2]}, rc_f2{t0[1], t0[3]});
        rc_f2 z23 = __builtin_elementwise_fma(y23, rc_f2{t1[0], t1[2]}, rc_f2{t1[1], t1[3]});
        z01 = rc_f2{act_t<ROD_ACT_RELU6>(z01.x), act_t<ROD_ACT_RELU6>(z01.y)};
        z23 = rc_f2{act_t<ROD_ACT_RELU6>(z23.x), act_t<ROD_ACT_RELU6>(z23.y)};
        const rc_b2 b01 = __builtin_convertvector(z01, rc_b2), b23 = __builtin_convertvector(z23, rc_b2);
        u32x2_t o;
        o[0] = ok ? __builtin_bit_cast(unsigned, b01) : 0u;
        o[1] = ok ? __builtin_bit_cast(unsigned, b23) : 0u;
        *(u32x2_t*)(ysl + px * ldy + c0) = o;
      }
    }
  };

  // ---- outputs and statistics (dw_lx_body's) --------------------------------------------------
  float piv[V], s1[V], s2[V];
#pragma unroll
  for (int v = 0; v < V; ++v) piv[v] = s1[v] = s2[v] = 0.f;
  const unsigned es = sizeof(T);
  T* yn = a.y + (long)n * Ho * Wo * C + c;
  const rsrc_t rys = rod_rsrc(yn - c, (unsigned)((long)Ho * Wo * C * es));
  const rsrc_t rnull = rod_rsrc(yn - c, 0u);
  const unsigned vy = comp ? (unsigned)(((long)wo * C + c) * es) : ROD_OOB;
  const unsigned rsy = (unsigned)(Wo * C * es);
  auto emit = [&](const float (&acc)[V], int ho, bool valid, bool first) {
    PK o;
#pragma unroll
    for (int v = 0; v < V; ++v) o.set(v, acc[v]);
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
  // this thread's tile pixels: S=2 the column pair 2p, 2p+1 and the right neighbour 2p+2;
  // S=1 p-1, p, p+1 (clamped into the tile: the clamped ones feed halo columns only)
  const int pc = S == 2 ? 2 * p : p;
  const int pa0 = S == 2 ? pc : (pc > 0 ? pc - 1 : 0);
  const int pb0 = S == 2 ? pc + 1 : pc;
  const int pr0 = pc + (S == 2 ? 2 : 1) < npix ? pc + (S == 2 ? 2 : 1) : npix - 1;
  const int ia = (p < P ? pa0 : 0) * ldy + cvb * V, ib = (p < P ? pb0 : 0) * ldy + cvb * V,
            ir = (p < P ? pr0 : 0) * ldy + cvb * V;
  auto rd = [&](int slot, int off, float (&o)[V]) {
    PK v;
    v.load(ys + slot * NPX * ldy + off);
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = v.get(e);
  };

  // ---- prologue: x rows 0, 1 staged, rows 2 .. D+1 in flight, ye of row 0 formed ----------------
  // x prefetch ring of D rows (the step loop's unroll: 3 for stride 1, 4 for stride 2): at step q
  // row q+2 is staged from slot (q+2) % D and row q+2+D loaded into it, D steps of latency cover
  constexpr int D = S == 1 ? 3 : 4;
  bf16x8 xr[D];
  xstage(xload(0), 0);
  xstage(xload(1), 1);
#pragma unroll
  for (int r = 2; r < 2 + D; ++r) xr[r % D] = xload(r);
  __syncthreads();
  form(0);
  __syncthreads();
  // one step (k = q mod D): (a) row q's tile -> taps / outputs, (b) row q+1's tile, (c) row q+2's
  // x staged and row q+2+D's loaded, (d) one barrier
  auto advance = [&](int q, int k) {
    form(q + 1);
    xstage(xr[(k + 2) % D], q & 1);
    xr[(k + 2) % D] = xload(q + 2 + D);
    __syncthreads();
  };
  if constexpr (S == 1) {
    float acc[3][V];
#pragma unroll
    for (int s_ = 0; s_ < 3; ++s_)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[s_][v] = 0.f;
    for (int q0 = 0; q0 < nin; q0 += 3) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int q = q0 + k;
        if (q >= nin) break;
        float L[V], cen[V], R[V];
        rd(q & 1, ia, L);
        rd(q & 1, ib, cen);
        rd(q & 1, ir, R);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int sl = (k - i + 3) % 3;
#pragma unroll
          for (int v = 0; v < V; ++v) {
            float t = acc[sl][v];
            t = fmaf(L[v], wr[i * 3][v], t);
            t = fmaf(cen[v], wr[i * 3 + 1][v], t);
            t = fmaf(R[v], wr[i * 3 + 2][v], t);
            acc[sl][v] = t;
          }
        }
        const int sd = (k + 1) % 3;
        const int m = q - 2;
        emit(acc[sd], ho0 + m, m >= 0 && ho0 + m < ho1, m == 0);
#pragma unroll
        for (int v = 0; v < V; ++v) acc[sd][v] = 0.f;
        advance(q, k);
      }
    }
  } else {
    float acc[2][V];
#pragma unroll
    for (int s_ = 0; s_ < 2; ++s_)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[s_][v] = 0.f;
    for (int q0 = 0; q0 < nin; q0 += 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = q0 + k;
        if (q >= nin) break;
        float c0v[V], c1v[V], R[V];
        rd(k & 1, ia, c0v);
        rd(k & 1, ib, c1v);
        rd(k & 1, ir, R);
        auto addrow = [&](int i, int sl) {
#pragma unroll
          for (int v = 0; v < V; ++v) {
            float t = acc[sl][v];
            t = fmaf(c0v[v], wr[i * 3][v], t);
            t = fmaf(c1v[v], wr[i * 3 + 1][v], t);
            t = fmaf(R[v], wr[i * 3 + 2][v], t);
            acc[sl][v] = t;
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
        advance(q, k);
      }
    }
  }

  if constexpr (STATS) {
    // dw_lx_body's merge: per thread (n, mean, M2), runs of 8 columns, then the runs -> part
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
      store_stat_part(a.parts, C, part, cg * Cc + ch, pn, pm, pq);
    }
  }
}

// =====================================================================================
// Stride-2 fused depthwise backward with the expanded input recomputed (ABI 23,
// rod_dw3x3_bwd_fused_rc): dw3x3_bwd_fused_s2p_kernel (2 channels a thread, 512-thread blocks,
// the BN_d backward apply + backward-data + filter gradient + BN_e backward sums in one pass) with
// its reads of ye — the 4 positions (rows 2a-pt, 2a-pt+1 x columns ci0, ci0+1) of each dy row
// step — served from an LDS tile of raw ye instead of HBM.  The tile of a step (2 rows x the
// block's 2P columns x its Cc channels) is formed one step ahead from the block input x with the
// expand forward's MFMA (operands swapped: bit-identical ye), by the 8 waves (one row x pixel tile
// each, every channel tile); x goes through a two-slot LDS ring with its prologue applied, loaded
// two steps ahead in registers like the kernel's other loads.  Everything after the ye values —
// BN_e apply, gates, dx order, filter and BN_e sums, the part structure — is the s2p kernel's, so
// dx, dw and the BN_e parts are bit-identical to rod_dw3x3_fwd_bwd_fused over the stored ye.
// =====================================================================================
constexpr int RCB_NPX = 64;   // tile pixels (2P <= 64)
template <int CIN, int NCT>
__global__ void __launch_bounds__(512, 4) dw3x3_bwd_fused_rc_kernel(
    const bf16_t* __restrict__ xin, BnPro xp, const bf16_t* __restrict__ wt0, const bf16_t* __restrict__ dz,
    const bf16_t* __restrict__ yd, const float* __restrict__ w, bf16_t* __restrict__ dx, float* __restrict__ slab,
    float* __restrict__ gparts, int H, int W, int C, int pt, int pl, int Ho, int Wo, DwTile tl, BnPro pro, DwBwdBn bd) {
  typedef bf16_t T;
  constexpr int nct = NCT, ldy = NCT * 16 + 8;
  constexpr int V = 2, VP = 1, TB = 512, D = 2;
  constexpr int KC = CIN / 8;
  typedef PackV<T, V> PK;
  // LDS: exchange slots [D][3][TB] fp32 pairs | x ring [2][2 rows][64][RC_XLD] | ye tile
  // [2][2 rows][64][ldy] | We [nct*16][RC_XLD] | x prologue table [CIN][2]; the epilogue's staged
  // column sums reuse the front
  extern __shared__ __attribute__((aligned(16))) char smem[];
  dw_f2* sl = (dw_f2*)smem;
  bf16_t* xs = (bf16_t*)(smem + D * 3 * TB * VP * sizeof(dw_f2));
  bf16_t* ys = xs + 2 * 2 * RCB_NPX * RC_XLD;
  bf16_t* wl = ys + 2 * 2 * RCB_NPX * ldy;
  float* xt = (float*)(wl + nct * 16 * RC_XLD);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int CVb = tl.CVb * 2, P = tl.P;
  const int p = tid / CVb, cvb = tid - (tid / CVb) * CVb;
  int bx, strip, n;
  xcd_block(bx, strip, n);
  const int cg = bx % tl.cgroups, ct = bx / tl.cgroups;
  const int Cc = CVb * V, cb = cg * Cc;
  const int c = cb + cvb * V;
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
  const int cbase = 2 * (ct * tl.TWo - 1) - pl;        // input column of tile pixel 0

  // ---- set-up: x prologue table, We rows (k zero-padded), zero k padding of the x ring ----------
  const bool xpro = xp.mean != nullptr;
  if (tid < CIN) {
    float sc = 1.f, sh = 0.f;
    if (xpro) bn_pro_affine(xp, tid, sc, sh);
    xt[2 * tid] = sc;
    xt[2 * tid + 1] = sh;
  }
  for (int i = tid; i < nct * 16 * (RC_XLD / 8); i += TB) {
    const int r = i / (RC_XLD / 8), k8 = i - r * (RC_XLD / 8);
    bf16x8 v = {};
    if (cb + r < C && k8 * 8 < CIN) v = *(const bf16x8*)(wt0 + (long)(cb + r) * CIN + k8 * 8);
    *(bf16x8*)(wl + r * RC_XLD + k8 * 8) = v;
  }
  for (int i = tid; i < 4 * RCB_NPX * (RC_XLD - CIN) / 8; i += TB) {
    const int row = i / ((RC_XLD - CIN) / 8), k8 = i - row * ((RC_XLD - CIN) / 8);
    *(bf16x8*)(xs + row * RC_XLD + CIN + k8 * 8) = bf16x8{};
  }

  dw_f2 wr[9][VP];
#pragma unroll
  for (int k = 0; k < 9; ++k) wr[k][0] = dw_f2{w[k * C + c], w[k * C + c + 1]};
  dw_f2 psc[VP], psh[VP], ers[VP], enb[VP];
  const int pact = pro.act;
  {
    float a0_, b0_, a1_, b1_;
    bn_pro_affine(pro, c, a0_, b0_);
    bn_pro_affine(pro, c + 1, a1_, b1_);
    psc[0] = dw_f2{a0_, a1_};
    psh[0] = dw_f2{b0_, b1_};
    ers[0] = dw_f2{pro.rstd[c], pro.rstd[c + 1]};
    enb[0] = dw_f2{-pro.mean[c] * ers[0].x, -pro.mean[c + 1] * ers[0].y};
  }
  dw_f2 dsc[VP], dsh[VP], da[VP], dk1[VP], dk0[VP];
  {
    const int c0 = c;
    float s0, t0, s1, t1, k10, k00, k11, k01;
    bn_affine(bd.mean, bd.rstd, bd.gamma, bd.beta, c0, s0, t0);
    bn_affine(bd.mean, bd.rstd, bd.gamma, bd.beta, c0 + 1, s1, t1);
    dsc[0] = dw_f2{s0, s1};
    dsh[0] = dw_f2{t0, t1};
    da[0] = dw_f2{bd.coef[c0], bd.coef[c0 + 1]};
    float m0, m1;
    bn_bwd_k<bf16_t>(da[0].x, bd.mean[c0], bd.rstd[c0], bd.coef[C + c0], bd.coef[2 * C + c0], k10, k00, m0);
    bn_bwd_k<bf16_t>(da[0].y, bd.mean[c0 + 1], bd.rstd[c0 + 1], bd.coef[C + c0 + 1], bd.coef[2 * C + c0 + 1], k11, k01,
                     m1);
    dk1[0] = dw_f2{k10, k11};
    dk0[0] = dw_f2{k00, k01};
  }
  dw_f2 sg[VP], sgx[VP];
  sg[0] = sgx[0] = dw_f2{0.f, 0.f};

  const unsigned es = sizeof(T);
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

  // x staging: thread u < 2*64*KC owns (row r = u / (64*KC), pixel, k8) of a step's two x rows
  const int xr_ = tid / (RCB_NPX * KC), xrem = tid - xr_ * (RCB_NPX * KC);
  const int xpx = xrem / KC, xk8 = xrem - (xrem / KC) * KC;
  const bool xown = tid < 2 * RCB_NPX * KC;
  const int xci = cbase + xpx;
  const bool xcol = xown && xpx < 2 * P && xci >= 0 && xci < W;
  const T* xn = xin + (long)n * H * W * CIN;
  const rsrc_t rxi = rod_rsrc(xn, (unsigned)((long)H * W * CIN * 2));
  const unsigned vxi = xcol ? (unsigned)((xci * CIN + xk8 * 8) * 2) : ROD_OOB;
  auto xload = [&](int q) -> bf16x8 {   // step q's x row xr_ (clamped into the map; masked at use)
    const int hh = 2 * (a0 - 1 + q) - pt + xr_;
    const int hc = hh < 0 ? 0 : (hh >= H ? H - 1 : hh);
    return buf_ld<bf16x8>(rxi, vxi, (unsigned)hc * (unsigned)(W * CIN * 2));
  };
  auto xstage = [&](bf16x8 v, int slot) {
    if (!xown) return;
    if (xpro) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = xk8 * 8 + e;
        v[e] = (bf16_t)act_fwd(fmaf((float)v[e], xt[2 * k], xt[2 * k + 1]), xp.act);
      }
    }
    *(bf16x8*)(xs + ((slot * 2 + xr_) * RCB_NPX + xpx) * RC_XLD + xk8 * 8) = v;
  };
  // raw ye of step q (both rows) into tile slot q & 1: wave w = (row w >> 2, pixel tile w & 3),
  // every channel tile
  const int frow = wave >> 2, fpt = wave & 3;
  auto form = [&](int slot) {
    const bf16_t* xsl = xs + ((slot * 2 + frow) * RCB_NPX + fpt * 16 + l16) * RC_XLD + 8 * g;
    const bf16x8 fb = *(const bf16x8*)xsl;
    bf16_t* ysl = ys + ((slot * 2 + frow) * RCB_NPX + fpt * 16 + l16) * ldy + 4 * g;
#pragma unroll
    for (int ct2 = 0; ct2 < nct; ++ct2) {
      const bf16x8 fw = *(const bf16x8*)(wl + (ct2 * 16 + l16) * RC_XLD + 8 * g);
      const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw, fb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const dw_b2 b01 = __builtin_convertvector(dw_f2{acc[0], acc[1]}, dw_b2);
      const dw_b2 b23 = __builtin_convertvector(dw_f2{acc[2], acc[3]}, dw_b2);
      u32x2_t o;
      o[0] = __builtin_bit_cast(unsigned, b01);
      o[1] = __builtin_bit_cast(unsigned, b23);
      *(u32x2_t*)(ysl + ct2 * 16) = o;
    }
  };
  // this thread's 4 ye positions in a tile slot: rows 0 / 1, pixels 2p / 2p+1 (clamped: halo lanes)
  const int tp = p < P ? 2 * p : 0;
  const int yo0 = tp * ldy + cvb * V, yo1 = (tp + 1) * ldy + cvb * V;

  PK rz[D], ry[D];
  bf16x8 xq;   // x of the step after next (one step of load latency cover; 128 VGPRs leave no room for two)
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
    }
  };
  const int nst = a1 - a0 + 2;
  // prologue: x of steps 0, 1 staged, steps 2, 3 in flight; ye of step 0 formed
  __syncthreads();   // the tables and the zero padding
  xstage(xload(0), 0);
  xstage(xload(1), 1);
  xq = xload(2);
#pragma unroll
  for (int k = 0; k < D; ++k) {
    issue(k, k);
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  form(0);
  __syncthreads();
  dw_f2 fa[9][VP], pv[VP], pL[VP];
  pv[0] = pL[0] = dw_f2{0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 9; ++k) fa[k][0] = dw_f2{0.f, 0.f};
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
        const dw_f2 z = f2fma(yv[0], dsc[0], dsh[0]);
        const dw_f2 gg = gate2<ROD_ACT_RELU6>(z, zv[0], bd.act);
        const dw_f2 o = f2fma(da[0], gg, f2fma(dk1[0], yv[0], dk0[0]));
        dv[0] = okd[k] ? round2(o, T{}) : zero2;
      }
      // ye at the 4 positions from the tile (slot k), the prologue, BN_e's pre-activation
      dw_f2 xv[4][VP], yr[4][VP], ez[4][VP];
      {
        const bf16_t* yt = ys + (k * 2) * RCB_NPX * ldy;
        PK r4[4];
        r4[0].load(yt + yo0);
        r4[1].load(yt + yo1);
        r4[2].load(yt + RCB_NPX * ldy + yo0);
        r4[3].load(yt + RCB_NPX * ldy + yo1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          unpackv(r4[i], yr[i]);
          const dw_f2 z = f2fma(yr[i][0], psc[0], psh[0]);
          const dw_f2 t = dw_f2{act_t<ROD_ACT_RELU6>(z.x), act_t<ROD_ACT_RELU6>(z.y)};
          ez[i][0] = z;
          xv[i][0] = okx[k][i] ? round2(t, T{}) : zero2;
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // the slots' reloads stay after their last reads
      issue(k, q + D);
      // the next step's ye tile, the x of the step after it staged, x two steps ahead loaded
      form((k + 1) & 1);
      xstage(xq, k);
      xq = xload(q + 3);
      dw_f2* S = sl + k * 3 * TB * VP;
      S[tid] = dv[0];
      S[TB + tid] = xv[0][0];
      S[2 * TB + tid] = xv[2][0];
      __syncthreads();
      const dw_f2 dL = S[li], r0 = S[TB + ri], r1 = S[2 * TB + ri];
      const bool own = a >= a0 && a < a1, ownp = a - 1 >= a0 && a - 1 < a1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hh = 2 * a - pt + (i >> 1);
        const bool hok = own && hh >= 0 && hh < H;
        const dw_f2 c1 = dv[0], c0 = dL, p1v = pv[0], p0v = pL[0];
        dw_f2 o;
        if (i == 0) o = f2fma(p0v, wr[8][0], f2fma(p1v, wr[6][0], f2fma(c0, wr[2][0], c1 * wr[0][0])));
        else if (i == 1) o = f2fma(p1v, wr[7][0], c1 * wr[1][0]);
        else if (i == 2) o = f2fma(c0, wr[5][0], c1 * wr[3][0]);
        else o = c1 * wr[4][0];
        PK pk;
        const dw_b2 bb = __builtin_convertvector(o, dw_b2);
        pk.v[0] = bb.x;
        pk.v[1] = bb.y;
        const unsigned u = __builtin_bit_cast(unsigned, bb);
        const dw_f2 orr = dw_f2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
        if (hok) {
          const bool cc = (i & 1) ? cok1 : cok0;
          const dw_f2 gg = cc ? gate2<ROD_ACT_RELU6>(ez[i][0], orr, pact) : zero2;
          sg[0] += gg;
          sgx[0] = f2fma(gg, f2fma(yr[i][0], ers[0], enb[0]), sgx[0]);
        }
        pk.bstore(hok ? rdx : rnull, (i & 1) ? vst1 : vst0, (unsigned)(hok ? hh : 0) * rsx);
      }
      if (own) {
        fa[0][0] = f2fma(dv[0], xv[0][0], fa[0][0]);
        fa[1][0] = f2fma(dv[0], xv[1][0], fa[1][0]);
        fa[2][0] = f2fma(dv[0], r0, fa[2][0]);
        fa[3][0] = f2fma(dv[0], xv[2][0], fa[3][0]);
        fa[4][0] = f2fma(dv[0], xv[3][0], fa[4][0]);
        fa[5][0] = f2fma(dv[0], r1, fa[5][0]);
      }
      if (ownp) {
        fa[6][0] = f2fma(pv[0], xv[0][0], fa[6][0]);
        fa[7][0] = f2fma(pv[0], xv[1][0], fa[7][0]);
        fa[8][0] = f2fma(pv[0], r0, fa[8][0]);
      }
      pv[0] = dv[0];
      pL[0] = dL;
    }
  }

  __syncthreads();
  float* red = (float*)smem;
  const long part = ((long)n * tl.strips + strip) * tl.coltiles + ct;
  auto stage = [&](const dw_f2 (&a)[VP], int qk) {
    red[(qk * TB + tid) * V] = comp ? a[0].x : 0.f;
    red[(qk * TB + tid) * V + 1] = comp ? a[0].y : 0.f;
  };
#pragma unroll
  for (int k = 0; k < 9; ++k) stage(fa[k], k);
  stage(sg, 9);
  stage(sgx, 10);
  __syncthreads();
  dw_colsum_emit<V>(red, 0, 11, TB, Cc, CVb, P, slab, gparts, part, C, cg);
}

inline size_t dw_bwd_rc_lds(int nct, int ldy) {
  const size_t main = 2 * 3 * 512 * sizeof(float) * 2 + (size_t)2 * 2 * RCB_NPX * RC_XLD * 2 +
                      (size_t)2 * 2 * RCB_NPX * ldy * 2 + (size_t)nct * 16 * RC_XLD * 2 + 32 * 2 * 4;
  const size_t red = (size_t)11 * 512 * 2 * 4;
  return main > red ? main : red;
}

// the plan rod_dw3x3_fwd would use for (x, y) 16-byte aligned, restricted to what the tile
// holds: the V pack of dw_fwd_v, whole 16-channel tiles on <= 8 tiles (2 per wave), <= 4 pixel
// tiles (64 input columns), Cin 16 / 24 / 32
static bool dw_rc_plan(int N, int Ho, int Wo, int C, int S, int Cin, DwTile& t, int& V, DwRcLds& l) {
  if (N <= 0 || Ho <= 0 || Wo <= 0 || C % 8 || (S != 1 && S != 2) || (Cin != 16 && Cin != 24 && Cin != 32))
    return false;
  V = dw_fwd_v(ROD_BF16, (long)N * Ho * Wo * S * S, C);
  t = dw_tile(N, Ho, Wo, C, S, V);
  l = dw_rc_lds(t, S, V, Cin);
  return l.npt <= 4 && l.nct <= 8 && l.npt * 16 * (Cin / 8) <= 256 && l.total <= 64 * 1024;
}

}  // namespace rod

using namespace rod;

extern "C" {

int rod_dw3x3_fwd_rc_supported(int N, int H, int W, int C, int Cin, int stride, int dtype) {
  if (dtype != ROD_BF16 || H <= 0 || W <= 0) return 0;
  const int Ho = (H + stride - 1) / stride, Wo = (W + stride - 1) / stride;
  DwTile t;
  int V;
  DwRcLds l;
  return dw_rc_plan(N, Ho, Wo, C, stride, Cin, t, V, l) ? 1 : 0;
}

int rod_dw3x3_fwd_rc(const void* x, const float* x_mean, const float* x_rstd, const float* x_gamma,
                     const float* x_beta, int x_act, const void* wt0, int Cin, const float* e_mean,
                     const float* e_rstd, const float* e_gamma, const float* e_beta, int e_act, const float* w,
                     void* y, float* stat_parts, int N, int H, int W, int C, int stride, int pad_t, int pad_l,
                     int Ho, int Wo, int dtype, void* stream) {
  ROD_CHECK_ARG(x && wt0 && e_mean && e_rstd && w && y, "rod_dw3x3_fwd_rc: NULL argument");
  ROD_CHECK_ARG(!x_mean || x_rstd, "rod_dw3x3_fwd_rc: the input prologue needs mean and rstd");
  ROD_CHECK_ARG(e_act == ROD_ACT_RELU6, "rod_dw3x3_fwd_rc: the expand BatchNorm's activation must be ReLU6");
  ROD_CHECK_ARG(x_act >= ROD_ACT_NONE && x_act <= ROD_ACT_RELU, "rod_dw3x3_fwd_rc: bad input act %d", x_act);
  ROD_CHECK_ARG(rod_dw3x3_fwd_rc_supported(N, H, W, C, Cin, stride, dtype),
                "rod_dw3x3_fwd_rc: unsupported N=%d H=%d W=%d C=%d Cin=%d stride=%d dtype=%d", N, H, W, C, Cin,
                stride, dtype);
  ROD_CHECK_ARG(Ho == (H + stride - 1) / stride && Wo == (W + stride - 1) / stride && pad_t >= 0 && pad_t <= 1 &&
                    pad_l >= 0 && pad_l <= 1,
                "rod_dw3x3_fwd_rc: output map / TF-SAME padding mismatch");
  ROD_CHECK_ARG(((((uintptr_t)x) | ((uintptr_t)wt0) | ((uintptr_t)y)) & 15) == 0,
                "rod_dw3x3_fwd_rc: x, wt0, y must be 16-byte aligned");
  ROD_CHECK_ARG((long)Ho * Wo * C * 2 < (1L << 31), "rod_dw3x3_fwd_rc: image over 2 GiB");
  DwTile t;
  int V;
  DwRcLds l;
  dw_rc_plan(N, Ho, Wo, C, stride, Cin, t, V, l);
  const DwRcArgs a{(const bf16_t*)x, BnPro{x_mean, x_rstd, x_gamma, x_beta, x_act}, (const bf16_t*)wt0,
                   BnPro{e_mean, e_rstd, e_gamma, e_beta, e_act}, w, (bf16_t*)y, stat_parts, H, W, C, pad_t, pad_l,
                   Ho, Wo};
  const dim3 grid(t.coltiles * t.cgroups, t.strips, N);
  hipStream_t s = ROD_STREAM(stream);
#define RCN(S_, V_, CI_, ST_)                                                                                  \
  do {                                                                                                         \
    if (l.npt <= 2)                                                                                            \
      hipLaunchKernelGGL((dw3x3_fwd_rc_kernel<S_, V_, CI_, ST_, 2>), grid, dim3(256), l.total, s, a, t, l.nct, \
                         l.ldy);                                                                               \
    else if (l.npt == 3)                                                                                       \
      hipLaunchKernelGGL((dw3x3_fwd_rc_kernel<S_, V_, CI_, ST_, 3>), grid, dim3(256), l.total, s, a, t, l.nct, \
                         l.ldy);                                                                               \
    else                                                                                                       \
      hipLaunchKernelGGL((dw3x3_fwd_rc_kernel<S_, V_, CI_, ST_, 4>), grid, dim3(256), l.total, s, a, t, l.nct, \
                         l.ldy);                                                                               \
  } while (0)
#define RCK(S_, V_, CI_)                         \
  do {                                           \
    if (stat_parts) RCN(S_, V_, CI_, true);      \
    else RCN(S_, V_, CI_, false);                \
  } while (0)
#define RCV(S_, CI_)                   \
  do {                                 \
    if (V == 8) RCK(S_, 8, CI_);       \
    else RCK(S_, 4, CI_);              \
  } while (0)
#define RCC(S_)                                    \
  do {                                             \
    if (Cin == 16) RCV(S_, 16);                    \
    else if (Cin == 24) RCV(S_, 24);               \
    else RCV(S_, 32);                              \
  } while (0)
  if (stride == 1) RCC(1);
  else RCC(2);
#undef RCC
#undef RCV
#undef RCK
#undef RCN
  return check_launch("rod_dw3x3_fwd_rc");
}


// the plan rod_dw3x3_bwd_fused takes for bf16 stride 2 (dw_tile over the (A, B) map, 4-channel
// units), restricted to what the recompute tile holds: 2P <= 64 pixels, <= 4 channel tiles
static bool dw_bwd_rc_plan(int N, int H, int W, int C, int pt, int pl, int Cin, DwTile& t, int& nct, int& ldy) {
  int A = 0, B = 0;
  if (C % 4 || (Cin != 16 && Cin != 24 && Cin != 32) || !dw_fused_geom(N, H, W, C, 2, pt, pl, A, B)) return false;
  t = dw_tile(N, A, B, C, 1, 4);
  const int Cc = t.CVb * 4;
  nct = std::max(2, (Cc + 15) / 16);   // the kernel instantiates 2, 3 or 4 channel tiles
  ldy = nct * 16 + 8;
  return 2 * t.P <= RCB_NPX && nct <= 4 && dw_bwd_rc_lds(nct, ldy) <= 160 * 1024;
}

int rod_dw3x3_bwd_fused_rc_supported(int N, int H, int W, int C, int Cin, int stride, int pad_t, int pad_l,
                                     int dtype) {
  DwTile t;
  int nct, ldy;
  return dtype == ROD_BF16 && stride == 2 && dw_bwd_rc_plan(N, H, W, C, pad_t, pad_l, Cin, t, nct, ldy) ? 1 : 0;
}

int rod_dw3x3_bwd_fused_rc(const void* x, const float* x_mean, const float* x_rstd, const float* x_gamma,
                           const float* x_beta, int x_act, const void* wt0, int Cin, const float* e_mean,
                           const float* e_rstd, const float* e_gamma, const float* e_beta, int e_act, const void* dz,
                           const void* yd, const float* bn_mean, const float* bn_rstd, const float* bn_gamma,
                           const float* bn_beta, int bn_act, const float* coef, const float* w, void* dx, float* dw,
                           float* gparts, void* workspace, int N, int H, int W, int C, int stride, int pad_t,
                           int pad_l, int Ho, int Wo, int dtype, void* stream) {
  ROD_CHECK_ARG(rod_dw3x3_bwd_fused_rc_supported(N, H, W, C, Cin, stride, pad_t, pad_l, dtype),
                "rod_dw3x3_bwd_fused_rc: unsupported N=%d H=%d W=%d C=%d Cin=%d stride=%d dtype=%d", N, H, W, C,
                Cin, stride, dtype);
  ROD_CHECK_ARG(x && wt0 && e_mean && e_rstd && dz && yd && bn_mean && bn_rstd && coef && w && dx && dw && gparts &&
                    workspace,
                "rod_dw3x3_bwd_fused_rc: NULL argument");
  ROD_CHECK_ARG(!x_mean || x_rstd, "rod_dw3x3_bwd_fused_rc: the input prologue needs mean and rstd");
  ROD_CHECK_ARG(e_act == ROD_ACT_RELU6 && bn_act == ROD_ACT_RELU6,
                "rod_dw3x3_bwd_fused_rc: both BatchNorms of the block must be ReLU6");
  ROD_CHECK_ARG(x_act >= ROD_ACT_NONE && x_act <= ROD_ACT_RELU, "rod_dw3x3_bwd_fused_rc: bad input act %d", x_act);
  ROD_CHECK_ARG(Ho == (H + 1) / 2 && Wo == (W + 1) / 2, "rod_dw3x3_bwd_fused_rc: output map mismatch");
  ROD_CHECK_ARG(((((uintptr_t)x) | ((uintptr_t)wt0) | ((uintptr_t)dz) | ((uintptr_t)yd) | ((uintptr_t)dx)) & 15) == 0,
                "rod_dw3x3_bwd_fused_rc: tensors must be 16-byte aligned");
  ROD_CHECK_ARG((long)H * W * C * 2 < (1L << 31), "rod_dw3x3_bwd_fused_rc: image over 2 GiB");
  DwTile t;
  int nct, ldy;
  dw_bwd_rc_plan(N, H, W, C, pad_t, pad_l, Cin, t, nct, ldy);
  const dim3 grid(t.coltiles * t.cgroups, t.strips, N);
  const size_t lds = dw_bwd_rc_lds(nct, ldy);
  const BnPro xp{x_mean, x_rstd, x_gamma, x_beta, x_act};
  const BnPro ep{e_mean, e_rstd, e_gamma, e_beta, e_act};
  const DwBwdBn bd{bn_mean, bn_rstd, bn_gamma, bn_beta, coef, bn_act};
  float* sl = (float*)workspace;
  hipStream_t s = ROD_STREAM(stream);
#define RCB0(CI_, NC_)                                                                                          \
  do {                                                                                                          \
    (void)hipFuncSetAttribute((const void*)dw3x3_bwd_fused_rc_kernel<CI_, NC_>,                                \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                           \
    hipLaunchKernelGGL((dw3x3_bwd_fused_rc_kernel<CI_, NC_>), grid, dim3(512), lds, s, (const bf16_t*)x, xp,   \
                       (const bf16_t*)wt0, (const bf16_t*)dz, (const bf16_t*)yd, w, (bf16_t*)dx, sl, gparts, H, W, C, \
                       pad_t, pad_l, Ho, Wo, t, ep, bd);                                                       \
  } while (0)
#define RCB(CI_)                      \
  do {                                \
    if (nct <= 2) RCB0(CI_, 2);       \
    else if (nct == 3) RCB0(CI_, 3);  \
    else RCB0(CI_, 4);                \
  } while (0)
  if (Cin == 16) RCB(16);
  else if (Cin == 24) RCB(24);
  else RCB(32);
#undef RCB
#undef RCB0
  const int rc = check_launch("rod_dw3x3_bwd_fused_rc");
  if (rc) return rc;
  slab_sum(sl, dw, (int)((long)N * t.strips * t.coltiles), 9L * C, s);
  return check_launch("rod_dw3x3_bwd_fused_rc");
}

}  // extern "C"
