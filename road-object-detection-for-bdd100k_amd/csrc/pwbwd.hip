// pwbwd.hip — the backward of a 1x1 conv and the BatchNorm after it, in one pass (bf16).
//
// Reference: slim.conv2d(.., [1, 1]) + slim.batch_norm (conv_blocks.py:263-294 expand /
// project, catch_net.py:301-304 head 1x1s); TF runs FusedBatchNormGrad, then
// Conv2DBackpropInput and Conv2DBackpropFilter, each a separate pass over the tensors.
//
// Unfused (rod_bn_bwd + rod_conv_fwd(mode 1) + rod_conv_wgrad) the [M, Cout] gradient dy is
// written once and read three times.  Here a block streams its chunk of rows, 64 at a time:
//   1. loads dz and the pre-BatchNorm y, forms dy = coef0*(g - coef1 - yhat*coef2) in
//      registers (rod_bn_bwd_apply's arithmetic, rounded to bf16) and stages it in LDS;
//      loads the conv input rows (BatchNorm-apply prologue when the input was Pending);
//   2. dW += dy^T . a  (16x16x32 bf16 MFMA, both operands read transposed with
//      ds_read_b64_tr_b16; the bias gradient is a ones column appended to a);
//      dx  = dy . W    (W = wt1 [Cin][Cout] held in LDS for the whole launch);
//   3. stages dx in LDS and writes whole 16-byte row segments.
// dW / db partials per block go to fp32 slabs summed in f64 in fixed order (slab_sum), so the
// result is deterministic.  Bytes per row: 2*Cout*2 (dz, y) + Cin*2 (x) + Cin*2 (dx).
//
// The kernel is latency-bound on its synchronous 64-row steps, so occupancy is what it runs
// on: the wave index is made scalar (readfirstlane: tile indices and their divisions in
// SGPRs), per-step offsets are recomputed from an opaque copy of the thread index instead of
// being hoisted as loop invariants, dz / y are batched two (not four) 16-byte loads deep, and
// the 7 coefficient fields are read four channels at a time.  The expand shapes went from
// 1-2 to 3 waves per SIMD: tools/pwbwd_bench.py 4715 -> 3326 us over its eight shapes,
// outputs bit-identical.
#include "rod_common.h"

namespace rod {

constexpr int PB_BM = 64;    // rows per step (4 waves x 16 rows of dx)
constexpr int PB_CF = 8;     // per-channel coefficient fields in the LDS table

struct PwBwdArgs {
  const bf16_t* dz;
  const bf16_t* y;
  const bf16_t* x;
  const bf16_t* wt1;
  bf16_t* dx;
  float* partw;  // [nblk][Cout][Cin]
  float* partb;  // [nblk][Cout] or NULL
  const float *mean, *rstd, *gamma, *beta, *coef;
  const float *xmean, *xrstd, *xgamma, *xbeta;
  int act, xact;
  long M, chunk;
  int Cin, Cout, kd, nci, nco, nxt;
  bf16_t* dyp = nullptr;   // rod_pw_bwd_gred_dyp: the BatchNorm-backward output rows [M][Cout] (dx not written)
  const bf16_t* wt0 = nullptr;   // RC (ABI 23): the forward weights [Cout][Cin]; y is recomputed, never read
};

typedef short pb_s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x4 pb_tr_read(const bf16_t* p) {
  pb_s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) pb_s16x4*)p);
  return __builtin_bit_cast(bf16x4, r);
}

template <int NX, int WT>
__global__ void __launch_bounds__(256) pw_bwd_kernel(PwBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Cin = a.Cin, Cout = a.Cout;
  const int CCH = Cout / 8, XCH = Cin / 8;
  const int LDD = a.kd + 8;           // 16-byte aligned rows, 8-byte aligned transposed reads
  const int LDX = a.nci * 16 + 8;
  // coefficient tables field-major ([PB_CF][Cout], [2][Cin]): a thread reads its chunk's 8
  // channels of a field as two 16-byte LDS reads, neighbouring lanes on neighbouring chunks
  float* ctab = (float*)smem;                                  // [PB_CF][Cout]
  float* xtab = ctab + (long)Cout * PB_CF;                     // [2][Cin]
  bf16_t* Ds = (bf16_t*)(xtab + 2 * Cin);                      // [64][LDD]   dy
  bf16_t* Xs = Ds + PB_BM * LDD;                               // [64][LDX]   a | 1 ; dx staging
  bf16_t* Ws = Xs + PB_BM * LDX;                               // [nxt*16][LDD] wt1
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: tile indices in SGPRs
  const bool prox = a.xmean != nullptr;
  const bool has_bias = a.partb != nullptr;
  // act_grad(z, act) as one select chain: z > 0 ? (z < hi ? 1 : 0) : lo — the same {0, 0.2, 1}
  // factors (NaN -> lo, as the compare-based forms give) without a per-element switch
  const float ghi = a.act == ROD_ACT_RELU6 ? 6.f : INFINITY;
  const float glo = a.act == ROD_ACT_LEAKY ? 0.2f : a.act == ROD_ACT_NONE ? 1.f : 0.f;

  for (int c = tid; c < Cout; c += 256) {
    float sc, sh;
    bn_affine(a.mean, a.rstd, a.gamma, a.beta, c, sc, sh);
    float* t = ctab + c;
    t[0] = a.mean[c];
    t[Cout] = a.rstd[c];
    t[2 * Cout] = sc;
    t[3 * Cout] = sh;
    t[4 * Cout] = a.coef[c];
    bn_bwd_k_fold(a.coef[c], a.mean[c], a.rstd[c], a.coef[Cout + c], a.coef[2 * Cout + c], t[5 * Cout], t[6 * Cout]);
    t[7 * Cout] = 0.f;
  }
  if (prox) {
    for (int c = tid; c < Cin; c += 256) {
      float sc, sh;
      bn_affine(a.xmean, a.xrstd, a.xgamma, a.xbeta, c, sc, sh);
      xtab[c] = sc;
      xtab[Cin + c] = sh;
    }
  }
  // zero padding: dy columns >= Cout, a columns >= Cin, the whole W image
  for (int i = tid; i < PB_BM * LDD; i += 256) Ds[i] = (bf16_t)0.f;
  for (int i = tid; i < PB_BM * LDX; i += 256) Xs[i] = (bf16_t)0.f;
  for (int i = tid; i < a.nxt * 16 * LDD; i += 256) Ws[i] = (bf16_t)0.f;
  __syncthreads();
  if (a.dx) {
    for (int i = tid; i < Cin * CCH; i += 256) {
      const int ci = i / CCH, cc = i - ci * CCH;
      *(bf16x8*)(Ws + ci * LDD + cc * 8) = *(const bf16x8*)(a.wt1 + (long)ci * Cout + cc * 8);
    }
  }

  const long mb = (long)blockIdx.x * a.chunk;
  const long me = mb + a.chunk < a.M ? mb + a.chunk : a.M;

  f32x4 accw[WT];
#pragma unroll
  for (int i = 0; i < WT; ++i) accw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntile = a.nco * a.nci;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;

  for (long m0 = mb; m0 < me; m0 += PB_BM) {
    __syncthreads();  // the previous step's readers of Ds / Xs are done
    // The thread index passes through an opaque copy each step, so the per-thread LDS / global
    // offsets below are recomputed in the loop (a few VALU ops) instead of being hoisted out of
    // it as loop invariants — each hoisted offset held a VGPR for the whole kernel and together
    // they cost two thirds of the occupancy.
    int tid_l = tid;
    asm volatile("" : "+v"(tid_l));
    const int tid = tid_l;
    const int g = (tid & 63) >> 4, li = tid & 15, q = li >> 2, p = li & 3;
    // ---- 1. dy = BatchNorm backward of (dz, y) -> Ds; a -> Xs ----------------------------
    // the conv-input rows are loaded first so their latency overlaps the dz / y loads
    constexpr int XR = NX / 2 > 0 ? NX / 2 : 1;   // 64 * Cin/8 chunks / 256 threads <= NX/2
    const int xtot = PB_BM * XCH;
    bf16x8 xr[XR];
#pragma unroll
    for (int k = 0; k < XR; ++k) {
      const int idx = tid + k * 256;
      const int r = idx / XCH, cc = idx - r * XCH;
      if (idx < xtot && m0 + r < me) xr[k] = *(const bf16x8*)(a.x + (m0 + r) * Cin + cc * 8);
    }
    const int tot = PB_BM * CCH;
    for (int base = tid; base < tot; base += 512) {
      bf16x8 dv[2], yv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int idx = base + u * 256;
        const int r = idx / CCH, cc = idx - r * CCH;
        const long m = m0 + r;
        if (idx < tot && m < me) {
          dv[u] = *(const bf16x8*)(a.dz + m * Cout + cc * 8);
          yv[u] = *(const bf16x8*)(a.y + m * Cout + cc * 8);
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int idx = base + u * 256;
        if (idx >= tot) continue;
        const int r = idx / CCH, cc = idx - r * CCH;
        const long m = m0 + r;
        bf16x8 o;
        if (m < me) {
          // two halves of 4 channels: 7 coefficient fields x 4 live at a time
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            f32x4 f[7];
#pragma unroll
            for (int k = 2; k < 7; ++k) f[k] = *(const f32x4*)(ctab + k * Cout + cc * 8 + 4 * h);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const int j = 4 * h + jj;
              const float yj = (float)yv[u][j];
              const float z = fmaf(yj, f[2][jj], f[3][jj]);
              const float gj = (float)dv[u][j] * (z > 0.f ? (z < ghi ? 1.f : 0.f) : glo);
              o[j] = (bf16_t)bn_bwd_apply1<bf16_t>(f[4][jj], gj, f[5][jj], f[6][jj], 0.f, yj);   // fields 5, 6: k1, k0
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (bf16_t)0.f;
        }
        *(bf16x8*)(Ds + r * LDD + cc * 8) = o;
      }
    }
#pragma unroll
    for (int k = 0; k < XR; ++k) {
      const int idx = tid + k * 256;
      if (idx >= xtot) continue;
      const int r = idx / XCH, cc = idx - r * XCH;
      bf16x8 v = xr[k];
      if (m0 + r < me) {
        if (prox) {
          const f32x4 s0 = *(const f32x4*)(xtab + cc * 8), s1 = *(const f32x4*)(xtab + cc * 8 + 4);
          const f32x4 h0 = *(const f32x4*)(xtab + Cin + cc * 8), h1 = *(const f32x4*)(xtab + Cin + cc * 8 + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = (bf16_t)act_fwd(fmaf((float)v[j], s0[j], h0[j]), a.xact);
            v[4 + j] = (bf16_t)act_fwd(fmaf((float)v[4 + j], s1[j], h1[j]), a.xact);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16_t)0.f;
      }
      *(bf16x8*)(Xs + r * LDX + cc * 8) = v;
    }
    if (has_bias && tid < PB_BM) Xs[tid * LDX + Cin] = (bf16_t)(m0 + tid < me ? 1.f : 0.f);
    __syncthreads();
    // ---- 2a. dW (+ db) += dy^T . [a | 1] over the 64 rows ----------------------------------
#pragma unroll
    for (int i = 0; i < WT; ++i) {
      const int t = wave + 4 * i;
      if (t >= ntile) continue;
      const int ct = t / a.nci, it = t - ct * a.nci;
#pragma unroll
      for (int ks = 0; ks < PB_BM / 32; ++ks) {
        const bf16_t* pd = Ds + (ks * 32 + 8 * g + q) * LDD + ct * 16 + 4 * p;
        const bf16_t* px = Xs + (ks * 32 + 8 * g + q) * LDX + it * 16 + 4 * p;
        const bf16x4 lo = pb_tr_read(pd), hi = pb_tr_read(pd + 4 * LDD);
        const bf16x4 l2 = pb_tr_read(px), h2 = pb_tr_read(px + 4 * LDX);
        const bf16x8 fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 fb = {l2[0], l2[1], l2[2], l2[3], h2[0], h2[1], h2[2], h2[3]};
        accw[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, accw[i], 0, 0, 0);
      }
    }
    if (!a.dx) continue;
    // ---- 2b. dx = dy . W for this wave's 16 rows -------------------------------------------
    f32x4 accx[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) accx[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < a.kd / 32; ++s) {
      const bf16x8 fa = *(const bf16x8*)(Ds + (wave * 16 + li) * LDD + s * 32 + 8 * g);
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        if (j >= a.nxt) continue;
        const bf16x8 fb = *(const bf16x8*)(Ws + (j * 16 + li) * LDD + s * 32 + 8 * g);
        accx[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, accx[j], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done reading Xs (dW) before it becomes the dx stage
    // ---- 3. dx -> Xs -> 16-byte row segments ------------------------------------------------
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      if (j >= a.nxt) continue;
      const int col = j * 16 + li;
      if (col < Cin) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Xs[(wave * 16 + 4 * g + r) * LDX + col] = (bf16_t)accx[j][r];
      }
    }
    __syncthreads();
    for (int idx = tid; idx < PB_BM * XCH; idx += 256) {
      const int r = idx / XCH, cc = idx - r * XCH;
      const long m = m0 + r;
      if (m < me) *(bf16x8*)(a.dx + m * Cin + cc * 8) = *(const bf16x8*)(Xs + r * LDX + cc * 8);
    }
  }
  // ---- partial dW / db of this block ------------------------------------------------------
  float* pw = a.partw + (long)blockIdx.x * Cout * Cin;
#pragma unroll
  for (int i = 0; i < WT; ++i) {
    const int t = wave + 4 * i;
    if (t >= ntile) continue;
    const int ct = t / a.nci, it = t - ct * a.nci;
    const int ci = it * 16 + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = ct * 16 + 4 * g + r;
      if (co >= Cout) continue;
      if (ci < Cin) pw[(long)co * Cin + ci] = accw[i][r];
      else if (has_bias && ci == Cin) a.partb[(long)blockIdx.x * Cout + co] = accw[i][r];
    }
  }
}


// =====================================================================================
// Streaming form (the expand shapes 16->96 and 24->144 without bias): every wave works on
// its own 32-row tiles with no block barrier inside the row loop — the 64-row block-synchronous
// steps above leave the memory system idle while all four waves sit in their MFMA phase.
//   * lane constants: a lane owns ONE 8-channel chunk cc of dz / y (lanes = RG row groups x
//     COUT/8 chunks) for the whole launch, so its BatchNorm-backward constants (sc, sh, a, k1,
//     k0 of 8 channels) sit in registers — no per-element coefficient reads from LDS;
//   * per 16-row half: dz / y / x arrive by buffer loads from a per-tile resource (rows past M
//     read 0, their dx stores are dropped), dy = bn_bwd_apply (rounded to bf16, the arithmetic of
//     the block kernel) goes to this wave's LDS tile, then the NEXT half's loads are issued into
//     the same registers before the MFMA work of this one (one half in flight per wave, no extra
//     registers);
//   * dx = dy . W for the half (A fragments straight from the dy rows, W staged once per block),
//     staged through a wave-private LDS slot and written as 16-byte row segments;
//   * after the second half, dW += dy^T . x over the 32 rows (both operands read transposed,
//     ds_read_b64_tr_b16, as above);
//   * at the end the four waves' dW add in wave order in LDS (one partial per block, slab_sum).
// dx is the block kernel's bit for bit (same dy, same MFMA k order); dW sums its rows in another
// grouping (fp32, within the float64 bounds of tests/test_gpu_pwbwd.py).
// =====================================================================================
typedef float pb_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 pb_b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pb_f2 pb_unpack(unsigned u) {   // bf16 pair (low, high) -> fp32 pair
  return pb_f2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}
__device__ __forceinline__ unsigned pb_round(pb_f2 v) {    // one v_cvt_pk_bf16_f32 (RNE per element)
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, pb_b2));
}
// ReLU6 gradient gate (0 < z < 6; NaN -> closed) as one unsigned compare on the bits
__device__ __forceinline__ bool pb_relu6_open(float z) { return __builtin_bit_cast(unsigned, z) - 1u < 0x40BFFFFFu; }

template <int CIN, int COUT>
struct PbsGeo {
  // CW channels per lane chunk: 4 (8-byte loads) where the chunks tile 64 lanes into whole rows
  // without waste (96: 2 row groups x 24 chunks, 16 rows in 8 steps, 20 constant registers
  // instead of 40), else 8
  static constexpr int CW = (64 / (COUT / 4)) * (COUT / 4) >= 48 && 16 % (64 / (COUT / 4)) == 0 ? 4 : 8;
  static constexpr int CCH = COUT / CW, RG = 64 / CCH, JN = (16 + RG - 1) / RG;
  static constexpr int KT = (COUT + 31) / 32, KD = KT * 32, LDD = KD + 8;
  static constexpr int NCO = COUT / 16, XCH = CIN / 8, NCI = (CIN + 15) / 16, LDX = NCI * 16 + 8;
  static constexpr int LDC = CIN + 8;
  static constexpr int WREG = 32 * LDD + 32 * LDX + 16 * LDC;    // bf16 elements per wave
  static constexpr int WS = NCI * 16 * LDD;                       // wt1 image (bf16 elements)
  static constexpr int XT = 3 * CIN * 2;                          // input-prologue table (bf16 slots)
  static constexpr int LDW = 40;                                  // RC: forward weight rows, k zero-padded to 32
  static constexpr int WF = COUT * LDW;                           // RC: forward weight image (bf16 elements)
  static constexpr size_t lds(bool rc = false) {
    const size_t main = (size_t)(WS + XT + 4 * WREG + (rc ? WF : 0)) * 2;
    const size_t red = (size_t)(WS + XT + (rc ? WF : 0)) * 2 + (size_t)COUT * NCI * 16 * 4 +
                       (size_t)4 * 16 * 2 * CIN * 4;
    return main > red ? main : red;
  }
};

template <int CW> struct PbsVec;
template <> struct PbsVec<4> { typedef bf16x4 T; };
template <> struct PbsVec<8> { typedef bf16x8 T; };

// XG (with the input prologue): also the input BatchNorm's backward sums over (dx, x) — the
// expand conv of a block whose input is the previous block's project output (linear BatchNorm):
// that BatchNorm's gradient is this dx, so its rod_bn_bwd_reduce pass is not needed
// (rod_pw_bwd_gred on the expand shapes); part blockIdx.x of [nblk][2][CIN]
// XL: the input BatchNorm is linear (act NONE; the project output chained into an expand) —
// its prologue and sums compile without the activation (a runtime branch costs the XG form
// 12 VGPRs and a wave per SIMD).
// RC (ABI 23, rod_pw_bwd_rc / rod_pw_bwd_gred_rc): the pre-BatchNorm y = x_act . W^T is not read
// but recomputed per 16-row half from the conv input already staged for the weight gradient — the
// forward's MFMA (v_mfma_f32_16x16x32_bf16, k zero-padded to 32) with the operands swapped, so the
// lane holds 4 consecutive channels of one row, rounded to bf16 once: the stored y bit for bit.
// It is written into the half's dy rows in LDS, where each lane reads its chunk and overwrites it
// with dy in place (the same lane reads and writes an element).  Saves the M x COUT y stream (the
// expanded tensor of an inverted-residual block: 1.42 GB at 720p b8 for 16 -> 96).
// Occupancy: the 16 -> 96 forms at 3 waves per SIMD — 120-168 VGPRs and no AGPRs, no spills
// (unbounded: 156 + 24 AGPRs, 2 waves), so the 768-block grid is resident at once: block 1's
// recomputing gred form 568.5 -> 557.8 us; the 24 -> 144 forms (200-250 + 72-76 AGPRs, 1 wave)
// measured slower at 2 waves (306 -> 321-327 us) and stay unbounded (profiles/r6_pwbwd_bounds_ab.txt).
template <int CIN, int COUT, bool PRO, bool DX, bool XG = false, bool XL = false, bool RC = false>
__global__ void __launch_bounds__(256, CIN == 16 ? 3 : 1) pw_bwd_stream_kernel(PwBwdArgs a, long ntiles, float* __restrict__ xparts) {
  using G = PbsGeo<CIN, COUT>;
  static_assert(!XG || (PRO && DX), "the input sums need the prologue and dx");
  static_assert(!RC || CIN <= 32, "the recompute is one k step");
  constexpr int CW = G::CW, CCH = G::CCH, RG = G::RG, JN = G::JN, KT = G::KT, LDD = G::LDD, NCO = G::NCO,
                XCH = G::XCH, NCI = G::NCI, LDX = G::LDX, LDC = G::LDC;
  typedef typename PbsVec<CW>::T VT;
  static_assert(COUT % 16 == 0 && CIN % 8 == 0 && 16 * XCH <= 64, "streaming pw_bwd geometry");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ws = (bf16_t*)smem;                                   // [NCI*16][LDD]: wt1 rows (ci), k = co
  float* xtab = (float*)(Ws + G::WS);                           // [3][CIN]: input prologue scale, shift, mean
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  bf16_t* Ds = Ws + G::WS + G::XT + wave * G::WREG;             // [32][LDD]  dy of the tile
  bf16_t* Xs = Ds + 32 * LDD;                                   // [32][LDX]  conv input of the tile
  bf16_t* Cx = Xs + 32 * LDX;                                   // [16][LDC]  dx staging
  bf16_t* Wf = Ws + G::WS + G::XT + 4 * G::WREG;                // RC: [COUT][LDW] forward weights
  // zero everything once (dy columns >= COUT, x columns >= CIN stay 0), then the weights
  for (int i = tid; i < (G::WS + G::XT + 4 * G::WREG + (RC ? G::WF : 0)) / 8; i += 256) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16_t)0.f;
    ((bf16x8*)smem)[i] = z;
  }
  __syncthreads();
  if constexpr (DX) {
    for (int i = tid; i < CIN * (COUT / 8); i += 256) {
      const int ci = i / (COUT / 8), c8 = i - ci * (COUT / 8);
      *(bf16x8*)(Ws + ci * LDD + c8 * 8) = *(const bf16x8*)(a.wt1 + (long)ci * COUT + c8 * 8);
    }
  }
  if constexpr (PRO) {
    for (int c = tid; c < CIN; c += 256) {
      bn_affine(a.xmean, a.xrstd, a.xgamma, a.xbeta, c, xtab[c], xtab[CIN + c]);
      xtab[2 * CIN + c] = a.xmean[c];
    }
  }
  if constexpr (RC) {
    for (int i = tid; i < COUT * (CIN / 8); i += 256) {
      const int co = i / (CIN / 8), k8 = i - co * (CIN / 8);
      *(bf16x8*)(Wf + co * G::LDW + k8 * 8) = *(const bf16x8*)(a.wt0 + (long)co * CIN + k8 * 8);
    }
  }
  __syncthreads();

  // ---- lane constants ---------------------------------------------------------------------
  float xsg[XG ? 8 : 1] = {}, xsgx[XG ? 8 : 1] = {};   // XG: sums of g and g*(x - mean), this lane's chunk
  const int rg = lane / CCH, cc = lane - (lane / CCH) * CCH;
  const bool dact = rg < RG;
  const int c0 = dact ? cc * CW : 0;
  float sc[CW], sh[CW], ca[CW], k1[CW], k0[CW];
#pragma unroll
  for (int e = 0; e < CW; ++e) {
    const int c = c0 + e;
    bn_affine(a.mean, a.rstd, a.gamma, a.beta, c, sc[e], sh[e]);
    ca[e] = a.coef[c];
    bn_bwd_k_fold(ca[e], a.mean[c], a.rstd[c], a.coef[COUT + c], a.coef[2 * COUT + c], k1[e], k0[e]);
  }
  const float ghi = a.act == ROD_ACT_RELU6 ? 6.f : INFINITY;
  const float glo = a.act == ROD_ACT_LEAKY ? 0.2f : a.act == ROD_ACT_NONE ? 1.f : 0.f;
  const int xr = lane / XCH, xc = lane - (lane / XCH) * XCH;
  const bool xact = lane < 16 * XCH;
  // lane offset of chunk j inside a half (bytes): vd0 + j * RG rows; ROD_OOB: no row there
  const unsigned vd0 = dact ? (unsigned)((rg * COUT + cc * CW) * 2) : ROD_OOB;
  auto vdj = [&](int j) -> unsigned {
    if constexpr (JN * RG == 16) return vd0 + (unsigned)(j * RG * COUT * 2);
    else return rg + RG * j < 16 ? vd0 + (unsigned)(j * RG * COUT * 2) : ROD_OOB;
  };
  const unsigned vx = xact ? (unsigned)((xr * CIN + xc * 8) * 2) : ROD_OOB;
  const long M = a.M;
  auto rsrc_rows = [&](const void* base, long row0, int rowbytes) {   // rows [row0, min(row0 + 32, M))
    const long rows = row0 < M ? (M - row0 < 32 ? M - row0 : 32) : 0;
    return rod_rsrc((const char*)base + (row0 < M ? row0 : 0) * rowbytes, (unsigned)(rows * rowbytes));
  };

  f32x4 accw[NCO][NCI];
#pragma unroll
  for (int i = 0; i < NCO; ++i)
#pragma unroll
    for (int j = 0; j < NCI; ++j) accw[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const long wstride = (long)gridDim.x * 4;
  long t = (long)blockIdx.x * 4 + wave;
  VT dzv[JN], yv[RC ? 1 : JN];
  bf16x8 xv;
  {   // the first half (t >= ntiles: an empty resource, the loads return 0)
    const rsrc_t rdz = rsrc_rows(a.dz, t * 32, COUT * 2);
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      dzv[j] = buf_ld<VT>(rdz, vdj(j), 0u);
      if constexpr (!RC) yv[j] = buf_ld<VT>(rsrc_rows(a.y, t * 32, COUT * 2), vdj(j), 0u);
    }
    xv = buf_ld<bf16x8>(rsrc_rows(a.x, t * 32, CIN * 2), vx, 0u);
  }
  for (; t < ntiles; t += wstride) {
    const long row0 = t * 32;
    // not unrolled: the reloads land in the registers just consumed (unrolled, the compiler
    // double-buffers them: +32 VGPRs)
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      // ---- dy = BatchNorm backward of (dz, y) -> Ds; x (+ prologue) -> Xs ------------------
      // each chunk's registers are reloaded with the NEXT half's chunk as soon as they are
      // consumed, so this wave keeps loads in flight through its VALU work as well
      // (RC: x first, then y recomputed from it into the dy rows, then dy over it in place)
      const long rown = (h == 0 ? t : t + wstride) * 32;
      const rsrc_t ndz = rsrc_rows(a.dz, rown, COUT * 2);
      const unsigned nso = (unsigned)((1 - h) * 16 * COUT * 2);
      auto dy_rows = [&]() {
        const rsrc_t ny = rsrc_rows(a.y, rown, COUT * 2);
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int r = rg + RG * j;
          const bool rok = dact && (JN * RG == 16 || r < 16);
          bf16_t* dp = Ds + (h * 16 + (rok ? r : 0)) * LDD + cc * CW;
          VT yj4;
          if constexpr (RC) yj4 = *(const VT*)dp;
          else yj4 = yv[j];
          typename PbsVec<CW>::T o;
#pragma unroll
          for (int e = 0; e < CW; ++e) {
            const float yj = (float)yj4[e];
            const float z = fmaf(yj, sc[e], sh[e]);
            const float gj = (float)dzv[j][e] * (z > 0.f ? (z < ghi ? 1.f : 0.f) : glo);
            o[e] = (bf16_t)bn_bwd_apply1<bf16_t>(ca[e], gj, k1[e], k0[e], 0.f, yj);
          }
          dzv[j] = buf_ld<VT>(ndz, vdj(j), nso);
          if constexpr (!RC) yv[j] = buf_ld<VT>(ny, vdj(j), nso);
          if (rok) *(VT*)dp = o;
        }
      };
      if constexpr (!RC) dy_rows();
      const bf16x8 xcur = xv;   // XG: the raw x of this half, for the sums at the dx write-back
      {
        bf16x8 v = xv;
        if constexpr (PRO) {
          const bool rok = row0 + h * 16 + xr < M;   // rows past M stay 0 (not act(shift))
          const f32x4 s0 = *(const f32x4*)(xtab + xc * 8), s1 = *(const f32x4*)(xtab + xc * 8 + 4);
          const f32x4 h0 = *(const f32x4*)(xtab + CIN + xc * 8), h1 = *(const f32x4*)(xtab + CIN + xc * 8 + 4);
          if constexpr (XL) {   // linear input BatchNorm: packed pairs
            const u32x4_t u = __builtin_bit_cast(u32x4_t, v);
            u32x4_t o;
#pragma unroll
            for (int h2 = 0; h2 < 4; ++h2) {
              const f32x4& sc4 = h2 < 2 ? s0 : s1;
              const f32x4& sh4 = h2 < 2 ? h0 : h1;
              const int b = (h2 & 1) * 2;
              const pb_f2 z2 = __builtin_elementwise_fma(pb_unpack(u[h2]), pb_f2{sc4[b], sc4[b + 1]},
                                                         pb_f2{sh4[b], sh4[b + 1]});
              o[h2] = rok ? pb_round(z2) : 0u;
            }
            v = __builtin_bit_cast(bf16x8, o);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = rok ? (bf16_t)act_fwd(fmaf((float)v[e], s0[e], h0[e]), a.xact) : (bf16_t)0.f;
              v[4 + e] = rok ? (bf16_t)act_fwd(fmaf((float)v[4 + e], s1[e], h1[e]), a.xact) : (bf16_t)0.f;
            }
          }
        }
        xv = buf_ld<bf16x8>(rsrc_rows(a.x, rown, CIN * 2), vx, (unsigned)((1 - h) * 16 * CIN * 2));
        if (xact) *(bf16x8*)(Xs + (h * 16 + xr) * LDX + xc * 8) = v;
      }
      __builtin_amdgcn_wave_barrier();
      if constexpr (RC) {
        // y^T tile by tile: A = W rows (16 channels x k), B = this half's x rows (k x 16 rows);
        // lane (g, li) gets channels 16ct + 4g .. +3 of row li -> one 8-byte LDS write per tile
        const bf16x8 zero8 = {};
        const bf16x8 fb = 8 * g < CIN ? *(const bf16x8*)(Xs + (h * 16 + li) * LDX + 8 * g) : zero8;
#pragma unroll
        for (int ct = 0; ct < NCO; ++ct) {
          const bf16x8 fw = 8 * g < CIN ? *(const bf16x8*)(Wf + (ct * 16 + li) * G::LDW + 8 * g) : zero8;
          const f32x4 yt = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw, fb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          const bf16x4 yb = {(bf16_t)yt[0], (bf16_t)yt[1], (bf16_t)yt[2], (bf16_t)yt[3]};
          *(bf16x4*)(Ds + (h * 16 + li) * LDD + ct * 16 + 4 * g) = yb;
        }
        __builtin_amdgcn_wave_barrier();
        dy_rows();
        __builtin_amdgcn_wave_barrier();
      }
      if constexpr (DX) {
        // ---- dx = dy . W for the 16 rows of this half -> Cx -> 16-byte row segments ---------
        f32x4 accx[NCI];
#pragma unroll
        for (int j = 0; j < NCI; ++j) accx[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KT; ++s) {
          const bf16x8 fa = *(const bf16x8*)(Ds + (h * 16 + li) * LDD + s * 32 + 8 * g);
#pragma unroll
          for (int j = 0; j < NCI; ++j) {
            const bf16x8 fb = *(const bf16x8*)(Ws + (j * 16 + li) * LDD + s * 32 + 8 * g);
            accx[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, accx[j], 0, 0, 0);
          }
        }
#pragma unroll
        for (int j = 0; j < NCI; ++j) {
          const int col = j * 16 + li;
          if (col < CIN) {
#pragma unroll
            for (int r = 0; r < 4; ++r) Cx[(4 * g + r) * LDC + col] = (bf16_t)accx[j][r];
          }
        }
        __builtin_amdgcn_wave_barrier();
        const rsrc_t rdx = rsrc_rows(a.dx, row0, CIN * 2);
        const bf16x8 ov = *(const bf16x8*)(Cx + (xact ? xr : 0) * LDC + xc * 8);
        buf_st(ov, rdx, vx, (unsigned)(h * 16 * CIN * 2));
        if constexpr (XG) {
          if (xact && row0 + h * 16 + xr < M) {
            if constexpr (XL) {   // linear input BatchNorm (the project's): g = dx
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float g = (float)ov[e];
                xsg[e] += g;
                xsgx[e] = fmaf(g, (float)xcur[e] - xtab[2 * CIN + xc * 8 + e], xsgx[e]);
              }
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float xe = (float)xcur[e];
                const float g = (float)ov[e] * act_grad(fmaf(xe, xtab[xc * 8 + e], xtab[CIN + xc * 8 + e]), a.xact);
                xsg[e] += g;
                xsgx[e] = fmaf(g, xe - xtab[2 * CIN + xc * 8 + e], xsgx[e]);
              }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    // ---- dW += dy^T . x over the tile's 32 rows ---------------------------------------------
#pragma unroll
    for (int ct = 0; ct < NCO; ++ct) {
      const bf16_t* pd = Ds + (8 * g + q) * LDD + ct * 16 + 4 * p;
      const bf16x4 lo = pb_tr_read(pd), hi = pb_tr_read(pd + 4 * LDD);
      const bf16x8 fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int it = 0; it < NCI; ++it) {
        const bf16_t* px = Xs + (8 * g + q) * LDX + it * 16 + 4 * p;
        const bf16x4 l2 = pb_tr_read(px), h2 = pb_tr_read(px + 4 * LDX);
        const bf16x8 fb = {l2[0], l2[1], l2[2], l2[3], h2[0], h2[1], h2[2], h2[3]};
        accw[ct][it] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, accw[ct][it], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();   // the next tile's dy / x writes stay after these reads
  }
  // ---- the block's dW: the four waves add in wave order -> part blockIdx.x -----------------
  float* red = (float*)(smem + (size_t)(G::WS + G::XT) * 2);   // [COUT][NCI*16]
  constexpr int LR = NCI * 16;
  __syncthreads();
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int ct = 0; ct < NCO; ++ct)
#pragma unroll
        for (int it = 0; it < NCI; ++it)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* d = red + (ct * 16 + 4 * g + r) * LR + it * 16 + li;
            *d = w == 0 ? accw[ct][it][r] : *d + accw[ct][it][r];
          }
    }
    __syncthreads();
  }
  float* pw = a.partw + (long)blockIdx.x * COUT * CIN;
  for (int i = tid; i < COUT * CIN; i += 256) {
    const int co = i / CIN, ci = i - co * CIN;
    pw[i] = red[co * LR + ci];
  }
  if constexpr (XG) {   // waves, then the 16 row lanes of each chunk, added in a fixed order
    float* gbuf = red + COUT * LR;                                // [4][16][2][CIN]
    if (xact) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        gbuf[((wave * 16 + xr) * 2 + 0) * CIN + xc * 8 + e] = xsg[e];
        gbuf[((wave * 16 + xr) * 2 + 1) * CIN + xc * 8 + e] = xsgx[e];
      }
    }
    __syncthreads();
    float* xp = xparts + (long)blockIdx.x * 2 * CIN;
    for (int i = tid; i < 2 * CIN; i += 256) {
      const int k = i / CIN, c = i - k * CIN;
      float sum = 0.f;
      for (int w = 0; w < 4; ++w)
        for (int r = 0; r < 16; ++r) sum += gbuf[((w * 16 + r) * 2 + k) * CIN + c];
      xp[i] = k ? sum * a.xrstd[c] : sum;
    }
  }
}


// =====================================================================================
// Project form with the input BatchNorm's backward sums (rod_pw_bwd_gred).  The conv input is
// x_p = act_x(BN_x(x)) with x the raw depthwise output; the block's backward needs, besides
// dx / dW, BN_x's backward sums over (dx, x) — which this kernel forms from the x it already
// reads for the weight gradient and the dx it writes.  Cout is small (16..64) and Cin large, so
// the grid splits Cin into groups of NW columns (blockIdx.y): a group re-reads only dz / y (4*Cout
// bytes a row) and owns its columns of x, dx, dW and the sums.  Per wave, 32-row tiles in two
// 16-row halves, no block barrier in the row loop:
//   * dy: a lane owns one 4-channel chunk of dz / y (constants in registers), reloaded with the
//     next half's chunk as soon as it is consumed; rows past M give dy = 0;
//   * x: a lane owns one 8-column chunk of the group (BN_x constants in registers) for RGX row
//     groups; x_p = act_x(BN_x(x)) (bf16) goes to LDS for the weight gradient, the raw x stays
//     in registers for the sums; the next half's x is loaded into a second register set at the
//     start of each half (the first form loaded it after the sums: 2.5 TB/s on 96->24);
//   * dx = dy . W for the half (A fragments from the dy rows in LDS, W's group rows in LDS),
//     staged in LDS, written by the x lanes, which add g and g*xhat of their chunk as they write;
//   * after the second half dW += dy^T . x_p over the 32 rows (transposed LDS reads);
//   * at the end the waves' dW and sums add in a fixed order -> part blockIdx.x.
// =====================================================================================
template <int COUT, int NW>
struct PbgGeo {
  static constexpr int CCH = COUT / 4, RG = 64 / CCH, JN = (16 + RG - 1) / RG;
  static constexpr int KT = (COUT + 31) / 32, KD = KT * 32, LDD = KD + 8;
  static constexpr int NCO = (COUT + 15) / 16;
  static constexpr int XCH = NW / 8, RGX = 64 / XCH, JX = (16 + RGX - 1) / RGX, NWT = NW / 16;
  static constexpr int LDX = NW + 8;
  static constexpr int WREG = 32 * LDD + 32 * LDX + 16 * LDX;     // bf16 elements per wave
  static constexpr int WS = NW * LDD;                              // the group's wt1 rows
  static constexpr int RED = NCO * 16 * NW + 4 * RGX * 2 * NW;     // fp32 end-of-launch buffer
  static constexpr size_t lds() {
    const size_t main = (size_t)(WS + 4 * WREG) * 2;
    const size_t red = (size_t)WS * 2 + (size_t)RED * 4;
    return main > red ? main : red;
  }
};

// FAST: the block's activations (linear output BatchNorm, ReLU6 input BatchNorm) at compile
// time, channel pairs as packed fp32 ops; otherwise both activations at run time, per element
// DYP (rod_pw_bwd_gred_dyp): dy written by column group 0, dx not stored — a template argument so
// the two entries are separate kernels in a trace / PMC pass (rod/roofline.py ENTRY_KERNELS)
template <int COUT, int NW, bool FAST, bool DYP = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) pw_bwd_gred_kernel(PwBwdArgs a, long ntiles, float* __restrict__ xparts) {
  using G = PbgGeo<COUT, NW>;
  constexpr int CCH = G::CCH, RG = G::RG, JN = G::JN, KT = G::KT, LDD = G::LDD, NCO = G::NCO, XCH = G::XCH,
                RGX = G::RGX, JX = G::JX, NWT = G::NWT, LDX = G::LDX;
  static_assert(COUT % 8 == 0 && NW % 16 == 0 && RG * CCH <= 64 && RGX * XCH <= 64, "gred pw_bwd geometry");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Cin = a.Cin;
  const int n0 = blockIdx.y * NW;                               // this group's first column
  bf16_t* Ws = (bf16_t*)smem;                                   // [NW][LDD]: wt1 rows n0.., k = co
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  bf16_t* Ds = Ws + G::WS + wave * G::WREG;                     // [32][LDD]  dy of the tile
  bf16_t* Xs = Ds + 32 * LDD;                                   // [32][LDX]  x_p of the tile
  bf16_t* Cx = Xs + 32 * LDX;                                   // [16][LDX]  dx staging
  for (int i = tid; i < (G::WS + 4 * G::WREG) / 8; i += 256) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16_t)0.f;
    ((bf16x8*)smem)[i] = z;
  }
  __syncthreads();
  for (int i = tid; i < NW * (COUT / 8); i += 256) {
    const int c = i / (COUT / 8), c8 = i - c * (COUT / 8);
    *(bf16x8*)(Ws + c * LDD + c8 * 8) = *(const bf16x8*)(a.wt1 + (long)(n0 + c) * COUT + c8 * 8);
  }
  __syncthreads();

  // ---- lane constants: dy chunk (4 channels of Cout) and x chunk (8 columns of the group) ----
  const int rg = lane / CCH, cc = lane - (lane / CCH) * CCH;
  const bool dact = rg < RG;
  float sc[4], sh[4], ca[4], k1[4], k0[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = (dact ? cc * 4 : 0) + e;
    bn_affine(a.mean, a.rstd, a.gamma, a.beta, c, sc[e], sh[e]);
    ca[e] = a.coef[c];
    bn_bwd_k_fold(ca[e], a.mean[c], a.rstd[c], a.coef[COUT + c], a.coef[2 * COUT + c], k1[e], k0[e]);
  }
  const float ghi = a.act == ROD_ACT_RELU6 ? 6.f : INFINITY;
  const float glo = a.act == ROD_ACT_LEAKY ? 0.2f : a.act == ROD_ACT_NONE ? 1.f : 0.f;
  const int rx = lane / XCH, xc = lane - (lane / XCH) * XCH;
  const bool xact = rx < RGX;
  // sgx sums g*(x - mean); the rstd factor is applied once per column at the end
  float xsc[8], xsh[8], xmu[8], sg[8], sgx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = n0 + (xact ? xc * 8 : 0) + e;
    bn_affine(a.xmean, a.xrstd, a.xgamma, a.xbeta, c, xsc[e], xsh[e]);
    xmu[e] = a.xmean[c];
    sg[e] = sgx[e] = 0.f;
  }
  // FAST: the same constants as register pairs (packed operands without pair-building moves)
  pb_f2 ca2[2], k12[2], k02[2], xsc2[4], xsh2[4], xmu2[4];
  if constexpr (FAST) {
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      ca2[h2] = pb_f2{ca[2 * h2], ca[2 * h2 + 1]};
      k12[h2] = pb_f2{k1[2 * h2], k1[2 * h2 + 1]};
      k02[h2] = pb_f2{k0[2 * h2], k0[2 * h2 + 1]};
    }
#pragma unroll
    for (int h2 = 0; h2 < 4; ++h2) {
      xsc2[h2] = pb_f2{xsc[2 * h2], xsc[2 * h2 + 1]};
      xsh2[h2] = pb_f2{xsh[2 * h2], xsh[2 * h2 + 1]};
      xmu2[h2] = pb_f2{xmu[2 * h2], xmu[2 * h2 + 1]};
    }
  }
  pb_f2 sg2[4] = {}, sgx2[4] = {};
  const unsigned vd0 = dact ? (unsigned)((rg * COUT + cc * 4) * 2) : ROD_OOB;
  auto vdj = [&](int j) -> unsigned {
    if constexpr (JN * RG == 16) return vd0 + (unsigned)(j * RG * COUT * 2);
    else return rg + RG * j < 16 ? vd0 + (unsigned)(j * RG * COUT * 2) : ROD_OOB;
  };
  const unsigned vx0 = xact ? (unsigned)((rx * Cin + xc * 8) * 2) : ROD_OOB;
  auto vxj = [&](int j) -> unsigned {
    if constexpr (JX * RGX == 16) return vx0 + (unsigned)(j * RGX * Cin * 2);
    else return rx + RGX * j < 16 ? vx0 + (unsigned)(j * RGX * Cin * 2) : ROD_OOB;
  };
  const long M = a.M;
  auto rows_of = [&](long row0) -> long { return row0 < M ? (M - row0 < 32 ? M - row0 : 32) : 0; };
  auto rsrc_d = [&](const void* base, long row0) {   // dz / y rows [row0, +32) of Cout channels
    return rod_rsrc((const char*)base + (row0 < M ? row0 : 0) * COUT * 2, (unsigned)(rows_of(row0) * COUT * 2));
  };
  auto rsrc_x = [&](const void* base, long row0) {   // x / dx rows of this group's columns
    const long r = rows_of(row0);
    return rod_rsrc((const char*)base + ((row0 < M ? row0 : 0) * Cin + n0) * 2,
                    r > 0 ? (unsigned)(((r - 1) * Cin + NW) * 2) : 0u);
  };

  f32x4 accw[NCO][NWT];
#pragma unroll
  for (int i = 0; i < NCO; ++i)
#pragma unroll
    for (int j = 0; j < NWT; ++j) accw[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const long wstride = (long)gridDim.x * 4;
  long t = (long)blockIdx.x * 4 + wave;
  bf16x4 dzv[JN], yv[JN];
  bf16x8 xv[JX];
  {
    const rsrc_t rdz = rsrc_d(a.dz, t * 32), ry = rsrc_d(a.y, t * 32), rxx = rsrc_x(a.x, t * 32);
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      dzv[j] = buf_ld<bf16x4>(rdz, vdj(j), 0u);
      yv[j] = buf_ld<bf16x4>(ry, vdj(j), 0u);
    }
#pragma unroll
    for (int j = 0; j < JX; ++j) xv[j] = buf_ld<bf16x8>(rxx, vxj(j), 0u);
  }
  for (; t < ntiles; t += wstride) {
    const long row0 = t * 32;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      const long rown = (h == 0 ? t : t + wstride) * 32;
      // the next half's x, in flight through this whole half (xv is needed until its sums)
      bf16x8 xn[JX];
      {
        const rsrc_t nx = rsrc_x(a.x, rown);
        const unsigned nso = (unsigned)((1 - h) * 16 * Cin * 2);
#pragma unroll
        for (int j = 0; j < JX; ++j) xn[j] = buf_ld<bf16x8>(nx, vxj(j), nso);
      }
      // ---- dy -> Ds (rows past M: 0); the next half's dz / y chunks reload as consumed --------
      {
        const rsrc_t ndz = rsrc_d(a.dz, rown), ny = rsrc_d(a.y, rown);
        const unsigned nso = (unsigned)((1 - h) * 16 * COUT * 2);
        // dyp (column group 0 only; other blocks and rows past M: the empty / range-checked resource)
        const rsrc_t rdp = DYP && blockIdx.y == 0 ? rsrc_d(a.dyp, row0) : rod_rsrc(a.dz, 0u);
        const unsigned dpso = (unsigned)(h * 16 * COUT * 2);
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int r = rg + RG * j;
          const bool rok = row0 + h * 16 + r < M;
          bf16x4 o;
          if constexpr (FAST) {   // linear output BatchNorm: g = dz; dy = fma(a, dz, fma(k1, y, k0))
            const u32x2_t yu = __builtin_bit_cast(u32x2_t, yv[j]), du = __builtin_bit_cast(u32x2_t, dzv[j]);
            u32x2_t ou;
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              const pb_f2 y2 = pb_unpack(yu[h2]), d2 = pb_unpack(du[h2]);
              const pb_f2 t2 = __builtin_elementwise_fma(k12[h2], y2, k02[h2]);
              ou[h2] = rok ? pb_round(__builtin_elementwise_fma(ca2[h2], d2, t2)) : 0u;
            }
            o = __builtin_bit_cast(bf16x4, ou);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float yj = (float)yv[j][e];
              const float z = fmaf(yj, sc[e], sh[e]);
              const float gj = (float)dzv[j][e] * (z > 0.f ? (z < ghi ? 1.f : 0.f) : glo);
              o[e] = rok ? (bf16_t)bn_bwd_apply1<bf16_t>(ca[e], gj, k1[e], k0[e], 0.f, yj) : (bf16_t)0.f;
            }
          }
          dzv[j] = buf_ld<bf16x4>(ndz, vdj(j), nso);
          yv[j] = buf_ld<bf16x4>(ny, vdj(j), nso);
          buf_st(o, rdp, vdj(j), dpso);   // dropped unless the dyp form (empty resource)
          if (dact && (JN * RG == 16 || r < 16)) *(bf16x4*)(Ds + (h * 16 + r) * LDD + cc * 4) = o;
        }
      }
      // ---- x_p = act_x(BN_x(x)) -> Xs (rows past M: 0) -------------------------------------
#pragma unroll
      for (int j = 0; j < JX; ++j) {
        const int r = rx + RGX * j;
        const bool rok = row0 + h * 16 + r < M;
        bf16x8 v;
        if constexpr (FAST) {   // ReLU6 input BatchNorm
          const u32x4_t xu = __builtin_bit_cast(u32x4_t, xv[j]);
          u32x4_t vu;
#pragma unroll
          for (int h2 = 0; h2 < 4; ++h2) {
            const pb_f2 z2 = __builtin_elementwise_fma(pb_unpack(xu[h2]), xsc2[h2], xsh2[h2]);
            const pb_f2 t2 = {act_t<ROD_ACT_RELU6>(z2.x), act_t<ROD_ACT_RELU6>(z2.y)};
            vu[h2] = rok ? pb_round(t2) : 0u;
          }
          v = __builtin_bit_cast(bf16x8, vu);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v[e] = rok ? (bf16_t)act_fwd(fmaf((float)xv[j][e], xsc[e], xsh[e]), a.xact) : (bf16_t)0.f;
        }
        if (xact && (JX * RGX == 16 || r < 16)) *(bf16x8*)(Xs + (h * 16 + r) * LDX + xc * 8) = v;
      }
      __builtin_amdgcn_wave_barrier();
      // ---- dx = dy . W for the half -> Cx; written by the x lanes with the BN_x sums ------------
      {
        f32x4 accx[NWT];
#pragma unroll
        for (int j = 0; j < NWT; ++j) accx[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KT; ++s) {
          const bf16x8 fa = *(const bf16x8*)(Ds + (h * 16 + li) * LDD + s * 32 + 8 * g);
#pragma unroll
          for (int j = 0; j < NWT; ++j) {
            const bf16x8 fb = *(const bf16x8*)(Ws + (j * 16 + li) * LDD + s * 32 + 8 * g);
            accx[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, accx[j], 0, 0, 0);
          }
        }
#pragma unroll
        for (int j = 0; j < NWT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) Cx[(4 * g + r) * LDX + j * 16 + li] = (bf16_t)accx[j][r];
        __builtin_amdgcn_wave_barrier();
        const rsrc_t rdx = !DYP ? rsrc_x(a.dx, row0) : rod_rsrc(a.x, 0u);   // dyp form: dx not stored
        const unsigned so = (unsigned)(h * 16 * Cin * 2);
#pragma unroll
        for (int j = 0; j < JX; ++j) {
          const int r = rx + RGX * j;
          const bool rok = row0 + h * 16 + r < M && xact && (JX * RGX == 16 || r < 16);
          const bf16x8 dv = *(const bf16x8*)(Cx + (r < 16 ? r : 0) * LDX + xc * 8);
          buf_st(dv, rdx, vxj(j), so);
          if (rok) {
            if constexpr (FAST) {   // g = dx where 0 < z < 6; sums of g and g*(x - mean), in pairs
              const u32x4_t du = __builtin_bit_cast(u32x4_t, dv), xu = __builtin_bit_cast(u32x4_t, xv[j]);
#pragma unroll
              for (int h2 = 0; h2 < 4; ++h2) {
                const pb_f2 x2 = pb_unpack(xu[h2]), d2 = pb_unpack(du[h2]);
                const pb_f2 z2 = __builtin_elementwise_fma(x2, xsc2[h2], xsh2[h2]);
                const pb_f2 g2 = {pb_relu6_open(z2.x) ? d2.x : 0.f, pb_relu6_open(z2.y) ? d2.y : 0.f};
                sg2[h2] += g2;
                sgx2[h2] = __builtin_elementwise_fma(g2, x2 - xmu2[h2], sgx2[h2]);
              }
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e)
                gred_acc((float)dv[e], (float)xv[j][e], xsc[e], xsh[e], xmu[e], 1.f, a.xact, sg[e], sgx[e]);
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
#pragma unroll
      for (int j = 0; j < JX; ++j) xv[j] = xn[j];
    }
    // ---- dW += dy^T . x_p over the tile's 32 rows -------------------------------------------
#pragma unroll
    for (int ct = 0; ct < NCO; ++ct) {
      const bf16_t* pd = Ds + (8 * g + q) * LDD + ct * 16 + 4 * p;
      const bf16x4 lo = pb_tr_read(pd), hi = pb_tr_read(pd + 4 * LDD);
      const bf16x8 fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int it = 0; it < NWT; ++it) {
        const bf16_t* px = Xs + (8 * g + q) * LDX + it * 16 + 4 * p;
        const bf16x4 l2 = pb_tr_read(px), h2 = pb_tr_read(px + 4 * LDX);
        const bf16x8 fb = {l2[0], l2[1], l2[2], l2[3], h2[0], h2[1], h2[2], h2[3]};
        accw[ct][it] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, accw[ct][it], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  // ---- end: dW (waves in order) and the BN_x sums (waves, then row groups, in order) -------
  float* red = (float*)(smem + (size_t)G::WS * 2);              // [NCO*16][NW]
  float* gbuf = red + NCO * 16 * NW;                            // [4][RGX][2][NW]
  __syncthreads();
  if constexpr (FAST) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sg[e] = sg2[e >> 1][e & 1];
      sgx[e] = sgx2[e >> 1][e & 1];
    }
  }
  if (xact) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gbuf[((wave * RGX + rx) * 2 + 0) * NW + xc * 8 + e] = sg[e];
      gbuf[((wave * RGX + rx) * 2 + 1) * NW + xc * 8 + e] = sgx[e];
    }
  }
#pragma unroll 1
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int ct = 0; ct < NCO; ++ct)
#pragma unroll
        for (int it = 0; it < NWT; ++it)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* d = red + (ct * 16 + 4 * g + r) * NW + it * 16 + li;
            *d = w == 0 ? accw[ct][it][r] : *d + accw[ct][it][r];
          }
    }
    __syncthreads();
  }
  float* pw = a.partw + (long)blockIdx.x * COUT * Cin;
  for (int i = tid; i < COUT * NW; i += 256) {
    const int co = i / NW, c = i - co * NW;
    pw[(long)co * Cin + n0 + c] = red[co * NW + c];
  }
  float* xp = xparts + (long)blockIdx.x * 2 * Cin;
  for (int i = tid; i < 2 * NW; i += 256) {
    const int k = i / NW, c = i - k * NW;
    float s = 0.f;
    for (int w = 0; w < 4; ++w)
      for (int r = 0; r < RGX; ++r) s += gbuf[((w * RGX + r) * 2 + k) * NW + c];
    xp[(long)k * Cin + n0 + c] = k ? s * a.xrstd[n0 + c] : s;
  }
}

// the group width of the gred form for (Cin, Cout); 0: not taken (ROD_PWB_GRED=0: never)
static int pw_bwd_gred_nw(int Cin, int Cout) {
  static const bool off = getenv("ROD_PWB_GRED") && atoi(getenv("ROD_PWB_GRED")) == 0;
  if (off || !(Cout == 16 || Cout == 24 || Cout == 32 || Cout == 64)) return 0;
  // Cout 64 at 48 columns spills under the 3-waves/SIMD bound (168 VGPRs); 32 columns fit (162)
  if (Cout == 64) return Cin % 32 == 0 ? 32 : 0;
  // 32-column groups wherever Cin allows (tools/pwgred_bench.py: 96->24 289 -> 256 us, 192->32
  // 139 -> 121 us against 48: no idle row group, 4 waves / SIMD), 48 for Cin = 144
  static const int force = getenv("ROD_PWB_GRED_NW") ? atoi(getenv("ROD_PWB_GRED_NW")) : 0;   // A/B switch
  if (force == 48 && Cin % 48 == 0) return 48;
  if (Cin % 32 == 0) return 32;
  if (Cin % 48 == 0) return 48;
  return 0;
}
static int pw_bwd_gred_rowblocks(long M, int Cin, int nw) {
  const long ntiles = cdivl(M, 32);
  const int groups = Cin / nw;
  const long want = std::max<long>(1, 768 / groups);   // ~3 resident blocks per CU over all groups
  return (int)std::max<long>(1, std::min<long>(cdivl(ntiles, 4), want));
}

struct PwBwdPlan {
  int kd, nci, nco, nxt, nx, wt, nblk;
  long chunk;
  size_t lds;
};

// the streaming kernel's shapes (expand convs without bias); ROD_PWB_STREAM=0 turns it off
static bool pw_bwd_stream_ok(int Cin, int Cout, bool bias) {
  static const bool off = getenv("ROD_PWB_STREAM") && atoi(getenv("ROD_PWB_STREAM")) == 0;
  // 32->192 stays on the block kernel: 248 VGPRs (2 waves / SIMD), measured slower (168 vs 152 us)
  return !off && !bias && ((Cin == 16 && Cout == 96) || (Cin == 24 && Cout == 144));
}
// blocks of the streaming launch: 3 per CU (the register budget of the 16->96 form), at most one
// 4-wave group per 4 tiles
static int pw_bwd_stream_blocks(long M) {
  const long ntiles = cdivl(M, 32);
  return (int)std::max<long>(1, std::min<long>(cdivl(ntiles, 4), 3L * 256));
}

static bool pw_bwd_ok(int Cin, int Cout) {
  if (Cin <= 0 || Cout <= 0 || Cin % 8 || Cout % 8 || Cin > 192 || Cout > 512) return false;
  const int nco = cdiv(Cout, 16), nci = cdiv(Cin + 1, 16);
  return nco * nci <= 64;
}

static PwBwdPlan pw_bwd_plan(long M, int Cin, int Cout, bool bias) {
  PwBwdPlan p;
  p.kd = cdiv(Cout, 32) * 32;
  p.nco = cdiv(Cout, 16);
  p.nci = cdiv(Cin + (bias ? 1 : 0), 16);
  p.nxt = cdiv(Cin, 16);
  p.nx = p.nxt <= 2 ? 2 : p.nxt <= 4 ? 4 : p.nxt <= 8 ? 8 : 12;
  const int per = cdiv(p.nco * p.nci, 4);
  p.wt = per <= 4 ? 4 : per <= 6 ? 6 : per <= 8 ? 8 : 16;
  p.lds = (size_t)Cout * PB_CF * 4 + (size_t)Cin * 2 * 4 +
          ((size_t)PB_BM * (p.kd + 8) + (size_t)PB_BM * (p.nci * 16 + 8) + (size_t)p.nxt * 16 * (p.kd + 8)) * 2;
  // two rounds of the 3 resident blocks per CU (measured: 768 / 1024 / 1280 / 1536 / 2048 /
  // 3072 blocks -> 3471 / 3722 / 3572 / 3326 / 3531 / 3519 us over tools/pwbwd_bench.py)
  const long steps = cdivl(M, PB_BM);
  p.nblk = (int)std::max<long>(1, std::min<long>(steps, 1536));
  p.chunk = cdivl(steps, p.nblk) * PB_BM;
  p.nblk = (int)cdivl(M, p.chunk);
  return p;
}

}  // namespace rod

using namespace rod;

extern "C" {

int rod_pw_bwd_supported(int Cin, int Cout, int dtype) { return dtype == ROD_BF16 && pw_bwd_ok(Cin, Cout) ? 1 : 0; }

size_t rod_pw_bwd_workspace(long M, int Cin, int Cout) {
  if (!pw_bwd_ok(Cin, Cout) || M <= 0) return 0;
  const PwBwdPlan p = pw_bwd_plan(M, Cin, Cout, true);
  const size_t blk = pw_bwd_stream_ok(Cin, Cout, false) ? (size_t)std::max(p.nblk, pw_bwd_stream_blocks(M)) : p.nblk;
  return blk * Cout * (Cin + 1) * sizeof(float) + 64;
}

int rod_pw_bwd_rc_supported(long M, int Cin, int Cout, int dtype) {
  return dtype == ROD_BF16 && M > 0 && pw_bwd_ok(Cin, Cout) && pw_bwd_stream_ok(Cin, Cout, false) ? 1 : 0;
}

static int pw_bwd_run(const void* dz, const void* y, const void* wt0, const float* mean, const float* rstd,
                      const float* gamma, const float* beta, int act, const float* coef, const void* x,
                      const float* xmean, const float* xrstd, const float* xgamma, const float* xbeta, int xact,
                      const void* wt1, void* dx, float* dw, float* db, void* workspace, long M, int Cin, int Cout,
                      int dtype, void* stream) {
  ROD_CHECK_ARG(dtype == ROD_BF16, "rod_pw_bwd: bf16 only");
  ROD_CHECK_ARG(M > 0 && pw_bwd_ok(Cin, Cout), "rod_pw_bwd: unsupported shape M=%ld Cin=%d Cout=%d", M, Cin, Cout);
  ROD_CHECK_ARG(dz && (y || wt0) && mean && rstd && coef && x && dw && workspace, "rod_pw_bwd: NULL argument");
  ROD_CHECK_ARG(!wt0 || (!db && rod_pw_bwd_rc_supported(M, Cin, Cout, dtype)),
                "rod_pw_bwd_rc: the recompute form takes the streaming shapes (16 -> 96, 24 -> 144) without bias");
  ROD_CHECK_ARG((((uintptr_t)wt0) & 15) == 0, "rod_pw_bwd_rc: wt0 must be 16-byte aligned");
  ROD_CHECK_ARG(!dx || wt1, "rod_pw_bwd: dx needs wt1");
  ROD_CHECK_ARG(!xmean || xrstd, "rod_pw_bwd: bad input prologue");
  ROD_CHECK_ARG(((((uintptr_t)dz) | ((uintptr_t)y) | ((uintptr_t)x) | ((uintptr_t)wt1) | ((uintptr_t)dx)) & 15) == 0,
                "rod_pw_bwd: tensors must be 16-byte aligned");
  const PwBwdPlan p = pw_bwd_plan(M, Cin, Cout, db != nullptr);
  ROD_CHECK_ARG(p.lds <= 160 * 1024, "rod_pw_bwd: LDS plan too large");
  hipStream_t s = ROD_STREAM(stream);
  float* partw = (float*)workspace;
  if (pw_bwd_stream_ok(Cin, Cout, db != nullptr)) {
    const int nblk = pw_bwd_stream_blocks(M);
    PwBwdArgs a{(const bf16_t*)dz, (const bf16_t*)y, (const bf16_t*)x, (const bf16_t*)wt1, (bf16_t*)dx, partw, nullptr,
                mean, rstd, gamma, beta, coef, xmean, xrstd, xgamma, xbeta, act, xact, M, 0, Cin, Cout, 0, 0, 0, 0,
                nullptr, (const bf16_t*)wt0};
    const long ntiles = cdivl(M, 32);
#define PBS0(CI, CO, PR, DXF, XLN, RCF)                                                                         \
  do {                                                                                                          \
    const size_t lds = PbsGeo<CI, CO>::lds(RCF);                                                                \
    (void)hipFuncSetAttribute((const void*)pw_bwd_stream_kernel<CI, CO, PR, DXF, false, XLN, RCF>,              \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                            \
    hipLaunchKernelGGL((pw_bwd_stream_kernel<CI, CO, PR, DXF, false, XLN, RCF>), dim3(nblk), dim3(256), lds, s, \
                       a, ntiles, nullptr);                                                                     \
  } while (0)
#define PBS1(CI, CO, PR, DXF, XLN)                  \
  do {                                              \
    if (wt0) PBS0(CI, CO, PR, DXF, XLN, true);      \
    else PBS0(CI, CO, PR, DXF, XLN, false);         \
  } while (0)
#define PBS(CI, CO, PR, DXF)                                      \
  do {                                                            \
    if (PR && xact == ROD_ACT_NONE) PBS1(CI, CO, PR, DXF, true);  \
    else PBS1(CI, CO, PR, DXF, false);                            \
  } while (0)
#define PBS2(CI, CO)                                        \
  if (Cin == CI) {                                          \
    if (xmean) {                                            \
      if (dx) PBS(CI, CO, true, true); else PBS(CI, CO, true, false);   \
    } else {                                                \
      if (dx) PBS(CI, CO, false, true); else PBS(CI, CO, false, false); \
    }                                                       \
  }
    PBS2(16, 96) else PBS2(24, 144)
#undef PBS2
#undef PBS
#undef PBS1
#undef PBS0
    slab_sum(partw, dw, nblk, (long)Cout * Cin, s);
    return check_launch("rod_pw_bwd");
  }
  float* partb = db ? partw + (size_t)p.nblk * Cout * Cin : nullptr;
  PwBwdArgs a{(const bf16_t*)dz, (const bf16_t*)y, (const bf16_t*)x, (const bf16_t*)wt1, (bf16_t*)dx, partw, partb,
              mean, rstd, gamma, beta, coef, xmean, xrstd, xgamma, xbeta, act, xact, M, p.chunk,
              Cin, Cout, p.kd, p.nci, p.nco, p.nxt};
#define PBL(NX_, WT_)                                                                                  \
  do {                                                                                                 \
    (void)hipFuncSetAttribute((const void*)pw_bwd_kernel<NX_, WT_>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                        (int)p.lds);                                                                   \
    hipLaunchKernelGGL((pw_bwd_kernel<NX_, WT_>), dim3(p.nblk), dim3(256), p.lds, s, a);               \
  } while (0)
#define PBW(NX_)                   \
  if (p.wt == 4) PBL(NX_, 4);      \
  else if (p.wt == 6) PBL(NX_, 6); \
  else if (p.wt == 8) PBL(NX_, 8); \
  else PBL(NX_, 16)
  if (p.nx == 2) PBW(2);
  else if (p.nx == 4) PBW(4);
  else if (p.nx == 8) PBW(8);
  else PBW(12);
#undef PBW
#undef PBL
  slab_sum(partw, dw, p.nblk, (long)Cout * Cin, s);
  if (db) slab_sum(partb, db, p.nblk, (long)Cout, s);
  return check_launch("rod_pw_bwd");
}

int rod_pw_bwd(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
               const float* beta, int act, const float* coef, const void* x, const float* xmean, const float* xrstd,
               const float* xgamma, const float* xbeta, int xact, const void* wt1, void* dx, float* dw, float* db,
               void* workspace, long M, int Cin, int Cout, int dtype, void* stream) {
  ROD_CHECK_ARG(y, "rod_pw_bwd: NULL y");
  return pw_bwd_run(dz, y, nullptr, mean, rstd, gamma, beta, act, coef, x, xmean, xrstd, xgamma, xbeta, xact, wt1, dx,
                    dw, db, workspace, M, Cin, Cout, dtype, stream);
}

int rod_pw_bwd_rc(const void* dz, const void* wt0, const float* mean, const float* rstd, const float* gamma,
                  const float* beta, int act, const float* coef, const void* x, const float* xmean, const float* xrstd,
                  const float* xgamma, const float* xbeta, int xact, const void* wt1, void* dx, float* dw,
                  void* workspace, long M, int Cin, int Cout, int dtype, void* stream) {
  ROD_CHECK_ARG(wt0, "rod_pw_bwd_rc: NULL wt0");
  return pw_bwd_run(dz, nullptr, wt0, mean, rstd, gamma, beta, act, coef, x, xmean, xrstd, xgamma, xbeta, xact, wt1,
                    dx, dw, nullptr, workspace, M, Cin, Cout, dtype, stream);
}


// expand shapes the gred entry takes (the streaming kernel with the input sums): 16 -> 96 only
// (168 VGPRs, 3 waves / SIMD); 24 -> 144 would need 268 (1 wave), and its input is usually also a
// residual source, whose gradient is a sum the sums could not be handed to anyway
static bool pw_bwd_xg_ok(int Cin, int Cout) { return Cin == 16 && Cout == 96 && pw_bwd_stream_ok(Cin, Cout, false); }

long rod_pw_bwd_gred_parts(long M, int Cin, int Cout, int dtype) {
  if (dtype == ROD_BF16 && M > 0 && pw_bwd_xg_ok(Cin, Cout)) return pw_bwd_stream_blocks(M);
  const int nw = dtype == ROD_BF16 && M > 0 ? pw_bwd_gred_nw(Cin, Cout) : 0;
  return nw ? pw_bwd_gred_rowblocks(M, Cin, nw) : 0;
}

size_t rod_pw_bwd_gred_workspace(long M, int Cin, int Cout) {
  if (M > 0 && pw_bwd_xg_ok(Cin, Cout)) return (size_t)pw_bwd_stream_blocks(M) * Cout * Cin * sizeof(float) + 64;
  const int nw = M > 0 ? pw_bwd_gred_nw(Cin, Cout) : 0;
  return nw ? (size_t)pw_bwd_gred_rowblocks(M, Cin, nw) * Cout * Cin * sizeof(float) + 64 : 0;
}

static int pw_bwd_gred_run(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                           const float* beta, int act, const float* coef, const void* x, const float* xmean,
                           const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1,
                           void* dx, void* dyp, float* dw, float* xparts, void* workspace, long M, int Cin, int Cout,
                           int dtype, void* stream, const void* wt0 = nullptr) {
  const bool sexp = dtype == ROD_BF16 && M > 0 && pw_bwd_xg_ok(Cin, Cout) && !dyp;
  const int nw = dtype == ROD_BF16 && M > 0 && !sexp ? pw_bwd_gred_nw(Cin, Cout) : 0;
  ROD_CHECK_ARG(nw || sexp, "rod_pw_bwd_gred: unsupported shape M=%ld Cin=%d Cout=%d dtype=%d", M, Cin, Cout,
                dtype);
  ROD_CHECK_ARG(!wt0 || sexp, "rod_pw_bwd_gred_rc: the recompute form takes the 16 -> 96 expand only");
  ROD_CHECK_ARG(dz && (y || wt0) && mean && rstd && coef && x && xmean && xrstd && dw && xparts && workspace,
                "rod_pw_bwd_gred: NULL argument");
  ROD_CHECK_ARG((((uintptr_t)wt0) & 15) == 0, "rod_pw_bwd_gred_rc: wt0 must be 16-byte aligned");
  ROD_CHECK_ARG((dx != nullptr) != (dyp != nullptr) && wt1,
                "rod_pw_bwd_gred: wt1 and exactly one of dx / dyp required (the sums are over dx)");
  ROD_CHECK_ARG(((((uintptr_t)dz) | ((uintptr_t)y) | ((uintptr_t)x) | ((uintptr_t)wt1) | ((uintptr_t)dx) |
                  ((uintptr_t)dyp)) & 15) == 0,
                "rod_pw_bwd_gred: tensors must be 16-byte aligned");
  ROD_CHECK_ARG(M * Cin * 2 < (1L << 31) && M * Cout * 2 < (1L << 31), "rod_pw_bwd_gred: tensor over 2 GiB");
  hipStream_t s = ROD_STREAM(stream);
  float* partw = (float*)workspace;
  if (sexp) {   // an expand shape: the streaming kernel with the input BatchNorm's sums
    const int nb = pw_bwd_stream_blocks(M);
    PwBwdArgs a{(const bf16_t*)dz, (const bf16_t*)y, (const bf16_t*)x, (const bf16_t*)wt1, (bf16_t*)dx, partw,
                nullptr, mean, rstd, gamma, beta, coef, xmean, xrstd, xgamma, xbeta, act, xact, M, 0, Cin, Cout, 0, 0,
                0, 0, nullptr, (const bf16_t*)wt0};
    const long nt = cdivl(M, 32);
#define PBX0(CI, CO, XLN, RCF)                                                                                 \
  do {                                                                                                         \
    const size_t lds = PbsGeo<CI, CO>::lds(RCF);                                                               \
    (void)hipFuncSetAttribute((const void*)pw_bwd_stream_kernel<CI, CO, true, true, true, XLN, RCF>,           \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                           \
    hipLaunchKernelGGL((pw_bwd_stream_kernel<CI, CO, true, true, true, XLN, RCF>), dim3(nb), dim3(256), lds, s, a, \
                       nt, xparts);                                                                            \
  } while (0)
#define PBX1(CI, CO, XLN)                      \
  do {                                         \
    if (wt0) PBX0(CI, CO, XLN, true);          \
    else PBX0(CI, CO, XLN, false);             \
  } while (0)
#define PBX(CI, CO)                                          \
  if (Cin == CI) {                                           \
    if (xact == ROD_ACT_NONE) PBX1(CI, CO, true);            \
    else PBX1(CI, CO, false);                                \
  }
    PBX(16, 96)
#undef PBX
#undef PBX1
#undef PBX0
    slab_sum(partw, dw, nb, (long)Cout * Cin, s);
    return check_launch("rod_pw_bwd_gred");
  }
  const int nblk = pw_bwd_gred_rowblocks(M, Cin, nw);
  PwBwdArgs a{(const bf16_t*)dz, (const bf16_t*)y, (const bf16_t*)x, (const bf16_t*)wt1, (bf16_t*)dx, partw, nullptr,
              mean, rstd, gamma, beta, coef, xmean, xrstd, xgamma, xbeta, act, xact, M, 0, Cin, Cout, 0, 0, 0, 0,
              (bf16_t*)dyp};
  const long ntiles = cdivl(M, 32);
  const dim3 grid(nblk, Cin / nw);
  // the inverted-residual block's case; at 48 columns the packed form measured slower (144->24:
  // 569 vs 433 us), so there the per-element form runs (ROD_PWB_GRED_FAST48=1: packed, A/B)
  static const bool fast48 = getenv("ROD_PWB_GRED_FAST48") && atoi(getenv("ROD_PWB_GRED_FAST48")) == 1;
  const bool fast = act == ROD_ACT_NONE && xact == ROD_ACT_RELU6 && (nw == 32 || fast48);
#define PBGD(CO, NW_, F, D)                                                                                     \
  do {                                                                                                          \
    const size_t lds = PbgGeo<CO, NW_>::lds();                                                                  \
    (void)hipFuncSetAttribute((const void*)pw_bwd_gred_kernel<CO, NW_, F, D>,                                   \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                            \
    hipLaunchKernelGGL((pw_bwd_gred_kernel<CO, NW_, F, D>), grid, dim3(256), lds, s, a, ntiles, xparts);        \
  } while (0)
#define PBG(CO, NW_, F)                  \
  do {                                   \
    if (dyp) PBGD(CO, NW_, F, true);     \
    else PBGD(CO, NW_, F, false);        \
  } while (0)
#define PBG1(CO, NW_)                        \
  if (fast) PBG(CO, NW_, true);              \
  else PBG(CO, NW_, false);
#define PBG2(CO)                                                                    \
  if (Cout == CO) {                                                                 \
    if (nw == 48 && CO != 64) { PBG1(CO, 48) }                                      \
    else { PBG1(CO, 32) }                                                           \
  }
  PBG2(16) else PBG2(24) else PBG2(32) else PBG2(64)
#undef PBG2
#undef PBG1
#undef PBG
#undef PBGD
  slab_sum(partw, dw, nblk, (long)Cout * Cin, s);
  return check_launch("rod_pw_bwd_gred");
}

int rod_pw_bwd_gred(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                    const float* beta, int act, const float* coef, const void* x, const float* xmean,
                    const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1,
                    void* dx, float* dw, float* xparts, void* workspace, long M, int Cin, int Cout, int dtype,
                    void* stream) {
  ROD_CHECK_ARG(dx, "rod_pw_bwd_gred: dx required");
  return pw_bwd_gred_run(dz, y, mean, rstd, gamma, beta, act, coef, x, xmean, xrstd, xgamma, xbeta, xact, wt1, dx,
                         nullptr, dw, xparts, workspace, M, Cin, Cout, dtype, stream);
}

int rod_pw_bwd_gred_dyp(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                        const float* beta, int act, const float* coef, const void* x, const float* xmean,
                        const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1,
                        void* dyp, float* dw, float* xparts, void* workspace, long M, int Cin, int Cout, int dtype,
                        void* stream) {
  ROD_CHECK_ARG(dyp, "rod_pw_bwd_gred_dyp: dyp required");
  return pw_bwd_gred_run(dz, y, mean, rstd, gamma, beta, act, coef, x, xmean, xrstd, xgamma, xbeta, xact, wt1,
                         nullptr, dyp, dw, xparts, workspace, M, Cin, Cout, dtype, stream);
}

int rod_pw_bwd_gred_rc(const void* dz, const void* wt0, const float* mean, const float* rstd, const float* gamma,
                       const float* beta, int act, const float* coef, const void* x, const float* xmean,
                       const float* xrstd, const float* xgamma, const float* xbeta, int xact, const void* wt1,
                       void* dx, float* dw, float* xparts, void* workspace, long M, int Cin, int Cout, int dtype,
                       void* stream) {
  ROD_CHECK_ARG(dx && wt0, "rod_pw_bwd_gred_rc: dx and wt0 required");
  return pw_bwd_gred_run(dz, nullptr, mean, rstd, gamma, beta, act, coef, x, xmean, xrstd, xgamma, xbeta, xact, wt1,
                         dx, nullptr, dw, xparts, workspace, M, Cin, Cout, dtype, stream, wt0);
}

}  // extern "C"
