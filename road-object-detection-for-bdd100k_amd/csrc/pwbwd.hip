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
    bn_bwd_k(a.coef[c], a.mean[c], a.rstd[c], a.coef[Cout + c], a.coef[2 * Cout + c], t[5 * Cout], t[6 * Cout]);
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
              o[j] = (bf16_t)bn_bwd_apply1(f[4][jj], gj, f[5][jj], f[6][jj], yj);   // fields 5, 6: k1, k0
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

struct PwBwdPlan {
  int kd, nci, nco, nxt, nx, wt, nblk;
  long chunk;
  size_t lds;
};

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
  return (size_t)p.nblk * Cout * (Cin + 1) * sizeof(float) + 64;
}

int rod_pw_bwd(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
               const float* beta, int act, const float* coef, const void* x, const float* xmean, const float* xrstd,
               const float* xgamma, const float* xbeta, int xact, const void* wt1, void* dx, float* dw, float* db,
               void* workspace, long M, int Cin, int Cout, int dtype, void* stream) {
  ROD_CHECK_ARG(dtype == ROD_BF16, "rod_pw_bwd: bf16 only");
  ROD_CHECK_ARG(M > 0 && pw_bwd_ok(Cin, Cout), "rod_pw_bwd: unsupported shape M=%ld Cin=%d Cout=%d", M, Cin, Cout);
  ROD_CHECK_ARG(dz && y && mean && rstd && coef && x && dw && workspace, "rod_pw_bwd: NULL argument");
  ROD_CHECK_ARG(!dx || wt1, "rod_pw_bwd: dx needs wt1");
  ROD_CHECK_ARG(!xmean || xrstd, "rod_pw_bwd: bad input prologue");
  ROD_CHECK_ARG(((((uintptr_t)dz) | ((uintptr_t)y) | ((uintptr_t)x) | ((uintptr_t)wt1) | ((uintptr_t)dx)) & 15) == 0,
                "rod_pw_bwd: tensors must be 16-byte aligned");
  const PwBwdPlan p = pw_bwd_plan(M, Cin, Cout, db != nullptr);
  ROD_CHECK_ARG(p.lds <= 160 * 1024, "rod_pw_bwd: LDS plan too large");
  hipStream_t s = ROD_STREAM(stream);
  float* partw = (float*)workspace;
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

}  // extern "C"
