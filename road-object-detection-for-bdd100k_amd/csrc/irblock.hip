// irblock.hip — the whole MobileNet-v2 inverted-residual block in one kernel (inference).
//
// Reference: expanded_conv (nets/backbone/mobilenet/conv_blocks.py:163-312): expand 1x1
// (+BatchNorm +ReLU6, 263-271) -> depthwise 3x3 stride s, TF-SAME (+BatchNorm +ReLU6,
// 238-247) -> project 1x1 (+BatchNorm, linear, 287-294) -> + input when s == 1 and
// Cin == Cout (302-311); eval-mode BatchNorm from the moving statistics (slim, is_training
// False: predict.py:106, evaluate.py:129).
//
// The expanded tensor (6x the block's input channels, the largest activations of the net)
// never touches HBM: a workgroup owns a TH x TW tile of output pixels, loads its input window
// (halo included) once into LDS, and walks the expanded channels in chunks of 32:
//   A. expand    E[e][p] = relu6(BN_e(x[p, :] . We[e, :]))     16x16x32 bf16 MFMA, K = Cin
//   B. depthwise D[e][q] = relu6(BN_d(sum_taps E[e][..] wd))   VALU, one output row per thread
//   C. project   acc[q, co] += D[., q]^T . Wp[co, e0..e0+31]    16x16x32 bf16 MFMA (A read
//                transposed from the channel-major D with ds_read_b64_tr_b16)
// and finally writes out[q, co] = BN_p(acc) (+ x[q, co]).  E and D are channel-major planes
// (the expand accumulators hold 4 consecutive pixels of one channel per lane, the depthwise
// walks rows of one channel).  The next chunk's weights and BatchNorm coefficients are
// fetched into registers while the current chunk computes and land in the other half of a
// double-buffered LDS parameter block, so no phase waits on an L2 round trip.
// HBM traffic per block: the input window and the output tile (plus L2-resident weights).
//
// Rounding (default): the expand / depthwise / project accumulators go through their BatchNorm
// (+ ReLU6) in fp32 and are rounded to bf16 once — the unfused chain rounds each conv output
// first, then the BatchNorm result again; skipping the first rounding is closer to the fp32
// reference and saves three packed instructions per pair of expanded values (the kernel is
// VALU-issue bound).  Exact mode (rod_ir_block_set_mode bit 1) follows the unfused librod eval
// path exactly — each conv output rounded to bf16, the BatchNorm prologue form
// act(fma(y, scale, offset)) rounded to bf16, the same MFMA k-step order for both GEMMs (32-deep
// steps in ascending k) and the depthwise taps in raster order — bit-identical to rod_conv_fwd
// -> rod_dw3x3_fwd -> rod_conv_fwd -> rod_bn_apply wherever those run without split-K
// (tests/test_gpu_irblock.py checks both modes).
#include "rod_common.h"

namespace rod {

constexpr int IR_CK = 32;  // expanded channels per chunk (one project k-step)
static int ir_persist_mode = 1;  // rod_ir_block_set_mode: 0 = one tile per workgroup only

template <int S> struct IrTile;
template <> struct IrTile<1> {
  static constexpr int TH = 8, TW = 16;
  static constexpr int IH = TH + 2, IW = TW + 2;          // 10 x 18
};
template <> struct IrTile<2> {
  static constexpr int TH = 8, TW = 8;
  static constexpr int IH = 2 * TH + 1, IW = 2 * TW + 2;  // 17 x 18 (one spare column: even rows)
};

struct IrArgs {
  const bf16_t* x;
  const bf16_t* we;   // [inner][Cin]
  const bf16_t* wp;   // [Cout][inner]
  const float* wd;    // [3][3][inner]
  BnPro be, bd, bp;   // eval BatchNorms
  bf16_t* y;
  int H, W, Cin, inner, Cout, Ho, Wo, pt, pl, residual;
};

typedef short ir_s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x4 ir_tr_read(const bf16_t* p) {
  ir_s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) ir_s16x4*)p);
  return __builtin_bit_cast(bf16x4, r);
}
typedef __bf16 ir_bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float relu6_bf16(float v, float sc, float sh) {
  return (float)(bf16_t)act_t<ROD_ACT_RELU6>(fmaf(v, sc, sh));
}
typedef float ir_f32x2 __attribute__((ext_vector_type(2)));
// two values of relu6_bf16((float)(bf16_t)a, sc, sh), packed as bf16x2 bits: the rounding pair
// and the BatchNorm fma pair each take one packed instruction (v_cvt_pk_bf16_f32, v_pk_fma_f32);
// per element the same operations, in the same order, as relu6_bf16
__device__ __forceinline__ unsigned relu6_pair(float a, float b, ir_f32x2 sc2, ir_f32x2 sh2) {
  const ir_bf16x2 r = ir_bf16x2{(bf16_t)a, (bf16_t)b};
  ir_f32x2 v = {(float)r[0], (float)r[1]};
  v = __builtin_elementwise_fma(v, sc2, sh2);
  const ir_bf16x2 o = ir_bf16x2{(bf16_t)act_t<ROD_ACT_RELU6>(v.x), (bf16_t)act_t<ROD_ACT_RELU6>(v.y)};
  return __builtin_bit_cast(unsigned, o);
}

// the single-rounding form (the default, EX = false): the BatchNorm fma on the fp32 accumulators
// themselves — no bf16 rounding of the conv / depthwise output before its BatchNorm, one rounding
// after the ReLU6 — three packed-pair instructions fewer per pair of expanded values
__device__ __forceinline__ unsigned relu6_pair_nr(float a, float b, ir_f32x2 sc2, ir_f32x2 sh2) {
  ir_f32x2 v = {a, b};
  v = __builtin_elementwise_fma(v, sc2, sh2);
  const ir_bf16x2 o = ir_bf16x2{(bf16_t)act_t<ROD_ACT_RELU6>(v.x), (bf16_t)act_t<ROD_ACT_RELU6>(v.y)};
  return __builtin_bit_cast(unsigned, o);
}
template <bool EX>
__device__ __forceinline__ unsigned relu6_pair_t(float a, float b, ir_f32x2 sc2, ir_f32x2 sh2) {
  if constexpr (EX) return relu6_pair(a, b, sc2, sh2);
  else return relu6_pair_nr(a, b, sc2, sh2);
}

// LDS layout (elements), all offsets multiples of 8 bf16 (16 bytes)
template <int S>
struct IrLayout {
  using Tl = IrTile<S>;
  static constexpr int PI = Tl::IH * Tl::IW;
  static constexpr int PIP = (PI + 15) / 16 * 16;
  static constexpr int PO = Tl::TH * Tl::TW;
  // E plane stride: an odd word count, chosen so the expand epilogue's b32 stores (16 channels
  // x 4 pixel groups per wave) meet at most 2 lanes per bank (PIP + 2: 4)
  static constexpr int LDE = PIP + 6;
  static constexpr int LDD = PO + 8;        // D plane stride (16-byte aligned rows)
  int KX, LDX, LDW, xs, we, wp, par, e, d, total;
  // nbuf parameter buffers: 2 (double-buffered chunk stream) or one per chunk (resident)
  __device__ __host__ IrLayout(int Cin, int Cout, int nbuf) {
    KX = (Cin + 31) / 32 * 32;
    LDX = KX + 8;
    LDW = IR_CK + 8;
    const int xs_in = PIP * LDX, xs_out = PO * (Cout + 8);
    xs = 0;
    const int xs_sz = xs_in > xs_out ? xs_in : xs_out;
    // one parameter buffer: We chunk [32][LDX], Wp chunk [Cout][LDW], then fp32 wd [9][32] and
    // (sc_e, sh_e, sc_d, sh_d) [4][32] (2 bf16 per float)
    we = 0;
    wp = IR_CK * LDX;
    par = wp + ((Cout + 15) / 16 * 16) * LDW;
    const int pbuf = par + 2 * (9 * IR_CK + 4 * IR_CK);
    e = xs_sz + nbuf * pbuf;
    d = e + IR_CK * LDE + 8;
    total = d + IR_CK * LDD;
    this->pbuf_ = pbuf;
    this->xs_sz_ = xs_sz;
  }
  int pbuf_, xs_sz_;
  __device__ __host__ int pbase(int b) const { return xs_sz_ + b * pbuf_; }
};

// XP == 0: one tile per workgroup, chunk parameters streamed through a double buffer.
// XP > 0 (persistent): every chunk's parameters resident in LDS, the workgroup walks tiles and
// holds the next tile's input window (XP 16-byte pieces per thread) in registers meanwhile.
template <int S, int NT, int XP, bool EX>
__global__ void __launch_bounds__(256) ir_block_fwd_kernel(IrArgs a, int ntiles) {
  constexpr bool PERSIST = XP > 0;
  using Tl = IrTile<S>;
  using Ly = IrLayout<S>;
  constexpr int TH = Tl::TH, TW = Tl::TW, IW = Tl::IW;
  constexpr int PI = Ly::PI, PIP = Ly::PIP, PO = Ly::PO, LDE = Ly::LDE, LDD = Ly::LDD;
  constexpr int MTE = (PIP / 16 + 3) / 4;                   // expand m-tiles per wave
  constexpr int MTP = PO / 64;                              // project m-tiles per wave
  static_assert(PO % 64 == 0 && TH == 8 && IR_CK == 32, "tile geometry");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* sm = (bf16_t*)smem_raw;
  const int Cin = a.Cin, Cout = a.Cout, inner = a.inner;
  const int nchunk = (inner + IR_CK - 1) / IR_CK;
  const Ly L(Cin, Cout, PERSIST ? nchunk : 2);
  const int KX = L.KX, LDX = L.LDX, LDW = L.LDW;
  bf16_t* Xs = sm;
  bf16_t* Es = sm + L.e;
  bf16_t* Dt = sm + L.d;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int ntx = (a.Wo + TW - 1) / TW, nty = (a.Ho + TH - 1) / TH;
  // tile t -> (image, tile row, tile column); one tile per block, or (PERSIST) a block walks
  // tiles t = blockIdx.x + k * gridDim.x with the next tile's input window in flight
  int t = PERSIST ? (int)blockIdx.x : (int)(blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z));
  int n = 0, ho0 = 0, wo0 = 0, hi0 = 0, wi0 = 0;
  auto set_tile = [&](int tt) {
    const int tx = tt % ntx, rest = tt / ntx;
    const int ty = rest % nty;
    n = rest / nty;
    ho0 = ty * TH;
    wo0 = tx * TW;
    hi0 = ho0 * S - a.pt;
    wi0 = wo0 * S - a.pl;
  };
  set_tile(t);

  // ---- chunk parameters: registers now, LDS buffer (c & 1) later ------------------------
  const int WE_CH = IR_CK * (KX / 8);                   // 16-byte pieces of the We chunk
  const int NTP = (Cout + 15) / 16;
  const int WP_CH = NTP * 16 * (IR_CK / 8);             // of the Wp chunk (rows padded to 16)
  constexpr int PF = PERSIST ? XP : 8;                  // pieces per thread (max)
  bf16x8 pf[PF];
  float pfs[2];                                         // wd / BN coefficient words
  auto fetch = [&](int e0) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int i = tid + u * 256;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[u][j] = (bf16_t)0.f;
      if (i < WE_CH) {
        const int r = i / (KX / 8), cc = i - r * (KX / 8);
        const int e = e0 + r;
        if (e < inner && cc * 8 < Cin) pf[u] = *(const bf16x8*)(a.we + (long)e * Cin + cc * 8);
      } else if (i < WE_CH + WP_CH) {
        const int k = i - WE_CH;
        const int co = k / (IR_CK / 8), cc = k - co * (IR_CK / 8);
        const int e = e0 + cc * 8;
        if (co < Cout && e < inner) pf[u] = *(const bf16x8*)(a.wp + (long)co * inner + e);
      }
    }
    // fp32 words: wd [9][32] (288) and the four coefficient rows [4][32] (128)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + u * 256;
      float v = 0.f;
      if (i < 9 * IR_CK) {
        const int k = i / IR_CK, c = i - k * IR_CK, e = e0 + c;
        if (e < inner) v = a.wd[k * inner + e];
      } else if (i < 13 * IR_CK) {
        const int k = (i - 9 * IR_CK) / IR_CK, c = (i - 9 * IR_CK) - k * IR_CK, e = e0 + c;
        if (e < inner) {
          float sc, sh;
          bn_pro_affine(k < 2 ? a.be : a.bd, e, sc, sh);
          v = (k & 1) ? sh : sc;
        }
      }
      pfs[u] = v;
    }
  };
  auto land = [&](int b) {
    bf16_t* P = sm + L.pbase(b);
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int i = tid + u * 256;
      if (i < WE_CH) {
        const int r = i / (KX / 8), cc = i - r * (KX / 8);
        *(bf16x8*)(P + r * LDX + cc * 8) = pf[u];
      } else if (i < WE_CH + WP_CH) {
        const int k = i - WE_CH;
        const int co = k / (IR_CK / 8), cc = k - co * (IR_CK / 8);
        *(bf16x8*)(P + IR_CK * LDX + co * LDW + cc * 8) = pf[u];
      }
    }
    float* F = (float*)(P + IR_CK * LDX + NTP * 16 * LDW);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + u * 256;
      if (i < 13 * IR_CK) F[i] = pfs[u];
    }
  };

  // persistent: chunk c's parameters straight into buffer c (once per launch)
  auto pdirect = [&](int c) {
    const int e0 = c * IR_CK;
    bf16_t* P = sm + L.pbase(c);
    for (int i = tid; i < WE_CH + WP_CH; i += 256) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16_t)0.f;
      if (i < WE_CH) {
        const int r = i / (KX / 8), cc = i - r * (KX / 8);
        const int e = e0 + r;
        if (e < inner && cc * 8 < Cin) v = *(const bf16x8*)(a.we + (long)e * Cin + cc * 8);
        *(bf16x8*)(P + r * LDX + cc * 8) = v;
      } else {
        const int k = i - WE_CH;
        const int co = k / (IR_CK / 8), cc = k - co * (IR_CK / 8);
        const int e = e0 + cc * 8;
        if (co < Cout && e < inner) v = *(const bf16x8*)(a.wp + (long)co * inner + e);
        *(bf16x8*)(P + IR_CK * LDX + co * LDW + cc * 8) = v;
      }
    }
    float* F = (float*)(P + IR_CK * LDX + NTP * 16 * LDW);
    for (int i = tid; i < 13 * IR_CK; i += 256) {
      float v = 0.f;
      if (i < 9 * IR_CK) {
        const int k = i / IR_CK, cl = i - k * IR_CK, e = e0 + cl;
        if (e < inner) v = a.wd[k * inner + e];
      } else {
        const int k = (i - 9 * IR_CK) / IR_CK, cl = (i - 9 * IR_CK) - k * IR_CK, e = e0 + cl;
        if (e < inner) {
          float sc, sh;
          bn_pro_affine(k < 2 ? a.be : a.bd, e, sc, sh);
          v = (k & 1) ? sh : sc;
        }
      }
      F[i] = v;
    }
  };
  // non-persistent: the window straight into Xs
  auto xdirect = [&]() {
    const bf16_t* xb = a.x + (long)n * a.H * a.W * Cin;
    for (int i = tid; i < PIP * (KX / 8); i += 256) {
      const int p = i / (KX / 8), cc = i - p * (KX / 8);
      const int r = p / IW, c = p - r * IW;
      const int hi = hi0 + r, wi = wi0 + c;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16_t)0.f;
      if (p < PI && cc * 8 < Cin && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W)
        v = *(const bf16x8*)(xb + ((long)hi * a.W + wi) * Cin + cc * 8);
      *(bf16x8*)(Xs + p * LDX + cc * 8) = v;
    }
  };
  // ---- input window of tile tt: 16-byte pieces (zero outside the image and past Cin) ------
  // the persistent variants have KX / 8 fixed by XP (ir_persist_pieces: 3 or 5 pieces <=> 4, 6
  // pieces <=> 8), so the piece -> (pixel, chunk) split is a shift
  constexpr int XCHC = XP == 6 ? 8 : 4;
  const int XCH = PERSIST ? XCHC : KX / 8;
  auto xfetch = [&](int tt) {   // -> pf (persistent prefetch); the host checks PIP*XCH <= XP*256
    const int tx = tt % ntx, rest = tt / ntx;
    const int nn = rest / nty, h0 = (rest % nty) * TH * S - a.pt, w0 = tx * TW * S - a.pl;
    const bf16_t* xb = a.x + (long)nn * a.H * a.W * Cin;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int i = tid + u * 256;
#pragma unroll
      for (int j = 0; j < 8; ++j) pf[u][j] = (bf16_t)0.f;
      if (i < PIP * XCH) {
        const int p = i / XCH, cc = i - p * XCH;
        const int r = p / IW, c = p - r * IW;
        const int hi = h0 + r, wi = w0 + c;
        if (p < PI && cc * 8 < Cin && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W)
          pf[u] = *(const bf16x8*)(xb + ((long)hi * a.W + wi) * Cin + cc * 8);
      }
    }
  };
  auto xland = [&]() {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int i = tid + u * 256;
      if (i < PIP * XCH) {
        const int p = i / XCH, cc = i - p * XCH;
        *(bf16x8*)(Xs + p * LDX + cc * 8) = pf[u];
      }
    }
  };
  // which of this lane's expand-output pixels lie inside the image (TF-SAME zero padding)
  unsigned inside = 0;
  auto set_inside = [&]() {
    // interior tiles (the window inside the image: all but the border tiles) in one
    // wave-uniform test
    if (hi0 >= 0 && hi0 + Tl::IH <= a.H && wi0 >= 0 && wi0 + IW <= a.W) {
      inside = 0xFFFFFFFFu;
#pragma unroll
      for (int i = 0; i < MTE; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if ((wave + 4 * i) * 16 + 4 * g + r >= PI) inside &= ~(1u << (i * 4 + r));
      return;
    }
    inside = 0;
#pragma unroll
    for (int i = 0; i < MTE; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = (wave + 4 * i) * 16 + 4 * g + r;
        const int pr = p / IW, pc = p - pr * IW;
        const int hi = hi0 + pr, wi = wi0 + pc;
        if (p < PI && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W) inside |= 1u << (i * 4 + r);
      }
  };
  if constexpr (PERSIST) {
    for (int c = 0; c < nchunk; ++c) pdirect(c);
    xfetch(t);
    xland();
  } else {
    fetch(0);
    land(0);
    xdirect();
  }
  set_inside();
  for (;;) {
  const int t_next = t + (int)gridDim.x;
  if (PERSIST && t_next < ntiles) xfetch(t_next);     // next window in flight under this tile
  f32x4 accp[MTP][NT];
#pragma unroll
  for (int i = 0; i < MTP; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) accp[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c < nchunk; ++c) {
    __syncthreads();  // parameters of chunk c landed; previous chunk's readers of Es / Dt done
    const bf16_t* P = sm + L.pbase(PERSIST ? c : (c & 1));
    const float* F = (const float*)(P + IR_CK * LDX + NTP * 16 * LDW);
    if (!PERSIST && c + 1 < nchunk) fetch((c + 1) * IR_CK);   // in flight under this chunk's work
    // ---- A. expand chunk -> Es (channel-major) ------------------------------------------------
    {
      f32x4 acc[MTE][2];
#pragma unroll
      for (int i = 0; i < MTE; ++i)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < KX; k0 += 32) {
        bf16x8 fb[2];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) fb[nt] = *(const bf16x8*)(P + (nt * 16 + li) * LDX + k0 + 8 * g);
#pragma unroll
        for (int i = 0; i < MTE; ++i) {
          const int mt = wave + 4 * i;
          if (mt * 16 >= PIP) continue;
          const bf16x8 fa = *(const bf16x8*)(Xs + (mt * 16 + li) * LDX + k0 + 8 * g);
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[nt], acc[i][nt], 0, 0, 0);
        }
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int e = nt * 16 + li;
        const float sc = F[9 * IR_CK + e], sh = F[10 * IR_CK + e];   // zero past inner
        const ir_f32x2 sc2 = {sc, sc}, sh2 = {sh, sh};
        const unsigned emask = c * IR_CK + e < inner ? 0xFFFFFFFFu : 0u;
#pragma unroll
        for (int i = 0; i < MTE; ++i) {
          const int mt = wave + 4 * i;
          if (mt * 16 >= PIP) continue;
          // conv output rounded (rod_conv_fwd), then the depthwise's BatchNorm + ReLU6
          // prologue (rounded); padding pixels and channels past inner are 0 (masked bits:
          // bf16 +0, as the unfused chain's zero padding)
          const unsigned in4 = (inside >> (i * 4)) & 15u;
          unsigned o[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            unsigned m = emask;
            if (in4 != 15u)
              m &= (((in4 >> (2 * h)) & 1u) ? 0x0000FFFFu : 0u) | (((in4 >> (2 * h + 1)) & 1u) ? 0xFFFF0000u : 0u);
            o[h] = relu6_pair_t<EX>(acc[i][nt][2 * h], acc[i][nt][2 * h + 1], sc2, sh2) & m;
          }
          unsigned* dst = (unsigned*)(Es + e * LDE + mt * 16 + 4 * g);
          dst[0] = o[0];
          dst[1] = o[1];
        }
      }
    }
    __syncthreads();
    // ---- B. depthwise: thread = (channel, output row), TW outputs -> Dt (channel-major) ---------
    {
      const int ch = tid & 31, oy = tid >> 5;
      const float* wdc = F + ch;
      float w[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) w[k] = wdc[k * IR_CK];
      const float dsc = F[11 * IR_CK + ch], dsh = F[12 * IR_CK + ch];
      const ir_f32x2 dsc2 = {dsc, dsc}, dsh2 = {dsh, dsh};
      const unsigned emask = c * IR_CK + ch < inner ? 0xFFFFFFFFu : 0u;
      // output pairs (2p, 2p + 1) accumulate as one packed fma per tap (v_pk_fma_f32)
      ir_f32x2 acc[TW / 2];
#pragma unroll
      for (int p = 0; p < TW / 2; ++p) acc[p] = ir_f32x2{0.f, 0.f};
      const bf16_t* ep = Es + ch * LDE;
      // taps in raster order (i, j): acc = fma(E, w, acc) per output, as rod_dw3x3_fwd
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        float rowv[IW];
        const bf16_t* rp = ep + (oy * S + i) * IW;
#pragma unroll
        for (int q = 0; q < IW / 2; ++q) {
          const ir_bf16x2 v = *(const ir_bf16x2*)(rp + 2 * q);
          rowv[2 * q] = (float)v[0];
          rowv[2 * q + 1] = (float)v[1];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const ir_f32x2 w2 = {w[i * 3 + j], w[i * 3 + j]};
#pragma unroll
          for (int p = 0; p < TW / 2; ++p) {
            const ir_f32x2 v = {rowv[(2 * p) * S + j], rowv[(2 * p + 1) * S + j]};
            acc[p] = __builtin_elementwise_fma(v, w2, acc[p]);
          }
        }
      }
      unsigned o[TW / 2];
#pragma unroll
      for (int p = 0; p < TW / 2; ++p) o[p] = relu6_pair_t<EX>(acc[p].x, acc[p].y, dsc2, dsh2) & emask;
#pragma unroll
      for (int h = 0; h < TW / 8; ++h)
        *(uint4*)(Dt + ch * LDD + oy * TW + 8 * h) = uint4{o[4 * h], o[4 * h + 1], o[4 * h + 2], o[4 * h + 3]};
    }
    __syncthreads();
    // ---- C. project: acc[q, co] += D^T[q, 32 chunk channels] . Wp[co, chunk] -------------------
    {
      const int q4 = li >> 2, p4 = li & 3;
#pragma unroll
      for (int i = 0; i < MTP; ++i) {
        const int mt = wave + 4 * i;
        const bf16_t* pd = Dt + (8 * g + q4) * LDD + mt * 16 + 4 * p4;
        const bf16x4 lo = ir_tr_read(pd), hi = ir_tr_read(pd + 4 * LDD);
        const bf16x8 fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          if (nt >= NTP) continue;
          const bf16x8 fb = *(const bf16x8*)(P + IR_CK * LDX + (nt * 16 + li) * LDW + 8 * g);
          accp[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, accp[i][nt], 0, 0, 0);
        }
      }
    }
    if (!PERSIST && c + 1 < nchunk) land((c + 1) & 1);
  }
  // ---- epilogue: BN_p (+ residual) -> staging -> 16-byte row segments ------------------------
  float out[MTP][NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    if (nt >= NTP) continue;
    const int co = nt * 16 + li;
    float sc = 0.f, sh = 0.f;
    if (co < Cout) bn_pro_affine(a.bp, co, sc, sh);
#pragma unroll
    for (int i = 0; i < MTP; ++i) {
      const int mt = wave + 4 * i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = mt * 16 + 4 * g + r;
        // linear BN of the project output (EX: rounded to bf16 first, as the unfused chain)
        float z = fmaf(EX ? (float)(bf16_t)accp[i][nt][r] : accp[i][nt][r], sc, sh);
        if (a.residual && co < Cout) {
          const int oy = q / TW, ox = q - oy * TW;   // S == 1: the input pixel under q
          z = z + (float)Xs[((oy + 1) * IW + ox + 1) * LDX + co];
        }
        out[i][nt][r] = z;
      }
    }
  }
  __syncthreads();  // Xs (residual source) consumed: reuse it as the output stage
  const int LDO = Cout + 8;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    if (nt >= NTP) continue;
    const int co = nt * 16 + li;
    if (co >= Cout) continue;
#pragma unroll
    for (int i = 0; i < MTP; ++i) {
      const int mt = wave + 4 * i;
#pragma unroll
      for (int r = 0; r < 4; ++r) Xs[(mt * 16 + 4 * g + r) * LDO + co] = (bf16_t)out[i][nt][r];
    }
  }
  __syncthreads();
  const int OCH = Cout / 8;
  bf16_t* yn = a.y + (long)n * a.Ho * a.Wo * Cout;
  for (int i = tid; i < PO * OCH; i += 256) {
    const int q = i / OCH, cc = i - q * OCH;
    const int ho = ho0 + q / TW, wo = wo0 + q % TW;
    if (ho < a.Ho && wo < a.Wo)
      *(bf16x8*)(yn + ((long)ho * a.Wo + wo) * Cout + cc * 8) = *(const bf16x8*)(Xs + q * LDO + cc * 8);
  }
  if (!PERSIST || t_next >= ntiles) break;
  __syncthreads();   // the output stage (Xs) has been read: the next window lands there
  xland();
  t = t_next;
  set_tile(t);
  set_inside();
  }
}

template <int S>
static size_t ir_lds(int Cin, int Cout, int nbuf) {
  IrLayout<S> L(Cin, Cout, nbuf);
  return (size_t)L.total * sizeof(bf16_t);
}

static bool ir_ok(int Cin, int inner, int Cout, int S, int residual) {
  if (Cin <= 0 || inner <= 0 || Cout <= 0 || Cin % 8 || Cout % 8 || inner % 8) return false;
  if (residual && (S != 1 || Cin != Cout)) return false;
  // the chunk parameters must fit the per-thread prefetch (8 x 16 bytes x 256 threads)
  const int KX = (Cin + 31) / 32 * 32;
  if (IR_CK * (KX / 8) + (Cout + 15) / 16 * 16 * (IR_CK / 8) > 8 * 256) return false;
  if (S == 1) return Cin <= 160 && Cout <= 160 && ir_lds<1>(Cin, Cout, 2) <= 160 * 1024;
  if (S == 2) return Cin <= 96 && Cout <= 320 && ir_lds<2>(Cin, Cout, 2) <= 160 * 1024;
  return false;
}

// persistent variant: prefetch pieces per thread for the input window (0 = not eligible)
static int ir_persist_pieces(int Cin, int inner, int Cout, int S) {
  const int KX = (Cin + 31) / 32 * 32;
  const int pip = S == 1 ? IrLayout<1>::PIP : IrLayout<2>::PIP;
  const int pieces = cdiv(pip * (KX / 8), 256);
  const int nchunk = cdiv(inner, IR_CK);
  const size_t lds = S == 1 ? ir_lds<1>(Cin, Cout, nchunk) : ir_lds<2>(Cin, Cout, nchunk);
  if (lds > 160 * 1024) return 0;
  if (S == 1) return pieces <= 3 ? 3 : pieces <= 6 ? 6 : 0;
  return pieces <= 5 ? 5 : 0;
}

static int ir_num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

template <int S, int NT, int XP, bool EX>
static void ir_launch(const IrArgs& a, int N, hipStream_t s) {
  using Tl = IrTile<S>;
  const int nchunk = cdiv(a.inner, IR_CK);
  const size_t lds = ir_lds<S>(a.Cin, a.Cout, XP ? nchunk : 2);
  const void* fn = (const void*)ir_block_fwd_kernel<S, NT, XP, EX>;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int ntx = cdiv(a.Wo, Tl::TW), nty = cdiv(a.Ho, Tl::TH);
  const int ntiles = ntx * nty * N;
  if (XP) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds) != hipSuccess || per_cu <= 0) per_cu = 1;
    const int grid = std::min(ntiles, per_cu * ir_num_cus());
    hipLaunchKernelGGL((ir_block_fwd_kernel<S, NT, XP, EX>), dim3(grid), dim3(256), lds, s, a, ntiles);
  } else {
    dim3 grid(ntx, nty, N);
    hipLaunchKernelGGL((ir_block_fwd_kernel<S, NT, XP, EX>), grid, dim3(256), lds, s, a, ntiles);
  }
}

template <int S, int NT, bool EX>
static void ir_launch_xp2(const IrArgs& a, int N, hipStream_t s) {
  const int xp = (ir_persist_mode & 1) ? ir_persist_pieces(a.Cin, a.inner, a.Cout, S) : 0;
  if constexpr (S == 1) {
    if (xp == 3) return ir_launch<S, NT, 3, EX>(a, N, s);
    if (xp == 6) return ir_launch<S, NT, 6, EX>(a, N, s);
  } else {
    if (xp == 5) return ir_launch<S, NT, 5, EX>(a, N, s);
  }
  ir_launch<S, NT, 0, EX>(a, N, s);
}
template <int S, int NT>
static void ir_launch_xp(const IrArgs& a, int N, hipStream_t s) {
  if (ir_persist_mode & 2) ir_launch_xp2<S, NT, true>(a, N, s);
  else ir_launch_xp2<S, NT, false>(a, N, s);
}

}  // namespace rod

using namespace rod;

extern "C" {

// bit 0 (default set): persistent resident-parameter variant where it fits (clear: never, A/B
// timing); bit 1: the exact-rounding form, bit-identical to the unfused librod eval chain (clear,
// the default: one rounding per expanded value, tests/test_gpu_irblock.py holds it to the oracle)
int rod_ir_block_set_mode(int mode) {
  const int old = ir_persist_mode;
  ir_persist_mode = mode & 3;
  return old;
}

int rod_ir_block_supported(int Cin, int inner, int Cout, int stride, int residual, int dtype) {
  return dtype == ROD_BF16 && ir_ok(Cin, inner, Cout, stride, residual) ? 1 : 0;
}

int rod_ir_block_persistent(int Cin, int inner, int Cout, int stride, int residual, int dtype) {
  return rod_ir_block_supported(Cin, inner, Cout, stride, residual, dtype) &&
                 ir_persist_pieces(Cin, inner, Cout, stride) > 0
             ? 1
             : 0;
}

int rod_ir_block_fwd(const void* x, const void* we, const float* e_mean, const float* e_rstd, const float* e_gamma,
                     const float* e_beta, const float* wd, const float* d_mean, const float* d_rstd,
                     const float* d_gamma, const float* d_beta, const void* wp, const float* p_mean,
                     const float* p_rstd, const float* p_gamma, const float* p_beta, int residual, void* y, int N,
                     int H, int W, int Cin, int inner, int Cout, int stride, int dtype, void* stream) {
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0, "rod_ir_block_fwd: bad shape");
  ROD_CHECK_ARG(dtype == ROD_BF16 && ir_ok(Cin, inner, Cout, stride, residual),
                "rod_ir_block_fwd: unsupported block Cin=%d inner=%d Cout=%d stride=%d residual=%d", Cin, inner, Cout,
                stride, residual);
  ROD_CHECK_ARG(x && we && wd && wp && y && e_mean && e_rstd && d_mean && d_rstd && p_mean && p_rstd,
                "rod_ir_block_fwd: NULL argument");
  ROD_CHECK_ARG(((((uintptr_t)x) | ((uintptr_t)we) | ((uintptr_t)wp) | ((uintptr_t)y)) & 15) == 0,
                "rod_ir_block_fwd: tensors must be 16-byte aligned");
  const int Ho = (H + stride - 1) / stride, Wo = (W + stride - 1) / stride;
  const int pth = std::max((Ho - 1) * stride + 3 - H, 0), ptw = std::max((Wo - 1) * stride + 3 - W, 0);
  IrArgs a{(const bf16_t*)x, (const bf16_t*)we, (const bf16_t*)wp, wd,
           BnPro{e_mean, e_rstd, e_gamma, e_beta, ROD_ACT_RELU6}, BnPro{d_mean, d_rstd, d_gamma, d_beta, ROD_ACT_RELU6},
           BnPro{p_mean, p_rstd, p_gamma, p_beta, ROD_ACT_NONE}, (bf16_t*)y, H, W, Cin, inner, Cout, Ho, Wo, pth / 2,
           ptw / 2, residual};
  hipStream_t s = ROD_STREAM(stream);
  const int ntp = (Cout + 15) / 16;
  if (stride == 1) {
    if (ntp <= 2) ir_launch_xp<1, 2>(a, N, s);
    else if (ntp <= 6) ir_launch_xp<1, 6>(a, N, s);
    else ir_launch_xp<1, 10>(a, N, s);
  } else {
    if (ntp <= 2) ir_launch_xp<2, 2>(a, N, s);
    else if (ntp <= 6) ir_launch_xp<2, 6>(a, N, s);
    else if (ntp <= 10) ir_launch_xp<2, 10>(a, N, s);
    else ir_launch_xp<2, 20>(a, N, s);
  }
  return check_launch("rod_ir_block_fwd");
}

}  // extern "C"
