// gemm.hip — dense convolutions as MFMA implicit GEMMs on gfx950.
//
//   rod_conv_fwd   : y[m, co] = sum_k A[m, k] * wt[co, k] (+ bias)          ("NT": k contiguous)
//   rod_conv_wgrad : dw[co, k] = sum_m dy[m, co] * A[m, k]                  ("TN": reduction over rows)
//
// A is either the activation rows (1x1 conv) or the 3x3 / stride-1 / TF-SAME im2col of x,
// gathered on the fly (no im2col buffer ever touches HBM).  bf16 storage uses
// v_mfma_f32_16x16x32_bf16; fp32 storage uses the exact-f32 v_mfma_f32_16x16x4_f32 (no
// reduced-precision path exists on gfx950), so fp32 parity runs are genuine fp32.
//
// Fragment maps (cdna_hip_programming.md §3): for 16x16x32 bf16 lane l holds
// A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], j=0..7; C/D col = l&15, row = 4(l>>4)+r.
// The f32 16x16x4 form is issued 8 times per 32-deep k-step with lane l contributing
// k = 8(l>>4)+j in issue j, so both dtypes read the same 8-element k-runs from LDS.
#include "rod_common.h"

namespace rod {

constexpr int BK = 32;

template <typename T> struct LdsPad;                       // row padding (elements)
template <> struct LdsPad<bf16_t> { static constexpr int v = 8; };   // 80-byte rows
template <> struct LdsPad<float> { static constexpr int v = 4; };    // 144-byte rows

// ---- 8-element chunk of T held in registers ------------------------------------
template <typename T> struct Chunk8;
// `ok`: the chunk holds raw loaded data that still needs the BatchNorm prologue (set by
// load_vec, cleared by zero()); the prologue runs when the chunk is stored to LDS, so the
// register prefetch of the next k step is not waited on at issue time.
template <> struct Chunk8<bf16_t> {
  bf16x8 v;
  bool ok;
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16_t)0.f;
    ok = false;
  }
  __device__ __forceinline__ void load_vec(const bf16_t* p) {
    v = *(const bf16x8*)p;
    ok = true;
  }
  __device__ __forceinline__ void set(int j, bf16_t x) { v[j] = x; }
  __device__ __forceinline__ void store_lds(bf16_t* p) const { *(bf16x8*)p = v; }
  // BatchNorm-apply prologue on channels c..c+7 (c % 8 == 0; LDS table of (scale, offset))
  template <int ACT>
  __device__ __forceinline__ void pro_t(const float* pt, int c) {
    const f32x4* q = (const f32x4*)(pt + 2 * c);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const f32x4 t = q[h];
      v[2 * h] = (bf16_t)act_t<ACT>(fmaf((float)v[2 * h], t[0], t[1]));
      v[2 * h + 1] = (bf16_t)act_t<ACT>(fmaf((float)v[2 * h + 1], t[2], t[3]));
    }
  }
  __device__ __forceinline__ void pro(const float* pt, int c, int act) {
    if (act == ROD_ACT_RELU6) pro_t<ROD_ACT_RELU6>(pt, c);
    else if (act == ROD_ACT_LEAKY) pro_t<ROD_ACT_LEAKY>(pt, c);
    else if (act == ROD_ACT_RELU) pro_t<ROD_ACT_RELU>(pt, c);
    else pro_t<ROD_ACT_NONE>(pt, c);
  }
};
template <> struct Chunk8<float> {
  f32x4 a, b;
  bool ok;
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = b[j] = 0.f;
    ok = false;
  }
  __device__ __forceinline__ void load_vec(const float* p) {
    a = *(const f32x4*)p;
    b = *(const f32x4*)(p + 4);
    ok = true;
  }
  __device__ __forceinline__ void set(int j, float x) {
    if (j < 4) a[j] = x; else b[j - 4] = x;
  }
  __device__ __forceinline__ void store_lds(float* p) const {
    *(f32x4*)p = a;
    *(f32x4*)(p + 4) = b;
  }
  template <int ACT>
  __device__ __forceinline__ void pro_t(const float* pt, int c) {
    const f32x4* q = (const f32x4*)(pt + 2 * c);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 t = q[h], u = q[h + 2];
      a[2 * h] = act_t<ACT>(fmaf(a[2 * h], t[0], t[1]));
      a[2 * h + 1] = act_t<ACT>(fmaf(a[2 * h + 1], t[2], t[3]));
      b[2 * h] = act_t<ACT>(fmaf(b[2 * h], u[0], u[1]));
      b[2 * h + 1] = act_t<ACT>(fmaf(b[2 * h + 1], u[2], u[3]));
    }
  }
  __device__ __forceinline__ void pro(const float* pt, int c, int act) {
    if (act == ROD_ACT_RELU6) pro_t<ROD_ACT_RELU6>(pt, c);
    else if (act == ROD_ACT_LEAKY) pro_t<ROD_ACT_LEAKY>(pt, c);
    else if (act == ROD_ACT_RELU) pro_t<ROD_ACT_RELU>(pt, c);
    else pro_t<ROD_ACT_NONE>(pt, c);
  }
};

// ---- A-row source: one output pixel of the conv (fixed for the whole K loop) --------
template <typename T, int KS, int CIN = 0>  // CIN > 0: Cin known at compile time (stem: 3)
struct RowSrc {
  const T* base;  // KS==1: &x[m*ldx]; KS==3: &x[pixel (n,0,0)]
  int y, x;       // KS==3 only
  bool valid;
  __device__ __forceinline__ void init(const T* X, long m, long M, int H, int W, int ldx) {
    valid = m < M;
    if (!valid) { base = X; y = x = 0; return; }
    if constexpr (KS == 1) {
      base = X + m * ldx;
    } else {
      const int xx = (int)(m % W);
      const long t = m / W;
      y = (int)(t % H);
      x = xx;
      const long n = t / H;
      base = X + n * (long)H * W * ldx;
    }
  }
  // load A[m, k..k+7]; K = KS*KS*Cin.  PRO: x holds the pre-BatchNorm tensor and every
  // in-bounds element goes through the BatchNorm-apply prologue (table pt = [Cin][2] of
  // (scale, offset) in LDS); padding taps and k >= K stay 0.
  template <bool VEC, bool PRO = false>
  __device__ __forceinline__ void load(Chunk8<T>& c, int k, int K, int Cin, int H, int W, int ldx,
                                       const float* pt = nullptr, int act = 0) const {
    if (!valid || k >= K) { c.zero(); return; }
    if constexpr (KS == 1) {
      if (VEC && k + 8 <= K) {
        c.load_vec(base + k);  // prologue deferred to pro_pending()
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          T v = (k + j < K) ? base[k + j] : (T)0.f;
          if constexpr (PRO) {
            if (k + j < K) v = from_f32<T>(act_fwd(fmaf(to_f32(v), pt[2 * (k + j)], pt[2 * (k + j) + 1]), act));
          }
          c.set(j, v);
        }
        c.ok = false;
      }
    } else {
      if (VEC) {  // Cin % 8 == 0 : the chunk lies inside one tap
        const int tap = k / Cin, ci = k - tap * Cin;
        const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) c.load_vec(base + ((long)yy * W + xx) * ldx + ci);
        else c.zero();  // prologue deferred to pro_pending()
      } else if constexpr (CIN == 0) {
        // Cin % 8 != 0 (the heads' last 3x3 convs: 4 or num_classes x anchors channels): one
        // division per chunk, then G-element sub-loads (G = the widest power of two dividing
        // Cin and ldx, so a sub-load never crosses a tap)
        const unsigned long al = (unsigned long)base;
        if (Cin % 4 == 0 && ldx % 4 == 0 && al % (4 * sizeof(T)) == 0) gather<4, PRO>(c, k, K, Cin, H, W, ldx, pt, act);
        else if (Cin % 2 == 0 && ldx % 2 == 0 && al % (2 * sizeof(T)) == 0)
          gather<2, PRO>(c, k, K, Cin, H, W, ldx, pt, act);
        else gather<1, PRO>(c, k, K, Cin, H, W, ldx, pt, act);
      } else {
        const int cin = CIN > 0 ? CIN : Cin;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int kk = k + j;
          T v = (T)0.f;
          if (kk < K) {
            const int tap = kk / cin, ci = kk - tap * cin;
            const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
            if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
              v = base[((long)yy * W + xx) * ldx + ci];
              if constexpr (PRO) v = from_f32<T>(act_fwd(fmaf(to_f32(v), pt[2 * ci], pt[2 * ci + 1]), act));
            }
          }
          c.set(j, v);
        }
        c.ok = false;
      }
    }
  }
  // Sequential im2col walk (KS == 3, Cin % 8 == 0) for a k loop that visits k, k + step, ...:
  // the chunk's tap / channel and the tap's pixel pointer are carried from step to step, so a
  // step costs a pointer add instead of a division and a 64-bit address rebuild per chunk
  int wtap, wci;
  const T* wp;
  bool wok;
  __device__ __forceinline__ void walk_set(int H, int W, int ldx) {
    const int yy = y + wtap / 3 - 1, xx = x + wtap % 3 - 1;
    wok = valid && wtap < 9 && yy >= 0 && yy < H && xx >= 0 && xx < W;
    wp = base + ((long)yy * W + xx) * ldx;
  }
  __device__ __forceinline__ void walk_init(int k, int Cin, int H, int W, int ldx) {
    wtap = k / Cin;
    wci = k - wtap * Cin;
    walk_set(H, W, ldx);
  }
  __device__ __forceinline__ void walk_next(int step, int Cin, int H, int W, int ldx) {
    wci += step;
    if (wci >= Cin) {
      do {
        wci -= Cin;
        ++wtap;
      } while (wci >= Cin);
      walk_set(H, W, ldx);
    }
  }
  __device__ __forceinline__ void walk_load(Chunk8<T>& c) const {
    if (wok) c.load_vec(wp + wci);  // prologue deferred (walk_pro)
    else c.zero();
  }
  template <bool PRO>
  __device__ __forceinline__ void walk_pro(Chunk8<T>& c, const float* pt, int act) const {
    if constexpr (PRO) {
      if (c.ok) c.pro(pt, wci, act);
    }
  }
  template <int G, bool PRO>
  __device__ __forceinline__ void gather(Chunk8<T>& c, int k, int K, int cin, int H, int W, int ldx, const float* pt,
                                         int act) const {
    struct alignas(sizeof(T) * G) Sub { T e[G]; };
    int tap = k / cin, ci = k - tap * cin;
#pragma unroll
    for (int j = 0; j < 8; j += G) {
      Sub v;
#pragma unroll
      for (int e = 0; e < G; ++e) v.e[e] = (T)0.f;
      if (k + j < K) {  // K % G == 0: the sub-load is all in or all out
        const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
          v = *(const Sub*)(base + ((long)yy * W + xx) * ldx + ci);
          if constexpr (PRO) {
#pragma unroll
            for (int e = 0; e < G; ++e)
              v.e[e] = from_f32<T>(act_fwd(fmaf(to_f32(v.e[e]), pt[2 * (ci + e)], pt[2 * (ci + e) + 1]), act));
          }
        }
      }
#pragma unroll
      for (int e = 0; e < G; ++e) c.set(j + e, v.e[e]);
      ci += G;
      if (ci >= cin) {
        ci -= cin;
        ++tap;
      }
    }
    c.ok = false;
  }
  // the deferred prologue of a chunk loaded for k (vector paths), just before it is stored
  template <bool PRO>
  __device__ __forceinline__ void pro_pending(Chunk8<T>& c, int k, int Cin, const float* pt, int act) const {
    if constexpr (PRO) {
      if (c.ok) c.pro(pt, KS == 1 ? k : k % Cin, act);
    }
  }
};

// chunk = p[0..7] with elements j >= left zero, in G-element loads (p G-aligned, left % G == 0)
template <int G, typename T>
__device__ __forceinline__ void load_sub(Chunk8<T>& c, const T* p, int left) {
  struct alignas(sizeof(T) * G) Sub { T e[G]; };
#pragma unroll
  for (int j = 0; j < 8; j += G) {
    Sub v;
    if (j < left) {
      v = *(const Sub*)(p + j);
    } else {
#pragma unroll
      for (int e = 0; e < G; ++e) v.e[e] = (T)0.f;
    }
#pragma unroll
    for (int e = 0; e < G; ++e) c.set(j + e, v.e[e]);
  }
  c.ok = false;
}

// Stage the prologue table [Cin][2] = (scale, offset) into LDS (caller syncs).
__device__ __forceinline__ void stage_pro(float* pt, const BnPro& p, int Cin) {
  for (int c = threadIdx.x; c < Cin; c += blockDim.x) bn_pro_affine(p, c, pt[2 * c], pt[2 * c + 1]);
}

// BatchNorm-backward prologue of the backward-data GEMM of a 1x1 conv (rod_conv_bwd_data_bn):
// the A operand is dy = the BatchNorm backward apply of (dz, y) (rod_bn_bwd_apply's arithmetic,
// rounded to bf16), formed as each 8-element chunk of dz / y is staged; the block of N tile 0
// also writes those rounded dy chunks out for the weight gradient.
struct BnBwd {
  const bf16_t* y;       // pre-BatchNorm conv output [M][K]
  const float *mean, *rstd, *gamma, *beta, *coef;
  int act;
  bf16_t* dy;            // [M][K]
};
constexpr int BWD_CF = 8;   // floats per channel in the prologue's LDS table: sc, sh, a, k1, k0, m

// ---- MFMA over one 32-deep k step for one 16x16 tile ---------------------------------
__device__ __forceinline__ void mma32(f32x4& acc, const bf16_t* a, const bf16_t* b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)a, *(const bf16x8*)b, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma32(f32x4& acc, const float* a, const float* b) {
  const f32x4 a0 = *(const f32x4*)a, a1 = *(const f32x4*)(a + 4);
  const f32x4 b0 = *(const f32x4*)b, b1 = *(const f32x4*)(b + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], b0[j], acc, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], b1[j], acc, 0, 0, 0);
}

// =====================================================================================
// forward: y[m, co] = sum_k A[m,k] wt[co,k] + bias[co]
// block 256 threads = 4 waves laid out WM x WN; tile BM x BN; wave tile (BM/WM) x (BN/WN)
// =====================================================================================
// BKT: k depth per LDS step.  32: one LDS buffer, two barriers per step (the next step's
// global loads in flight under the MFMAs).  64 (bf16): two LDS buffers, ONE barrier per step,
// twice the MFMAs per wave between barriers — the deep-K 3x3 convs (K = 9 x 128), which at 32
// were load-latency bound (a k step's MFMAs per SIMD shorter than the im2col gather latency).
template <typename T, int KS, int BN, bool VA, bool VB, bool VY, bool SPLIT = false, bool STATS = false,
          bool PRO = false, bool GRED = false, int BKT = BK, bool EPI = false, bool BWD = false>
__global__ void __launch_bounds__(256) conv_fwd_kernel(const T* __restrict__ X, const T* __restrict__ Wt,
                                                       const float* __restrict__ bias, T* __restrict__ Y, long M,
                                                       int H, int W, int Cin, int Cout, int ldx, int ldy,
                                                       float* __restrict__ part = nullptr, int kper = 0,
                                                       BnPro pro = BnPro{}, BnGred gr = BnGred{},
                                                       BnEpi ep = BnEpi{}, BnBwd bw = BnBwd{}) {
  static_assert(!EPI || (!SPLIT && !STATS && !GRED), "the BatchNorm-apply epilogue is inference-only");
  static_assert(!BWD || (KS == 1 && VA && !PRO && !STATS && !GRED && !EPI && BKT == BK && sizeof(T) == 2),
                "the BatchNorm-backward prologue: bf16 1x1 backward-data only");
  constexpr int BM = 128;
  constexpr int WN = BN >= 64 ? 2 : 1;
  constexpr int WM = 4 / WN;
  constexpr int MT = BM / WM / 16;
  constexpr int NT = BN / WN / 16;
  static_assert(BKT == BK || (BKT == 64 && sizeof(T) == 2 && !SPLIT), "BKT 64: bf16, no split-K");
  constexpr bool DB = BKT == 64;                  // double-buffered LDS
  constexpr int CPR = BKT / 8;                    // 16-byte k chunks per tile row
  constexpr int RPP = 256 / CPR;                  // tile rows per pass of the block
  constexpr int LD = BKT + LdsPad<T>::v;
  constexpr int ACH = BM * BKT / 8 / 256;          // A chunks per thread (2, or 4 at BKT 64)
  constexpr int BCH = (BN * BKT / 8 + 255) / 256;  // B chunks per thread
  // epilogue staging: one 64-row half of the tile at a time, row pad keeps 16-byte alignment
  constexpr int EV = 16 / sizeof(T);
  constexpr int LDC = BN + EV;
  constexpr int MAIN_BYTES = (DB ? 2 : 1) * (BM + BN) * LD * sizeof(T);
  constexpr int EPI_BYTES = VY ? 64 * LDC * sizeof(T) : 0;
  constexpr int ST_BYTES = 0;
  constexpr int SM1 = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  constexpr int SMEM = SM1 > ST_BYTES ? SM1 : ST_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  T* As = (T*)smem;  // LDS buffer b: A tile at As + b(BM+BN)LD, B tile after it

  const int K = KS * KS * Cin;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware order when Cout spans several N tiles (Cout > 256): the host pads gridDim.x to a
  // multiple of 8 and the N tiles of one M tile run on one XCD, so its A rows are fetched into
  // that XCD's L2 once; padding blocks exit before any barrier
  long mt = blockIdx.x;
  int nt = blockIdx.y;
  if (!SPLIT && gridDim.y > 1 && (gridDim.x & 7) == 0) {
    const long pl = blockIdx.x + (long)blockIdx.y * gridDim.x;
    const long q = pl >> 3;
    nt = (int)(q % gridDim.y);
    mt = (q / gridDim.y) * 8 + (pl & 7);
    if (mt * BM >= M) return;
  }
  const long m0 = mt * BM;
  const int n0 = nt * BN;
  const int kc = (tid % CPR) * 8;

  RowSrc<T, KS> rows[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) rows[i].init(X, m0 + tid / CPR + i * RPP, M, H, W, ldx);
  extern __shared__ float pro_lds[];  // PRO: [Cin][2] prologue table; BWD: [K][BWD_CF] (dynamic LDS)
  if constexpr (PRO) {
    stage_pro(pro_lds, pro, Cin);
    __syncthreads();
  }
  if constexpr (BWD) {
    for (int c = tid; c < K; c += 256) {
      float* t = pro_lds + c * BWD_CF;
      bn_affine(bw.mean, bw.rstd, bw.gamma, bw.beta, c, t[0], t[1]);
      t[2] = bw.coef[c];
      bn_bwd_k<T>(t[2], bw.mean[c], bw.rstd[c], bw.coef[K + c], bw.coef[2 * K + c], t[3], t[4], t[5]);
    }
    __syncthreads();
  }

  Chunk8<T> ra[ACH], rb[BCH];
  Chunk8<T> ryb[BWD ? ACH : 1];   // BWD: the y chunks beside the dz chunks in ra
  // 3x3 with 16-byte A chunks: the k loop is sequential (k0 = kb, kb + BKT, ...), so the rows
  // walk their taps incrementally (RowSrc::walk_*); the state always matches the chunk held in ra
  constexpr bool WALK = KS == 3 && VA;
  bool first = true;
  auto load_tiles = [&](int k0) {
    if constexpr (WALK) {
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        if (first) rows[i].walk_init(k0 + kc, Cin, H, W, ldx);
        else rows[i].walk_next(BKT, Cin, H, W, ldx);
        rows[i].walk_load(ra[i]);
      }
      first = false;
    } else {
#pragma unroll
      for (int i = 0; i < ACH; ++i)
        rows[i].template load<VA, PRO>(ra[i], k0 + kc, K, Cin, H, W, ldx, pro_lds, pro.act);
      if constexpr (BWD) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
          if (rows[i].valid && k0 + kc < K) ryb[i].load_vec(bw.y + (rows[i].base - X) + k0 + kc);
          else ryb[i].zero();
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int cid = tid + i * 256;
      const int r = cid / CPR;
      const int co = n0 + r;
      const int k = k0 + kc;
      if (cid >= BN * BKT / 8) continue;
      if (co >= Cout || k >= K) {
        rb[i].zero();
      } else if (VB && k + 8 <= K) {
        rb[i].load_vec(Wt + (long)co * K + k);
      } else {
        // unaligned rows (K % 8 != 0: the heads' last 3x3 convs): G-element sub-loads, G the
        // widest power of two dividing K (Wt is 16-byte aligned, so the row start is G-aligned)
        const T* wrow = Wt + (long)co * K + k;
        if (K % 4 == 0) load_sub<4>(rb[i], wrow, K - k);
        else if (K % 2 == 0) load_sub<2>(rb[i], wrow, K - k);
        else load_sub<1>(rb[i], wrow, K - k);
      }
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[a][b][r] = 0.f;

  // split-K: this workgroup reduces k in [kb, ke) only
  const int kb = SPLIT ? blockIdx.z * kper : 0;
  const int ke = SPLIT ? (kb + kper < K ? kb + kper : K) : K;
  // stage the registers of the k step at k0 into LDS buffer `buf`
  auto store_tiles = [&](int k0, int buf) {
    T* as = As + buf * (BM + BN) * LD;
    T* bs = as + BM * LD;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      if constexpr (WALK) rows[i].template walk_pro<PRO>(ra[i], pro_lds, pro.act);
      else rows[i].template pro_pending<PRO>(ra[i], k0 + kc, Cin, pro_lds, pro.act);
      if constexpr (BWD) {
        if (ra[i].ok) {   // a valid row and k < K (K % 8 == 0: whole chunks)
          const int k = k0 + kc;
          const float* t = pro_lds + k * BWD_CF;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const f32x4 c0 = *(const f32x4*)(t + j * BWD_CF), c1 = *(const f32x4*)(t + j * BWD_CF + 4);
            const float yv = (float)ryb[i].v[j];
            const float z = fmaf(yv, c0[0], c0[1]);
            const float g = (float)ra[i].v[j] * act_grad(z, bw.act);
            ra[i].v[j] = (bf16_t)bn_bwd_apply1<T>(c0[2], g, c0[3], c1[0], c1[1], yv);
          }
          if (nt == 0) *(bf16x8*)(bw.dy + (rows[i].base - X) + k) = ra[i].v;
        }
      }
      ra[i].store_lds(as + (tid / CPR + i * RPP) * LD + kc);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int cid = tid + i * 256;
      if (cid < BN * BKT / 8) rb[i].store_lds(bs + (cid / CPR) * LD + kc);
    }
  };
  auto mma_step = [&](int buf) {
    const T* as = As + buf * (BM + BN) * LD;
    const T* bs = as + BM * LD;
    const int fr = lane & 15, fk = (lane >> 4) * 8;
#pragma unroll
    for (int kk = 0; kk < BKT; kk += 32)
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const T* pa = as + (wm * (BM / WM) + a * 16 + fr) * LD + kk + fk;
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const T* pb = bs + (wn * (BN / WN) + b * 16 + fr) * LD + kk + fk;
          mma32(acc[a][b], pa, pb);
        }
      }
  };
  load_tiles(kb);
  if constexpr (DB) {
    // buffer b is read in step i and rewritten in step i+1 (after that step's barrier)
    store_tiles(kb, 0);
    __syncthreads();
    int buf = 0;
    for (int k0 = kb; k0 < ke; k0 += BKT) {
      const bool more = k0 + BKT < ke;
      if (more) load_tiles(k0 + BKT);  // next step's global loads in flight under the MFMAs
      mma_step(buf);
      if (more) store_tiles(k0 + BKT, buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  } else {
    for (int k0 = kb; k0 < ke; k0 += BKT) {
      __syncthreads();
      store_tiles(k0, 0);
      __syncthreads();
      if (k0 + BKT < ke) load_tiles(k0 + BKT);  // next tile in flight under the MFMAs
      mma_step(0);
    }
  }

  if constexpr (SPLIT) {
    // fp32 partial tile -> part[split][m][co]; bias and rounding happen in the combine
    float* out = part + (long)blockIdx.z * M * Cout;
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int col = n0 + wn * (BN / WN) + b * 16 + (lane & 15);
      if (col >= Cout) continue;
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long row = m0 + wm * (BM / WM) + a * 16 + (lane >> 4) * 4 + r;
          if (row < M) out[row * Cout + col] = acc[a][b][r];
        }
    }
  } else if constexpr (VY) {
    // epilogue through LDS: the accumulators (row = 4(l>>4)+r, col = l&15 of each 16x16
    // tile) are rounded to T into a 64-row staging tile, then every thread stores 16-byte
    // row segments, so each wave writes whole contiguous rows of Y.
    float bv[NT];
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int col = n0 + wn * (BN / WN) + b * 16 + (lane & 15);
      bv[b] = (bias && col < Cout) ? bias[col] : 0.f;
    }
    T* Cs = (T*)smem;
    constexpr int WROWS = BM / WM;  // rows per wave
    // BatchNorm partial statistics of this 128-row tile (STATS) and the gred sums (GRED) walk
    // the staged (already rounded) rows of each half: a thread owns one EV-wide column chunk
    // and the rows GRPP apart, reading 16-byte LDS chunks.  STATS: one pass of sums shifted by
    // a pivot per column common to the whole tile (the mean of its first <= 8 rows, so the
    // shifted sums do not cancel), combined over the row groups by plain addition.
    // GRED: BatchNorm-backward sums of this tile's rounded outputs (dz, staged in Cs) against
    // y_in; a thread owns one EV-wide column chunk and walks rows GRPP apart, so each pass of
    // the block reads whole 16-byte row segments of y_in (coalesced, all loads independent)
    constexpr int GCPR = BN / EV;
    constexpr int GRPP = 256 / GCPR;
    const int gcc = (tid % GCPR) * EV, grg = tid / GCPR;
    const int gcol = n0 + gcc;
    const bool gact = GRED && grg < GRPP && gcol < Cout;
    // STATS from the accumulators, before staging: a column of a 16x16 MFMA tile lives in the
    // four lanes l, l^16, l^32, l^48 (rows 4(l>>4)+r).  Per wave and column: pivot = mean of the
    // wave strip's first (up to) 8 valid rows, then sums of (v - pivot), (v - pivot)^2 over the
    // strip's valid rows (v = the output rounded to T), combined across the four lane groups by
    // shuffles -> (n, mean, M2) per wave; the WM waves are Chan-merged in order at the end.
    // per-wave (count, mean, M2) of each column: [WM][3][BN] floats in their own LDS (written
    // here, read after the staging loop, whose barriers order the two)
    __shared__ float wst[(VY && STATS) ? WM * 3 * BN : 1];
    if constexpr (STATS) {
      // round once, in place: the statistics and the staging below use the stored values
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[a][b][r] = to_f32(from_f32<T>(acc[a][b][r] + bv[b]));
      const int lg = lane >> 4;
      // rows of this wave's strip still inside M (all of them except in the last tile)
      const long left_l = M - (m0 + wm * WROWS);
      const int left = left_l > WROWS ? WROWS : (left_l < 0 ? 0 : (int)left_l);
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        float p = 0.f, pc = 0.f;
        if (lg < 2) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (lg * 4 + r < left) {
              p += acc[0][b][r];
              pc += 1.f;
            }
          }
        }
        p += __shfl_xor(p, 16, 64);
        pc += __shfl_xor(pc, 16, 64);
        p = __shfl(p, lane & 15, 64);
        pc = __shfl(pc, lane & 15, 64);
        // full strips: pc = 8 and the division is an exact scaling
        const float piv = left >= 8 ? p * 0.125f : (pc > 0.f ? p / pc : 0.f);
        float s1 = 0.f, s2 = 0.f, n = 0.f;
        if (left == WROWS) {  // full strip: no row checks
#pragma unroll
          for (int a = 0; a < MT; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float d = acc[a][b][r] - piv;
              s1 += d;
              s2 = fmaf(d, d, s2);
            }
          n = (float)(MT * 4);
        } else {
#pragma unroll
          for (int a = 0; a < MT; ++a)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (a * 16 + lg * 4 + r < left) {
                const float d = acc[a][b][r] - piv;
                s1 += d;
                s2 = fmaf(d, d, s2);
                n += 1.f;
              }
            }
        }
        s1 += __shfl_xor(s1, 16, 64);
        s2 += __shfl_xor(s2, 16, 64);
        n += __shfl_xor(n, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        n += __shfl_xor(n, 32, 64);
        if (lane < 16) {
          static_assert((WROWS & (WROWS - 1)) == 0, "wave strip must be a power of two");
          const float dm = left == WROWS ? s1 * (1.0f / WROWS) : (n > 0.f ? s1 / n : 0.f);
          const int cl = wn * (BN / WN) + b * 16 + lane;
          wst[(wm * 3 + 0) * BN + cl] = n;
          wst[(wm * 3 + 1) * BN + cl] = piv + dm;
          wst[(wm * 3 + 2) * BN + cl] = fmaxf(s2 - s1 * dm, 0.f);
        }
      }
    }
    // EPI: the block's columns' BatchNorm (scale, offset), staged once (the store loop's first
    // barrier publishes it)
    __shared__ float2 etab[EPI ? BN : 1];
    if constexpr (EPI) {
      if (tid < BN && n0 + tid < Cout) {
        float sc, sh;
        bn_affine(ep.mean, ep.rstd, ep.gamma, ep.beta, n0 + tid, sc, sh);
        etab[tid] = float2{sc, sh};
      }
    }
    constexpr int GV = GRED ? EV : 1;
    float gsc[GV], gsh[GV], gmu[GV], grs[GV], gs[GV], gsx[GV];
#pragma unroll
    for (int v = 0; v < GV; ++v) {
      gsc[v] = gsh[v] = gmu[v] = grs[v] = gs[v] = gsx[v] = 0.f;
      if (GRED && gact && gcol + v < Cout) gred_coef(gr.p, gcol + v, gsc[v], gsh[v], gmu[v], grs[v]);
    }
#pragma unroll
    for (int h = 0; h < BM / 64; ++h) {
      __syncthreads();
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        const int r_tile = wm * WROWS + a * 16;  // first row of this 16-row tile in the block
        if (r_tile < h * 64 || r_tile >= h * 64 + 64) continue;
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const int cl = wn * (BN / WN) + b * 16 + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(r_tile - h * 64 + (lane >> 4) * 4 + r) * LDC + cl] =
                from_f32<T>(STATS ? acc[a][b][r] : acc[a][b][r] + bv[b]);  // STATS: already rounded
        }
      }
      __syncthreads();
      if constexpr (GRED) {
        const long left = M - (m0 + h * 64);
        const int nrows = left < 64 ? (int)left : 64;
        if (gact) {
          const T* yin = (const T*)gr.y + (m0 + h * 64) * ldy + gcol;
          const bool full = gcol + EV <= Cout;
#pragma unroll 2
          for (int r = grg; r < nrows; r += GRPP) {
            Vec16<T> yv, dv;
            if (full) {
              yv.load(yin + (long)r * ldy);
            } else {
#pragma unroll
              for (int v = 0; v < EV; ++v) yv.set(v, gcol + v < Cout ? to_f32(yin[(long)r * ldy + v]) : 0.f);
            }
            dv.v = *(const decltype(dv.v)*)(Cs + r * LDC + gcc);
#pragma unroll
            for (int v = 0; v < EV; ++v)
              gred_acc(dv.get(v), yv.get(v), gsc[v], gsh[v], gmu[v], grs[v], gr.p.act, gs[v], gsx[v]);
          }
        }
      }
      constexpr int CPR = BN / EV;  // 16-byte chunks per row
      for (int idx = tid; idx < 64 * CPR; idx += 256) {
        const int rr = idx / CPR, cc = (idx - rr * CPR) * EV;
        const long row = m0 + h * 64 + rr;
        const int col = n0 + cc;
        if (row >= M || col >= Cout) continue;
        const T* src = Cs + rr * LDC + cc;
        T* dst = Y + row * ldy + col;
        if constexpr (EPI) {   // z = act(BN(y)) (+ res) from the staged, already rounded y
          if (col + EV <= Cout) {
            Vec16<T> yv, rv, o;
            yv.v = *(const decltype(yv.v)*)src;
            if (ep.res) rv.load((const T*)ep.res + row * ep.ldr + col);
#pragma unroll
            for (int j = 0; j < EV; ++j) {
              const float2 t = etab[cc + j];
              float z = act_fwd(fmaf(yv.get(j), t.x, t.y), ep.act);
              if (ep.res) z = z + rv.get(j);
              o.set(j, z);
            }
            o.store(dst);
          } else {
            for (int j = 0; j < Cout - col; ++j) {
              const float2 t = etab[cc + j];
              dst[j] = from_f32<T>(bn_epi1<T>(ep, t.x, t.y, to_f32(src[j]), row, col + j));
            }
          }
        } else if (col + EV <= Cout) {
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          ROD_ST_OUT((u32x4*)dst, *(const u32x4*)src);
        } else {
          for (int j = 0; j < Cout - col; ++j) dst[j] = src[j];
        }
      }
    }
    if constexpr (GRED) {
      // per channel: the GRPP row groups of its chunk, in order -> part blockIdx.x
      __shared__ float gsum[2][256];
#pragma unroll
      for (int v = 0; v < GV; ++v) {
        __syncthreads();
        gsum[0][tid] = gs[v];
        gsum[1][tid] = gsx[v];
        __syncthreads();
        if (gact && grg == 0 && gcol + v < Cout) {
          float a = 0.f, b = 0.f;
          for (int q = 0; q < GRPP; ++q) {
            a += gsum[0][q * GCPR + tid];
            b += gsum[1][q * GCPR + tid];
          }
          gr.parts[mt * 2 * Cout + gcol + v] = a;
          gr.parts[mt * 2 * Cout + Cout + gcol + v] = b;
        }
      }
    }
    if constexpr (STATS) {
      const float* st = wst;
      if (tid < BN && n0 + tid < Cout) {
        float n = st[tid], mu = st[BN + tid], m2 = st[2 * BN + tid];
        for (int w = 1; w < WM; ++w) {  // Chan merge in wave order
          const float nb = st[(w * 3) * BN + tid];
          if (nb <= 0.f) continue;
          const float mb = st[(w * 3 + 1) * BN + tid], m2b = st[(w * 3 + 2) * BN + tid];
          const float nn = n + nb;
          const float d = mb - mu;
          mu = mu + d * (nb / nn);
          m2 = m2 + m2b + d * d * (n * nb / nn);
          n = nn;
        }
        store_stat_part(part, Cout, mt, n0 + tid, n, mu, m2);
      }
    }
  } else {
    // direct epilogue: bias + store (row = 4(l>>4)+r, col = l&15)
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int col = n0 + wn * (BN / WN) + b * 16 + (lane & 15);
      if (col >= Cout) continue;
      const float bv = bias ? bias[col] : 0.f;
      float esc = 1.f, esh = 0.f;
      if constexpr (EPI) bn_affine(ep.mean, ep.rstd, ep.gamma, ep.beta, col, esc, esh);
#pragma unroll
      for (int a = 0; a < MT; ++a) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long row = m0 + wm * (BM / WM) + a * 16 + (lane >> 4) * 4 + r;
          if (row < M) {
            float v = acc[a][b][r] + bv;
            if constexpr (EPI) v = bn_epi1<T>(ep, esc, esh, v, row, col);
            Y[row * ldy + col] = from_f32<T>(v);
          }
        }
      }
    }
  }
}

// =====================================================================================
// Streaming 1x1 GEMM (bf16, K <= 96, no bias / prologue): y[m, n0 .. n0 + 16*NT) = x[m, :K] *
// wt[n0 .., :K]^T over N groups of 16*NT columns (blockIdx.y), with an optional epilogue:
//   MODE 1: the BatchNorm statistics parts of y ([ceil(M/128)][3][Cout], the forward expand);
//   MODE 3: those statistics only, y not written (ABI 23, rod_conv_fwd_stats: an expand whose
//           consumers recompute y from x);
//   MODE 2: "gred" — the BatchNorm-backward sums of y taken as dz against the pre-BatchNorm
//           tensor gr.y at the same positions ([ceil(M/128)][2][Cout]: sum g, sum g*yhat,
//           g = dz * act'(BN(gr.y))), for a backward-data whose output is the gradient of a
//           BatchNorm's output (the project conv's dx = the depthwise BatchNorm's dz): the
//           separate rod_bn_bwd_reduce pass over (dz, y) is not needed.
//
// The tiled kernel above spends a whole 256-thread block (two barriers, a 128x160 LDS tile, a
// block-wide epilogue) on one 128-row tile whose single k step is a handful of MFMAs: at K = 24
// it is latency-bound (24->144 at 360x640: 2.8 TB/s).  Here every wave streams on its own:
//   * the weights of the N group [16*NT][K] are staged in LDS once per block (zero-padded to
//     KT*32);
//   * a wave owns whole 128-row tiles (the statistics / sums part unit) and walks each in 16-row
//     sub-steps (one MFMA row tile: fewest VGPRs, most waves in flight; measured faster than
//     32-row ones: 24->144 at 360x640 with statistics 195 vs 218 us); the A fragments (lane l:
//     row l & 15, k 8(l >> 4) .. +7 — exactly the MFMA operand layout) load straight from global
//     into registers, the next sub-step's while the current one computes and stores;
//   * the sub-tile's output rows are rounded once, staged in a wave-private LDS slot and
//     written back as 16-byte row segments;
//   * statistics: each lane owns one column per 16-wide N tile (rows 4(l>>4) + r of the MFMA
//     tile), sums (v - pivot) and (v - pivot)^2 over the tile's rows in registers (pivot = mean
//     of the tile's first 8 rows, values rounded to bf16), and the four lane groups combine by
//     two xor-shuffles -> (n, mean, M2) of the tile;
//   * gred: the write-back gives every lane a FIXED 8-channel chunk (lane = row group rg x
//     chunk cc, rows rg, rg + RG, ...), so the lane's BatchNorm constants stay in registers and
//     its sums run over its rows in order; gr.y's rows are loaded (16-byte chunks) before the
//     sub-step's MFMAs; at the tile's end the RG row groups are added in order (shuffles).
// No block barrier after the weight staging.
// =====================================================================================
constexpr int PWS_WAVES = 4;
// PRO: the BatchNorm-apply prologue on x — act(fma(x, scale, offset)) rounded to bf16, the value
// rod_bn_apply would have written.  KT == 1: the lane's 8 channels' constants in registers (its k
// range is fixed: 8*(lane >> 4)); KT > 1 (the projects, K = 96 .. 192): a [K][2] LDS table read
// per chunk, the tiled kernel's Chunk8::pro_t (the same rounding), its activation a template
// argument (ReLU6, the projects' depthwise BatchNorm: a runtime switch there kept every variant's
// table reads live, 150-190 VGPRs).  Rows past M stay 0.
// Cout need not fill the last 16-wide N tile (Cout % 8 == 0: the 24-channel projects): weight
// rows past Cout are zero, their columns are neither stored nor counted.
// (KT >= 5 with the table prologue: at least 4 waves per SIMD, 128 VGPRs — unbounded the compiler
// took 144-172 and 2 waves per SIMD)
template <int NT, int KT, int MODE, bool PRO = false, int PACT = ROD_ACT_RELU6>
__global__ void __launch_bounds__(256, (PRO && KT >= 5) ? 4 : (MODE == 3 ? 5 : 1)) pw_stream_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                                                        bf16_t* __restrict__ Y, long M, int K, int Cout, int ldx,
                                                        int ldy, float* __restrict__ part, BnGred gr,
                                                        BnPro pro = BnPro{}) {
  static_assert(!PRO || MODE != 2, "the prologue form has no gred epilogue");
  constexpr int NP = NT * 16;       // columns of the N group
  constexpr int LDB = KT * 32 + 8;  // weight row stride in LDS (elements)
  constexpr int LDC = NP + 8;       // staging row stride (elements; 16-byte multiple)
  constexpr int SUB = 8;            // 16-row sub-steps per 128-row tile
  constexpr int CPR = NP / 8;       // 16-byte chunks per output row of the group
  constexpr int RG = 64 / CPR;      // gred: row groups of lanes (lanes >= RG*CPR idle)
  constexpr int JN = (16 + RG - 1) / RG;
  constexpr bool STATS = MODE == 1 || MODE == 3, GRED = MODE == 2, NOSTORE = MODE == 3;
  __shared__ __attribute__((aligned(16))) bf16_t Bs[NP * LDB];
  __shared__ __attribute__((aligned(16))) bf16_t Cs[PWS_WAVES][16 * LDC];
  constexpr bool PTAB = PRO && KT > 1;
  __shared__ __attribute__((aligned(16))) float Pt[PTAB ? KT * 32 * 2 : 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, lg = lane >> 4;
  const int n0 = blockIdx.y * NP;

  if constexpr (PTAB) stage_pro(Pt, pro, K);
  for (int idx = tid; idx < NP * KT * 4; idx += 256) {  // weights -> LDS, k >= K / rows >= Cout zero
    const int r = idx / (KT * 4), k = (idx - r * (KT * 4)) * 8;
    bf16x8 v;
    if (k < K && n0 + r < Cout) v = *(const bf16x8*)(Wt + (long)(n0 + r) * K + k);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16_t)0.f;
    }
    *(bf16x8*)(Bs + r * LDB + k) = v;
  }
  __syncthreads();

  const long ntiles = (M + 127) >> 7;
  const long tstride = (long)gridDim.x * PWS_WAVES;
  long t = (long)blockIdx.x * PWS_WAVES + wave;
  bf16_t* cs = Cs[wave];
  // gred: this lane's fixed chunk (row group rg, channels gc .. gc+7) and its BatchNorm constants
  const int rg = lane / CPR, cc = lane - (lane / CPR) * CPR;
  const bool gact = GRED && rg < RG;
  const int gc = n0 + cc * 8;
  constexpr int GV = GRED ? 8 : 1;
  float gsc[GV], gsh[GV], gmu[GV], grs[GV], sg[GV], sgx[GV];
  if constexpr (GRED) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gred_coef(gr.p, gc + e, gsc[e], gsh[e], gmu[e], grs[e]);
      sg[e] = sgx[e] = 0.f;
    }
  }

  float psc[PRO && !PTAB ? 8 : 1], psh[PRO && !PTAB ? 8 : 1];
  if constexpr (PRO && !PTAB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = lg * 8 + e;
      psc[e] = psh[e] = 0.f;
      if (k < K) bn_pro_affine(pro, k, psc[e], psh[e]);
    }
  }
  // A fragments of sub-step (tile, s): rows tile*128 + 16s + fr, k 32kt + 8lg
  auto load_a = [&](bf16x8 (&a)[KT], long tile, int s) {
    const long row = tile * 128 + s * 16 + fr;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int k = kt * 32 + lg * 8;
      if (row < M && k < K) a[kt] = *(const bf16x8*)(X + row * ldx + k);
      else {
#pragma unroll
        for (int e = 0; e < 8; ++e) a[kt][e] = (bf16_t)0.f;
      }
    }
  };
  // the prologue on a loaded fragment (at use, so the load stays in flight meanwhile)
  auto pro_a = [&](bf16x8 (&a)[KT], long tile, int s) {
    if constexpr (PTAB) {
      // applied per k step inside the MFMA loop (pro_k): one chunk's table reads live at a time
    } else if constexpr (PRO) {
      const bool ok = tile * 128 + s * 16 + fr < M && lg * 8 < K;
      if (pro.act == ROD_ACT_NONE) {   // the linear (project) BatchNorm: packed pairs, one rounding each
        typedef float pf2 __attribute__((ext_vector_type(2)));
        typedef __bf16 pb2 __attribute__((ext_vector_type(2)));
        typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
        const u32x4v u = __builtin_bit_cast(u32x4v, a[0]);
        u32x4v o;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const pf2 x2 = {__builtin_bit_cast(float, u[h] << 16), __builtin_bit_cast(float, u[h] & 0xffff0000u)};
          const pf2 z2 = __builtin_elementwise_fma(x2, pf2{psc[2 * h], psc[2 * h + 1]}, pf2{psh[2 * h], psh[2 * h + 1]});
          o[h] = ok ? __builtin_bit_cast(unsigned, __builtin_convertvector(z2, pb2)) : 0u;
        }
        a[0] = __builtin_bit_cast(bf16x8, o);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          a[0][e] = ok ? (bf16_t)act_fwd(fmaf((float)a[0][e], psc[e], psh[e]), pro.act) : (bf16_t)0.f;
      }
    }
  };
  auto pro_k = [&](bf16x8& a, bool rok, int kt) {
    const int k = kt * 32 + lg * 8;
    Chunk8<bf16_t> c;
    c.v = a;
    if (rok && k < K) c.template pro_t<PACT>(Pt, k);
    else c.zero();
    a = c.v;
  };
  // gred: this lane's rows of gr.y for the sub-step starting at row rs (one sub-step ahead)
  auto load_y = [&](bf16x8 (&yv)[GRED ? JN : 1], long rs) {
    if constexpr (GRED) {
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int rr = rg + RG * j;
        if (gact && rr < 16 && rs + rr < M) yv[j] = *(const bf16x8*)((const bf16_t*)gr.y + (rs + rr) * ldy + gc);
      }
    }
  };
  bf16x8 ab[KT], an[KT];
  bf16x8 yb[GRED ? JN : 1], yn[GRED ? JN : 1];
  if (t < ntiles) {
    load_a(ab, t, 0);
    load_y(yb, t * 128);
  }
  for (; t < ntiles; t += tstride) {
    const long row0 = t * 128;
    const int left = M - row0 < 128 ? (int)(M - row0) : 128;  // valid rows of this tile
    const bool full = left == 128;
    float piv[NT], s1[NT], s2[NT];
#pragma unroll
    for (int b = 0; b < NT; ++b) piv[b] = s1[b] = s2[b] = 0.f;
#pragma unroll 1
    for (int s = 0; s < SUB; ++s) {
      const long rs = row0 + s * 16;
      {  // prefetch the next sub-step (the next tile's first one after the last): A and gr.y
        const long tn = s + 1 < SUB ? t : t + tstride;
        if (tn < ntiles) {
          load_a(an, tn, s + 1 < SUB ? s + 1 : 0);
          if constexpr (GRED) load_y(yn, tn * 128 + (s + 1 < SUB ? s + 1 : 0) * 16);
        }
      }
      pro_a(ab, t, s);
      // the weight fragments are re-read from LDS every sub-step (kept out of registers)
      asm volatile("" ::: "memory");
      f32x4 acc[NT];
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        if constexpr (PTAB) {
          pro_k(ab[kt], rs + fr < M, kt);
          asm volatile("" ::: "memory");   // the next chunk's table reads stay after this step
        }
#pragma unroll
        for (int b = 0; b < NT; ++b) {
          const bf16x8 bf = *(const bf16x8*)(Bs + (b * 16 + fr) * LDB + kt * 32 + lg * 8);
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab[kt], bf, acc[b], 0, 0, 0);
        }
      }
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) ab[kt] = an[kt];
      // epilogue, one 16-wide N tile at a time: round once (the statistics and the staged value
      // are the stored one), statistics, stage into this wave's LDS slot
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (float)(bf16_t)acc[b][r];
        if constexpr (STATS) {
          if (s == 0) {  // pivot: mean of the tile's first (up to) 8 valid rows, this column
            float p = 0.f;
            if (lg < 2) {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (full || lg * 4 + r < left) p += v[r];
            }
            p += __shfl_xor(p, 16, 64);
            p = __shfl(p, fr, 64);
            const int pc = left < 8 ? left : 8;
            piv[b] = full ? p * 0.125f : p / (float)pc;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (full || s * 16 + lg * 4 + r < left) {
              const float d = v[r] - piv[b];
              s1[b] += d;
              s2[b] = fmaf(d, d, s2[b]);
            }
          }
        }
        if constexpr (!NOSTORE) {
#pragma unroll
          for (int r = 0; r < 4; ++r) cs[(lg * 4 + r) * LDC + b * 16 + fr] = (bf16_t)v[r];
        }
      }
      __builtin_amdgcn_wave_barrier();
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      if constexpr (NOSTORE) {
      } else if constexpr (GRED) {
        // fixed-chunk write-back + the BatchNorm-backward sums of the stored values
        if (gact) {
#pragma unroll
          for (int j = 0; j < JN; ++j) {
            const int rr = rg + RG * j;
            if (rr >= 16 || rs + rr >= M) continue;
            const bf16x8 dv = *(const bf16x8*)(cs + rr * LDC + cc * 8);
            ROD_ST_OUT((u32x4*)(Y + (rs + rr) * ldy + gc), __builtin_bit_cast(u32x4, dv));
#pragma unroll
            for (int e = 0; e < 8; ++e)
              gred_acc((float)dv[e], (float)yb[j][e], gsc[e], gsh[e], gmu[e], grs[e], gr.p.act, sg[e], sgx[e]);
          }
        }
      } else {
#pragma unroll
        for (int it = 0; it < (16 * CPR + 63) / 64; ++it) {
          const int idx = it * 64 + lane;
          if ((16 * CPR) % 64 != 0 && idx >= 16 * CPR) break;
          const int rr = idx / CPR, c8 = idx - rr * CPR;
          const u32x4 v = *(const u32x4*)(cs + rr * LDC + c8 * 8);
          if (rs + rr < M && n0 + c8 * 8 < Cout) ROD_ST_OUT((u32x4*)(Y + (rs + rr) * ldy + n0 + c8 * 8), v);
        }
      }
      __builtin_amdgcn_wave_barrier();
      if constexpr (GRED) {
#pragma unroll
        for (int j = 0; j < JN; ++j) yb[j] = yn[j];
      }
    }
    if constexpr (STATS) {
      const float n = (float)left;
#pragma unroll
      for (int b = 0; b < NT; ++b) {
        float a = s1[b], q = s2[b];
        a += __shfl_xor(a, 16, 64);
        q += __shfl_xor(q, 16, 64);
        a += __shfl_xor(a, 32, 64);
        q += __shfl_xor(q, 32, 64);
        if (lane < 16 && n0 + b * 16 + lane < Cout) {
          const float dm = full ? a * (1.0f / 128.0f) : a / n;
          store_stat_part(part, Cout, t, n0 + b * 16 + lane, n, piv[b] + dm, fmaxf(q - a * dm, 0.f));
        }
      }
    }
    if constexpr (GRED) {
      // the tile's part: row groups added in order (lane rg*CPR + cc holds group rg of chunk cc)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float a = sg[e], q = sgx[e];
#pragma unroll
        for (int k = 1; k < RG; ++k) {
          a += __shfl(sg[e], cc + k * CPR, 64);
          q += __shfl(sgx[e], cc + k * CPR, 64);
        }
        if (gact && rg == 0) {
          gr.parts[t * 2 * Cout + gc + e] = a;
          gr.parts[t * 2 * Cout + Cout + gc + e] = q;
        }
        sg[e] = sgx[e] = 0.f;
      }
    }
  }
}

// rod_conv_fwd's streaming path (pw_stream_kernel): bf16 1x1, no bias / prologue, K <= 96
// (K % 8 == 0), Cout a multiple of 96, 144 or 192 (N groups of 6, 9 or 12 MFMA tiles),
// 16-byte aligned rows, M >= 65536; statistics parts or the gred sums (dense y) or neither.
// ROD_PW_STREAM=0 turns it off (A/B measurement switch).
static int pw_stream_groups(long M, int K, int Cout, int& nt, bool gred = false) {
  static const bool off = getenv("ROD_PW_STREAM") && atoi(getenv("ROD_PW_STREAM")) == 0;
  // >= 512 row tiles: on the 45x80 maps (225 tiles) the tiled kernel measured faster
  // (tools/conv_bench.py: 96->576 18.2 vs 23.1 us)
  if (off || K > 96 || K % 8 || Cout % 16 || M < 65536) return 0;
  // gred: narrow groups (3 MFMA tiles: the lane's fixed chunks span more rows, fewer VGPRs for
  // its BatchNorm constants, row sums and prefetched gr.y); otherwise the widest that divides Cout
  static const int gred_first[] = {3, 2, 4, 6, 9, 12, 8};
  static const int wide_first[] = {12, 9, 6, 8, 4, 3, 2};
  for (int c : gred ? gred_first : wide_first) {
    if (Cout % (16 * c) == 0) {
      nt = c;
      return Cout / (16 * c);
    }
  }
  return 0;
}
static bool pw_stream_launch(const bf16_t* x, const bf16_t* wt, bf16_t* y, long M, int K, int Cout, int ldx, int ldy,
                             float* stats, const BnGred* gr, hipStream_t s, const BnPro* pro = nullptr) {
  if (y == nullptr) {   // statistics only (rod_conv_fwd_stats): K <= 32, one k step
    int nt = 0;
    const int ng = pw_stream_groups(M, K, Cout, nt, false);
    if (ng == 0 || !stats || gr || K > 32) return false;
    // no store to stream behind: latency-bound on its A loads, so up to 5 blocks of 4 waves per CU
    // (<= 102 VGPRs: 5 waves per SIMD) instead of the storing kernel's 3.  (Measured slower: a
    // dedicated kernel with a 2- / 4-deep A ring and the sub-steps unrolled, 232 -> 280 us at 720p
    // b8 16 -> 96, its registers up to 144-220; one that loads the next whole 128-row tile (4 KB a
    // wave) before computing the current one through a register queue, 158 VGPRs at 3 waves per
    // SIMD, 227 -> 253 us (24 -> 144: 80 -> 90) — the sub-step's MFMA -> rounding -> statistics
    // chain, not the loads, is what the waves wait on.)
    const long ntiles = cdivl(M, 128);
    const BnPro pv = pro ? *pro : BnPro{};
    const long maxw = cdivl(256L * 5 * PWS_WAVES, ng);
    const long per = cdivl(ntiles, maxw);
    const dim3 grid((unsigned)cdivl(cdivl(ntiles, per), PWS_WAVES), ng);
    const BnGred g{};
#define PWN(NT_)                                                                                               \
  if (nt == NT_) {                                                                                             \
    if (pro)                                                                                                   \
      hipLaunchKernelGGL((pw_stream_kernel<NT_, 1, 3, true>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout, ldx, \
                         ldy, stats, g, pv);                                                                   \
    else                                                                                                       \
      hipLaunchKernelGGL((pw_stream_kernel<NT_, 1, 3>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout, ldx, ldy,  \
                         stats, g);                                                                            \
    return true;                                                                                               \
  }
    PWN(2) PWN(3) PWN(4) PWN(6) PWN(8) PWN(9) PWN(12)
#undef PWN
    return false;
  }
  int nt = 0;
  const int ng = pw_stream_groups(M, K, Cout, nt, gr != nullptr);
  if (ng == 0 || (gr && (stats || ldy != Cout))) return false;
  const int kt = K > 64 ? 3 : K > 32 ? 2 : 1;
  if (pro && (kt != 1 || gr)) return false;   // the prologue form: K <= 32, no gred epilogue
  const long ntiles = cdivl(M, 128);
  // waves: <= 3 blocks of 4 waves per CU (over all N groups), every wave the same number of
  // tiles (+-1)
  const long maxw = cdivl(256L * 3 * PWS_WAVES, ng);
  const long per = cdivl(ntiles, maxw);
  const dim3 grid((unsigned)cdivl(cdivl(ntiles, per), PWS_WAVES), ng);
  const BnGred g = gr ? *gr : BnGred{};
#define PWS(NT_, KT_)                                                                                           \
  do {                                                                                                          \
    if constexpr (KT_ == 1) {                                                                                   \
      if (pro) {                                                                                                \
        if (stats)                                                                                              \
          hipLaunchKernelGGL((pw_stream_kernel<NT_, 1, 1, true>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout,  \
                             ldx, ldy, stats, g, *pro);                                                         \
        else                                                                                                    \
          hipLaunchKernelGGL((pw_stream_kernel<NT_, 1, 0, true>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout,  \
                             ldx, ldy, nullptr, g, *pro);                                                       \
        return true;                                                                                            \
      }                                                                                                         \
    }                                                                                                           \
    if (gr)                                                                                                     \
      hipLaunchKernelGGL((pw_stream_kernel<NT_, KT_, 2>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout, ldx, ldy, \
                         nullptr, g);                                                                           \
    else if (stats)                                                                                             \
      hipLaunchKernelGGL((pw_stream_kernel<NT_, KT_, 1>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout, ldx, ldy, \
                         stats, g);                                                                             \
    else                                                                                                        \
      hipLaunchKernelGGL((pw_stream_kernel<NT_, KT_, 0>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout, ldx, ldy, \
                         nullptr, g);                                                                           \
    return true;                                                                                                \
  } while (0)
#define PWK(NT_)                  \
  if (nt == NT_) {                \
    if (kt == 1) PWS(NT_, 1);     \
    else if (kt == 2) PWS(NT_, 2); \
    else PWS(NT_, 3);             \
  }
  PWK(2) PWK(3) PWK(4) PWK(6) PWK(8) PWK(9) PWK(12)
#undef PWK
#undef PWS
  return false;
}

// The projects (the streaming form past K = 96): a 1x1 conv whose input
// BatchNorm is still pending (the prologue), K = 40 .. 192 input channels (ReLU6 prologue), Cout = 16 .. 32 outputs
// (one N group of 1 or 2 MFMA tiles), M >= 65536 rows, with or without the statistics epilogue.
// tools/conv_bench.py (fwd_stats, 8 images): 96 -> 24 at 360x640 100 -> 95 us, 144 -> 24 162 -> 139,
// 192 -> 32 at 180x320 44 -> 42, 144 -> 32 44 -> 36 (3.7-4.7 -> 4.5-5.0 TB/s).
// The tiled kernel ran these at 3.5-4.5 TB/s: a 128 x 32 output tile per block behind two barriers
// per 32-deep k step.  Here each wave streams its 16-row sub-steps with all KT A fragments in
// flight and no block barrier.  y is bit-identical (the same MFMA k order and prologue rounding);
// the statistics parts are per 128-row tile as before, summed in another order.
// ROD_PW_PROJ=0 turns it off (A/B switch).
static bool pw_proj_launch(const bf16_t* x, const bf16_t* wt, bf16_t* y, long M, int K, int Cout, int ldx, int ldy,
                           float* stats, hipStream_t s, const BnPro& pro) {
  const char* e = getenv("ROD_PW_PROJ");   // read per call (tests A/B it in one process)
  const bool off = e != nullptr && atoi(e) == 0;
  if (off || K > 192 || K % 8 || Cout > 32 || Cout % 8 || M < 65536) return false;
  const int kt = cdiv(K, 32), nt = cdiv(Cout, 16);
  // K <= 32 (the 720p block-1 project 32 -> 16, one 16-wide N tile) measured no faster here
  // (229 vs 224 us): the tiled kernel keeps it; the table form is built for ReLU6
  if (kt == 1 || pro.act != ROD_ACT_RELU6) return false;
  const long ntiles = cdivl(M, 128);
  const long maxw = 256L * 3 * PWS_WAVES;
  const long per = cdivl(ntiles, maxw);
  const dim3 grid((unsigned)cdivl(cdivl(ntiles, per), PWS_WAVES), 1);
  const BnGred g{};
#define PJ(NT_, KT_)                                                                                             \
  do {                                                                                                           \
    if (stats)                                                                                                   \
      hipLaunchKernelGGL((pw_stream_kernel<NT_, KT_, 1, true>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout, ldx, \
                         ldy, stats, g, pro);                                                                    \
    else                                                                                                         \
      hipLaunchKernelGGL((pw_stream_kernel<NT_, KT_, 0, true>), grid, dim3(256), 0, s, x, wt, y, M, K, Cout, ldx, \
                         ldy, nullptr, g, pro);                                                                  \
    return true;                                                                                                 \
  } while (0)
#define PJK(NT_)                     \
  switch (kt) {                      \
    case 1: PJ(NT_, 1);              \
    case 2: PJ(NT_, 2);              \
    case 3: PJ(NT_, 3);              \
    case 4: PJ(NT_, 4);              \
    case 5: PJ(NT_, 5);              \
    default: PJ(NT_, 6);             \
  }
  if (nt == 1) PJK(1) else PJK(2)
#undef PJK
#undef PJ
  return false;
}

// split-K combine: y[m, co] = round(sum_s part[s][m][co] + bias[co]), fixed split order
template <typename T, bool EPI = false>
__global__ void splitk_combine_kernel(const float* __restrict__ part, const float* __restrict__ bias,
                                      T* __restrict__ Y, long M, int Cout, int ldy, int splits, BnEpi ep = BnEpi{}) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = M * Cout;
  if (i >= n) return;
  const long m = i / Cout;
  const int co = (int)(i - m * Cout);
  float acc = 0.f;
  for (int z = 0; z < splits; ++z) acc += part[(long)z * n + i];
  if (bias) acc += bias[co];
  if constexpr (EPI) {
    float sc, sh;
    bn_affine(ep.mean, ep.rstd, ep.gamma, ep.beta, co, sc, sh);
    acc = bn_epi1<T>(ep, sc, sh, acc, m, co);
  }
  Y[m * ldy + co] = from_f32<T>(acc);
}

struct SplitPlan {
  int splits, kper;
};
// split K when the output has fewer than 128 tiles of 128 rows x 128 columns and K is
// at least 8 k-steps deep: ~256 workgroups, each >= 2 k-steps
static SplitPlan split_plan(long M, int Cout, int K) {
  SplitPlan p{1, K};
  const long tiles = cdivl(M, 128) * cdivl(Cout, 128);
  const int ksteps = cdiv(K, BK);
  if (tiles >= 128 || ksteps < 8) return p;
  int splits = (int)std::min<long>(ksteps / 2, cdivl(256, tiles));
  if (splits < 2) return p;
  const int per = cdiv(ksteps, splits);
  p.kper = per * BK;
  p.splits = cdiv(ksteps, per);
  return p;
}

// =====================================================================================
// stem: 3x3 / stride 1 / TF-SAME conv with Cin = 3 (the normalised image, mobilenet_v2.py
// Conv layer) — a direct VALU convolution.  A block makes TW = 4096/CO consecutive pixels
// of one image row: the 3 x (TW+2) x 3 input patch and the [27][CO] weights are staged in
// LDS, each thread makes one pixel x 16 channels (27 taps, fp32 FMAs) and stores them as
// two 16-byte vectors, so a wave writes whole contiguous output rows.
// =====================================================================================
template <typename T, int CO>
__global__ void __launch_bounds__(256) stem_conv_fwd_kernel(const T* __restrict__ X, const T* __restrict__ Wt,
                                                            const float* __restrict__ bias, T* __restrict__ Y, int H,
                                                            int W, int ldx, int ldy) {
  constexpr int G = CO / 16;         // 16-channel groups per pixel
  constexpr int TW = 256 / G;        // pixels per block
  __shared__ float patch[3][TW + 2][3];
  __shared__ __attribute__((aligned(16))) float ws[27][CO];
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * TW;
  const int yy = blockIdx.y;
  const int n = blockIdx.z;
  for (int e = tid; e < 3 * (TW + 2) * 3; e += 256) {
    const int ci = e % 3, t = e / 3;
    const int cx = t % (TW + 2), r = t / (TW + 2);
    const int iy = yy + r - 1, ix = x0 + cx - 1;
    float v = 0.f;
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = to_f32(X[(((long)n * H + iy) * W + ix) * ldx + ci]);
    patch[r][cx][ci] = v;
  }
  for (int e = tid; e < 27 * CO; e += 256) {
    const int co = e / 27, k = e - co * 27;  // Wt is [CO][27] (k = (i*3 + j)*3 + ci)
    ws[k][co] = to_f32(Wt[e]);
  }
  __syncthreads();
  const int p = tid / G, cg = (tid % G) * 16;
  const int xo = x0 + p;
  if (xo >= W) return;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = bias ? bias[cg + j] : 0.f;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) {
        const float a = patch[r][p + c][ci];
        const f32x4* wv = (const f32x4*)&ws[(r * 3 + c) * 3 + ci][cg];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 w4 = wv[q];
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[q * 4 + u] = fmaf(a, w4[u], acc[q * 4 + u]);
        }
      }
  T* dst = Y + (((long)n * H + yy) * W + xo) * ldy + cg;
  constexpr int EV = Vec16<T>::N;
#pragma unroll
  for (int q = 0; q < 16 / EV; ++q) {
    Vec16<T> o;
#pragma unroll
    for (int u = 0; u < EV; ++u) o.set(u, acc[q * EV + u]);
    o.store(dst + q * EV);
  }
}

constexpr int SW_TW = 128;  // stem kernels: pixels per block row
constexpr int SW_LD = 40;   // stem kernels: LDS row (elements), 80 B

// =====================================================================================
// stem forward on MFMA (bf16, Cout = 32): a block makes 128 consecutive pixels of one image
// row.  Each thread gathers 16 taps of one pixel's 3x3x3 patch (as stem_wgrad_kernel) into
// an im2col tile Xs[128][32] (taps 27..31 zero); wave w multiplies pixels [32w, 32w+32) by
// the [32 taps][32 co] weights held in registers (2 x 2 16x16x32 MFMAs: A rows = pixels read
// straight from Xs, B = Wt rows), adds the bias, rounds, and stages the [128][32] tile in
// LDS so each thread stores 32 contiguous bytes.  STATS (W % 128 == 0, so the block is
// exactly the 128-row tile blockIdx of the rod_conv_fwd stat_parts contract): per channel,
// 8 lanes x 16 pixels of pivot-shifted sums of the rounded outputs, xor-shuffle combined.
// =====================================================================================
// Taps [16*HALF, 16*HALF + 16) of pixel (n, y, xx)'s 3x3x3 SAME patch (tap = (r*3 + c)*3 + ci;
// taps >= 27 and padding read as zero).  HALF is a template argument so every tap's
// (r, c, ci) folds to constants; callers make it wave-uniform.
template <int HALF>
__device__ __forceinline__ void stem_gather(const unsigned short* __restrict__ Xu, long nH, int y, int xx, int H,
                                            int W, int ldx, unsigned short (&tv)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = HALF * 16 + j;
    unsigned short v = 0;
    if (k < 27) {
      const int r = k / 9, c = (k / 3) % 3, ci = k % 3;
      const int iy = y + r - 1, ix = xx + c - 1;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W && xx < W)
        v = Xu[((nH + iy) * W + ix) * ldx + ci];
    }
    tv[j] = v;
  }
}

template <bool STATS>
__global__ void __launch_bounds__(256) stem_fwd_mfma_kernel(const bf16_t* __restrict__ X,
                                                            const bf16_t* __restrict__ Wt,
                                                            const float* __restrict__ bias, bf16_t* __restrict__ Y,
                                                            float* __restrict__ stats, int H, int W, int ldx,
                                                            int ldy, int rb) {
  // input rows through an LDS ring of three (130 pixels x 3 channels each: one 2-byte load per
  // element per row, issued a whole row ahead), the 3x3x3 patches gathered from LDS — the
  // first form gathered every tap from global memory (16 two-byte loads per thread per row,
  // each input element fetched 9 times)
  constexpr int RIN = (SW_TW + 2) * 3;
  __shared__ __attribute__((aligned(16))) bf16_t Xs[SW_TW * SW_LD];
  __shared__ __attribute__((aligned(16))) bf16_t Ys[SW_TW * SW_LD];
  __shared__ unsigned short Rin[3][RIN + 2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int x0 = blockIdx.x * SW_TW, n = blockIdx.z;
  const int ya = blockIdx.y * rb;
  const int yz = ya + rb < H ? ya + rb : H;
  const int px = tid >> 1, half = tid & 1;  // output store: pixel, 16-channel half
  const int xx = x0 + px;
  const bool inx = xx < W;
  const int pg = tid & 127, hg = tid >> 7;  // gather: pixel, wave-uniform tap half
  typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
  const unsigned short* Xu = (const unsigned short*)X;
  unsigned short tv[16], rv[2];
  auto load_in = [&](int iy) {   // this thread's elements of input row iy (zero outside the image)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * 256;
      const int pxe = x0 - 1 + e / 3, ci = e - (e / 3) * 3;
      rv[u] = 0;
      if (e < RIN && iy >= 0 && iy < H && pxe >= 0 && pxe < W) rv[u] = Xu[(((long)n * H + iy) * W + pxe) * ldx + ci];
    }
  };
  auto store_in = [&](int iy) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * 256;
      if (e < RIN) Rin[(iy + 3) % 3][e] = rv[u];
    }
  };
  // taps [16*HG, 16*HG + 16) of pixel pg's patch, tap = (r*3 + c)*3 + ci (HG constant: every
  // tap's row / column / channel folds; callers pick HG = hg, which is wave-uniform)
  auto gather_h = [&](auto hgc, int y) {
    constexpr int HG = decltype(hgc)::value;
    const unsigned short* rows[3] = {Rin[(y + 2) % 3], Rin[(y + 3) % 3], Rin[(y + 4) % 3]};   // y-1, y, y+1
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = HG * 16 + j;
      if (k < 27) {
        const int r = k / 9, c = (k / 3) % 3, ci = k % 3;
        tv[j] = rows[r][(pg + c) * 3 + ci];
      } else {
        tv[j] = 0;
      }
    }
  };
  auto gather = [&](int y) {
    if (hg) gather_h(std::integral_constant<int, 1>{}, y);
    else gather_h(std::integral_constant<int, 0>{}, y);
  };
  const int g = lane >> 4, i = lane & 15;
  bf16x8 fb[2];  // B[k = 8g + j][co = ct*16 + i] = Wt[co][k]
  float bv[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * g + j;
      fb[ct][j] = k < 27 ? Wt[(ct * 16 + i) * 27 + k] : (bf16_t)0.f;
    }
    bv[ct] = bias ? bias[ct * 16 + i] : 0.f;
  }
  if (ya < yz) {   // rows ya-1 .. ya+1 into the ring (loads issued together), row ya+2 in flight
    unsigned short pre[3][2];
#pragma unroll
    for (int i3 = 0; i3 < 3; ++i3) {
      load_in(ya - 1 + i3);
      pre[i3][0] = rv[0];
      pre[i3][1] = rv[1];
    }
#pragma unroll
    for (int i3 = 0; i3 < 3; ++i3) {
      rv[0] = pre[i3][0];
      rv[1] = pre[i3][1];
      store_in(ya - 1 + i3);
    }
    load_in(ya + 2);
    __syncthreads();
    gather(ya);
  }
  for (int y = ya; y < yz; ++y) {
    __syncthreads();   // Ys of the previous row stored; every gather of row y done
    {
      u16x8 t0, t1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        t0[j] = tv[j];
        t1[j] = tv[8 + j];
      }
      *(u16x8*)(Xs + pg * SW_LD + hg * 16) = t0;
      *(u16x8*)(Xs + pg * SW_LD + hg * 16 + 8) = t1;
    }
    if (y + 1 < yz) store_in(y + 2);   // the slot of row y - 1 (no longer gathered)
    __syncthreads();
    if (y + 2 < yz) load_in(y + 3);    // a whole row ahead
    const int m0 = wave * 32;
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      const bf16x8 fa = *(const bf16x8*)(Xs + (m0 + pt * 16 + i) * SW_LD + 8 * g);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb[ct], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) Ys[(m0 + pt * 16 + g * 4 + r) * SW_LD + ct * 16 + i] = (bf16_t)(acc[r] + bv[ct]);
      }
    }
    __syncthreads();
    if (inx) {
      bf16_t* dst = Y + (((long)n * H + y) * W + xx) * ldy + half * 16;
      ROD_ST_OUT((bf16x8*)dst, *(const bf16x8*)(Ys + px * SW_LD + half * 16));
      ROD_ST_OUT((bf16x8*)(dst + 8), *(const bf16x8*)(Ys + px * SW_LD + half * 16 + 8));
    }
    if constexpr (STATS) {
      const int c = tid >> 3, sub = tid & 7;
      const float k = (float)Ys[c];  // pivot: pixel 0 of the tile
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float d = (float)Ys[(sub * 16 + j) * SW_LD + c] - k;
        s1 += d;
        s2 = fmaf(d, d, s2);
      }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
      }
      if (sub == 0) {
        const long tile = (((long)n * H + y) * W + x0) / SW_TW;
        const double nb = (double)SW_TW;
        const double m2 = (double)s2 - (double)s1 * (double)s1 / nb;
        store_stat_part(stats, 32, tile, c, (float)nb, (float)((double)k + (double)s1 / nb),
                        (float)(m2 > 0.0 ? m2 : 0.0));
      }
    }
    if (y + 1 < yz) gather(y + 1);   // rows y .. y+2 are in the ring (barrier above)
  }
}

// =====================================================================================
// weight gradient: part[s][co][k] = sum_{m in split s} dy[m, co] * A[m, k]
// tile 64 (co) x 64 (k); rows staged m-major in LDS and read transposed
// (ds_read_b64_tr_b16 for bf16, plain b32 lane-per-column reads for f32).
// =====================================================================================
constexpr int WG_T = 64;            // co / k tile
constexpr int WG_LD = WG_T + 4;     // LDS row (elements): 136 B bf16 / 272 B f32

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x4 tr_read(const bf16_t* p) {
  s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
  return __builtin_bit_cast(bf16x4, r);
}

// RPT row chunks per thread per step (bf16: 2, so a block keeps two 32-row steps of loads in
// flight per barrier pair; the kernel is load-latency bound at <= 8 resident blocks per CU)
template <typename T, int KS, bool VA, bool VD, int CIN = 0, bool PRO = false>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(const T* __restrict__ X, const T* __restrict__ DY,
                                                         float* __restrict__ part, long M, int H, int W, int Cin,
                                                         int Cout, int ldx, int lddy, long chunk, int ktiles,
                                                         BnPro pro = BnPro{}) {
  constexpr int RPT = sizeof(T) == 2 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) T Ds[RPT * BK * WG_LD];  // [m][co]
  __shared__ __attribute__((aligned(16))) T Xs[RPT * BK * WG_LD];  // [m][k]
  extern __shared__ float pro_lds[];  // PRO: [Cin][2] prologue table (dynamic LDS)
  if constexpr (PRO) {
    stage_pro(pro_lds, pro, Cin);
    __syncthreads();
  }
  const int K = KS * KS * Cin;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // 2x2 waves of 32x32
  // XCD-aware order: the gridDim.x tiles of one row split run on one XCD (the hardware
  // deals blocks to the 8 XCDs round-robin by linear id), so the dy / x rows the tiles share
  // are fetched into that XCD's L2 once (wgrad_plan makes the split count a multiple of 8)
  int tile = blockIdx.x, split = blockIdx.y;
  if (gridDim.x > 1 && (gridDim.y & 7) == 0) {
    const long pl = blockIdx.x + (long)blockIdx.y * gridDim.x;
    const long q = pl >> 3;
    tile = (int)(q % gridDim.x);
    split = (int)((q / gridDim.x) * 8 + (pl & 7));
  }
  const int co0 = (tile / ktiles) * WG_T;
  const int k0 = (tile % ktiles) * WG_T;
  const long mb = (long)split * chunk;
  const long me = mb + chunk < M ? mb + chunk : M;

  // each thread stages one 8-wide chunk of a Ds row and one of an Xs row per step
  const int lr = tid >> 3;       // row within the 32-row step
  const int lc = (tid & 7) * 8;  // column chunk within the 64-wide tile

  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[a][b][r] = 0.f;

  Chunk8<T> rdv[RPT], rxv[RPT];
  // 3x3 with 16-byte chunks: the thread's im2col column k0 + lc (tap, channel) is fixed for the
  // whole block and its rows walk forward, so the pixel coordinates are carried from step to
  // step instead of re-derived by 64-bit divisions per row (RowSrc::init)
  constexpr bool WALKW = KS == 3 && VA && CIN == 0;
  int wy[RPT], wx[RPT], wnn[RPT], kdy = 0, kdx = 0, kci = 0;
  bool kok = false;
  if constexpr (WALKW) {
    const int kk = k0 + lc;
    kok = kk < K;
    const int tap = kok ? kk / Cin : 0;
    kci = kk - tap * Cin;
    kdy = tap / 3 - 1;
    kdx = tap % 3 - 1;
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const long row = mb + lr + u * BK;
      wx[u] = (int)(row % W);
      const long t = row / W;
      wy[u] = (int)(t % H);
      wnn[u] = (int)(t / H);
    }
  }
  auto load_one = [&](long row, Chunk8<T>& rd, Chunk8<T>& rx) {
    // dy[row, co0+lc .. +7]
    if (row >= me || co0 + lc >= Cout) {
      rd.zero();
    } else if (VD && co0 + lc + 8 <= Cout) {
      rd.load_vec(DY + row * lddy + co0 + lc);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) rd.set(j, (co0 + lc + j < Cout) ? DY[row * lddy + co0 + lc + j] : (T)0.f);
    }
    if constexpr (!WALKW) {
      RowSrc<T, KS, CIN> rs;
      rs.init(X, row < me ? row : M, M, H, W, ldx);
      rs.template load<VA, PRO>(rx, k0 + lc, K, Cin, H, W, ldx, pro_lds, pro.act);
    }
  };
  auto load_step = [&](long m) {
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      load_one(m + lr + u * BK, rdv[u], rxv[u]);
      if constexpr (WALKW) {
        // the thread's k (tap, channel) is fixed; its rows advance by RPT * BK pixels per step
        const long row = m + lr + u * BK;
        const int yy = wy[u] + kdy, xx = wx[u] + kdx;
        if (kok && row < me && yy >= 0 && yy < H && xx >= 0 && xx < W)
          rxv[u].load_vec(X + (((long)wnn[u] * H + yy) * W + xx) * ldx + kci);
        else
          rxv[u].zero();
        wx[u] += RPT * BK;
        while (wx[u] >= W) {
          wx[u] -= W;
          if (++wy[u] == H) {
            wy[u] = 0;
            ++wnn[u];
          }
        }
      }
    }
  };

  if (mb < me) load_step(mb);
  for (long m = mb; m < me; m += RPT * BK) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      rdv[u].store_lds(Ds + (lr + u * BK) * WG_LD + lc);
      if constexpr (PRO && WALKW) {
        if (rxv[u].ok) rxv[u].pro(pro_lds, kci, pro.act);
      } else if constexpr (PRO) {
        RowSrc<T, KS, CIN> rp;  // (pro_pending only needs KS)
        rp.template pro_pending<PRO>(rxv[u], k0 + lc, Cin, pro_lds, pro.act);
      }
      rxv[u].store_lds(Xs + (lr + u * BK) * WG_LD + lc);
    }
    __syncthreads();
    if (m + RPT * BK < me) load_step(m + RPT * BK);
#pragma unroll
    for (int u = 0; u < RPT; ++u)
    if constexpr (sizeof(T) == 2) {
      // A operand (rows = co): lane needs Ds[8g+j][co]; B (cols = k): Xs[8g+j][k]
      const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int cb = wm * 32 + a * 16;
        const bf16x4 lo = tr_read((const bf16_t*)Ds + (u * BK + 8 * g + q) * WG_LD + cb + 4 * p);
        const bf16x4 hi = tr_read((const bf16_t*)Ds + (u * BK + 8 * g + 4 + q) * WG_LD + cb + 4 * p);
        bf16x8 fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int kb = wn * 32 + b * 16;
          const bf16x4 l2 = tr_read((const bf16_t*)Xs + (u * BK + 8 * g + q) * WG_LD + kb + 4 * p);
          const bf16x4 h2 = tr_read((const bf16_t*)Xs + (u * BK + 8 * g + 4 + q) * WG_LD + kb + 4 * p);
          bf16x8 fb = {l2[0], l2[1], l2[2], l2[3], h2[0], h2[1], h2[2], h2[3]};
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[a][b], 0, 0, 0);
        }
      }
    } else {
      // f32 16x16x4: lane l contributes A[i=l&15][k=l>>4] = Ds[kk*4 + (l>>4)][co]
      const int i = lane & 15, q = lane >> 4;
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        const int mr = u * BK + kk * 4 + q;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const float av = ((const float*)Ds)[mr * WG_LD + wm * 32 + a * 16 + i];
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const float bv = ((const float*)Xs)[mr * WG_LD + wn * 32 + b * 16 + i];
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[a][b], 0, 0, 0);
          }
        }
      }
    }
  }
  // write the partial tile: rows co, cols k
  float* out = part + (long)split * Cout * K;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int k = k0 + wn * 32 + b * 16 + (lane & 15);
      if (k >= K) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 32 + a * 16 + (lane >> 4) * 4 + r;
        if (co < Cout) out[(long)co * K + k] = acc[a][b][r];
      }
    }
}

// =====================================================================================
// stem weight gradient (3x3 / stride 1 / SAME, Cin = 3, Cout = 32, bf16):
// part[blk][co][k] = sum over the block's pixels of dy[px, co] * im2col[px, k], k = 27 taps.
// A block owns 128 consecutive pixels of one image row for RB image rows.  Per row, each
// thread loads 32 bytes of dy (one pixel, 16 channels) and gathers its 16 taps of that
// pixel's 3x3x3 patch (contiguous 9-element runs of the three input rows; SAME padding
// and x >= W read as zero), so the [128][32] dy tile and the [128][32] im2col tile (taps
// 27..31 zero) are built in LDS with one 16-byte store per 8 values; the next row's loads
// are issued before the MFMAs of the current one.  Wave w contracts pixels [32w, 32w+32)
// with 2 x 2 16x16x32 bf16 MFMAs (co tiles x tap tiles, operands read transposed with
// ds_read_b64_tr_b16 as in conv_wgrad_kernel); the four waves' tiles are summed in LDS in
// a fixed order and the block writes its 32 x 27 partial (summed by slab_sum).
// =====================================================================================

struct StemWgradPlan {
  int xb, yb, rb, nblk;
};
static StemWgradPlan stem_wgrad_plan(int N, int H, int W) {
  StemWgradPlan p;
  p.xb = cdiv(W, SW_TW);
  const long segs = (long)N * H * p.xb;
  p.rb = (int)std::max<long>(1, cdivl(segs, 2048));  // <= ~2048 partials
  p.yb = cdiv(H, p.rb);
  p.nblk = N * p.yb * p.xb;
  return p;
}

// BNB: dy is not read but formed in the loader from the stem BatchNorm's (dz, y) — the apply of
// rod_bn_bwd_apply (bn_bwd_apply1, rounded to bf16), so dy never crosses HBM (rod_stem_wgrad_bn)
struct StemBnb {
  const bf16_t* dz;
  const bf16_t* y;
  const float *mean, *rstd, *gamma, *beta, *coef;
  int act;
};
template <bool BNB>
__global__ void __launch_bounds__(256) stem_wgrad_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ DY,
                                                         float* __restrict__ part, int H, int W, int ldx, int lddy,
                                                         int rb, StemBnb bb) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * SW_TW * SW_LD];  // Ds [px][co] | Xs [px][tap]
  bf16_t* Ds = lds;
  bf16_t* Xs = lds + SW_TW * SW_LD;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int x0 = blockIdx.x * SW_TW;
  const int n = blockIdx.z;
  const int ya = blockIdx.y * rb;
  const int yz = ya + rb < H ? ya + rb : H;
  // dy loader: pixel + 16-channel half (BNB: pixels px, px + 64 and a fixed 8-channel chunk, so
  // the chunk's BatchNorm-backward constants stay in registers)
  const int px = BNB ? tid >> 2 : tid >> 1, half = tid & 1, ck = tid & 3;
  const int xx = x0 + px;
  const bool inx = xx < W, inx2 = xx + 64 < W;
  const int pg = tid & 127, hg = tid >> 7;  // gather: pixel, wave-uniform tap half
  float sc[BNB ? 8 : 1], sh[BNB ? 8 : 1], ca[BNB ? 8 : 1], k1[BNB ? 8 : 1], k0[BNB ? 8 : 1];
  float ghi = 0.f, glo = 0.f;
  if constexpr (BNB) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = ck * 8 + e;
      bn_affine(bb.mean, bb.rstd, bb.gamma, bb.beta, c, sc[e], sh[e]);
      ca[e] = bb.coef[c];
      bn_bwd_k_fold(ca[e], bb.mean[c], bb.rstd[c], bb.coef[32 + c], bb.coef[64 + c], k1[e], k0[e]);
    }
    ghi = bb.act == ROD_ACT_RELU6 ? 6.f : INFINITY;
    glo = bb.act == ROD_ACT_LEAKY ? 0.2f : bb.act == ROD_ACT_NONE ? 1.f : 0.f;
  }
  auto apply = [&](const bf16x8& dzv, const bf16x8& yv) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float yj = (float)yv[e];
      const float z = fmaf(yj, sc[e], sh[e]);
      const float gj = (float)dzv[e] * (z > 0.f ? (z < ghi ? 1.f : 0.f) : glo);
      o[e] = (bf16_t)bn_bwd_apply1<bf16_t>(ca[e], gj, k1[e], k0[e], 0.f, yj);
    }
    return o;
  };

  bf16x8 d0, d1, y0, y1;
  unsigned short tv[16];
  const unsigned short* Xu = (const unsigned short*)X;
  auto load_row = [&](int y) {
#pragma unroll
    for (int j = 0; j < 8; ++j) d0[j] = d1[j] = y0[j] = y1[j] = (bf16_t)0.f;
    if constexpr (BNB) {   // (dz, y) of pixels xx and xx + 64, channels ck*8 .. +7
      const long r = ((long)n * H + y) * W;
      if (inx) {
        d0 = *(const bf16x8*)(bb.dz + (r + xx) * 32 + ck * 8);
        y0 = *(const bf16x8*)(bb.y + (r + xx) * 32 + ck * 8);
      }
      if (inx2) {
        d1 = *(const bf16x8*)(bb.dz + (r + xx + 64) * 32 + ck * 8);
        y1 = *(const bf16x8*)(bb.y + (r + xx + 64) * 32 + ck * 8);
      }
    } else if (inx) {
      const bf16_t* src = DY + (((long)n * H + y) * W + xx) * lddy + half * 16;
      d0 = *(const bf16x8*)src;
      d1 = *(const bf16x8*)(src + 8);
    }
    if (hg) stem_gather<1>(Xu, (long)n * H, y, x0 + pg, H, W, ldx, tv);
    else stem_gather<0>(Xu, (long)n * H, y, x0 + pg, H, W, ldx, tv);
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[a][b][r] = 0.f;

  if (ya < yz) load_row(ya);
  for (int y = ya; y < yz; ++y) {
    __syncthreads();
    if constexpr (BNB) {   // pixels past W: dy 0 (the apply of zeros is not 0)
      bf16x8 z8;
#pragma unroll
      for (int j = 0; j < 8; ++j) z8[j] = (bf16_t)0.f;
      *(bf16x8*)(Ds + px * SW_LD + ck * 8) = inx ? apply(d0, y0) : z8;
      *(bf16x8*)(Ds + (px + 64) * SW_LD + ck * 8) = inx2 ? apply(d1, y1) : z8;
    } else {
      *(bf16x8*)(Ds + px * SW_LD + half * 16) = d0;
      *(bf16x8*)(Ds + px * SW_LD + half * 16 + 8) = d1;
    }
    {
      typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
      u16x8 t0, t1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        t0[j] = tv[j];
        t1[j] = tv[8 + j];
      }
      *(u16x8*)(Xs + pg * SW_LD + hg * 16) = t0;
      *(u16x8*)(Xs + pg * SW_LD + hg * 16 + 8) = t1;
    }
    __syncthreads();
    if (y + 1 < yz) load_row(y + 1);
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int m0 = wave * 32;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const bf16x4 lo = tr_read(Ds + (m0 + 8 * g + q) * SW_LD + a * 16 + 4 * p);
      const bf16x4 hi = tr_read(Ds + (m0 + 8 * g + 4 + q) * SW_LD + a * 16 + 4 * p);
      bf16x8 fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const bf16x4 l2 = tr_read(Xs + (m0 + 8 * g + q) * SW_LD + b * 16 + 4 * p);
        const bf16x4 h2 = tr_read(Xs + (m0 + 8 * g + 4 + q) * SW_LD + b * 16 + 4 * p);
        bf16x8 fb = {l2[0], l2[1], l2[2], l2[3], h2[0], h2[1], h2[2], h2[3]};
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[a][b], 0, 0, 0);
      }
    }
  }
  // fixed-order sum of the four waves' 32 x 32 tiles: red[wave][co][tap]
  __syncthreads();
  float* red = (float*)lds;  // 4 * 32 * 32 floats = 16 KB <= 20 KB
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = a * 16 + (lane >> 4) * 4 + r, k = b * 16 + (lane & 15);
        red[(wave * 32 + co) * 32 + k] = acc[a][b][r];
      }
  __syncthreads();
  const long blk = ((long)n * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  float* out = part + blk * 32 * 27;
  for (int e = tid; e < 32 * 27; e += 256) {
    const int co = e / 27, k = e - co * 27;
    float s = red[co * 32 + k];
    s += red[(32 + co) * 32 + k];
    s += red[(64 + co) * 32 + k];
    s += red[(96 + co) * 32 + k];
    out[e] = s;
  }
}

__global__ void split_reduce_kernel(const float* __restrict__ part, float* __restrict__ out, int splits, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int b = 0; b < splits; ++b) s += part[(long)b * n + i];
  out[i] = s;
}

// column sums of dy[M, C] (row stride ld): slab [nblk][C] then reduce
// (bias gradients of the head convs, whose C is 24..36: all 256 threads work — 256 / C row
// lanes per column, four independent chains per lane, lanes added in a fixed order)
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ dy, long M, int C, int ld, long chunk,
                                                     float* __restrict__ slab) {
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const int CB = C < 256 ? C : 256;
  const int lanes = 256 / CB;
  const int cl = tid % CB, ln = tid / CB;
  const int c = blockIdx.y * 256 + cl;
  const long r0 = (long)blockIdx.x * chunk;
  const long r1 = r0 + chunk < M ? r0 + chunk : M;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (ln < lanes && c < C) {
    long r = r0 + ln;
    for (; r + 3L * lanes < r1; r += 4L * lanes) {
      s0 += to_f32(dy[r * ld + c]);
      s1 += to_f32(dy[(r + lanes) * ld + c]);
      s2 += to_f32(dy[(r + 2L * lanes) * ld + c]);
      s3 += to_f32(dy[(r + 3L * lanes) * ld + c]);
    }
    for (; r < r1; r += lanes) s0 += to_f32(dy[r * ld + c]);
  }
  red[tid] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ln == 0 && c < C) {
    float t = 0.f;
    for (int l = 0; l < lanes; ++l) t += red[l * CB + cl];
    slab[(long)blockIdx.x * C + c] = t;
  }
}

template <typename T>
__global__ void weight_prep_kernel(const float* __restrict__ w, T* __restrict__ wt, int Cout, int Cin, int ks,
                                   int mode) {
  const long n = (long)Cout * ks * ks * Cin;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  if (mode == 0) {
    wt[idx] = from_f32<T>(w[idx]);
    return;
  }
  // destination index -> [ci][i][j][co]
  const int co = (int)(idx % Cout);
  long t = idx / Cout;
  const int j = (int)(t % ks);
  t /= ks;
  const int i = (int)(t % ks);
  const int ci = (int)(t / ks);
  const int si = ks - 1 - i, sj = ks - 1 - j;
  wt[idx] = from_f32<T>(w[(((long)co * ks + si) * ks + sj) * Cin + ci]);
}

// batched weight_prep: one launch over the concatenated element ranges of every table entry
struct PrepEntry {
  const float* w;
  void* wt;
  long start;
  int Cout, Cin, ksize, mode;
};
static_assert(sizeof(PrepEntry) == 40, "rod_prep_entry layout");

template <typename T>
__global__ void __launch_bounds__(256) weight_prep_batch_kernel(const PrepEntry* __restrict__ tab, int n, long total) {
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    int lo = 0, hi = n - 1;  // last entry with start <= idx
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tab[mid].start <= idx) lo = mid;
      else hi = mid - 1;
    }
    const PrepEntry e = tab[lo];
    const long i = idx - e.start;
    T* wt = (T*)e.wt;
    if (e.mode == 0) {
      wt[i] = from_f32<T>(e.w[i]);
      continue;
    }
    const int co = (int)(i % e.Cout);
    long t = i / e.Cout;
    const int j = (int)(t % e.ksize);
    t /= e.ksize;
    const int ii = (int)(t % e.ksize);
    const int ci = (int)(t / e.ksize);
    wt[i] = from_f32<T>(e.w[(((long)co * e.ksize + (e.ksize - 1 - ii)) * e.ksize + (e.ksize - 1 - j)) * e.Cin + ci]);
  }
}

struct WgradPlan {
  int ctiles, ktiles, splits;
  long chunk;
};
static WgradPlan wgrad_plan(long M, int Cin, int Cout, int ks) {
  WgradPlan p;
  const int K = ks * ks * Cin;
  p.ctiles = cdiv(Cout, WG_T);
  p.ktiles = cdiv(K, WG_T);
  const int tiles = p.ctiles * p.ktiles;
  // measurement switches: ROD_WG_TARGET (blocks, 2048), ROD_WG_MINROWS (rows per split, 128:
  // the heads' small-map 3x3 convs walk 2 row steps per block instead of 8; bench 384.6 (512)
  // -> 386.9 img/s, 64 rows 386.1)
  static const long wg_target = getenv("ROD_WG_TARGET") ? atol(getenv("ROD_WG_TARGET")) : 2048;
  static const long wg_minrows = getenv("ROD_WG_MINROWS") ? atol(getenv("ROD_WG_MINROWS")) : 128;
  long splits = std::max<long>(1, std::min<long>(cdivl(wg_target, tiles), cdivl(M, wg_minrows)));
  long chunk = cdivl(M, splits);
  chunk = cdivl(chunk, BK) * BK;
  p.chunk = chunk;
  p.splits = (int)cdivl(M, chunk);
  // several tiles share each row split: a multiple of 8 splits lets the kernel keep them on
  // one XCD (splits past M are empty and write zero partials)
  if (tiles > 1 && p.splits >= 8) p.splits = (p.splits + 7) / 8 * 8;
  return p;
}

template <typename T>
static bool aligned16(const void* p) {
  return ((uintptr_t)p & 15) == 0;
}

// `pro` (nullable): BatchNorm-apply prologue on the A operand; its table takes 8*Cin bytes of
// dynamic LDS.
template <typename T, int KS, int BN, bool VA, bool VB, bool VY, bool PRO, int BKT = BK>
static void conv_fwd_launch(const void* x, const void* wt, const float* bias, void* y, long M, int H, int W, int Cin,
                            int Cout, int ldx, int ldy, float* stats, const BnPro& pro, const BnGred* gr,
                            hipStream_t s, const BnEpi* ep = nullptr, const BnBwd* bw = nullptr) {
  dim3 grid(cdivl(M, 128), cdiv(Cout, BN));
  if (grid.y > 1) grid.x = (grid.x + 7) / 8 * 8;  // XCD-aware N-tile order (see the kernel)
  const size_t lds = PRO ? 8 * (size_t)Cin : 0;
  if constexpr (sizeof(T) == 2 && BKT == BK && KS == 1 && !PRO && VA) {   // the backward-data BatchNorm prologue
    if (bw) {
      hipLaunchKernelGGL((conv_fwd_kernel<T, KS, BN, VA, VB, VY, false, false, false, false, BKT, false, true>), grid,
                         dim3(256), (size_t)Cin * BWD_CF * sizeof(float), s, (const T*)x, (const T*)wt, bias, (T*)y, M,
                         H, W, Cin, Cout, ldx, ldy, nullptr, 0, pro, BnGred{}, BnEpi{}, *bw);
      return;
    }
  }
  if constexpr (sizeof(T) == 2 && BKT == BK) {   // the inference BatchNorm-apply epilogue (bf16)
    if (ep) {
      hipLaunchKernelGGL((conv_fwd_kernel<T, KS, BN, VA, VB, VY, false, false, PRO, false, BKT, true>), grid,
                         dim3(256), lds, s, (const T*)x, (const T*)wt, bias, (T*)y, M, H, W, Cin, Cout, ldx, ldy,
                         nullptr, 0, pro, BnGred{}, *ep);
      return;
    }
  }
  if constexpr (VY) {
    if (gr) {
      hipLaunchKernelGGL((conv_fwd_kernel<T, KS, BN, VA, VB, VY, false, false, PRO, true, BKT>), grid, dim3(256), lds, s,
                         (const T*)x, (const T*)wt, bias, (T*)y, M, H, W, Cin, Cout, ldx, ldy, nullptr, 0, pro, *gr);
      return;
    }
    if (stats) {
      hipLaunchKernelGGL((conv_fwd_kernel<T, KS, BN, VA, VB, VY, false, true, PRO, false, BKT>), grid, dim3(256), lds, s,
                         (const T*)x, (const T*)wt, bias, (T*)y, M, H, W, Cin, Cout, ldx, ldy, stats, 0, pro);
      return;
    }
  }
  hipLaunchKernelGGL((conv_fwd_kernel<T, KS, BN, VA, VB, VY, false, false, PRO, false, BKT>), grid, dim3(256), lds, s,
                     (const T*)x, (const T*)wt, bias, (T*)y, M, H, W, Cin, Cout, ldx, ldy, nullptr, 0, pro);
}

// k depth 64 with double-buffered LDS (bf16) for the 3x3 convs with K % 64 == 0 and a 97..128-wide
// N tile (the heads' 128 -> 128 3x3), ROD_GEMM_BK64=1 (2: also the 1x1 convs with K >= 256).  Off
// by default: measured no faster at b = 8 (87.5 vs 87.1 us) and slower at b = 32 (217 vs 185 us per
// call): 184 VGPRs and 74 KB of LDS drop the kernel from 3 to 2 waves per SIMD.
static int bk64_mode() {
  static const int m = [] {
    const char* e = getenv("ROD_GEMM_BK64");
    return e ? atoi(e) : 0;
  }();
  return m;
}

// N tile: the whole of Cout in one tile up to 256 (A is read once), else 128-wide tiles.
// The fully vectorisable case (16-byte A, B and Y rows) gets the full tile menu and the
// LDS-staged epilogue; the rest (stem Cin=3, odd strides) the 32/64/128 direct-store kernel
// (with a prologue: the 128-wide one only).
template <typename T, int KS, bool PRO>
static void conv_fwd_dispatch(bool va, bool vb, bool vy, const void* x, const void* wt, const float* bias, void* y,
                              long M, int H, int W, int Cin, int Cout, int ldx, int ldy, float* stats,
                              const BnPro& pro, const BnGred* gr, hipStream_t s, const BnEpi* ep = nullptr,
                              const BnBwd* bw = nullptr) {
#define CF(BN_, VA_, VB_, VY_) \
  conv_fwd_launch<T, KS, BN_, VA_, VB_, VY_, PRO>(x, wt, bias, y, M, H, W, Cin, Cout, ldx, ldy, stats, pro, gr, s, ep, bw)
  if (va && vb && vy) {
    if constexpr (sizeof(T) == 2) {
      const int K = KS * KS * Cin;
      const int mode = bk64_mode();
      if (!ep && !bw && mode > 0 && K % 64 == 0 && Cout > 96 && Cout <= 128 && (KS == 3 || (mode > 1 && K >= 256))) {
        conv_fwd_launch<T, KS, 128, true, true, true, PRO, 64>(x, wt, bias, y, M, H, W, Cin, Cout, ldx, ldy, stats,
                                                                pro, gr, s);
        return;
      }
    }
    if (Cout <= 32) CF(32, true, true, true);
    else if (Cout <= 64) CF(64, true, true, true);
    else if (Cout <= 96) CF(96, true, true, true);
    else if (Cout <= 128) CF(128, true, true, true);
    else if (Cout <= 160) CF(160, true, true, true);
    else if (Cout <= 192) CF(192, true, true, true);
    else if (Cout <= 256) CF(256, true, true, true);
    else CF(128, true, true, true);
    return;
  }
  // direct-store epilogue (Cout or ldy not a multiple of 8: the heads' last convs, 4 / 11 x
  // anchors channels): the N tile is the smallest of 32 / 64 / 96 / 128 covering Cout (a 128-wide
  // tile for 36 or 66 outputs wasted half the MFMAs and B loads); B rows load in G-element
  // pieces (VB false), which also covers the aligned case at two 8-byte loads per chunk
  if (Cout <= 32) {
    if (va) CF(32, true, false, false); else CF(32, false, false, false);
  } else if (Cout <= 64) {
    if (va) CF(64, true, false, false); else CF(64, false, false, false);
  } else if (Cout <= 96) {
    if (va) CF(96, true, false, false); else CF(96, false, false, false);
  } else {
    if (va) CF(128, true, false, false); else CF(128, false, false, false);
  }
#undef CF
}

template <typename T, int KS, bool PRO, bool VA, bool VB>
static void conv_fwd_split_t(const SplitPlan& p, const void* x, const void* wt, float* part, long M, int H, int W,
                             int Cin, int Cout, int ldx, const BnPro& pro, hipStream_t s, const BnBwd* bw = nullptr) {
  dim3 grid(cdivl(M, 128), cdiv(Cout, 128), p.splits);
  const size_t lds = PRO ? 8 * (size_t)Cin : 0;
  if constexpr (sizeof(T) == 2 && KS == 1 && !PRO && VA) {
    if (bw) {
      hipLaunchKernelGGL((conv_fwd_kernel<T, KS, 128, VA, VB, false, true, false, false, false, BK, false, true>), grid,
                         dim3(256), (size_t)Cin * BWD_CF * sizeof(float), s, (const T*)x, (const T*)wt, nullptr,
                         nullptr, M, H, W, Cin, Cout, ldx, 0, part, p.kper, pro, BnGred{}, BnEpi{}, *bw);
      return;
    }
  }
  hipLaunchKernelGGL((conv_fwd_kernel<T, KS, 128, VA, VB, false, true, false, PRO>), grid, dim3(256), lds, s,
                     (const T*)x, (const T*)wt, nullptr, nullptr, M, H, W, Cin, Cout, ldx, 0, part, p.kper, pro);
}
// split-K over the k-steps (small maps with a deep K).  The non-vector operand paths (the heads'
// last 3x3 convs, Cin % 8 != 0 on 3x5 .. 23x40 maps) split too: one 128-row tile per image level
// would otherwise walk all of K in a single workgroup (~50 us of load latency).
template <typename T, int KS, bool PRO>
static void conv_fwd_split(bool va, bool vb, const SplitPlan& p, const void* x, const void* wt, float* part, long M,
                           int H, int W, int Cin, int Cout, int ldx, const BnPro& pro, hipStream_t s,
                           const BnBwd* bw = nullptr) {
  if (va && vb) conv_fwd_split_t<T, KS, PRO, true, true>(p, x, wt, part, M, H, W, Cin, Cout, ldx, pro, s, bw);
  else if (va) conv_fwd_split_t<T, KS, PRO, true, false>(p, x, wt, part, M, H, W, Cin, Cout, ldx, pro, s, bw);
  else if (vb) conv_fwd_split_t<T, KS, PRO, false, true>(p, x, wt, part, M, H, W, Cin, Cout, ldx, pro, s);
  else conv_fwd_split_t<T, KS, PRO, false, false>(p, x, wt, part, M, H, W, Cin, Cout, ldx, pro, s);
}

template <typename T>
static void conv_fwd_typed(const void* x, const BnPro* pro, const void* wt, const float* bias, void* y, void* ws,
                           float* stats, const BnGred* gr, int N, int H, int W, int Cin, int Cout, int ksize, int ldx,
                           int ldy, hipStream_t s, const BnEpi* ep = nullptr, const BnBwd* bw = nullptr) {
  const long M = (long)N * H * W;
  const int K = ksize * ksize * Cin;
  const int eV = Vec16<T>::N;
  const bool va = aligned16<T>(x) && (ldx % eV == 0) && (ksize == 1 ? true : (Cin % 8 == 0));
  const bool vb = aligned16<T>(wt) && (K % eV == 0);
  const bool vy = aligned16<T>(y) && (ldy % eV == 0);
  const SplitPlan sp = split_plan(M, Cout, K);
  const int nparts = (int)cdivl(M, 128);
  const int dt = sizeof(T) == 4 ? ROD_F32 : ROD_BF16;
  const BnPro pv = pro ? *pro : BnPro{};
  static const bool old_stem_fwd = getenv("ROD_DEBUG_OLDSTEMFWD") != nullptr;  // A/B against the VALU kernel
  if constexpr (sizeof(T) == 2) {
    if (!pro && !gr && !ep && !bw && ksize == 3 && Cin == 3 && Cout == 32 && vy && !old_stem_fwd) {
      const bool fuse = stats != nullptr && W % SW_TW == 0;  // block == stat tile
      // rows per block: >= ~4 blocks' worth per CU of rows, pipelined within a block
      const int xb = cdiv(W, SW_TW);
      const int rb = (int)std::max<long>(1, std::min<long>(8, (long)N * H * xb / 8192));
      const dim3 grid(xb, cdiv(H, rb), N);
      if (fuse)
        hipLaunchKernelGGL(stem_fwd_mfma_kernel<true>, grid, dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)wt,
                           bias, (bf16_t*)y, stats, H, W, ldx, ldy, rb);
      else
        hipLaunchKernelGGL(stem_fwd_mfma_kernel<false>, grid, dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)wt,
                           bias, (bf16_t*)y, nullptr, H, W, ldx, ldy, rb);
      if (stats && !fuse) stat_parts(dt, y, M, Cout, ldy, stats, nparts, s);
      return;
    }
  }
  if (ws != nullptr && sp.splits > 1 && !(ksize == 3 && Cin == 3)) {
    float* part = (float*)ws;
    if (ksize == 1) {
      if (pro) conv_fwd_split<T, 1, true>(va, vb, sp, x, wt, part, M, H, W, Cin, Cout, ldx, pv, s);
      else conv_fwd_split<T, 1, false>(va, vb, sp, x, wt, part, M, H, W, Cin, Cout, ldx, pv, s, bw);
    } else {
      if (pro) conv_fwd_split<T, 3, true>(va, vb, sp, x, wt, part, M, H, W, Cin, Cout, ldx, pv, s);
      else conv_fwd_split<T, 3, false>(va, vb, sp, x, wt, part, M, H, W, Cin, Cout, ldx, pv, s);
    }
    if (ep)
      hipLaunchKernelGGL((splitk_combine_kernel<T, true>), dim3(cdivl(M * Cout, 256)), dim3(256), 0, s,
                         (const float*)part, bias, (T*)y, M, Cout, ldy, sp.splits, *ep);
    else
      hipLaunchKernelGGL(splitk_combine_kernel<T>, dim3(cdivl(M * Cout, 256)), dim3(256), 0, s, (const float*)part,
                         bias, (T*)y, M, Cout, ldy, sp.splits);
    if (stats) stat_parts(dt, y, M, Cout, ldy, stats, nparts, s);
    if (gr) gred_parts(dt, y, gr->y, gr->p, M, Cout, gr->parts, nparts, s);
    return;
  }
  if ((stats || gr) && !(va && vb && vy)) {  // no fused epilogue on this path: separate pass
    conv_fwd_typed<T>(x, pro, wt, bias, y, ws, nullptr, nullptr, N, H, W, Cin, Cout, ksize, ldx, ldy, s);
    if (stats) stat_parts(dt, y, M, Cout, ldy, stats, nparts, s);
    if (gr) gred_parts(dt, y, gr->y, gr->p, M, Cout, gr->parts, nparts, s);
    return;
  }
  static const bool no_stem = getenv("ROD_DEBUG_NOSTEM") != nullptr;  // debug bisection
  if (!pro && !gr && !ep && ksize == 3 && Cin == 3 && (Cout == 32 || Cout == 64) && vy && !no_stem) {
    if (Cout == 32)
      hipLaunchKernelGGL((stem_conv_fwd_kernel<T, 32>), dim3(cdiv(W, 128), H, N), dim3(256), 0, s, (const T*)x,
                         (const T*)wt, bias, (T*)y, H, W, ldx, ldy);
    else
      hipLaunchKernelGGL((stem_conv_fwd_kernel<T, 64>), dim3(cdiv(W, 64), H, N), dim3(256), 0, s, (const T*)x,
                         (const T*)wt, bias, (T*)y, H, W, ldx, ldy);
    return;
  }
  if constexpr (sizeof(T) == 2) {
    if (!ep && !bw && !gr && pro && ksize == 1 && !bias && va && vb && vy && Cin <= PRO_MAXC &&
        pw_proj_launch((const bf16_t*)x, (const bf16_t*)wt, (bf16_t*)y, M, K, Cout, ldx, ldy, stats, s, pv))
      return;
    // the prologue form only for the block-to-block case it serves (K <= 32 input channels of a
    // project BatchNorm left pending: the 720p expand 16 -> 96)
    if (!ep && !bw && ksize == 1 && !bias && va && vb && vy && (!pro || (K <= 32 && Cin <= PRO_MAXC)) &&
        pw_stream_launch((const bf16_t*)x, (const bf16_t*)wt, (bf16_t*)y, M, K, Cout, ldx, ldy, stats, gr, s,
                         pro ? &pv : nullptr))
      return;
  }
  if (ksize == 1) {
    if (pro) conv_fwd_dispatch<T, 1, true>(va, vb, vy, x, wt, bias, y, M, H, W, Cin, Cout, ldx, ldy, stats, pv, gr, s, ep);
    else conv_fwd_dispatch<T, 1, false>(va, vb, vy, x, wt, bias, y, M, H, W, Cin, Cout, ldx, ldy, stats, pv, gr, s, ep,
                                        bw);
  } else {
    if (pro) conv_fwd_dispatch<T, 3, true>(va, vb, vy, x, wt, bias, y, M, H, W, Cin, Cout, ldx, ldy, stats, pv, gr, s, ep);
    else conv_fwd_dispatch<T, 3, false>(va, vb, vy, x, wt, bias, y, M, H, W, Cin, Cout, ldx, ldy, stats, pv, gr, s, ep);
  }
}

template <typename T, int KS, bool VA, bool VD, bool PRO>
static void wgrad_launch(const WgradPlan& p, const void* x, const void* dy, float* part, long M, int H, int W,
                         int Cin, int Cout, int ldx, int lddy, const BnPro& pro, hipStream_t s) {
  dim3 grid(p.ctiles * p.ktiles, p.splits);
  const size_t lds = PRO ? 8 * (size_t)Cin : 0;
  hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, VA, VD, 0, PRO>), grid, dim3(256), lds, s, (const T*)x, (const T*)dy,
                     part, M, H, W, Cin, Cout, ldx, lddy, p.chunk, p.ktiles, pro);
}

template <typename T, int KS, bool PRO>
static void wgrad_va_vd(bool va, bool vd, const WgradPlan& p, const void* x, const void* dy, float* part, long M,
                        int H, int W, int Cin, int Cout, int ldx, int lddy, const BnPro& pro, hipStream_t s) {
  if (va && vd) wgrad_launch<T, KS, true, true, PRO>(p, x, dy, part, M, H, W, Cin, Cout, ldx, lddy, pro, s);
  else if (va) wgrad_launch<T, KS, true, false, PRO>(p, x, dy, part, M, H, W, Cin, Cout, ldx, lddy, pro, s);
  else if (vd) wgrad_launch<T, KS, false, true, PRO>(p, x, dy, part, M, H, W, Cin, Cout, ldx, lddy, pro, s);
  else wgrad_launch<T, KS, false, false, PRO>(p, x, dy, part, M, H, W, Cin, Cout, ldx, lddy, pro, s);
}

// workspace layout: [weight-gradient partials][bias column-sum partials].  Separate regions:
// while rod_slab_defer is on, the weight partials are summed only at rod_slab_flush, after the
// bias partials have been written.
static long wgrad_part_floats(int N, int H, int W, int Cin, int Cout, int ksize) {
  const long M = (long)N * H * W;
  WgradPlan p = wgrad_plan(M, Cin, Cout, ksize);
  const long K = (long)ksize * ksize * Cin;
  if (ksize == 3 && Cin == 3 && Cout == 32) p.splits = std::max(p.splits, stem_wgrad_plan(N, H, W).nblk);
  return ((long)p.splits * Cout * K + 3) / 4 * 4;
}

template <typename T>
static void wgrad_typed(const void* x, const BnPro* pro, const void* dy, float* dw, float* db, float* part, int N,
                        int H, int W, int Cin, int Cout, int ksize, int ldx, int lddy, hipStream_t s) {
  const long M = (long)N * H * W;
  const long K = (long)ksize * ksize * Cin;
  WgradPlan p = wgrad_plan(M, Cin, Cout, ksize);
  const int eV = Vec16<T>::N;
  const bool va = aligned16<T>(x) && (ldx % eV == 0) && (ksize == 1 ? true : (Cin % 8 == 0));
  const bool vd = aligned16<T>(dy) && (lddy % eV == 0);
  const BnPro pv = pro ? *pro : BnPro{};
  static const bool old_stem = getenv("ROD_DEBUG_OLDSTEMWG") != nullptr;  // A/B against the generic kernel
  bool stem = false;
  if constexpr (sizeof(T) == 2) {
    if (!pro && ksize == 3 && Cin == 3 && Cout == 32 && vd && !old_stem) {
      const StemWgradPlan sp = stem_wgrad_plan(N, H, W);
      hipLaunchKernelGGL(stem_wgrad_kernel<false>, dim3(sp.xb, sp.yb, N), dim3(256), 0, s, (const bf16_t*)x,
                         (const bf16_t*)dy, part, H, W, ldx, lddy, sp.rb, StemBnb{});
      p.splits = sp.nblk;
      stem = true;
    }
  }
  if (stem) {
  } else if (!pro && ksize == 3 && Cin == 3 && vd) {
    dim3 grid(p.ctiles * p.ktiles, p.splits);
    hipLaunchKernelGGL((conv_wgrad_kernel<T, 3, false, true, 3>), grid, dim3(256), 0, s, (const T*)x, (const T*)dy,
                       part, M, H, W, Cin, Cout, ldx, lddy, p.chunk, p.ktiles, pv);
  } else if (ksize == 1) {
    if (pro) wgrad_va_vd<T, 1, true>(va, vd, p, x, dy, part, M, H, W, Cin, Cout, ldx, lddy, pv, s);
    else wgrad_va_vd<T, 1, false>(va, vd, p, x, dy, part, M, H, W, Cin, Cout, ldx, lddy, pv, s);
  } else {
    if (pro) wgrad_va_vd<T, 3, true>(va, vd, p, x, dy, part, M, H, W, Cin, Cout, ldx, lddy, pv, s);
    else wgrad_va_vd<T, 3, false>(va, vd, p, x, dy, part, M, H, W, Cin, Cout, ldx, lddy, pv, s);
  }
  const long n = (long)Cout * K;
  slab_sum(part, dw, p.splits, n, s);
  if (db) {
    long cchunk = std::max<long>(64, cdivl(M, 512));
    int nb = (int)cdivl(M, cchunk);
    float* partb = part + wgrad_part_floats(N, H, W, Cin, Cout, ksize);
    hipLaunchKernelGGL(colsum_kernel<T>, dim3(nb, cdiv(Cout, 256)), dim3(256), 0, s, (const T*)dy, M, Cout, lddy,
                       cchunk, partb);
    slab_sum(partb, db, nb, (long)Cout, s);
  }
}

}  // namespace rod

using namespace rod;

extern "C" {

int rod_conv_fwd_stream_ok(long M, int K, int Cout, int dtype) {
  int nt = 0;
  return dtype == ROD_BF16 && pw_stream_groups(M, K, Cout, nt) > 0 ? 1 : 0;
}

size_t rod_conv_fwd_workspace(int N, int H, int W, int Cin, int Cout, int ksize) {
  const long M = (long)N * H * W;
  const SplitPlan p = split_plan(M, Cout, ksize * ksize * Cin);
  return p.splits > 1 ? (size_t)p.splits * M * Cout * sizeof(float) : 0;
}

int rod_conv_fwd(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                 const float* pro_beta, int pro_act, const void* wt, const float* bias, void* y, void* workspace,
                 float* stat_parts, const void* gred_y, const float* gred_mean, const float* gred_rstd,
                 const float* gred_gamma, const float* gred_beta, int gred_act, float* gred_parts, int N, int H, int W,
                 int Cin, int Cout, int ksize, int ldx, int ldy, int dtype, void* stream) {
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0, "rod_conv_fwd: bad shape");
  ROD_CHECK_ARG(ksize == 1 || ksize == 3, "rod_conv_fwd: ksize must be 1 or 3");
  if (ldx == 0) ldx = Cin;
  if (ldy == 0) ldy = Cout;
  ROD_CHECK_ARG(ldx >= Cin && ldy >= Cout, "rod_conv_fwd: leading dim too small");
  ROD_CHECK_ARG(!pro_mean || (pro_rstd && Cin <= PRO_MAXC), "rod_conv_fwd: bad BatchNorm prologue (Cin %d)", Cin);
  ROD_CHECK_ARG(!gred_parts || (gred_y && gred_mean && gred_rstd && ldy == Cout && !stat_parts),
                "rod_conv_fwd: gred needs y, mean, rstd, a dense output and no stat_parts");
  const BnPro pro{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  const BnGred gr{gred_y, BnPro{gred_mean, gred_rstd, gred_gamma, gred_beta, gred_act}, gred_parts};
  ROD_DISPATCH_DTYPE(dtype, conv_fwd_typed<T>(x, pro_mean ? &pro : nullptr, wt, bias, y, workspace, stat_parts,
                                              gred_parts ? &gr : nullptr, N, H, W, Cin, Cout, ksize, ldx, ldy,
                                              ROD_STREAM(stream)));
  return check_launch("rod_conv_fwd");
}

int rod_conv_fwd_stats_supported(long M, int Cin, int Cout, int dtype) {
  int nt = 0;
  return dtype == ROD_BF16 && Cin <= 32 && pw_stream_groups(M, Cin, Cout, nt, false) > 0 ? 1 : 0;
}

int rod_conv_fwd_stats(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                       const float* pro_beta, int pro_act, const void* wt, float* stat_parts, long M, int Cin, int Cout,
                       int dtype, void* stream) {
  ROD_CHECK_ARG(rod_conv_fwd_stats_supported(M, Cin, Cout, dtype),
                "rod_conv_fwd_stats: unsupported M=%ld Cin=%d Cout=%d dtype=%d", M, Cin, Cout, dtype);
  ROD_CHECK_ARG(x && wt && stat_parts, "rod_conv_fwd_stats: NULL argument");
  ROD_CHECK_ARG(!pro_mean || pro_rstd, "rod_conv_fwd_stats: bad BatchNorm prologue");
  ROD_CHECK_ARG(((((uintptr_t)x) | ((uintptr_t)wt)) & 15) == 0, "rod_conv_fwd_stats: x, wt must be 16-byte aligned");
  const BnPro pro{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  if (!pw_stream_launch((const bf16_t*)x, (const bf16_t*)wt, nullptr, M, Cin, Cout, Cin, Cout, stat_parts, nullptr,
                        ROD_STREAM(stream), pro_mean ? &pro : nullptr)) {
    set_error("rod_conv_fwd_stats: no statistics-only plan for M=%ld Cin=%d Cout=%d", M, Cin, Cout);
    return ROD_EINVAL;
  }
  return check_launch("rod_conv_fwd_stats");
}

int rod_conv_fwd_bnact(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                       const float* pro_beta, int pro_act, const void* wt, const float* bias, void* z, void* workspace,
                       const float* bn_mean, const float* bn_rstd, const float* bn_gamma, const float* bn_beta,
                       int bn_act, const void* res, int ldr, int N, int H, int W, int Cin, int Cout, int ksize,
                       int ldx, int ldy, int dtype, void* stream) {
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0, "rod_conv_fwd_bnact: bad shape");
  ROD_CHECK_ARG(ksize == 1 || ksize == 3, "rod_conv_fwd_bnact: ksize must be 1 or 3");
  ROD_CHECK_ARG(dtype == ROD_BF16, "rod_conv_fwd_bnact: bf16 only (dtype %d)", dtype);
  ROD_CHECK_ARG(bn_mean && bn_rstd && z, "rod_conv_fwd_bnact: BatchNorm mean / rstd and the output required");
  ROD_CHECK_ARG(bn_act >= ROD_ACT_NONE && bn_act <= ROD_ACT_RELU, "rod_conv_fwd_bnact: bad act %d", bn_act);
  if (ldx == 0) ldx = Cin;
  if (ldy == 0) ldy = Cout;
  if (ldr == 0) ldr = Cout;
  ROD_CHECK_ARG(ldx >= Cin && ldy >= Cout && (!res || ldr >= Cout), "rod_conv_fwd_bnact: leading dim too small");
  ROD_CHECK_ARG(!res || (((uintptr_t)res & 15) == 0 && ldr % 8 == 0), "rod_conv_fwd_bnact: res 16-byte rows");
  ROD_CHECK_ARG(!pro_mean || (pro_rstd && Cin <= PRO_MAXC), "rod_conv_fwd_bnact: bad BatchNorm prologue (Cin %d)", Cin);
  const BnPro pro{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  const BnEpi ep{bn_mean, bn_rstd, bn_gamma, bn_beta, res, ldr, bn_act};
  conv_fwd_typed<bf16_t>(x, pro_mean ? &pro : nullptr, wt, bias, z, workspace, nullptr, nullptr, N, H, W, Cin, Cout,
                         ksize, ldx, ldy, ROD_STREAM(stream), &ep);
  return check_launch("rod_conv_fwd_bnact");
}

// The BWD loader's per-channel table takes Cout * BWD_CF floats of dynamic LDS beside the GEMM's
// static tiles (<= BWD_STATIC_LDS bytes for every tile configuration): the bound is the device's
// LDS per workgroup (160 KB on gfx950 -> Cout <= 4096), read once.
constexpr int BWD_STATIC_LDS = 32 * 1024;
static int bwd_data_bn_max_cout() {
  static int cached = -1;
  if (cached < 0) {
    int dev = 0, lds = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || lds <= 0)
      lds = 64 * 1024;   // no device (CPU-side query): the smallest LDS of any target
    cached = (lds - BWD_STATIC_LDS) / (BWD_CF * (int)sizeof(float)) / 8 * 8;
  }
  return cached;
}

int rod_conv_bwd_data_bn_supported(int Cout, int Cin, int dtype) {
  return dtype == ROD_BF16 && Cout % 8 == 0 && Cin % 8 == 0 && Cout > 0 && Cout <= bwd_data_bn_max_cout() ? 1 : 0;
}

int rod_conv_bwd_data_bn(const void* dz, const void* y, const float* mean, const float* rstd, const float* gamma,
                         const float* beta, int act, const float* coef, const void* wt1, void* dy, void* dx,
                         void* workspace, long M, int Cout, int Cin, int dtype, void* stream) {
  ROD_CHECK_ARG(M > 0 && rod_conv_bwd_data_bn_supported(Cout, Cin, dtype),
                "rod_conv_bwd_data_bn: unsupported M=%ld Cout=%d Cin=%d dtype=%d", M, Cout, Cin, dtype);
  ROD_CHECK_ARG(dz && y && mean && rstd && coef && wt1 && dy && dx, "rod_conv_bwd_data_bn: NULL argument");
  ROD_CHECK_ARG(act >= ROD_ACT_NONE && act <= ROD_ACT_RELU, "rod_conv_bwd_data_bn: bad act %d", act);
  ROD_CHECK_ARG(((((uintptr_t)dz) | ((uintptr_t)y) | ((uintptr_t)wt1) | ((uintptr_t)dy) | ((uintptr_t)dx)) & 15) == 0,
                "rod_conv_bwd_data_bn: tensors must be 16-byte aligned");
  ROD_CHECK_ARG(M <= 0x7fffffffL, "rod_conv_bwd_data_bn: M too large");
  const BnBwd bw{(const bf16_t*)y, mean, rstd, gamma, beta, coef, act, (bf16_t*)dy};
  // the GEMM dx[M][Cin] = dy[M][Cout] . wt1[Cin][Cout]^T: rod_conv_fwd's 1x1 form with K = Cout
  conv_fwd_typed<bf16_t>(dz, nullptr, wt1, nullptr, dx, workspace, nullptr, nullptr, 1, 1, (int)M, Cout, Cin, 1, Cout,
                         Cin, ROD_STREAM(stream), nullptr, &bw);
  return check_launch("rod_conv_bwd_data_bn");
}

int rod_conv_weight_prep(const float* w, void* wt, int Cout, int Cin, int ksize, int mode, int dtype,
                         void* stream) {
  ROD_CHECK_ARG(Cout > 0 && Cin > 0 && (ksize == 1 || ksize == 3), "rod_conv_weight_prep: bad shape");
  ROD_CHECK_ARG(mode == 0 || mode == 1, "rod_conv_weight_prep: bad mode %d", mode);
  const long n = (long)Cout * ksize * ksize * Cin;
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(weight_prep_kernel<T>, dim3(cdivl(n, 256)), dim3(256), 0,
                                               ROD_STREAM(stream), w, (T*)wt, Cout, Cin, ksize, mode));
  return check_launch("rod_conv_weight_prep");
}

int rod_conv_weight_prep_batch(const void* table, int n, long total, int dtype, void* stream) {
  ROD_CHECK_ARG(table != nullptr && n > 0 && total > 0, "rod_conv_weight_prep_batch: bad arguments");
  const int blocks = (int)std::min<long>(cdivl(total, 256), 4096);
  ROD_DISPATCH_DTYPE(dtype, hipLaunchKernelGGL(weight_prep_batch_kernel<T>, dim3(blocks), dim3(256), 0,
                                               ROD_STREAM(stream), (const PrepEntry*)table, n, total));
  return check_launch("rod_conv_weight_prep_batch");
}

size_t rod_conv_wgrad_workspace(int N, int H, int W, int Cin, int Cout, int ksize) {
  const long M = (long)N * H * W;
  long cchunk = std::max<long>(64, cdivl(M, 512));
  size_t cs = (size_t)cdivl(M, cchunk) * Cout * sizeof(float);
  return (size_t)wgrad_part_floats(N, H, W, Cin, Cout, ksize) * sizeof(float) + cs;
}

int rod_conv_wgrad(const void* x, const float* pro_mean, const float* pro_rstd, const float* pro_gamma,
                   const float* pro_beta, int pro_act, const void* dy, float* dw, float* db, void* workspace, int N,
                   int H, int W, int Cin, int Cout, int ksize, int ldx, int lddy, int dtype, void* stream) {
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0, "rod_conv_wgrad: bad shape");
  ROD_CHECK_ARG(ksize == 1 || ksize == 3, "rod_conv_wgrad: ksize must be 1 or 3");
  ROD_CHECK_ARG(workspace != nullptr, "rod_conv_wgrad: workspace is NULL");
  if (ldx == 0) ldx = Cin;
  if (lddy == 0) lddy = Cout;
  ROD_CHECK_ARG(ldx >= Cin && lddy >= Cout, "rod_conv_wgrad: leading dim too small");
  ROD_CHECK_ARG(!pro_mean || (pro_rstd && Cin <= PRO_MAXC), "rod_conv_wgrad: bad BatchNorm prologue (Cin %d)", Cin);
  const BnPro pro{pro_mean, pro_rstd, pro_gamma, pro_beta, pro_act};
  ROD_DISPATCH_DTYPE(dtype, wgrad_typed<T>(x, pro_mean ? &pro : nullptr, dy, dw, db, (float*)workspace, N, H, W, Cin,
                                           Cout, ksize, ldx, lddy, ROD_STREAM(stream)));
  return check_launch("rod_conv_wgrad");
}


int rod_stem_wgrad_bn_supported(int Cin, int Cout, int ksize, int dtype) {
  return dtype == ROD_BF16 && ksize == 3 && Cin == 3 && Cout == 32 ? 1 : 0;
}

int rod_stem_wgrad_bn(const void* x, const void* dz, const void* y, const float* mean, const float* rstd,
                      const float* gamma, const float* beta, int act, const float* coef, float* dw, void* workspace,
                      int N, int H, int W, int Cin, int Cout, int ksize, int dtype, void* stream) {
  ROD_CHECK_ARG(N > 0 && H > 0 && W > 0 && rod_stem_wgrad_bn_supported(Cin, Cout, ksize, dtype),
                "rod_stem_wgrad_bn: unsupported shape N=%d H=%d W=%d Cin=%d Cout=%d ksize=%d", N, H, W, Cin, Cout,
                ksize);
  ROD_CHECK_ARG(x && dz && y && mean && rstd && coef && dw && workspace, "rod_stem_wgrad_bn: NULL argument");
  ROD_CHECK_ARG(((((uintptr_t)dz) | ((uintptr_t)y)) & 15) == 0, "rod_stem_wgrad_bn: dz / y must be 16-byte aligned");
  hipStream_t s = ROD_STREAM(stream);
  const StemWgradPlan sp = stem_wgrad_plan(N, H, W);
  const StemBnb bb{(const bf16_t*)dz, (const bf16_t*)y, mean, rstd, gamma, beta, coef, act};
  float* part = (float*)workspace;
  hipLaunchKernelGGL(stem_wgrad_kernel<true>, dim3(sp.xb, sp.yb, N), dim3(256), 0, s, (const bf16_t*)x, nullptr,
                     part, H, W, Cin, Cout, sp.rb, bb);
  slab_sum(part, dw, sp.nblk, (long)Cout * 27, s);
  return check_launch("rod_stem_wgrad_bn");
}

}  // extern "C"
