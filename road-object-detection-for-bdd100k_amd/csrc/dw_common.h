// dw_common.h — pieces of the depthwise LDS-exchange engine shared by depthwise.hip and
// dwrc.hip (the expand-recompute forward, ABI 23): register packs, the tile plan and its
// XCD-aware block order, the forward pack width.  The tile plan fixes the statistics part
// structure, so every kernel that writes those parts must share it.
#pragma once
#include "rod_common.h"

namespace rod {

// V contiguous elements of T held in registers (bf16 x4 = 8-byte, f32 x4 = 16-byte loads).
template <typename T, int V> struct PackV;
template <> struct PackV<float, 4> {
  f32x4 v;
  __device__ __forceinline__ void bload(rsrc_t r, unsigned vo, unsigned so) { v = buf_ld<decltype(v)>(r, vo, so); }
  __device__ __forceinline__ void bstore(rsrc_t r, unsigned vo, unsigned so) const { buf_st(v, r, vo, so); }
  __device__ __forceinline__ void load(const float* p) { v = *(const f32x4*)p; }
  __device__ __forceinline__ void zero() { v = f32x4{0.f, 0.f, 0.f, 0.f}; }
  __device__ __forceinline__ float get(int i) const { return v[i]; }
  __device__ __forceinline__ void set(int i, float a) { v[i] = a; }
  __device__ __forceinline__ void store(float* p) const { *(f32x4*)p = v; }
  __device__ __forceinline__ void store_out(float* p) const { ROD_ST_OUT((f32x4*)p, v); }
};
template <> struct PackV<bf16_t, 4> {
  bf16x4 v;
  __device__ __forceinline__ void bload(rsrc_t r, unsigned vo, unsigned so) { v = buf_ld<decltype(v)>(r, vo, so); }
  __device__ __forceinline__ void bstore(rsrc_t r, unsigned vo, unsigned so) const { buf_st(v, r, vo, so); }
  __device__ __forceinline__ void load(const bf16_t* p) { v = *(const bf16x4*)p; }
  __device__ __forceinline__ void zero() { v = bf16x4{(bf16_t)0.f, (bf16_t)0.f, (bf16_t)0.f, (bf16_t)0.f}; }
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
  __device__ __forceinline__ void set(int i, float a) { v[i] = (bf16_t)a; }
  __device__ __forceinline__ void store(bf16_t* p) const { *(bf16x4*)p = v; }
  __device__ __forceinline__ void store_out(bf16_t* p) const { ROD_ST_OUT((bf16x4*)p, v); }
};
template <> struct PackV<bf16_t, 8> {
  bf16x8 v;
  __device__ __forceinline__ void bload(rsrc_t r, unsigned vo, unsigned so) { v = buf_ld<decltype(v)>(r, vo, so); }
  __device__ __forceinline__ void bstore(rsrc_t r, unsigned vo, unsigned so) const { buf_st(v, r, vo, so); }
  __device__ __forceinline__ void load(const bf16_t* p) { v = *(const bf16x8*)p; }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (bf16_t)0.f;
  }
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
  __device__ __forceinline__ void set(int i, float a) { v[i] = (bf16_t)a; }
  __device__ __forceinline__ void store(bf16_t* p) const { *(bf16x8*)p = v; }
  __device__ __forceinline__ void store_out(bf16_t* p) const { ROD_ST_OUT((bf16x8*)p, v); }
};
template <> struct PackV<bf16_t, 2> {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  bf16x2_t v;
  __device__ __forceinline__ void bload(rsrc_t r, unsigned vo, unsigned so) { v = buf_ld<decltype(v)>(r, vo, so); }
  __device__ __forceinline__ void bstore(rsrc_t r, unsigned vo, unsigned so) const { buf_st(v, r, vo, so); }
  __device__ __forceinline__ void load(const bf16_t* p) { v = *(const bf16x2_t*)p; }
  __device__ __forceinline__ void zero() { v = bf16x2_t{(bf16_t)0.f, (bf16_t)0.f}; }
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
  __device__ __forceinline__ void set(int i, float a) { v[i] = (bf16_t)a; }
  __device__ __forceinline__ void store(bf16_t* p) const { *(bf16x2_t*)p = v; }
  __device__ __forceinline__ void store_out(bf16_t* p) const { ROD_ST_OUT((bf16x2_t*)p, v); }
};
template <typename T> struct PackV<T, 1> {
  T v;
  __device__ __forceinline__ void load(const T* p) { v = *p; }
  __device__ __forceinline__ void zero() { v = (T)0.f; }
  __device__ __forceinline__ float get(int) const { return to_f32(v); }
  __device__ __forceinline__ void set(int, float a) { v = from_f32<T>(a); }
  __device__ __forceinline__ void store(T* p) const { *p = v; }
  __device__ __forceinline__ void store_out(T* p) const { *p = v; }
};


struct DwTile {
  int CVb, P, TWo, cgroups, coltiles, RB, strips;
};

// Tile plan for a V-wide 16-byte pack: CVb a divisor of C/V (whole 128-byte pixel segments
// preferred), P columns (<= the columns the map has), RB output rows (>= 8: the prologue / epilogue are per block) so that the grid has
// ~1024 blocks.  Deterministic in (N, Ho, Wo, C, S, V): the statistics part count depends
// on it.
inline DwTile dw_tile(int N, int Ho, int Wo, int C, int S, int V) {
  DwTile t;
  const int CV = C / V;
  const int halo = S == 1 ? 2 : 1;
  double best = -1.0;
  t.CVb = 1;
  for (int d = 1; d <= std::min(CV, 32); ++d) {
    if (CV % d) continue;
    const int P = std::min(256 / d, Wo + halo);
    if (P <= halo) continue;
    const double eff = (double)(P - halo) / P * (double)(P * d) / 256.0;
    const double seg = (d * 16 >= 128 || d == CV) ? 1.0 : 0.8;
    const double sc = eff * seg;
    if (sc > best + 1e-9) {
      best = sc;
      t.CVb = d;
    }
  }
  t.P = std::min(256 / t.CVb, Wo + halo);
  t.TWo = t.P - halo;
  t.cgroups = CV / t.CVb;
  t.coltiles = cdiv(Wo, t.TWo);
  const long base = (long)N * t.coltiles * t.cgroups;
  // >= 16 output rows per block: fewer, longer strips on the small deep maps, whose per-block
  // prologue / epilogue and 3-row ramp dominated short strips (tools/dw_bench.py, round 2:
  // 45x80x576 forward with prologue + statistics 40.8 -> 33.7 us, filter gradient 53.7 -> 43.4;
  // 23x40x960 25.7 -> 19.7 and 34.4 -> 24.0; round 5 step: 466.5 / 466.7 -> 469.5 / 469.2 img/s
  // against 8, 24: 468.5 / 467.8).  It regroups the statistic / filter partial sums (a
  // rounding-level change); round 2 kept 8 because the ALL-mode step test then moved — a kink
  // flip the fp64 truth itself shows under 1e-6 input noise, which that test now measures.
  // Measurement switches: ROD_DW_WANT (target blocks, 1024), ROD_DW_RBMIN (minimum rows per block)
  static const long want_blocks = getenv("ROD_DW_WANT") ? atol(getenv("ROD_DW_WANT")) : 1024;
  static const long rb_min = getenv("ROD_DW_RBMIN") ? atol(getenv("ROD_DW_RBMIN")) : 16;
  const long want = std::max<long>(1, cdivl(want_blocks, base));
  t.RB = (int)std::min<long>(64, std::max<long>(rb_min, cdivl(Ho, want)));
  t.strips = cdiv(Ho, t.RB);
  return t;
}

// blockIdx -> (x, y, z) after an XCD-aware remap: consecutive tiles (which share halo
// rows / columns) are placed on the same XCD (the dispatcher deals blocks round-robin).
__device__ __forceinline__ void xcd_block(int& bx, int& by, int& bz) {
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const int nb = gx * gy * gz;
  int lin = (blockIdx.z * gy + blockIdx.y) * gx + blockIdx.x;
  if ((nb & 7) == 0) lin = (lin & 7) * (nb >> 3) + (lin >> 3);
  bx = lin % gx;
  lin /= gx;
  by = lin % gy;
  bz = lin / gy;
}

// channel pack of the forward LX kernel: 16-byte packs, or (bf16) 8-byte packs with half the
// per-thread weights / accumulators / statistics in registers (106 instead of 192 VGPRs with the
// prologue and statistics: 4 waves / SIMD instead of 2).  tools/dw_bench.py fwdpro, per shape
// with ROD_DW_FWD_V=4 / 8 (round 4): 8 bytes on the narrow or small maps — 720x1280x32 s1 229.6
// vs 258.3 us, 180x320x192 s1 104 vs 113, 90x160x384 52 vs 62, 45x80x576 30 vs 39 — and 16
// bytes on the wide large ones — 720x1280x96 s2 387 vs 420, 360x640x144 s1 306 vs 341,
// 360x640x144 s2 187 vs 206.  So 16 bytes when C >= 96 and the INPUT map has > 1M pixels.
// ROD_DW_FWD_V=4 / 8 forces one width (A/B switch).
inline int dw_fwd_v(int dtype, long in_pixels, int C) {
  static const int env = getenv("ROD_DW_FWD_V") ? atoi(getenv("ROD_DW_FWD_V")) : 0;
  if (dtype == ROD_F32) return 4;
  if (env == 4 || env == 8) return env;
  return C >= 96 && in_pixels > 1024L * 1024 ? 8 : 4;
}

struct DwBwdBn {
  const float *mean, *rstd, *gamma, *beta, *coef;  // BN_d and its backward coefficients [3][C]
  int act;
};

typedef float dw_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ dw_f2 f2fma(dw_f2 a, dw_f2 b, dw_f2 c) { return __builtin_elementwise_fma(a, b, c); }
template <int ACT>
__device__ __forceinline__ float agrad(float z, int act) {
  if constexpr (ACT == ROD_ACT_RELU6) return (z > 0.f && !(z >= 6.f)) ? 1.f : 0.f;  // == act_grad(z, RELU6)
  else return act_grad(z, act);
}
template <typename T>
__device__ __forceinline__ void unpack4(const PackV<T, 4>& p, dw_f2& a, dw_f2& b) {
  a = dw_f2{p.get(0), p.get(1)};
  b = dw_f2{p.get(2), p.get(3)};
}
template <typename T, int V>
__device__ __forceinline__ void unpackv(const PackV<T, V>& p, dw_f2 (&o)[V / 2]) {
#pragma unroll
  for (int h = 0; h < V / 2; ++h) o[h] = dw_f2{p.get(2 * h), p.get(2 * h + 1)};
}
// one v_cvt_pk_bf16_f32 for the pair (RNE, as (bf16_t)x per element), unpacked by a shift / mask
typedef __bf16 dw_b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ dw_f2 round2(dw_f2 v, bf16_t) {
  const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(v, dw_b2));
  return dw_f2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}
// ReLU6 gradient gate (z > 0 && z < 6, NaN -> 0: agrad<ROD_ACT_RELU6>) as one unsigned compare
// on the bits: positive floats order as integers, negative ones and NaN land above 6.0's bits
__device__ __forceinline__ bool relu6_open(float z) {
  return __builtin_bit_cast(unsigned, z) - 1u < 0x40BFFFFFu;
}
template <int ACT>
__device__ __forceinline__ dw_f2 gate2(dw_f2 z, dw_f2 v, int act) {
  if constexpr (ACT == ROD_ACT_RELU6) return dw_f2{relu6_open(z.x) ? v.x : 0.f, relu6_open(z.y) ? v.y : 0.f};
  else return dw_f2{v.x * act_grad(z.x, act), v.y * act_grad(z.y, act)};
}
__device__ __forceinline__ dw_f2 round2(dw_f2 v, float) { return v; }

// Epilogue of the packed depthwise backward kernels: the per-block column sums of the nq staged
// quantities (the 9 filter taps, then with the BatchNorm sums g and g*yhat; red = [nq][TB][V]
// floats, halo lanes staged as 0) — every (quantity, channel) summed over the computing columns
// 1 .. P-2 in column order by one thread, after ONE barrier for all quantities (the
// one-quantity-at-a-time form took two barriers a quantity with Cc of the TB threads working;
// the sums, and so the parts, are bit-identical).
template <int V>
__device__ __forceinline__ void dw_colsum_emit(const float* red, int q0, int nq, int TB, int Cc, int CVb, int P,
                                               float* slab, float* gparts, long part, int C, int cg) {
  for (int e = threadIdx.x; e < nq * Cc; e += TB) {
    const int qs = e / Cc, ce = e - qs * Cc, qk = q0 + qs;
    const int cve = ce / V, v = ce - cve * V;
    const float* r = red + qs * TB * V;
    float s = 0.f;
    for (int pp = 1; pp <= P - 2; ++pp) s += r[(pp * CVb + cve) * V + v];
    float* dst = qk < 9 ? slab + (part * 9 + qk) * C : gparts + (part * 2 + (qk - 9)) * C;
    dst[cg * Cc + ce] = s;
  }
}


// Both strides tile a map with one halo column each side (the S=1 plan geometry): stride 1
// the output (= input) map, stride 2 the (A, B) map of dy positions that own a dx row / column.
inline bool dw_fused_geom(int N, int H, int W, int C, int S, int pt, int pl, int& A, int& B) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 4) return false;
  if (S == 1) {
    if (pt != 1 || pl != 1) return false;
    A = H, B = W;
    return true;
  }
  if (S != 2 || pt < 0 || pt > 1 || pl < 0 || pl > 1) return false;
  A = ((H - 1 + pt) >> 1) + 1, B = ((W - 1 + pl) >> 1) + 1;
  return true;
}


}  // namespace rod
