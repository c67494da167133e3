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
}  // namespace rod
