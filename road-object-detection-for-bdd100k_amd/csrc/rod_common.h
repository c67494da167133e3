// rod_common.h — shared device/host helpers for librod (gfx950 / CDNA4 only).
//
// Conventions (see include/rod.h):
//   * every tensor is NHWC, row-major, C innermost;
//   * dtype codes: ROD_F32 = 0, ROD_BF16 = 1 (storage type; arithmetic is fp32);
//   * every entry point returns 0 or an error code and records a message in
//     rod_last_error(); launches are stream-ordered on the caller's hipStream_t.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/rod.h"

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace rod {

void set_error(const char* fmt, ...);
int check_launch(const char* what);
// out[i] = sum_b slab[b*n + i] (fp32 partials, f64 accumulation, fixed order).
// Blocks of CB columns x 256/CB slab lanes (CB adapts to n), so long slabs and wide rows both parallelise.
// deferrable: a parameter-gradient sum that rod_slab_defer(1) may queue for rod_slab_flush (its
// output is read by no kernel before the flush); false for sums a later kernel of the same call reads.
void slab_sum(const float* slab, float* out, int nslab, long n, hipStream_t s, bool deferrable = true);
int slab_cb(int nslab, long n);  // the column-block width slab_sum launches with
// Grid size for a grid-stride loop over rows x CV channel vectors in which every thread
// keeps ONE channel vector: (blocks * 256) % CV == 0 and blocks ~ target.
int const_channel_blocks(int CV, long total, int target = 2048);

// ---- scalar conversions -------------------------------------------------
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16_t v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float v) { return (bf16_t)v; }

// 16-byte vector of T: 4 x f32 or 8 x bf16.
// Global stores of kernel outputs that are streamed (written once, read by a later launch):
// ROD_NT_OUT builds mark them non-temporal.
#ifdef ROD_NT_OUT
#define ROD_ST_OUT(p, v) __builtin_nontemporal_store((v), (p))
#else
#define ROD_ST_OUT(p, v) (*(p) = (v))
#endif

template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  f32x4 v;
  __device__ __forceinline__ void load(const float* p) { v = *(const f32x4*)p; }
  __device__ __forceinline__ void store(float* p) const { *(f32x4*)p = v; }
  __device__ __forceinline__ void store_out(float* p) const { ROD_ST_OUT((f32x4*)p, v); }
  __device__ __forceinline__ float get(int i) const { return v[i]; }
  __device__ __forceinline__ void set(int i, float x) { v[i] = x; }
};
template <> struct Vec16<bf16_t> {
  static constexpr int N = 8;
  bf16x8 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *(const bf16x8*)p; }
  __device__ __forceinline__ void store(bf16_t* p) const { *(bf16x8*)p = v; }
  __device__ __forceinline__ void store_out(bf16_t* p) const { ROD_ST_OUT((bf16x8*)p, v); }
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
  __device__ __forceinline__ void set(int i, float x) { v[i] = (bf16_t)x; }
};

// Buffer-resource I/O for streaming kernels with a register prefetch ring.  A load or store
// inside a branch (a row outside the strip, a halo lane) makes the compiler's wait-count pass
// lose track of how many vector-memory operations are in flight, and it then drains them all
// (s_waitcnt vmcnt(0)) every step — the ring prefetches nothing.  With buffer instructions every
// load / store is issued unconditionally: the 32-bit lane offset `vo` carries the per-lane
// column, the wave-uniform `so` (SGPR) the row.  A lane that must not store has vo = ROD_OOB
// (fixed for the whole kernel), which the hardware range check (offset >= num_records) drops;
// a whole row that must not store goes to an empty resource (rod_rsrc(base, 0), chosen in
// SGPRs).  Store hazard: the compiler inserts the wait state between a >8-byte buffer store and
// a VALU overwrite of its data registers only for stores whose SGPR offset is the constant 0 (its
// MUBUF rule); these stores carry the row in an SGPR offset, and a VALU write of the data
// registers in the very next instruction corrupted stored elements on the MI355X (fp32
// depthwise outputs, different run to run; tests/test_gpu_dwsweep.py).  buf_st therefore fences
// every store with s_nop 4 (5 wait states) between scheduling barriers, so nothing that writes a
// VGPR issues within 5 cycles of the store.  Base and size must be wave-uniform; one resource's
// byte range fits in 31 bits.
constexpr unsigned ROD_OOB = 0x80000000u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t rod_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
template <typename V> __device__ __forceinline__ V buf_ld(rsrc_t r, unsigned vo, unsigned so) {
  constexpr int NB = sizeof(V);
  static_assert(NB == 4 || NB == 8 || NB == 16, "buffer load of 4 / 8 / 16 bytes");
  if constexpr (NB == 4) return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  else if constexpr (NB == 8) return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
  else return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
}
template <typename V> __device__ __forceinline__ void buf_st(const V& v, rsrc_t r, unsigned vo, unsigned so) {
  constexpr int NB = sizeof(V);
  static_assert(NB == 4 || NB == 8 || NB == 16, "buffer store of 4 / 8 / 16 bytes");
  if constexpr (NB == 4) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, vo, so, 0);
  else if constexpr (NB == 8) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, vo, so, 0);
  else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, vo, so, 0);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Correctly-rounded f32 transcendental functions (evaluated in f64 and
// rounded once).  The oracle uses the same definition (np.float64 then cast),
// so integer decisions downstream of exp/log are reproducible bit for bit.
__device__ __forceinline__ float exp_cr(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float log_cr(float x) { return (float)log((double)x); }

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// BatchNorm partial statistics: slab [nparts][3][C] of (count, mean, M2) per part and
// channel, part-major so that a producer block writes its 3*C values contiguously (parts
// with count 0 are ignored by the merge).  Written by bn_stats_kernel and by the epilogues
// of the producers that fuse it (rod_conv_fwd, rod_dw3x3_fwd).
__device__ __forceinline__ void store_stat_part(float* slab, int C, long part, int c, float n, float mean, float m2) {
  float* p = slab + part * 3 * C + c;
  p[0] = n;
  p[C] = mean;
  p[2 * C] = m2;
}

// fp32 Chan merge of (n, mean, M2) accumulators
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  if (nb == 0.f) return;
  if (n == 0.f) {
    n = nb;
    mean = meanb;
    m2 = m2b;
    return;
  }
  const float nt = n + nb;
  const float d = meanb - mean;
  mean = fmaf(d, nb / nt, mean);
  m2 = m2 + m2b + d * d * (n * nb / nt);
  n = nt;
}

// ---- activations (after BatchNorm) ---------------------------------------------
// relu6 = clamp (v_med3_f32), leaky = max(z, 0.2 z) (== z > 0 ? z : 0.2 z bit for bit)
template <int ACT>
__device__ __forceinline__ float act_t(float z) {
  if constexpr (ACT == ROD_ACT_RELU6) return __builtin_amdgcn_fmed3f(z, 0.f, 6.f);  // tf.nn.relu6
  else if constexpr (ACT == ROD_ACT_LEAKY) return fmaxf(z, z * 0.2f);                // leaky_relu(0.2)
  else if constexpr (ACT == ROD_ACT_RELU) return fmaxf(z, 0.f);                      // tf.nn.relu (VGG)
  else return z;
}
__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == ROD_ACT_RELU6) return act_t<ROD_ACT_RELU6>(z);
  if (act == ROD_ACT_LEAKY) return act_t<ROD_ACT_LEAKY>(z);
  if (act == ROD_ACT_RELU) return act_t<ROD_ACT_RELU>(z);
  return z;
}
// Relu6Grad (0 < z < 6), LeakyReluGrad (z > 0 ? 1 : 0.2), ReluGrad (z > 0), none (1) as ONE
// branch-free select chain: z > 0 ? (!(z >= hi) ? 1 : 0) : lo with (lo, hi) from the
// activation (hi = NaN: no upper bound; the unordered compare keeps +inf at 1).  Same value
// as the per-activation forms for every z, NaN and inf included.  The (lo, hi) selects depend
// only on the wave-uniform act, so they hoist out of the loops: no per-element branches.
__device__ __forceinline__ float act_grad(float z, int act) {
  const float lo = act == ROD_ACT_LEAKY ? 0.2f : ((act == ROD_ACT_RELU6 || act == ROD_ACT_RELU) ? 0.f : 1.f);
  const float hi = act == ROD_ACT_RELU6 ? 6.f : __builtin_nanf("");
  return z > 0.f ? (!(z >= hi) ? 1.f : 0.f) : lo;
}

// ---- BatchNorm affine -------------------------------------------------------------
// z = x*scale + offset (one FMA), scale = rstd*gamma, offset = beta - mean*scale — the form of
// TF's fused batch-norm kernel; every librod kernel that forms z (rod_bn_apply, the backward's
// activation mask, the consumer prologues) uses exactly this, so they agree bit for bit.
__device__ __forceinline__ void bn_affine(const float* mean, const float* rstd, const float* gamma,
                                          const float* beta, int c, float& sc, float& sh) {
  sc = gamma ? rstd[c] * gamma[c] : rstd[c];
  sh = (beta ? beta[c] : 0.f) - mean[c] * sc;
}

// ---- BatchNorm-backward apply --------------------------------------------------------
// TF's FusedBatchNormGrad: dy = a*(g - mean(g) - yhat*mean(g*yhat)), yhat = (y - mean)*rstd,
// with coef = (a, mean(g), mean(g*yhat)) per channel (rod_bn_bwd_finalize).  Every librod kernel
// that applies it (rod_bn_bwd_apply, the one-launch small-tensor form, the fused depthwise and
// 1x1 backwards) evaluates it with the per-channel constants below, so all of them round
// identically for a given storage type T:
//   * bf16 storage:  fma(a, g, fma(k1, y, k0)), the mean folded into k0 (two FMAs per element).
//     Folding costs ~|mean|/std * 2^-24 relative in k0; the bf16 input y itself carries
//     |y| * 2^-9 ~ |mean| * 2^-9 of quantisation, 2^15 times more, so the fold is invisible;
//   * fp32 storage:  fma(a, g, fma(k1, y - mean, k0')), k0' = -a*mean(g) — y is centred first,
//     as FusedBatchNormGrad does ((y - mean) is exact near the mean), so a channel with
//     |mean| >> std keeps full fp32 precision (tests/test_gpu_bnred.py, mean 50 / rstd 100).
// `m` is the centring shift: the mean for fp32, unused (0) for bf16.
template <typename T>
__device__ __forceinline__ void bn_bwd_k(float a, float mu, float rs, float mg, float mgx, float& k1, float& k0,
                                         float& m) {
  const float t = rs * mgx;
  k1 = -(a * t);
  if constexpr (sizeof(T) == 4) {
    k0 = -(a * mg);
    m = mu;
  } else {
    k0 = a * fmaf(t, mu, -mg);
    m = 0.f;
  }
}
// bf16-only kernels (1x1 backwards, the stem weight gradient): the folded constants
__device__ __forceinline__ void bn_bwd_k_fold(float a, float mu, float rs, float mg, float mgx, float& k1, float& k0) {
  float m;
  bn_bwd_k<bf16_t>(a, mu, rs, mg, mgx, k1, k0, m);
}
template <typename T>
__device__ __forceinline__ float bn_bwd_apply1(float a, float g, float k1, float k0, float m, float y) {
  if constexpr (sizeof(T) == 4) return fmaf(a, g, fmaf(k1, y - m, k0));
  else return fmaf(a, g, fmaf(k1, y, k0));
}

// ---- BatchNorm-apply prologue -----------------------------------------------------
// A consumer kernel that reads the PRE-BatchNorm tensor y instead of the BatchNorm output:
// z = act(fma(y, scale, offset)), rounded to the storage type — exactly the value
// rod_bn_apply would have written — is formed in registers as each element is consumed, so
// the normalised activation never crosses HBM.  Padding taps stay 0.
struct BnPro {
  const float* mean;
  const float* rstd;
  const float* gamma;  // NULL => 1
  const float* beta;   // NULL => 0
  int act;
};
constexpr int PRO_MAXC = 2048;  // channel limit of the LDS-staged prologue tables
__device__ __forceinline__ void bn_pro_affine(const BnPro& p, int c, float& sc, float& sh) {
  bn_affine(p.mean, p.rstd, p.gamma, p.beta, c, sc, sh);
}

// BatchNorm-apply epilogue (ABI 21, inference): the producer of y writes z = act(BN(y)) (+ res)
// instead of y — the value rod_bn_apply would write from the stored (rounded) y: y is rounded to
// the storage type first, then z = act(fma(y, scale, offset)) (+ res) rounded once, so the
// predict path's result is bit-identical to conv -> rod_bn_apply while y never crosses HBM.
struct BnEpi {
  const float* mean;
  const float* rstd;
  const float* gamma;  // NULL => 1
  const float* beta;   // NULL => 0
  const void* res;     // residual added after the activation (nullable), row stride ldr
  int ldr;
  int act;
};
template <typename T>
__device__ __forceinline__ float bn_epi1(const BnEpi& e, float sc, float sh, float v, long row, int col) {
  float z = act_fwd(fmaf(to_f32(from_f32<T>(v)), sc, sh), e.act);
  if (e.res) z = z + to_f32(((const T*)e.res)[row * e.ldr + col]);
  return z;
}

// Fallback: parts of y[M, C] computed by a separate pass (batchnorm.hip).
void stat_parts(int dtype, const void* y, long M, int C, int ld, float* parts, int nparts, hipStream_t s);
// Fallback: BatchNorm-backward partial sums [nparts][2][C] of (g, g*yhat) from dz and the
// pre-BatchNorm y (both [M, C] contiguous) by a separate pass (batchnorm.hip).
void gred_parts(int dtype, const void* dz, const void* y, const BnPro& p, long M, int C, float* parts, int nparts,
                hipStream_t s);

// BatchNorm-backward reduction in a producer's epilogue ("gred"): for the BatchNorm whose
// output z = act(y*scale + offset) a consumer read through its prologue, the kernel that
// writes dz (that consumer's backward-data) also reads y at the same positions and sums,
// per channel, g = dz*act'(y*scale + offset) and g*yhat, yhat = (y - mean)*rstd — the
// arithmetic of bn_bwd_reduce_kernel, on the rounded dz it stores.
struct BnGred {
  const void* y;
  BnPro p;
  float* parts;  // [nparts][2][C]
};
__device__ __forceinline__ void gred_coef(const BnPro& p, int c, float& sc, float& sh, float& mu, float& rs) {
  bn_pro_affine(p, c, sc, sh);
  mu = p.mean[c];
  rs = p.rstd[c];
}
__device__ __forceinline__ void gred_acc(float dz, float y, float sc, float sh, float mu, float rs, int act, float& sg,
                                         float& sgx) {
  const float d = y - mu;
  const float g = dz * act_grad(fmaf(y, sc, sh), act);
  sg += g;
  sgx = fmaf(g, d * rs, sgx);
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
inline long cdivl(long a, long b) { return (a + b - 1) / b; }

}  // namespace rod

#define ROD_CHECK_ARG(cond, ...)             \
  do {                                       \
    if (!(cond)) {                           \
      ::rod::set_error(__VA_ARGS__);         \
      return ROD_EINVAL;                     \
    }                                        \
  } while (0)

#define ROD_STREAM(s) ((hipStream_t)(s))

// dispatch on storage dtype: defines `T` inside the body
#define ROD_DISPATCH_DTYPE(dt, ...)                                   \
  do {                                                                \
    if ((dt) == ROD_F32) {                                            \
      typedef float T;                                                \
      __VA_ARGS__;                                                    \
    } else if ((dt) == ROD_BF16) {                                    \
      typedef bf16_t T;                                               \
      __VA_ARGS__;                                                    \
    } else {                                                          \
      ::rod::set_error("unsupported dtype code %d", (int)(dt));        \
      return ROD_EINVAL;                                              \
    }                                                                 \
  } while (0)
