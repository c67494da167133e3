// nms.hip — detected_bboxes (reference utils/net_tools.py:739-758) for every (image, class)
// in one launch: one 1024-thread workgroup per (image, class c = 1..K-1) performs
//
//   select   s_i = p_i * (p_i >= select_threshold), box_i * (p_i >= thr)  (net_tools.py:689-692)
//   sort     top_k(s, top_k, sorted=True): score desc, ties -> lower index (bboxes.py:86)
//   nms      tf.image.non_max_suppression(boxes, s, keep_top_k, nms_threshold) with
//            score_threshold = -inf: greedy in score order, suppress when IoU > thr; IoU on
//            min/max-normalised corners, 0 if either area <= 0 (bboxes.py:182)
//   pad      zero-pad the kept scores/boxes to keep_top_k (tensors.py:59-86)
//
// Two implementations with identical output:
//  * compacted (select_threshold > 0, workspace given — the CLIs' 0.1 / 0.3): ONE row-wise,
//    coalesced pass over probs appends every selected (nonzero) score of every class as a
//    64-bit key (~score bits, anchor index) to a per-(image, class) list
//    (nms_compact_kernel); then one workgroup per (image, class) sorts its list in LDS (or,
//    past 4096 candidates, radix-selects the top_k-th key over the list first) and runs the
//    greedy NMS (nms_select_kernel).  The entries top_k would take beyond the selected ones
//    have score 0 and a zeroed box (p < threshold): zero area, they suppress nothing and are
//    output as the zero padding — so they need not be materialised.
//  * direct (any threshold): per (image, class) an exact in-workgroup 4 x 8-bit radix select
//    on the (non-negative) f32 score bits read column-wise from probs; candidates compacted in
//    index order (ties resolved by index), then bitonic-sorted by (score desc, index asc).
// Compiled with -ffp-contract=off.
#include <math.h>

#include "rod_common.h"

namespace rod {

constexpr int NMS_T = 1024;  // threads per workgroup = max top_k

__device__ __forceinline__ float sel_score(const float* probs, long row, int K, int c, float thr) {
  const float p = probs[row * K + c];
  return p * (p >= thr ? 1.f : 0.f);  // scores * cast(greater_equal(scores, thr))
}

// count of values with digit > d / == d handled via histogram over the prefix-matching set
__device__ unsigned block_radix_kth_largest(const float* probs, long base, int A, int K, int c, float thr, int k,
                                            unsigned* hist, unsigned* sh) {
  unsigned prefix = 0, rank = (unsigned)k;  // k-th largest, 1-based
  for (int shift = 24; shift >= 0; shift -= 8) {
    const unsigned hmask = shift >= 24 ? 0u : (0xFFFFFFFFu << (shift + 8));
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0u;
    __syncthreads();
    for (int a0 = 0; a0 < A; a0 += blockDim.x) {  // uniform trip count: ballots see every lane
      const int a = a0 + threadIdx.x;
      const unsigned b = a < A ? __float_as_uint(sel_score(probs, base + a, K, c, thr)) : 0xFFFFFFFFu;
      const bool match = a < A && (b & hmask) == (prefix & hmask);
      // scores below the select threshold are exactly 0: count them per wave, not per lane
      if (match && b != 0u) atomicAdd(&hist[(b >> shift) & 255u], 1u);
      const unsigned long long zm = __ballot(match && b == 0u);
      if ((threadIdx.x & 63) == 0 && zm) atomicAdd(&hist[0], (unsigned)__popcll(zm));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned acc = 0;
      int d = 255;
      for (; d >= 0; --d) {
        if (acc + hist[d] >= rank) break;
        acc += hist[d];
      }
      if (d < 0) d = 0;
      sh[0] = prefix | ((unsigned)d << shift);
      sh[1] = rank - acc;
    }
    __syncthreads();
    prefix = sh[0];
    rank = sh[1];
    __syncthreads();
  }
  return prefix;  // bits of the k-th largest score
}

__device__ __forceinline__ float tf_iou(const float* bi, const float* bj) {
  const float ymin_i = fminf(bi[0], bi[2]), xmin_i = fminf(bi[1], bi[3]);
  const float ymax_i = fmaxf(bi[0], bi[2]), xmax_i = fmaxf(bi[1], bi[3]);
  const float ymin_j = fminf(bj[0], bj[2]), xmin_j = fminf(bj[1], bj[3]);
  const float ymax_j = fmaxf(bj[0], bj[2]), xmax_j = fmaxf(bj[1], bj[3]);
  const float area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i);
  const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
  if (area_i <= 0.f || area_j <= 0.f) return 0.f;
  const float iy0 = fmaxf(ymin_i, ymin_j), ix0 = fmaxf(xmin_i, xmin_j);
  const float iy1 = fminf(ymax_i, ymax_j), ix1 = fminf(xmax_i, xmax_j);
  const float inter = fmaxf(iy1 - iy0, 0.f) * fmaxf(ix1 - ix0, 0.f);
  return inter / (area_i + area_j - inter);
}

__global__ void __launch_bounds__(NMS_T) select_topk_nms_kernel(const float* __restrict__ probs,
                                                                 const float* __restrict__ boxes, int A, int K,
                                                                 float sel_thr, int top_k, int keep_k, float nms_thr,
                                                                 float* __restrict__ out_scores,
                                                                 float* __restrict__ out_boxes) {
  __shared__ unsigned hist[256];
  __shared__ unsigned sh[4];
  __shared__ unsigned long long key[NMS_T];
  __shared__ float bx[NMS_T][4];
  __shared__ float sc[NMS_T];
  __shared__ unsigned char dead[NMS_T];
  __shared__ int wsum[NMS_T / 64];
  __shared__ int kept_idx[NMS_T];

  const int b = blockIdx.y;
  const int c = blockIdx.x + 1;  // classes 1..K-1 (ignore_class = 0)
  const long base = (long)b * A;
  const int k = min(top_k, A);
  const int tid = threadIdx.x;

  // 1) exact value of the k-th largest score and how many ties to take
  const unsigned tbits = block_radix_kth_largest(probs, base, A, K, c, sel_thr, k, hist, sh);
  if (tid == 0) sh[2] = 0;
  __syncthreads();
  for (int a = tid; a < A; a += NMS_T) {
    const unsigned bb = __float_as_uint(sel_score(probs, base + a, K, c, sel_thr));
    if (bb > tbits) atomicAdd(&sh[2], 1u);
  }
  __syncthreads();
  const int need_ties = k - (int)sh[2];

  // 2) ordered compaction (index order): all s > T, and the first need_ties with s == T
  int n_out = 0, ties_seen = 0;
  for (int a0 = 0; a0 < A; a0 += NMS_T) {
    const int a = a0 + tid;
    unsigned bb = 0;
    bool gt = false, eq = false;
    if (a < A) {
      bb = __float_as_uint(sel_score(probs, base + a, K, c, sel_thr));
      gt = bb > tbits;
      eq = bb == tbits;
    }
    // exclusive scan of eq within the chunk (wave ballots + LDS)
    const unsigned long long eqm = __ballot(eq);
    const unsigned long long gtm = __ballot(gt);
    const int lane = tid & 63, w = tid >> 6;
    const unsigned long long lower = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (lane == 0) wsum[w] = __popcll(eqm) | (__popcll(gtm) << 16);
    __syncthreads();
    int eq_before = 0, gt_before = 0, eq_tot = 0, gt_tot = 0;
    for (int q = 0; q < NMS_T / 64; ++q) {
      const int v = wsum[q];
      if (q < w) {
        eq_before += v & 0xFFFF;
        gt_before += v >> 16;
      }
      eq_tot += v & 0xFFFF;
      gt_tot += v >> 16;
    }
    const int eq_rank = ties_seen + eq_before + __popcll(eqm & lower);
    const bool take_eq = eq && eq_rank < need_ties;
    // slots: gt elements and admitted ties, in index order
    const int tie_taken_before = min(max(need_ties - ties_seen, 0), eq_before + __popcll(eqm & lower));
    const int slot = n_out + gt_before + __popcll(gtm & lower) + tie_taken_before;
    if ((gt || take_eq) && slot < NMS_T) {
      key[slot] = ((unsigned long long)(~bb) << 32) | (unsigned)a;  // score desc, index asc
    }
    const int ties_taken_chunk = min(max(need_ties - ties_seen, 0), eq_tot);
    n_out += gt_tot + ties_taken_chunk;
    ties_seen += eq_tot;
    __syncthreads();
  }
  const int n = min(n_out, k);
  // 3) bitonic sort of n keys (pad to NMS_T)
  for (int i = tid; i < NMS_T; i += NMS_T)
    if (i >= n) key[i] = ~0ull;
  __syncthreads();
  for (int size = 2; size <= NMS_T; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int i = tid;
      const int j = i ^ stride;
      if (j > i) {
        const bool up = (i & size) == 0;
        const unsigned long long ki = key[i], kj = key[j];
        if ((ki > kj) == up) {
          key[i] = kj;
          key[j] = ki;
        }
      }
      __syncthreads();
    }
  }
  // 4) gather candidate boxes (masked like the reference) and scores
  if (tid < n) {
    const int a = (int)(key[tid] & 0xFFFFFFFFu);
    const float p = probs[(base + a) * K + c];
    const float fm = p >= sel_thr ? 1.f : 0.f;
    sc[tid] = p * fm;
    const float* bp = boxes + (base + a) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) bx[tid][q] = bp[q] * fm;
    dead[tid] = 0;
  }
  __syncthreads();
  // 5) greedy NMS in sorted order
  int kept = 0;
  for (int i = 0; i < n && kept < keep_k; ++i) {
    if (dead[i]) continue;  // uniform: dead[] only changes between barriers
    if (tid == 0) kept_idx[kept] = i;
    ++kept;
    for (int j = i + 1 + tid; j < n; j += NMS_T)
      if (!dead[j] && tf_iou(bx[i], bx[j]) > nms_thr) dead[j] = 1;
    __syncthreads();
  }
  __syncthreads();
  // 6) write kept entries and zero padding
  float* os = out_scores + ((long)b * (K - 1) + (c - 1)) * keep_k;
  float* ob = out_boxes + ((long)b * (K - 1) + (c - 1)) * keep_k * 4;
  for (int j = tid; j < keep_k; j += NMS_T) {
    if (j < kept) {
      const int i = kept_idx[j];
      os[j] = sc[i];
#pragma unroll
      for (int q = 0; q < 4; ++q) ob[j * 4 + q] = bx[i][q];
    } else {
      os[j] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) ob[j * 4 + q] = 0.f;
    }
  }
}


// ----------------------------------------------------------------- compacted implementation
constexpr int NMS_CT = 2048;     // anchors per compaction workgroup (8 per thread)
constexpr int NMS_SORT = 4096;   // candidate lists up to this size are sorted whole in LDS
constexpr int NMS_MAXC = 32;     // classes per launch (K - 1)

__global__ void nms_zero_kernel(unsigned* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0u;
}

__global__ void __launch_bounds__(256) nms_compact_kernel(const float* __restrict__ probs, int A, int K,
                                                          float sel_thr, unsigned* __restrict__ counts,
                                                          unsigned long long* __restrict__ keys) {
  __shared__ unsigned lcnt[NMS_MAXC], lbase[NMS_MAXC];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int C = K - 1;
  const long base = (long)b * A;
  const int a0 = blockIdx.x * NMS_CT;
  const unsigned long long lower = lane ? (~0ull >> (64 - lane)) : 0ull;
  if (tid < C) lcnt[tid] = 0u;
  __syncthreads();
  // pass 1: candidates per class in this tile
  for (int u = 0; u < NMS_CT / 256; ++u) {
    const int a = a0 + u * 256 + tid;
    for (int c = 1; c <= C; ++c) {
      const bool cand = a < A && __float_as_uint(sel_score(probs, base + a, K, c, sel_thr)) != 0u;
      const unsigned long long m = __ballot(cand);
      if (lane == 0 && m) atomicAdd(&lcnt[c - 1], (unsigned)__popcll(m));
    }
  }
  __syncthreads();
  if (tid < C) {
    lbase[tid] = lcnt[tid] ? atomicAdd(&counts[b * C + tid], lcnt[tid]) : 0u;
    lcnt[tid] = 0u;
  }
  __syncthreads();
  // pass 2 (rows now in L1/L2): append keys; list order is irrelevant (sorted later)
  for (int u = 0; u < NMS_CT / 256; ++u) {
    const int a = a0 + u * 256 + tid;
    for (int c = 1; c <= C; ++c) {
      const unsigned bits = a < A ? __float_as_uint(sel_score(probs, base + a, K, c, sel_thr)) : 0u;
      const bool cand = bits != 0u;
      const unsigned long long m = __ballot(cand);
      if (!m) continue;
      unsigned off = 0;
      if (lane == 0) off = atomicAdd(&lcnt[c - 1], (unsigned)__popcll(m));
      off = __shfl(off, 0);
      if (cand)
        keys[((long)b * C + (c - 1)) * A + lbase[c - 1] + off + __popcll(m & lower)] =
            ((unsigned long long)(~bits) << 32) | (unsigned)a;
    }
  }
}

// bitonic sort (ascending) of key[0..P), P a power of two <= NMS_SORT, 1024 threads
__device__ void lds_bitonic(unsigned long long* key, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < P; i += NMS_T) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const unsigned long long ki = key[i], kj = key[j];
          if ((ki > kj) == up) {
            key[i] = kj;
            key[j] = ki;
          }
        }
      }
      __syncthreads();
    }
  }
}

__global__ void __launch_bounds__(NMS_T) nms_select_kernel(const float* __restrict__ probs,
                                                           const float* __restrict__ boxes, int A, int K,
                                                           float sel_thr, int top_k, int keep_k, float nms_thr,
                                                           const unsigned* __restrict__ counts,
                                                           const unsigned long long* __restrict__ keys,
                                                           float* __restrict__ out_scores,
                                                           float* __restrict__ out_boxes) {
  __shared__ unsigned long long key[NMS_SORT];
  __shared__ unsigned hist[256];
  __shared__ unsigned long long sh64[2];
  __shared__ unsigned shn[1];
  __shared__ float bx[NMS_T][4];
  __shared__ float sc[NMS_T];
  __shared__ unsigned char dead[NMS_T];
  __shared__ int kept_idx[NMS_T];

  const int b = blockIdx.y, c = blockIdx.x + 1, C = K - 1, tid = threadIdx.x;
  const long base = (long)b * A;
  const int k = min(top_k, A);
  const int n = (int)counts[b * C + c - 1];
  const unsigned long long* list = keys + ((long)b * C + (c - 1)) * A;
  int m;
  if (n <= NMS_SORT) {
    int P = 64;
    while (P < n) P <<= 1;
    for (int i = tid; i < P; i += NMS_T) key[i] = i < n ? list[i] : ~0ull;
    __syncthreads();
    lds_bitonic(key, P);
    m = min(n, k);
  } else {
    // k-th smallest key (keys are distinct: the index is part of the key), 8 x 8-bit digits
    unsigned long long prefix = 0;
    unsigned rank = (unsigned)k;
    for (int shift = 56; shift >= 0; shift -= 8) {
      const unsigned long long hmask = shift >= 56 ? 0ull : (~0ull << (shift + 8));
      for (int i = tid; i < 256; i += NMS_T) hist[i] = 0u;
      __syncthreads();
      for (int i = tid; i < n; i += NMS_T) {
        const unsigned long long v = list[i];
        if ((v & hmask) == (prefix & hmask)) atomicAdd(&hist[(v >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (tid == 0) {
        unsigned acc = 0;
        int d = 0;
        for (; d < 256; ++d) {
          if (acc + hist[d] >= rank) break;
          acc += hist[d];
        }
        sh64[0] = prefix | ((unsigned long long)d << shift);
        sh64[1] = rank - acc;
      }
      __syncthreads();
      prefix = sh64[0];
      rank = (unsigned)sh64[1];
      __syncthreads();
    }
    // the k keys <= the k-th, in any order, then sorted
    if (tid == 0) shn[0] = 0u;
    __syncthreads();
    for (int i = tid; i < n; i += NMS_T) {
      const unsigned long long v = list[i];
      if (v <= prefix) key[atomicAdd(&shn[0], 1u)] = v;
    }
    __syncthreads();
    int P = 64;
    while (P < k) P <<= 1;
    for (int i = k + tid; i < P; i += NMS_T) key[i] = ~0ull;
    __syncthreads();
    lds_bitonic(key, P);
    m = k;
  }
  // gather the m candidates (score desc, index asc), boxes masked as the reference
  if (tid < m) {
    const int a = (int)(key[tid] & 0xFFFFFFFFu);
    const float p = probs[(base + a) * K + c];
    const float fm = p >= sel_thr ? 1.f : 0.f;
    sc[tid] = p * fm;
    const float* bp = boxes + (base + a) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) bx[tid][q] = bp[q] * fm;
    dead[tid] = 0;
  }
  __syncthreads();
  int kept = 0;
  for (int i = 0; i < m && kept < keep_k; ++i) {
    if (dead[i]) continue;  // uniform: dead[] only changes between barriers
    if (tid == 0) kept_idx[kept] = i;
    ++kept;
    for (int j = i + 1 + tid; j < m; j += NMS_T)
      if (!dead[j] && tf_iou(bx[i], bx[j]) > nms_thr) dead[j] = 1;
    __syncthreads();
  }
  __syncthreads();
  float* os = out_scores + ((long)b * C + (c - 1)) * keep_k;
  float* ob = out_boxes + ((long)b * C + (c - 1)) * keep_k * 4;
  for (int j = tid; j < keep_k; j += NMS_T) {
    const bool kk = j < kept;
    const int i = kk ? kept_idx[j] : 0;
    os[j] = kk ? sc[i] : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) ob[j * 4 + q] = kk ? bx[i][q] : 0.f;
  }
}

static size_t nms_counts_bytes(int B, int K) { return ((size_t)B * (K - 1) * sizeof(unsigned) + 255) / 256 * 256; }

}  // namespace rod

using namespace rod;

extern "C" {

size_t rod_select_topk_nms_workspace(int B, int A, int K) {
  if (B <= 0 || A <= 0 || K < 2) return 0;
  return nms_counts_bytes(B, K) + (size_t)B * (K - 1) * A * sizeof(unsigned long long);
}

int rod_select_topk_nms(const float* probs, const float* boxes, int B, int A, int K, float select_threshold,
                        int top_k, int keep_top_k, float nms_threshold, float* out_scores, float* out_boxes,
                        void* workspace, void* stream) {
  ROD_CHECK_ARG(B > 0 && A > 0 && K > 1, "rod_select_topk_nms: bad shape");
  ROD_CHECK_ARG(top_k > 0 && top_k <= NMS_T, "rod_select_topk_nms: top_k must be in [1, %d]", NMS_T);
  ROD_CHECK_ARG(keep_top_k > 0 && keep_top_k <= NMS_T, "rod_select_topk_nms: keep_top_k must be in [1, %d]", NMS_T);
  ROD_CHECK_ARG(B <= 65535, "rod_select_topk_nms: B too large");
  hipStream_t s = ROD_STREAM(stream);
  if (workspace && select_threshold > 0.f && K - 1 <= NMS_MAXC) {
    unsigned* counts = (unsigned*)workspace;
    unsigned long long* keys = (unsigned long long*)((char*)workspace + nms_counts_bytes(B, K));
    hipLaunchKernelGGL(nms_zero_kernel, dim3(cdiv((long)B * (K - 1), 256)), dim3(256), 0, s, counts, B * (K - 1));
    hipLaunchKernelGGL(nms_compact_kernel, dim3(cdiv(A, NMS_CT), B), dim3(256), 0, s, probs, A, K, select_threshold,
                       counts, keys);
    hipLaunchKernelGGL(nms_select_kernel, dim3(K - 1, B), dim3(NMS_T), 0, s, probs, boxes, A, K, select_threshold,
                       top_k, keep_top_k, nms_threshold, counts, keys, out_scores, out_boxes);
  } else {
    hipLaunchKernelGGL(select_topk_nms_kernel, dim3(K - 1, B), dim3(NMS_T), 0, s, probs, boxes, A, K,
                       select_threshold, top_k, keep_top_k, nms_threshold, out_scores, out_boxes);
  }
  return check_launch("rod_select_topk_nms");
}

}  // extern "C"
