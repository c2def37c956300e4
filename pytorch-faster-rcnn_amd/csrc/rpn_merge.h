// The RPN proposals' cross-level merge (reference lib/heads/rpn_head.py:81-118: concatenate the
// levels' NMS survivors, then the top max_num by score), shared by proposals.hip
// (rpn_merge_wide_kernel, its own launch) and nms.hip (the one-launch NMS's merge workgroups).
#pragma once
#include "common.h"
#include "seg_topk.h"

namespace frh {

struct MergeArgs {
  const float* sel_boxes;
  const float* sel_scores;
  const int32_t* keep;
  const int32_t* keep_count;
  int L, P;
  int max_num;  // <= 0: no cut
  int64_t out_cap;
  float* out_boxes;   // [B][4][out_cap]
  float* out_scores;  // [B][out_cap]
  int32_t* out_counts;
};

// The merge over the one-launch NMS's compact kept scores (nms.hip kscore: [seg][j] = the
// score of keep[j]): grid (survivor chunks of kMwThreads, level, image), ONE survivor per
// thread, so the image's ranks are spread over ~40 CUs instead of one workgroup per level
// (rpn_merge_lds_kernel: the binary searches of 2 survivors per thread against 4 levels are
// LDS-bound on 10 CUs -- as were the same searches run by the NMS launch's own scan
// workgroups, a folded form measured and removed in round 5).  Each workgroup stages the
// other levels' kept scores of its image (one round trip, kMwGather loads per thread in
// flight; no keep-index indirection) and searches them with kMwSearch levels in lock step.
constexpr int kMwThreads = 512;
constexpr int kMwGather = 16;
constexpr int kMwSearch = 4;

// kXwg: the keep lists, counts and kept scores were written by other workgroups of the SAME
// launch (nms_fused_kernel's scans, write-through) -- read them with sc1 loads (hand-off table
// row 1); else by an earlier launch -- plain loads.  ms: (L - 1) * P floats of LDS.
template <bool kXwg>
__device__ __forceinline__ int32_t mw_load(const int32_t* q) {
  if constexpr (kXwg) return xwg_load(q);
  else return *q;
}
template <bool kXwg>
__device__ __forceinline__ uint32_t mw_load(const uint32_t* q) {
  if constexpr (kXwg) return xwg_load(q);
  else return *q;
}

template <bool kXwg>
__device__ __forceinline__ void merge_wide_body(MergeArgs p, const uint32_t* __restrict__ kscore, int chunk, int l,
                                                int b, float* ms) {
  __shared__ int cnt_s[FRH_MAX_LEVELS], beg_s[FRH_MAX_LEVELS];
  const int L = p.L, t = threadIdx.x;
  const int seg = b * L + l, j = chunk * kMwThreads + t, jc = min(j, p.P - 1);
  const int cv = t < L ? mw_load<kXwg>(p.keep_count + b * L + t) : 0;  // in flight with the own survivor
  const int pos_raw = mw_load<kXwg>(p.keep + (int64_t)seg * p.P + jc);
  const uint32_t scb = mw_load<kXwg>(kscore + (int64_t)seg * p.P + jc);
  if (t < L) cnt_s[t] = min(max(cv, 0), p.P);
  __syncthreads();
  if (t == 0) {
    int o = 0;
    for (int q = 0; q < L; ++q) {
      beg_s[q] = o;
      o += q == l ? 0 : cnt_s[q];
    }
  }
  int total = 0, base = 0;
  for (int q = 0; q < L; ++q) {
    const int c = cnt_s[q];
    base += q < l ? c : 0;
    total += c;
  }
  const int own_n = cnt_s[l];
  const bool cut = p.max_num > 0 && total > p.max_num;
  if (chunk == 0 && l == 0 && t == 0) p.out_counts[b] = cut ? p.max_num : total;
  if (chunk * kMwThreads >= own_n) return;  // workgroup-uniform
  const bool live = j < own_n;
  const float4 bx = reinterpret_cast<const float4*>(p.sel_boxes)[(int64_t)seg * p.P + min(max(pos_raw, 0), p.P - 1)];
  __syncthreads();  // beg_s
  if (cut) {
    const int n_other = total - own_n;
    for (int e0 = 0; e0 < n_other; e0 += kMwThreads * kMwGather) {
      uint32_t v[kMwGather];
#pragma unroll
      for (int u = 0; u < kMwGather; ++u) {
        const int e = e0 + u * kMwThreads + t;
        int q = l == 0 ? 1 : 0;  // the level holding packed entry e
#pragma unroll 1
        for (int r = q + 1; r < L; ++r)
          if (r != l && beg_s[r] <= e) q = r;
        v[u] = e < n_other ? mw_load<kXwg>(kscore + (int64_t)(b * L + q) * p.P + (e - beg_s[q])) : 0u;
      }
#pragma unroll
      for (int u = 0; u < kMwGather; ++u) {
        const int e = e0 + u * kMwThreads + t;
        if (e < n_other) ms[e] = __uint_as_float(v[u]);
      }
    }
    __syncthreads();
  }
  const float sc = __uint_as_float(scb);
  int rank = base + j;
  if (cut) {
    rank = j;
    for (int k0 = 0; k0 < L - 1; k0 += kMwSearch) {
      int qv[kMwSearch], qb[kMwSearch], qc[kMwSearch], lo[kMwSearch], hi[kMwSearch];
      int steps = 0;
#pragma unroll
      for (int i = 0; i < kMwSearch; ++i) {  // other level k = k0 + i is level k + (k >= l)
        const int q = k0 + i + (k0 + i >= l ? 1 : 0);
        qv[i] = q;
        qc[i] = q < L ? __builtin_amdgcn_readfirstlane(cnt_s[q]) : 0;
        qb[i] = q < L ? __builtin_amdgcn_readfirstlane(beg_s[q]) : 0;
        lo[i] = 0;
        hi[i] = qc[i];
        steps = max(steps, 32 - __builtin_clz((uint32_t)qc[i] | 1u));
      }
      for (int n = 0; n < steps; ++n) {  // survivors of level q ordered before (sc, level l)
        float v[kMwSearch];
#pragma unroll
        for (int i = 0; i < kMwSearch; ++i) v[i] = ms[qb[i] + min((lo[i] + hi[i]) >> 1, max(qc[i] - 1, 0))];
#pragma unroll
        for (int i = 0; i < kMwSearch; ++i) {
          const int mid = (lo[i] + hi[i]) >> 1;
          const bool before = qv[i] < l ? (v[i] >= sc) : (v[i] > sc);
          const bool act = lo[i] < hi[i];
          lo[i] = act && before ? mid + 1 : lo[i];
          hi[i] = act && !before ? mid : hi[i];
        }
      }
#pragma unroll
      for (int i = 0; i < kMwSearch; ++i) rank += lo[i];
    }
  }
  if (!live || (cut && rank >= p.max_num)) return;
  float* ob = p.out_boxes + (int64_t)b * 4 * p.out_cap;
  ob[rank] = bx.x;
  ob[p.out_cap + rank] = bx.y;
  ob[2 * p.out_cap + rank] = bx.z;
  ob[3 * p.out_cap + rank] = bx.w;
  p.out_scores[(int64_t)b * p.out_cap + rank] = sc;
}

}  // namespace frh
