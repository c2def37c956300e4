// a6/a7/a8/a12: target gathers + delta encode/decode.
// Reference: lib/anchor.py:11-76 (anchor_target), lib/bbox.py:6-82 (bbox_target),
// lib/utils.py:40-70 (bbox2param), lib/utils.py:83-144 (param2bbox, clamp_bbox).
#include "block_ops.h"

namespace frh {

int32_t launch_compact_lists(int32_t S, const int64_t* labels, int64_t label_seg_stride, const int32_t* num,
                             int64_t max_n, int npred, const int* preds, int32_t** lists,
                             int64_t list_seg_stride, int32_t* counts, int32_t* chunk_counts, hipStream_t st);
size_t compact_workspace(int32_t S, int64_t max_n);

// bbox2param then (p - mean) / std, in the reference's operation order.
__device__ __forceinline__ void encode(float bx1, float by1, float bx2, float by2, float gx1, float gy1,
                                       float gx2, float gy2, const float* m, const float* sd, float out[4]) {
  float bw = (bx2 - bx1) + 1.0f, bh = (by2 - by1) + 1.0f;
  float gw = (gx2 - gx1) + 1.0f, gh = (gy2 - gy1) + 1.0f;
  float bcx = (bx2 + bx1) / 2.0f, bcy = (by2 + by1) / 2.0f;
  float gcx = (gx2 + gx1) / 2.0f, gcy = (gy2 + gy1) / 2.0f;
  float t[4];
  t[0] = (gcx - bcx) / bw;
  t[1] = (gcy - bcy) / bh;
  t[2] = logf(gw / bw);
  t[3] = logf(gh / bh);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float v = (t[k] - 0.0f) / 1.0f;  // bbox2param's own default normalisation
    out[k] = m ? (v - m[k]) / sd[k] : v;
  }
}

__device__ __forceinline__ float clampf_ref(float x, float lo, float hi) {
  // torch.clamp: min(max(x, lo), hi), NaN propagates
  float y = (x < lo) ? lo : x;
  return (y > hi) ? hi : y;
}

// _param2bbox_ (utils.py:134-144) after param*std+mean (utils.py:88); no dw clamp.
__device__ __forceinline__ void decode(float ax1, float ay1, float ax2, float ay2, float p0, float p1, float p2,
                                       float p3, const float* m, const float* sd, int clamp, float img_h,
                                       float img_w, float out[4]) {
  float tx = p0 * sd[0] + m[0];
  float ty = p1 * sd[1] + m[1];
  float tw = p2 * sd[2] + m[2];
  float th = p3 * sd[3] + m[3];
  float bw = (ax2 - ax1) + 1.0f, bh = (ay2 - ay1) + 1.0f;
  float bcx = (ax2 + ax1) / 2.0f, bcy = (ay2 + ay1) / 2.0f;
  float cx = tx * bw + bcx;
  float cy = ty * bh + bcy;
  float w = expf(tw) * bw;
  float h = expf(th) * bh;
  float hw = w / 2.0f, hh = h / 2.0f;
  out[0] = cx - hw;
  out[1] = cy - hh;
  out[2] = cx + hw;
  out[3] = cy + hh;
  if (clamp) {
    float wm = img_w - 1.0f, hm = img_h - 1.0f;
    out[0] = clampf_ref(out[0], 0.0f, wm);
    out[1] = clampf_ref(out[1], 0.0f, hm);
    out[2] = clampf_ref(out[2], 0.0f, wm);
    out[3] = clampf_ref(out[3], 0.0f, hm);
  }
}

struct Norm4 {
  float m[4], s[4];
  int has;
};

__global__ void bbox2param_kernel(const float* base, int64_t ldb, const float* bbox, int64_t ldx, int64_t n,
                                  Norm4 nm, float* out, int64_t ldo) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float r[4];
  encode(base[i], base[ldb + i], base[2 * ldb + i], base[3 * ldb + i], bbox[i], bbox[ldx + i],
         bbox[2 * ldx + i], bbox[3 * ldx + i], nm.has ? nm.m : nullptr, nm.s, r);
#pragma unroll
  for (int k = 0; k < 4; ++k) out[k * ldo + i] = r[k];
}

__global__ void param2bbox_kernel(const float* base, int64_t ldb, const float* param, int64_t ldp, int64_t n,
                                  int ncls, Norm4 nm, int clamp, float img_h, float img_w, float* out,
                                  int64_t ldo) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * ncls) return;
  int64_t c = idx / n, i = idx - c * n;
  float r[4];
  decode(base[i], base[ldb + i], base[2 * ldb + i], base[3 * ldb + i], param[(0 * ncls + c) * ldp + i],
         param[(1 * ncls + c) * ldp + i], param[(2 * ncls + c) * ldp + i], param[(3 * ncls + c) * ldp + i],
         nm.m, nm.s, clamp, img_h, img_w, r);
#pragma unroll
  for (int k = 0; k < 4; ++k) out[(k * ncls + c) * ldo + i] = r[k];
}

__device__ __forceinline__ int64_t seg_prefix(const int32_t* counts, int s, int64_t cap) {
  int64_t off = 0;
  for (int q = 0; q < s; ++q) {
    int64_t c = counts[q * 2];
    off += c < cap ? c : cap;
  }
  return off;
}

struct AnchorTargetArgs {
  const int64_t* labels;
  int64_t label_seg_stride;
  const int32_t* chosen;  // [S, max_boxes] ascending box indices
  const int32_t* counts;  // [S, 2] (slot 0 = chosen count)
  int64_t list_seg_stride;
  const float* anchors;
  int64_t anchor_ld, anchor_seg_stride;
  const float* gts;
  int64_t gt_ld, gt_seg_stride;
  const int64_t* gt_labels;
  int64_t gt_label_seg_stride;
  Norm4 nm;
  int64_t cap;
  int64_t* chosen_idx;
  int32_t* seg_of;
  int64_t* tar_labels;
  float *tar_anchors, *tar_bbox, *tar_param;
  int64_t out_ld;
  int32_t* out_counts;
  int S;
  const int32_t* sel;      // nullable: the device sampler's lists [S][2][sel_ld] (positives, negatives)
  const int32_t* sel_cnt;  // [S][2]
  int64_t sel_ld;
};

__device__ void anchor_target_item(const AnchorTargetArgs& p, int s, int64_t n, int64_t o);

__global__ void anchor_target_kernel(AnchorTargetArgs p) {
  const int s = blockIdx.y;
  int64_t cnt = p.counts[s * 2];
  if (cnt > p.cap) cnt = p.cap;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t off = seg_prefix(p.counts, s, p.cap);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    p.out_counts[s] = (int32_t)cnt;
    if (s == p.S - 1) p.out_counts[p.S] = (int32_t)(off + cnt);
  }
  if (j >= cnt) return;
  anchor_target_item(p, s, p.chosen[(int64_t)s * p.list_seg_stride + j], off + j);
}

// The image's selected boxes = its two sampler lists (disjoint, any order), in ascending
// box order: each item's output position is the number of listed boxes below it (rank by
// counting over the list staged in LDS) -- the reference's nonzero(labels >= 0) order
// (anchor.py:49-50, bbox.py:52-58) without a compaction pass over every box.
// Dynamic LDS: 2 * sel_ld + 4 int32.  Counts are clamped to the capacity and box indices
// to [0, lim): a no-op for a sampler call that completed, and memory safety for one whose
// in-launch wait ran out (its lists are undefined; the status word says so).
template <class F, class P>
__device__ __forceinline__ void ranked_selection(const int32_t* sel, const int32_t* sel_cnt, int64_t sel_ld, int S,
                                                 int32_t* out_counts, int64_t cap, int64_t lim, F&& item, P&& pad) {
  extern __shared__ __attribute__((aligned(16))) int32_t su[];
  const int s = blockIdx.y;
  const int icap = (int)min(cap, sel_ld);
  auto counts_of = [&](int q, int& pos) {
    const int a = min(max(sel_cnt[2 * q], 0), icap);
    pos = a;
    return a + min(max(sel_cnt[2 * q + 1], 0), icap - a);
  };
  int np;
  const int cnt = counts_of(s, np);
  int64_t off = 0, total = 0;
  for (int q = 0; q < S; ++q) {
    int pq;
    const int64_t c = counts_of(q, pq);
    off += q < s ? c : 0;
    total += c;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out_counts[s] = cnt;
    if (s == S - 1) out_counts[S] = (int32_t)total;
  }
  // rows [total, S * cap) of the output get neutral values (ignored label), so a caller may
  // consume the whole capacity with the device count instead of synchronising on it: this
  // segment writes its cap - cnt share, starting at total + s * cap - off
  {
    const int64_t jp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (jp >= cnt && jp < cap) pad(total + (int64_t)s * cap - off + (jp - cnt));
  }
  if ((int64_t)blockIdx.x * blockDim.x >= cnt) return;  // uniform per workgroup
  const int32_t* pos = sel + (int64_t)(2 * s) * sel_ld;
  const int32_t* neg = pos + sel_ld;
  const int cnt4 = (cnt + 3) & ~3;  // padded with INT32_MAX (never below an index): 16-B LDS reads
  for (int q = threadIdx.x; q < cnt4; q += blockDim.x) su[q] = q < np ? pos[q] : (q < cnt ? neg[q - np] : INT32_MAX);
  __syncthreads();
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cnt) return;
  // rank among the listed values, equal values by list position: a permutation of [0, cnt)
  // whatever the lists hold (a valid selection lists distinct boxes; the lists of an aborted
  // call -- status word set -- may repeat values, and every output row must still be written)
  const int32_t raw = su[j];
  const int32_t x = min(max(raw, 0), (int32_t)(lim > 0 ? lim - 1 : 0));
  int rank = 0;
  const int4* s4 = reinterpret_cast<const int4*>(su);
  // (one comparison per value: <= before position j, < from it on)
  const int jq = j >> 2, jr = j & 3;
  for (int q = 0; q < jq; ++q) {
    const int4 v = s4[q];
    rank += (v.x <= raw) + (v.y <= raw) + (v.z <= raw) + (v.w <= raw);
  }
  {
    const int4 v = s4[jq];
    rank += (jr > 0 ? v.x <= raw : v.x < raw) + (jr > 1 ? v.y <= raw : v.y < raw) + (jr > 2 ? v.z <= raw : v.z < raw) +
            (v.w < raw);
  }
  for (int q = jq + 1; q < cnt4 / 4; ++q) {
    const int4 v = s4[q];
    rank += (v.x < raw) + (v.y < raw) + (v.z < raw) + (v.w < raw);
  }
  item(s, (int64_t)x, off + rank);
}

__global__ void anchor_target_sel_kernel(AnchorTargetArgs p) {
  ranked_selection(p.sel, p.sel_cnt, p.sel_ld, p.S, p.out_counts, p.cap, p.list_seg_stride,
                   [&](int s, int64_t n, int64_t o) { anchor_target_item(p, s, n, o); },
                   [&](int64_t o) {  // padding row: no anchor (seg -1), label -1 (ignored), zero targets
                     p.chosen_idx[o] = 0;
                     p.seg_of[o] = -1;
                     p.tar_labels[o] = -1;
#pragma unroll
                     for (int k = 0; k < 4; ++k)
                       p.tar_anchors[k * p.out_ld + o] = p.tar_bbox[k * p.out_ld + o] = p.tar_param[k * p.out_ld + o] = 0.0f;
                   });
}

__device__ void anchor_target_item(const AnchorTargetArgs& p, int s, int64_t n, int64_t o) {
  const int64_t lab = p.labels[(int64_t)s * p.label_seg_stride + n];
  const int64_t g = lab > 0 ? lab - 1 : 0;
  const float* a = p.anchors + (int64_t)s * p.anchor_seg_stride;
  const float* gt = p.gts + (int64_t)s * p.gt_seg_stride;
  float ax1 = a[n], ay1 = a[p.anchor_ld + n], ax2 = a[2 * p.anchor_ld + n], ay2 = a[3 * p.anchor_ld + n];
  float gx1 = gt[g], gy1 = gt[p.gt_ld + g], gx2 = gt[2 * p.gt_ld + g], gy2 = gt[3 * p.gt_ld + g];
  float r[4];
  encode(ax1, ay1, ax2, ay2, gx1, gy1, gx2, gy2, p.nm.has ? p.nm.m : nullptr, p.nm.s, r);
  p.chosen_idx[o] = n;
  p.seg_of[o] = s;
  int64_t tl = 0;
  if (lab > 0) tl = p.gt_labels ? p.gt_labels[(int64_t)s * p.gt_label_seg_stride + g] : 1;
  p.tar_labels[o] = tl;
  const float av[4] = {ax1, ay1, ax2, ay2}, gv[4] = {gx1, gy1, gx2, gy2};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    p.tar_anchors[k * p.out_ld + o] = av[k];
    p.tar_bbox[k * p.out_ld + o] = gv[k];
    p.tar_param[k * p.out_ld + o] = r[k];
  }
}

// Per-level head outputs [B, C * A, H, W] with explicit element strides (b, c, y, x):
// NCHW and channels-last alike.  Level-local anchor index loc = a * H * W + y * W + x (the
// reference's [C, A * H * W] view, anchor_head.py:82); output channel c of anchor a is
// tensor channel c * A + a.
struct LevelMap {
  const float* ptr[FRH_MAX_LEVELS];
  int64_t off[FRH_MAX_LEVELS + 1];
  int64_t sb[FRH_MAX_LEVELS], sc[FRH_MAX_LEVELS], sy[FRH_MAX_LEVELS], sx[FRH_MAX_LEVELS];
  uint32_t hw[FRH_MAX_LEVELS], w[FRH_MAX_LEVELS];
  int A;
  int n;
};

__device__ __forceinline__ int64_t level_elem(const LevelMap& lm, int l, int b, int c, int64_t loc) {
  const uint32_t u = (uint32_t)loc, a = u / lm.hw[l], sp = u - a * lm.hw[l], y = sp / lm.w[l], x = sp - y * lm.w[l];
  return (int64_t)b * lm.sb[l] + (int64_t)(c * lm.A + (int)a) * lm.sc[l] + (int64_t)y * lm.sy[l] +
         (int64_t)x * lm.sx[l];
}

__global__ void gather_levels_kernel(LevelMap lm, int C, int64_t total, const int64_t* chosen,
                                     const int32_t* seg_of, float* out, int64_t out_ld) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  int64_t n = chosen[j];
  int b = seg_of[j];
  if (b < 0) {  // padding row of a fixed-capacity target buffer
    for (int c = 0; c < C; ++c) out[c * out_ld + j] = 0.0f;
    return;
  }
  int l = 0;
  while (l + 1 < lm.n && n >= lm.off[l + 1]) ++l;
  const int64_t loc = n - lm.off[l];
  for (int c = 0; c < C; ++c) out[c * out_ld + j] = lm.ptr[l][level_elem(lm, l, b, c, loc)];
}

__global__ void scatter_levels_kernel(LevelMap lm, int C, int64_t total, const int64_t* chosen,
                                      const int32_t* seg_of, const float* grad, int64_t grad_ld) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  int64_t n = chosen[j];
  int b = seg_of[j];
  if (b < 0) return;  // padding row: no gradient (and no read-modify-write race with a real row)
  int l = 0;
  while (l + 1 < lm.n && n >= lm.off[l + 1]) ++l;
  const int64_t loc = n - lm.off[l];
  float* dst = const_cast<float*>(lm.ptr[l]);
  for (int c = 0; c < C; ++c) dst[level_elem(lm, l, b, c, loc)] += grad[c * grad_ld + j];
}

__global__ void prepend_gt_kernel(const int64_t* prop_labels, int64_t pstride, const int32_t* num_props,
                                  const int32_t* num_gts, int64_t max_rows, int64_t* rows, int64_t rstride,
                                  int32_t* num_rows) {
  const int s = blockIdx.y;
  const int64_t G = num_gts[s], n = num_props[s];
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j == 0) num_rows[s] = (int32_t)(G + n);
  if (j >= max_rows) return;  // rows past G + n: padding label -1
  rows[(int64_t)s * rstride + j] = j < G ? j + 1 : (j < G + n ? prop_labels[(int64_t)s * pstride + (j - G)] : -1);
}

struct BBoxTargetArgs {
  const int64_t* labels;
  int64_t label_seg_stride;
  const int32_t* chosen;
  const int32_t* counts;
  int64_t list_seg_stride;
  const int32_t* num_gts;
  const float* props;
  int64_t prop_ld, prop_seg_stride;
  const float* gts;
  int64_t gt_ld, gt_seg_stride;
  const int64_t* gt_labels;
  int64_t gt_label_seg_stride;
  Norm4 nm;
  int64_t cap;
  float *tar_props, *tar_bbox, *tar_param;
  int64_t *tar_label, *tar_is_gt;
  int64_t out_ld;
  int32_t* out_counts;
  int S;
  const int32_t* sel;      // nullable: the device sampler's lists [S][2][sel_ld]
  const int32_t* sel_cnt;  // [S][2]
  int64_t sel_ld;
};

__device__ void bbox_target_item(const BBoxTargetArgs& p, int s, int64_t row, int64_t o);

__global__ void bbox_target_kernel(BBoxTargetArgs p) {
  const int s = blockIdx.y;
  int64_t cnt = p.counts[s * 2];
  if (cnt > p.cap) cnt = p.cap;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t off = seg_prefix(p.counts, s, p.cap);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    p.out_counts[s] = (int32_t)cnt;
    if (s == p.S - 1) p.out_counts[p.S] = (int32_t)(off + cnt);
  }
  if (j >= cnt) return;
  bbox_target_item(p, s, p.chosen[(int64_t)s * p.list_seg_stride + j], off + j);
}

__global__ void bbox_target_sel_kernel(BBoxTargetArgs p) {
  ranked_selection(p.sel, p.sel_cnt, p.sel_ld, p.S, p.out_counts, p.cap, p.list_seg_stride,
                   [&](int s, int64_t row, int64_t o) { bbox_target_item(p, s, row, o); },
                   [&](int64_t o) {  // padding row: zero box, label -1 (ignored), not a gt
                     p.tar_label[o] = -1;
                     p.tar_is_gt[o] = 0;
#pragma unroll
                     for (int k = 0; k < 4; ++k)
                       p.tar_props[k * p.out_ld + o] = p.tar_bbox[k * p.out_ld + o] = p.tar_param[k * p.out_ld + o] = 0.0f;
                   });
}

__device__ void bbox_target_item(const BBoxTargetArgs& p, int s, int64_t row, int64_t o) {
  const int64_t lab = p.labels[(int64_t)s * p.label_seg_stride + row];
  const int64_t G = p.num_gts[s];
  const int64_t g = lab > 0 ? lab - 1 : 0;
  const float* gt = p.gts + (int64_t)s * p.gt_seg_stride;
  float bv[4];
  if (row < G) {
#pragma unroll
    for (int k = 0; k < 4; ++k) bv[k] = gt[k * p.gt_ld + row];
  } else {
    const float* pr = p.props + (int64_t)s * p.prop_seg_stride;
#pragma unroll
    for (int k = 0; k < 4; ++k) bv[k] = pr[k * p.prop_ld + (row - G)];
  }
  float gv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) gv[k] = gt[k * p.gt_ld + g];
  float r[4];
  encode(bv[0], bv[1], bv[2], bv[3], gv[0], gv[1], gv[2], gv[3], p.nm.has ? p.nm.m : nullptr, p.nm.s, r);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    p.tar_props[k * p.out_ld + o] = bv[k];
    p.tar_bbox[k * p.out_ld + o] = gv[k];
    p.tar_param[k * p.out_ld + o] = r[k];
  }
  p.tar_label[o] = lab > 0 ? p.gt_labels[(int64_t)s * p.gt_label_seg_stride + g] : 0;
  p.tar_is_gt[o] = row < G ? 1 : 0;
}

static Norm4 make_norm(const float* means, const float* stds) {
  Norm4 nm{};
  nm.has = (means && stds) ? 1 : 0;
  for (int k = 0; k < 4; ++k) {
    nm.m[k] = means ? means[k] : 0.f;
    nm.s[k] = stds ? stds[k] : 1.f;
  }
  return nm;
}

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

}  // namespace frh

using namespace frh;

extern "C" int32_t frh_bbox2param(const float* base, int64_t ldb, const float* bbox, int64_t ldx, int64_t n,
                                  const float* means, const float* stds, float* out, int64_t ldo,
                                  void* stream) {
  FRH_REQUIRE(n >= 0, "negative size");
  if (n == 0) return FRH_OK;
  FRH_REQUIRE(base && bbox && out, "null pointer argument");
  hipLaunchKernelGGL(bbox2param_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), base,
                     ldb, bbox, ldx, n, make_norm(means, stds), out, ldo);
  return check_launch("frh_bbox2param");
}

extern "C" int32_t frh_param2bbox(const float* base, int64_t ldb, const float* param, int64_t ldp, int64_t n,
                                  int32_t ncls, const float* means, const float* stds, int32_t clamp,
                                  float img_h, float img_w, float* out, int64_t ldo, void* stream) {
  FRH_REQUIRE(n >= 0 && ncls >= 1, "bad sizes");
  if (n == 0) return FRH_OK;
  FRH_REQUIRE(base && param && out, "null pointer argument");
  Norm4 nm = make_norm(means, stds);
  int64_t total = n * ncls;
  hipLaunchKernelGGL(param2bbox_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                     base, ldb, param, ldp, n, ncls, nm, clamp, img_h, img_w, out, ldo);
  return check_launch("frh_param2bbox");
}

extern "C" size_t frh_anchor_target_workspace(int32_t num_segs, int64_t max_boxes) {
  return align256(compact_workspace(num_segs, max_boxes)) +
         align256((size_t)num_segs * (size_t)(max_boxes > 0 ? max_boxes : 1) * sizeof(int32_t)) +
         (size_t)num_segs * 2 * sizeof(int32_t);
}

extern "C" int32_t frh_anchor_target(int32_t num_segs, const int64_t* labels, int64_t label_seg_stride,
                                     const int32_t* num_boxes, int64_t max_boxes, const float* anchors,
                                     int64_t anchor_ld, int64_t anchor_seg_stride, const float* gts,
                                     int64_t gt_ld, int64_t gt_seg_stride, const int64_t* gt_labels,
                                     int64_t gt_label_seg_stride, const float* means, const float* stds,
                                     int64_t max_out_per_seg, const int32_t* sel, const int32_t* sel_counts,
                                     int64_t* chosen_idx, int32_t* seg_of,
                                     int64_t* tar_labels, float* tar_anchors, float* tar_bbox,
                                     float* tar_param, int64_t out_ld, int32_t* out_counts, void* workspace,
                                     size_t ws_bytes, void* stream) {
  FRH_REQUIRE(num_segs >= 1 && max_boxes >= 0 && max_out_per_seg >= 0, "bad sizes");
  FRH_REQUIRE(labels && num_boxes && anchors && gts && chosen_idx && seg_of && tar_labels && tar_anchors &&
                  tar_bbox && tar_param && out_counts,
              "null pointer argument");
  FRH_REQUIRE(out_ld >= (int64_t)num_segs * max_out_per_seg, "out_ld too small");
  FRH_REQUIRE(!sel == !sel_counts, "sel and sel_counts go together");
  hipStream_t st = as_stream(stream);
  unsigned gx = (unsigned)((max_out_per_seg + 255) / 256);
  if (sel) {  // the device sampler's lists: no compaction pass (sel_ld = max_out_per_seg)
    FRH_REQUIRE((2 * max_out_per_seg + 4) * sizeof(int32_t) <= 65536, "sampler lists exceed the LDS stage");
    // sel mode: list_seg_stride carries max_boxes, the bound of the lists' box indices
    AnchorTargetArgs p{labels, label_seg_stride, nullptr, nullptr, max_boxes, anchors, anchor_ld, anchor_seg_stride,
                       gts, gt_ld, gt_seg_stride, gt_labels, gt_label_seg_stride, make_norm(means, stds),
                       max_out_per_seg, chosen_idx, seg_of, tar_labels, tar_anchors, tar_bbox, tar_param, out_ld,
                       out_counts, num_segs, sel, sel_counts, max_out_per_seg};
    hipLaunchKernelGGL(anchor_target_sel_kernel, dim3(gx > 0 ? gx : 1, (unsigned)num_segs), dim3(256),
                       (2 * max_out_per_seg + 4) * sizeof(int32_t), st, p);
    return check_launch("frh_anchor_target");
  }
  FRH_REQUIRE(workspace && ws_bytes >= frh_anchor_target_workspace(num_segs, max_boxes), "workspace too small");
  char* ws = reinterpret_cast<char*>(workspace);
  int32_t* chunk_counts = reinterpret_cast<int32_t*>(ws);
  size_t a = align256(compact_workspace(num_segs, max_boxes));
  int32_t* chosen = reinterpret_cast<int32_t*>(ws + a);
  size_t b = align256((size_t)num_segs * (size_t)(max_boxes > 0 ? max_boxes : 1) * sizeof(int32_t));
  int32_t* counts = reinterpret_cast<int32_t*>(ws + a + b);
  int preds[1] = {kChosen};
  int32_t* lists[1] = {chosen};
  int32_t r = launch_compact_lists(num_segs, labels, label_seg_stride, num_boxes, max_boxes, 1, preds, lists,
                                   max_boxes, counts, chunk_counts, st);
  if (r) return r;
  AnchorTargetArgs p{labels, label_seg_stride, chosen, counts, max_boxes, anchors, anchor_ld, anchor_seg_stride,
                     gts, gt_ld, gt_seg_stride, gt_labels, gt_label_seg_stride, make_norm(means, stds),
                     max_out_per_seg, chosen_idx, seg_of, tar_labels, tar_anchors, tar_bbox, tar_param, out_ld,
                     out_counts, num_segs, nullptr, nullptr, 0};
  hipLaunchKernelGGL(anchor_target_kernel, dim3(gx > 0 ? gx : 1, (unsigned)num_segs), dim3(256), 0, st, p);
  return check_launch("frh_anchor_target");
}

// strides: [L][4] element strides (b, c, y, x); hw: [L][2] grid (H, W); A anchors per cell
static int32_t make_levelmap(int32_t L, const float* const* ptrs, const int64_t* off, const int32_t* hw,
                             const int64_t* strides, int32_t A, LevelMap* lm) {
  FRH_REQUIRE(L >= 1 && L <= FRH_MAX_LEVELS, "bad level count");
  FRH_REQUIRE(ptrs && off && hw && strides && A >= 1, "null pointer argument");
  lm->n = L;
  lm->A = A;
  for (int l = 0; l < L; ++l) {
    lm->ptr[l] = ptrs[l];
    lm->off[l] = off[l];
    FRH_REQUIRE(hw[2 * l] >= 1 && hw[2 * l + 1] >= 1, "empty level %d", l);
    lm->w[l] = (uint32_t)hw[2 * l + 1];
    lm->hw[l] = (uint32_t)hw[2 * l] * (uint32_t)hw[2 * l + 1];
    lm->sb[l] = strides[4 * l];
    lm->sc[l] = strides[4 * l + 1];
    lm->sy[l] = strides[4 * l + 2];
    lm->sx[l] = strides[4 * l + 3];
  }
  lm->off[L] = off[L - 1] + (int64_t)A * hw[2 * L - 2] * hw[2 * L - 1];
  return FRH_OK;
}

// the contiguous [B, C, A*H*W] form of the non-strided entries: one anchor per "cell", W = A*H*W
static int32_t contiguous_levelmap(int32_t L, const float* const* ptrs, const int64_t* off, const int64_t* hwa,
                                   int32_t channels, LevelMap* lm) {
  FRH_REQUIRE(L >= 1 && L <= FRH_MAX_LEVELS, "bad level count");
  FRH_REQUIRE(hwa, "null pointer argument");
  int32_t hw[2 * FRH_MAX_LEVELS];
  int64_t st[4 * FRH_MAX_LEVELS];
  for (int l = 0; l < L; ++l) {
    FRH_REQUIRE(hwa[l] >= 1 && hwa[l] < ((int64_t)1 << 31), "bad level size");
    hw[2 * l] = 1;
    hw[2 * l + 1] = (int32_t)hwa[l];
    st[4 * l] = (int64_t)channels * hwa[l];
    st[4 * l + 1] = hwa[l];
    st[4 * l + 2] = hwa[l];
    st[4 * l + 3] = 1;
  }
  return make_levelmap(L, ptrs, off, hw, st, 1, lm);
}

static int32_t launch_gather(const LevelMap& lm, int32_t channels, int64_t total, const int64_t* chosen_idx,
                             const int32_t* seg_of, float* out, int64_t out_ld, void* stream) {
  FRH_REQUIRE(channels >= 1 && total >= 0, "bad sizes");
  if (total == 0) return FRH_OK;
  FRH_REQUIRE(chosen_idx && seg_of && out, "null pointer argument");
  hipLaunchKernelGGL(gather_levels_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                     lm, channels, total, chosen_idx, seg_of, out, out_ld);
  return check_launch("frh_gather_level_outputs");
}

static int32_t launch_scatter(const LevelMap& lm, int32_t channels, int64_t total, const int64_t* chosen_idx,
                              const int32_t* seg_of, const float* grad, int64_t grad_ld, void* stream) {
  FRH_REQUIRE(channels >= 1 && total >= 0, "bad sizes");
  if (total == 0) return FRH_OK;
  FRH_REQUIRE(chosen_idx && seg_of && grad, "null pointer argument");
  hipLaunchKernelGGL(scatter_levels_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     as_stream(stream), lm, channels, total, chosen_idx, seg_of, grad, grad_ld);
  return check_launch("frh_scatter_level_grads");
}

extern "C" int32_t frh_gather_level_outputs(int32_t num_levels, const float* const* level_ptrs,
                                            const int64_t* level_off, const int64_t* level_hw_a,
                                            int32_t channels, int64_t total, const int64_t* chosen_idx,
                                            const int32_t* seg_of, float* out, int64_t out_ld, void* stream) {
  LevelMap lm;
  int32_t r = contiguous_levelmap(num_levels, level_ptrs, level_off, level_hw_a, channels, &lm);
  if (r) return r;
  return launch_gather(lm, channels, total, chosen_idx, seg_of, out, out_ld, stream);
}

extern "C" int32_t frh_scatter_level_grads(int32_t num_levels, float* const* level_grads,
                                           const int64_t* level_off, const int64_t* level_hw_a, int32_t channels,
                                           int64_t total, const int64_t* chosen_idx, const int32_t* seg_of,
                                           const float* grad, int64_t grad_ld, void* stream) {
  LevelMap lm;
  int32_t r = contiguous_levelmap(num_levels, const_cast<const float* const*>(level_grads), level_off, level_hw_a,
                                  channels, &lm);
  if (r) return r;
  return launch_scatter(lm, channels, total, chosen_idx, seg_of, grad, grad_ld, stream);
}

extern "C" int32_t frh_gather_level_outputs_strided(int32_t num_levels, const float* const* level_ptrs,
                                                    const int64_t* level_off, const int32_t* level_hw,
                                                    const int64_t* level_strides, int32_t num_anchors,
                                                    int32_t channels, int64_t total, const int64_t* chosen_idx,
                                                    const int32_t* seg_of, float* out, int64_t out_ld,
                                                    void* stream) {
  LevelMap lm;
  int32_t r = make_levelmap(num_levels, level_ptrs, level_off, level_hw, level_strides, num_anchors, &lm);
  if (r) return r;
  return launch_gather(lm, channels, total, chosen_idx, seg_of, out, out_ld, stream);
}

extern "C" int32_t frh_scatter_level_grads_strided(int32_t num_levels, float* const* level_grads,
                                                   const int64_t* level_off, const int32_t* level_hw,
                                                   const int64_t* level_strides, int32_t num_anchors,
                                                   int32_t channels, int64_t total, const int64_t* chosen_idx,
                                                   const int32_t* seg_of, const float* grad, int64_t grad_ld,
                                                   void* stream) {
  LevelMap lm;
  int32_t r = make_levelmap(num_levels, const_cast<const float* const*>(level_grads), level_off, level_hw,
                            level_strides, num_anchors, &lm);
  if (r) return r;
  return launch_scatter(lm, channels, total, chosen_idx, seg_of, grad, grad_ld, stream);
}

extern "C" int32_t frh_prepend_gt_labels(int32_t num_segs, const int64_t* prop_labels,
                                         int64_t prop_label_seg_stride, const int32_t* num_props,
                                         const int32_t* num_gts, int64_t max_rows, int64_t* rows_out,
                                         int64_t rows_seg_stride, int32_t* num_rows, void* stream) {
  FRH_REQUIRE(num_segs >= 0 && max_rows >= 0, "bad sizes");
  if (num_segs == 0) return FRH_OK;
  FRH_REQUIRE(prop_labels && num_props && num_gts && rows_out && num_rows, "null pointer argument");
  unsigned gx = (unsigned)((max_rows + 255) / 256);
  hipLaunchKernelGGL(prepend_gt_kernel, dim3(gx > 0 ? gx : 1, (unsigned)num_segs), dim3(256), 0, as_stream(stream),
                     prop_labels, prop_label_seg_stride, num_props, num_gts, max_rows, rows_out, rows_seg_stride,
                     num_rows);
  return check_launch("frh_prepend_gt_labels");
}

extern "C" size_t frh_bbox_target_workspace(int32_t num_segs, int64_t max_rows) {
  return frh_anchor_target_workspace(num_segs, max_rows);
}

extern "C" int32_t frh_bbox_target(int32_t num_segs, const int64_t* labels, int64_t label_seg_stride,
                                   const int32_t* num_rows, const int32_t* num_gts, int64_t max_rows,
                                   const float* props, int64_t prop_ld, int64_t prop_seg_stride, const float* gts,
                                   int64_t gt_ld, int64_t gt_seg_stride, const int64_t* gt_labels,
                                   int64_t gt_label_seg_stride, const float* means, const float* stds,
                                   int64_t max_out_per_seg, const int32_t* sel, const int32_t* sel_counts,
                                   float* tar_props, float* tar_bbox,
                                   int64_t* tar_label, float* tar_param, int64_t* tar_is_gt, int64_t out_ld,
                                   int32_t* out_counts, void* workspace, size_t ws_bytes, void* stream) {
  FRH_REQUIRE(num_segs >= 1 && max_rows >= 0 && max_out_per_seg >= 0, "bad sizes");
  FRH_REQUIRE(labels && num_rows && num_gts && props && gts && gt_labels && tar_props && tar_bbox && tar_label &&
                  tar_param && tar_is_gt && out_counts,
              "null pointer argument");
  FRH_REQUIRE(out_ld >= (int64_t)num_segs * max_out_per_seg, "out_ld too small");
  FRH_REQUIRE(!sel == !sel_counts, "sel and sel_counts go together");
  hipStream_t st = as_stream(stream);
  unsigned gx = (unsigned)((max_out_per_seg + 255) / 256);
  if (sel) {  // the device sampler's lists: no compaction pass (sel_ld = max_out_per_seg)
    FRH_REQUIRE((2 * max_out_per_seg + 4) * sizeof(int32_t) <= 65536, "sampler lists exceed the LDS stage");
    // sel mode: list_seg_stride carries max_rows, the bound of the lists' row indices
    BBoxTargetArgs p{labels, label_seg_stride, nullptr, nullptr, max_rows, num_gts, props, prop_ld, prop_seg_stride,
                     gts, gt_ld, gt_seg_stride, gt_labels, gt_label_seg_stride, make_norm(means, stds),
                     max_out_per_seg, tar_props, tar_bbox, tar_param, tar_label, tar_is_gt, out_ld, out_counts,
                     num_segs, sel, sel_counts, max_out_per_seg};
    hipLaunchKernelGGL(bbox_target_sel_kernel, dim3(gx > 0 ? gx : 1, (unsigned)num_segs), dim3(256),
                       (2 * max_out_per_seg + 4) * sizeof(int32_t), st, p);
    return check_launch("frh_bbox_target");
  }
  FRH_REQUIRE(workspace && ws_bytes >= frh_bbox_target_workspace(num_segs, max_rows), "workspace too small");
  char* ws = reinterpret_cast<char*>(workspace);
  int32_t* chunk_counts = reinterpret_cast<int32_t*>(ws);
  size_t a = align256(compact_workspace(num_segs, max_rows));
  int32_t* chosen = reinterpret_cast<int32_t*>(ws + a);
  size_t b = align256((size_t)num_segs * (size_t)(max_rows > 0 ? max_rows : 1) * sizeof(int32_t));
  int32_t* counts = reinterpret_cast<int32_t*>(ws + a + b);
  int preds[1] = {kChosen};
  int32_t* lists[1] = {chosen};
  int32_t r = launch_compact_lists(num_segs, labels, label_seg_stride, num_rows, max_rows, 1, preds, lists,
                                   max_rows, counts, chunk_counts, st);
  if (r) return r;
  BBoxTargetArgs p{labels, label_seg_stride, chosen, counts, max_rows, num_gts, props, prop_ld, prop_seg_stride,
                   gts, gt_ld, gt_seg_stride, gt_labels, gt_label_seg_stride, make_norm(means, stds),
                   max_out_per_seg, tar_props, tar_bbox, tar_param, tar_label, tar_is_gt, out_ld, out_counts,
                   num_segs, nullptr, nullptr, 0};
  hipLaunchKernelGGL(bbox_target_kernel, dim3(gx > 0 ? gx : 1, (unsigned)num_segs), dim3(256), 0, st, p);
  return check_launch("frh_bbox_target");
}
