// a9: RPN proposals for all (image, level) segments at once.
// Reference: lib/heads/rpn_head.py:68-120 (predict_single_image), decode from
// lib/utils.py:83-144, NMS = torchvision.ops.nms semantics (nms.hip).
//
//  1. select  (1 block of 1024 per segment): radix top-k of the scores
//     (score = sigmoid or 2-way softmax of the logits, recomputed per radix
//     pass straight from the head output), LDS bitonic sort by
//     (score desc, index asc), decode + clamp, min-size compaction.
//  2. NMS mask + scan over all segments (nms.hip), keep <= post_nms.
//  3. merge   (1 block per image): concatenate the levels' survivors and, if
//     more than max_num, keep the best max_num by (score desc, concat order).
#include "seg_topk.h"

namespace frh {

int32_t launch_nms_sorted(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                          double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                          uint64_t* mask, hipStream_t st);
size_t nms_mask_bytes(int32_t S, int32_t n_max);

constexpr int kPropThreads = 1024;
constexpr int kMaxSort = 16384;

struct PropArgs {
  const float* cls[FRH_MAX_LEVELS];
  const float* reg[FRH_MAX_LEVELS];
  int32_t h[FRH_MAX_LEVELS], w[FRH_MAX_LEVELS];
  int64_t off[FRH_MAX_LEVELS];
  int L, A, C;  // levels, anchors per location, cls channels (1 sigmoid, 2 softmax)
  const float* anchors;
  int64_t anchor_ld;
  float m[4], sd[4];
  int pre_nms;
  int P;  // per-segment capacity (max selected)
  // workspace
  float* sel_boxes;   // [S][P][4]
  float* sel_scores;  // [S][P]
  int32_t* sel_idx;   // [S][P] scratch for the selection
  int32_t* sel_count; // [S]
};

struct ImgArgs {
  float hw[2 * 64];
  float min_size[64];
};

__device__ __forceinline__ float score_of(const float* cls, int64_t hwa, int C, int64_t i) {
  if (C == 1) {
    float x = cls[i];
    return 1.0f / (1.0f + expf(-x));
  }
  float x0 = cls[i], x1 = cls[hwa + i];  // softmax over the 2 channels, score = channel 1
  float mx = fmaxf(x0, x1);
  float e0 = expf(x0 - mx), e1 = expf(x1 - mx);
  return e1 / (e0 + e1);
}

// keys = order-preserving u32 of the score; also seeds the top-k state
__global__ void rpn_keys_kernel(PropArgs p, uint32_t* keys, int64_t kld, int32_t* state) {
  const int seg = blockIdx.y;
  const int b = seg / p.L, l = seg % p.L;
  const int64_t hwa = (int64_t)p.A * p.h[l] * p.w[l];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    int n = (int)hwa;
    state[seg * TK_WORDS + TK_N] = n;
    state[seg * TK_WORDS + TK_K] = (p.pre_nms > 0 && p.pre_nms < n) ? p.pre_nms : n;
  }
  if (i >= hwa) return;
  const float* cls = p.cls[l] + (int64_t)b * p.C * hwa;
  keys[(int64_t)seg * kld + i] = float_key(score_of(cls, hwa, p.C, i));
}

// one 1024-thread block per segment: order the selected anchors by
// (score desc, index asc), decode + clamp, min-size filter (order preserving)
__global__ void __launch_bounds__(kPropThreads) rpn_sort_decode_kernel(PropArgs p, ImgArgs ia, const uint32_t* keys,
                                                                       int64_t kld, const int32_t* state,
                                                                       const int32_t* sel, int64_t sel_ld) {
  extern __shared__ uint64_t skeys[];
  __shared__ int wave_tot[kPropThreads / 64];
  const int seg = blockIdx.x;
  const int b = seg / p.L, l = seg % p.L;
  const int64_t hwa = (int64_t)p.A * p.h[l] * p.w[l];
  const float* reg = p.reg[l] + (int64_t)b * 4 * hwa;
  const int m = state[seg * TK_WORDS + TK_K];
  const int P2 = next_pow2(m > 1 ? m : 1);
  const uint32_t* kk = keys + (int64_t)seg * kld;
  const int32_t* sl = sel + (int64_t)seg * sel_ld;
  for (int j = threadIdx.x; j < P2; j += blockDim.x) {
    uint64_t key = 0;
    if (j < m) {
      int i = sl[j];
      key = ((uint64_t)kk[i] << 32) | (uint32_t)(~(uint32_t)i);
    }
    skeys[j] = key;
  }
  __syncthreads();
  block_bitonic_sort_desc(skeys, P2);
  // decode + clamp + min-size filter, order-preserving compaction
  const float img_h = ia.hw[2 * b], img_w = ia.hw[2 * b + 1];
  const float min_size = ia.min_size[b];
  float* ob = p.sel_boxes + (int64_t)seg * p.P * 4;
  float* os = p.sel_scores + (int64_t)seg * p.P;
  int written = 0;
  for (int base = 0; base < m; base += blockDim.x) {
    int j = base + threadIdx.x;
    bool live = j < m;
    float box[4] = {0.f, 0.f, 0.f, 0.f};
    float score = 0.f;
    if (live) {
      uint64_t key = skeys[j];
      int i = (int)(~(uint32_t)key);
      score = key_float((uint32_t)(key >> 32));
      int64_t ai = p.off[l] + i;
      const float* an = p.anchors;
      const int64_t ld = p.anchor_ld;
      float ax1 = an[ai], ay1 = an[ld + ai], ax2 = an[2 * ld + ai], ay2 = an[3 * ld + ai];
      float tx = reg[i] * p.sd[0] + p.m[0];
      float ty = reg[hwa + i] * p.sd[1] + p.m[1];
      float tw = reg[2 * hwa + i] * p.sd[2] + p.m[2];
      float th = reg[3 * hwa + i] * p.sd[3] + p.m[3];
      float bw = (ax2 - ax1) + 1.0f, bh = (ay2 - ay1) + 1.0f;
      float bcx = (ax2 + ax1) / 2.0f, bcy = (ay2 + ay1) / 2.0f;
      float cx = tx * bw + bcx, cy = ty * bh + bcy;
      float ww = expf(tw) * bw, hh = expf(th) * bh;
      float hw2 = ww / 2.0f, hh2 = hh / 2.0f;
      float v[4] = {cx - hw2, cy - hh2, cx + hw2, cy + hh2};
      float hi[4] = {img_w - 1.0f, img_h - 1.0f, img_w - 1.0f, img_h - 1.0f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float y = (v[q] < 0.0f) ? 0.0f : v[q];
        box[q] = (y > hi[q]) ? hi[q] : y;
      }
      if (min_size > 0.0f) {  // rpn_head.py:86-90
        live = (((box[2] - box[0]) + 1.0f) >= min_size) && (((box[3] - box[1]) + 1.0f) >= min_size);
      }
    }
    int tot;
    int r = block_rank(live, wave_tot, &tot);
    if (live) {
      int o = written + r;
      reinterpret_cast<float4*>(ob)[o] = make_float4(box[0], box[1], box[2], box[3]);
      os[o] = score;
    }
    written += tot;
  }
  if (threadIdx.x == 0) p.sel_count[seg] = written;
}

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

// Cross-level top-k as a merge: each level's survivors are already in
// (score desc) order, so the rank of survivor j of level l among all levels
// (score desc, concatenation order on ties) is j + sum over other levels of
// a binary search (upper bound for earlier levels, lower bound for later).
// Grid: (survivor chunks of 256, level, image); no sort, no LDS.
__device__ __forceinline__ float kept_score(const MergeArgs& p, int seg, int j) {
  return p.sel_scores[(int64_t)seg * p.P + p.keep[(int64_t)seg * p.P + j]];
}

__global__ void __launch_bounds__(256) rpn_merge_kernel(MergeArgs p) {
  const int b = blockIdx.z, l = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int seg = b * p.L + l;
  const int cnt = p.keep_count[seg];
  int total = 0, base = 0;
  for (int q = 0; q < p.L; ++q) {
    int c = p.keep_count[b * p.L + q];
    base += q < l ? c : 0;
    total += c;
  }
  const bool cut = p.max_num > 0 && total > p.max_num;
  if (blockIdx.x == 0 && threadIdx.x == 0 && l == 0) p.out_counts[b] = cut ? p.max_num : total;
  if (j >= cnt) return;
  const int pos = p.keep[(int64_t)seg * p.P + j];
  const float s = p.sel_scores[(int64_t)seg * p.P + pos];
  int rank = base + j;
  if (cut) {
    rank = j;
    for (int q = 0; q < p.L; ++q) {
      if (q == l) continue;
      const int oseg = b * p.L + q;
      int lo = 0, hi = p.keep_count[oseg];
      // count of survivors of level q ordered before (s, this level)
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        float o = kept_score(p, oseg, mid);
        bool before = q < l ? (o >= s) : (o > s);
        if (before)
          lo = mid + 1;
        else
          hi = mid;
      }
      rank += lo;
    }
    if (rank >= p.max_num) return;
  }
  float4 bx = reinterpret_cast<const float4*>(p.sel_boxes)[(int64_t)seg * p.P + pos];
  float* ob = p.out_boxes + (int64_t)b * 4 * p.out_cap;
  ob[rank] = bx.x;
  ob[p.out_cap + rank] = bx.y;
  ob[2 * p.out_cap + rank] = bx.z;
  ob[3 * p.out_cap + rank] = bx.w;
  p.out_scores[(int64_t)b * p.out_cap + rank] = s;
}

static size_t al(size_t v) { return (v + 255) & ~(size_t)255; }

struct PropLayout {
  int P;
  size_t boxes, scores, idx, cnt, keep, kcnt, mask, keys, hist, state, cand, total;
  int64_t nmax;
};

static PropLayout prop_layout(int32_t B, int32_t L, const int32_t* grid_hw, int32_t A, int32_t pre_nms) {
  PropLayout z{};
  int P = 1;
  for (int l = 0; l < L; ++l) {
    int64_t n = (int64_t)A * grid_hw[2 * l] * grid_hw[2 * l + 1];
    int64_t k = (pre_nms > 0 && pre_nms < n) ? pre_nms : n;
    if (k > P) P = (int)k;
  }
  z.P = P;
  int64_t nmax = 1;
  for (int l = 0; l < L; ++l) {
    int64_t n = (int64_t)A * grid_hw[2 * l] * grid_hw[2 * l + 1];
    if (n > nmax) nmax = n;
  }
  z.nmax = nmax;
  const size_t S = (size_t)B * L;
  z.boxes = 0;
  z.scores = z.boxes + al(S * P * 4 * sizeof(float));
  z.idx = z.scores + al(S * P * sizeof(float));
  z.cnt = z.idx + al(S * P * sizeof(int32_t));
  z.keep = z.cnt + al(S * sizeof(int32_t));
  z.kcnt = z.keep + al(S * P * sizeof(int32_t));
  z.mask = z.kcnt + al(S * sizeof(int32_t));
  z.keys = z.mask + al(nms_mask_bytes((int32_t)S, P));
  z.hist = z.keys + al(S * (size_t)nmax * sizeof(uint32_t));
  z.state = z.hist + al(tk_hist_bytes((int)S));
  z.cand = z.state + al(tk_state_bytes((int)S));
  z.total = z.cand + al(tk_cand_bytes((int)S));
  return z;
}

}  // namespace frh

using namespace frh;

extern "C" size_t frh_rpn_proposals_workspace(int32_t num_imgs, int32_t num_levels, const int32_t* grid_hw,
                                              int32_t num_anchors, int32_t pre_nms) {
  if (num_imgs <= 0 || num_levels <= 0 || !grid_hw) return 0;
  return prop_layout(num_imgs, num_levels, grid_hw, num_anchors, pre_nms).total;
}

// Where frh_rpn_proposals leaves its per-level NMS input in the workspace (measurement:
// bench.py replays that NMS alone).  out = {boxes byte offset ([S, P, 4] f32, rows in
// descending-score order), counts byte offset ([S] int32), P, S}.
extern "C" int32_t frh_rpn_proposals_nms_view(int32_t num_imgs, int32_t num_levels, const int32_t* grid_hw,
                                              int32_t num_anchors, int32_t pre_nms, int64_t* out) {
  FRH_REQUIRE(num_imgs >= 1 && num_levels >= 1 && grid_hw && out, "bad arguments");
  const PropLayout z = prop_layout(num_imgs, num_levels, grid_hw, num_anchors, pre_nms);
  out[0] = (int64_t)z.boxes;
  out[1] = (int64_t)z.cnt;
  out[2] = z.P;
  out[3] = (int64_t)num_imgs * num_levels;
  return FRH_OK;
}

extern "C" int32_t frh_rpn_proposals(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                     const float* const* reg_ptrs, const int32_t* grid_hw, int32_t num_anchors,
                                     int32_t cls_channels, const float* anchors, int64_t anchor_ld,
                                     const float* means, const float* stds, const float* img_hw,
                                     const float* min_size, int32_t pre_nms, int32_t post_nms, int32_t max_num,
                                     double nms_iou, float* out_boxes, float* out_scores, int32_t* out_counts,
                                     void* workspace, size_t ws_bytes, void* stream) {
  FRH_REQUIRE(num_imgs >= 1 && num_imgs <= 64, "num_imgs %d must be in [1, 64]", num_imgs);
  FRH_REQUIRE(num_levels >= 1 && num_levels <= FRH_MAX_LEVELS, "bad level count %d", num_levels);
  FRH_REQUIRE(cls_channels == 1 || cls_channels == 2, "cls_channels must be 1 (sigmoid) or 2 (softmax)");
  FRH_REQUIRE(cls_ptrs && reg_ptrs && grid_hw && anchors && img_hw && min_size && out_boxes && out_scores &&
                  out_counts && means && stds,
              "null pointer argument");
  PropLayout z = prop_layout(num_imgs, num_levels, grid_hw, num_anchors, pre_nms);
  FRH_REQUIRE(z.P <= kMaxSort, "per-level candidate count %d exceeds %d (set pre_nms)", z.P, kMaxSort);
  int64_t post = (post_nms > 0 && post_nms < z.P) ? post_nms : z.P;
  FRH_REQUIRE(post * num_levels <= kMaxSort, "levels x post_nms exceeds %d", kMaxSort);
  FRH_REQUIRE(workspace && ws_bytes >= z.total, "workspace too small");
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  PropArgs p{};
  int64_t off = 0;
  for (int l = 0; l < num_levels; ++l) {
    p.cls[l] = cls_ptrs[l];
    p.reg[l] = reg_ptrs[l];
    p.h[l] = grid_hw[2 * l];
    p.w[l] = grid_hw[2 * l + 1];
    p.off[l] = off;
    off += (int64_t)num_anchors * p.h[l] * p.w[l];
  }
  FRH_REQUIRE(anchor_ld >= off, "anchor_ld smaller than the total anchor count");
  p.L = num_levels;
  p.A = num_anchors;
  p.C = cls_channels;
  p.anchors = anchors;
  p.anchor_ld = anchor_ld;
  for (int q = 0; q < 4; ++q) {
    p.m[q] = means[q];
    p.sd[q] = stds[q];
  }
  p.pre_nms = pre_nms;
  p.P = z.P;
  p.sel_boxes = reinterpret_cast<float*>(ws + z.boxes);
  p.sel_scores = reinterpret_cast<float*>(ws + z.scores);
  p.sel_idx = reinterpret_cast<int32_t*>(ws + z.idx);
  p.sel_count = reinterpret_cast<int32_t*>(ws + z.cnt);
  // per-image sizes travel by value in the kernel arguments
  ImgArgs ia{};
  for (int b = 0; b < num_imgs; ++b) {
    ia.hw[2 * b] = img_hw[2 * b];
    ia.hw[2 * b + 1] = img_hw[2 * b + 1];
    ia.min_size[b] = min_size[b];
  }
  const int S = num_imgs * num_levels;
  // 1. keys + top-k state, 2. segmented top-k, 3. order + decode + min-size
  uint32_t* keys = reinterpret_cast<uint32_t*>(ws + z.keys);
  TopkBuffers tb{keys, z.nmax, reinterpret_cast<uint32_t*>(ws + z.hist), reinterpret_cast<int32_t*>(ws + z.state),
                 p.sel_idx, z.P, reinterpret_cast<int32_t*>(ws + z.cand), S};
  FRH_HIP(hipMemsetAsync(ws + z.hist, 0, z.cand - z.hist, st));  // hist + state
  hipLaunchKernelGGL(rpn_keys_kernel, dim3((unsigned)((z.nmax + 255) / 256), (unsigned)S), dim3(256), 0, st, p, keys,
                     z.nmax, tb.state);
  tk_launch(tb, z.nmax, st);
  const size_t lds_sel = (size_t)next_pow2(z.P) * sizeof(uint64_t);
  if (lds_sel > 65536)
    FRH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(rpn_sort_decode_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sel));
  hipLaunchKernelGGL(rpn_sort_decode_kernel, dim3(S), dim3(kPropThreads), lds_sel, st, p, ia, keys, z.nmax,
                     tb.state, p.sel_idx, (int64_t)z.P);
  int32_t r = check_launch("rpn_select");
  if (r) return r;
  int32_t* keep = reinterpret_cast<int32_t*>(ws + z.keep);
  int32_t* kcnt = reinterpret_cast<int32_t*>(ws + z.kcnt);
  r = launch_nms_sorted(S, p.sel_boxes, (int64_t)z.P * 4, p.sel_count, z.P, nms_iou,
                        (post_nms > 0) ? post_nms : -1, keep, z.P, kcnt, reinterpret_cast<uint64_t*>(ws + z.mask), st);
  if (r) return r;
  MergeArgs mp{p.sel_boxes, p.sel_scores, keep, kcnt, num_levels, z.P, max_num,
               (int64_t)(max_num > 0 ? max_num : post * num_levels), out_boxes, out_scores, out_counts};
  dim3 mg((unsigned)((post + 255) / 256), (unsigned)num_levels, (unsigned)num_imgs);
  hipLaunchKernelGGL(rpn_merge_kernel, mg, dim3(256), 0, st, mp);
  return check_launch("rpn_merge");
}
