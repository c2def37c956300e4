// a11: class-wise batched multiclass NMS over (image x class) segments.
// Reference: lib/utils.py:211-269 (multiclass_nms + batched_nms), called per
// image from anchor_head.py:207-262, fcos_head.py:566-627, bbox_head.py:122-146.
//
// The reference builds the candidate (box, class) pairs of one image, shifts
// every box by label * max(candidate coordinates) so that classes cannot
// overlap, and runs ONE torchvision nms over all of them; the keep list comes
// out in (score desc) order and is cut to max_num.  Here every (image, class)
// pair is a segment of its own -- the shifted boxes of different classes never
// overlap when coordinates are >= 0 (the callers clamp to the image), so the
// per-class greedy passes keep exactly what the single pass keeps -- and all
// segments of all images run in one NMS launch:
//   prepare  candidates : one thread per (row, class) [official] or row
//                         [strict]: channel / min_score / row-valid filter,
//                         score x score_factor, record key << 32 | ~candidate
//                         appended to its segment; per-image max coordinate.
//            sort       : one workgroup per segment orders its records by
//                         (score desc, candidate asc) -- the reference's stable
//                         sort order -- in LDS and writes the shifted boxes
//                         (box + float(label) * max, in f32 as the reference).
//            summary    : one workgroup: the largest segment count, the negative-
//                         coordinate flag and each segment's NMS mask offset (its
//                         own triangle of 64x64 tiles) into a caller-provided device
//                         `info` / the workspace.  The caller copies `info` back (its
//                         one sync) to size the sort and the NMS workspace.
//   finish   sort       : as above; segments above 16384 candidates are sorted in
//                         16384-record chunks and merged by rank (binary searches).
//            nms        : nms.hip over all segments, max_num keeps per segment, each
//                         segment's mask sized by its own count.
//            merge      : per image, the kept pairs of all classes ranked by
//                         (score desc, candidate asc) with binary searches
//                         into the other classes' keep lists; the first
//                         max_num are written in that order.
// A candidate coordinate < 0 can make the reference's shifted classes overlap;
// prepare reports it and the caller redoes the call with one segment per image
// (by_class = 0): the reference's single pass, exactly.  (With coordinates >= 0
// the split is exact for any nms_iou above the ~1e-10 IoU a one-ulp rounding
// overlap of two shifted classes could produce.)
// "candidate" is the pair's position in the reference's flattened candidate
// array (row * classes + class official, row strict): ties order exactly as
// its stable sort does, also when rows the reference drops before the call
// (row_valid = 0) are kept in place here.
#include <algorithm>

#include "block_ops.h"

namespace frh {

int32_t launch_nms_sorted(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                          double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                          uint64_t* mask, const int64_t* seg_base, hipStream_t st, int64_t* stamps = nullptr);

constexpr int kMcMaxSeg = 65536;    // per-segment candidates (the NMS limit)
constexpr int kMcSortChunk = 16384; // records sorted per workgroup in LDS (128 KB)

struct McArgs {
  int B, C;
  int64_t n_max;
  int64_t seg_ld;  // record / row capacity per segment
  const int32_t* num_rows;
  const float* boxes;
  int64_t box_ld;   // per image
  int per_class;    // boxes [n][4 * C] viewed (n, 4, C)
  const float* scores;
  int64_t score_ld;
  const float* sf;  // score factor [n] or [n][C] (sf_per_class) per image, nullable
  int64_t sf_ld;
  int sf_per_class;
  const uint8_t* valid;  // nullable
  int64_t valid_ld;
  const uint8_t* chan;   // [C]
  int strict;
  int by_class;      // segments: 1 = (image, class), 0 = image (the reference's single pass)
  float min_score;
  // workspace
  int32_t* cnt;      // [S]
  uint32_t* maxk;    // [B] float_key of the largest candidate coordinate
  uint32_t* negk;    // [B] ~float_key of the smallest (nonzero: some coordinate < 0)
  uint64_t* rec;     // [segments][seg_ld] (B * C * n_max entries in all)
  int64_t* seg_base; // [S + 1] NMS mask tile offset of each segment (summary kernel)
  float4* rows;      // shifted boxes, sorted
  float* ssc;        // scores, sorted
  int32_t* scand;    // candidates, sorted
};

__device__ __forceinline__ float mc_coord(const McArgs& a, int b, int64_t i, int q, int c) {
  const float* bx = a.boxes + (int64_t)b * a.box_ld;
  return a.per_class ? bx[i * 4 * a.C + (int64_t)q * a.C + c] : bx[i * 4 + q];
}

// score.max(1) of row i: the first maximum (strict mode's label)
__device__ __forceinline__ int mc_argmax(const McArgs& a, int b, int64_t i, float* best) {
  const float* sc = a.scores + (int64_t)b * a.score_ld + i * a.C;
  float s = sc[0];
  int c = 0;
  for (int q = 1; q < a.C; ++q) {
    const float v = sc[q];
    if (v > s) {
      s = v;
      c = q;
    }
  }
  if (best) *best = s;
  return c;
}

// (row, label) of candidate cand
__device__ __forceinline__ int64_t mc_row(const McArgs& a, int b, uint32_t cand, int* label) {
  if (a.strict) {
    *label = mc_argmax(a, b, (int64_t)cand, nullptr);
    return (int64_t)cand;
  }
  *label = (int)(cand % (uint32_t)a.C);
  return (int64_t)(cand / (uint32_t)a.C);
}

static __global__ void __launch_bounds__(256) mc_candidates_kernel(McArgs a) {
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = a.num_rows[b];
  const int64_t i = a.strict ? e : e / a.C;
  bool chosen = false;
  float s = 0.f;
  int c = 0;
  if (i < n) {
    if (a.strict) {
      c = mc_argmax(a, b, i, &s);
    } else {
      c = (int)(e - i * a.C);
      s = a.scores[(int64_t)b * a.score_ld + i * a.C + c];
    }
    chosen = a.chan[c] && s >= a.min_score && (!a.valid || a.valid[(int64_t)b * a.valid_ld + i]);
    if (a.sf) s = s * a.sf[(int64_t)b * a.sf_ld + (a.sf_per_class ? i * a.C + c : i)];
  }
  uint32_t mk = 0u, nk = 0u;
  if (chosen) {
    const int seg = a.by_class ? b * a.C + c : b;
    const int pos = atomicAdd(&a.cnt[seg], 1);
    const uint32_t cand = (uint32_t)(a.strict ? i : i * a.C + c);
    a.rec[(int64_t)seg * a.seg_ld + pos] = ((uint64_t)float_key(s) << 32) | (uint32_t)~cand;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float v = mc_coord(a, b, i, q, c);
      const uint32_t k = float_key(v);
      mk = k > mk ? k : mk;
      nk = (v < 0.0f && ~k > nk) ? ~k : nk;
    }
  }
  mk = wave_max_u32(mk);
  nk = wave_max_u32(nk);
  if (lane_id() == 0 && mk) atomicMax(&a.maxk[b], mk);
  if (lane_id() == 0 && nk) atomicMax(&a.negk[b], nk);
}

// sorted record r of segment seg at position j: the shifted box, the score, the candidate
__device__ __forceinline__ void mc_emit(const McArgs& a, int seg, int b, int64_t j, uint64_t r) {
  const float M = key_float(a.maxk[b]);
  const uint32_t cand = ~(uint32_t)r;
  int c;
  const int64_t i = mc_row(a, b, cand, &c);
  const float off = (float)c * M;  // (label * max_range) in f32, utils.py:218-219
  float4 v;
  v.x = mc_coord(a, b, i, 0, c) + off;
  v.y = mc_coord(a, b, i, 1, c) + off;
  v.z = mc_coord(a, b, i, 2, c) + off;
  v.w = mc_coord(a, b, i, 3, c) + off;
  const int64_t o = (int64_t)seg * a.seg_ld + j;
  a.rows[o] = v;
  a.ssc[o] = key_float((uint32_t)(r >> 32));
  a.scand[o] = (int32_t)cand;
}

// one 1024-thread workgroup per (segment, 16384-record chunk); dynamic LDS
// next_pow2(chunk) u64.  One chunk: the sorted records are emitted directly; several:
// each chunk is written back sorted (descending; keys are unique: the candidate is in
// the low word) and mc_rank_kernel merges them.
static __global__ void __launch_bounds__(1024) mc_sort_kernel(McArgs a, int chunked) {
  extern __shared__ uint64_t sk[];
  const int seg = blockIdx.x, b = a.by_class ? seg / a.C : seg;
  const int m = a.cnt[seg];
  const int q0 = blockIdx.y * kMcSortChunk;
  if (q0 >= m) return;
  const int mq = min(m - q0, kMcSortChunk);
  const int P2 = next_pow2(mq);
  uint64_t* rec = a.rec + (int64_t)seg * a.seg_ld + q0;
  for (int j = threadIdx.x; j < P2; j += blockDim.x) sk[j] = j < mq ? rec[j] : 0ull;
  __syncthreads();
  block_bitonic_sort_desc(sk, P2);
  for (int j = threadIdx.x; j < mq; j += blockDim.x) {
    if (chunked)
      rec[j] = sk[j];
    else
      mc_emit(a, seg, b, j, sk[j]);
  }
}

// position of each record among all chunks of its segment: its index in its own chunk
// plus, per other chunk, the number of records ordered before it (binary search)
static __global__ void __launch_bounds__(256) mc_rank_kernel(McArgs a) {
  const int seg = blockIdx.y, b = a.by_class ? seg / a.C : seg;
  const int m = a.cnt[seg];
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint64_t* rec = a.rec + (int64_t)seg * a.seg_ld;
  const uint64_t key = rec[j];
  const int q = (int)(j / kMcSortChunk);
  int64_t rank = j - (int64_t)q * kMcSortChunk;
  for (int q2 = 0; q2 * kMcSortChunk < m; ++q2) {
    if (q2 == q) continue;
    const uint64_t* c = rec + (int64_t)q2 * kMcSortChunk;
    int lo = 0, hi = min(m - q2 * kMcSortChunk, kMcSortChunk);
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (c[mid] > key)
        lo = mid + 1;
      else
        hi = mid;
    }
    rank += lo;
  }
  mc_emit(a, seg, b, rank, key);
}

// one workgroup: info = {largest segment count, some coordinate < 0, total NMS mask
// tiles (lo, hi)} and seg_base[s] = sum over earlier segments of tri(ceil(cnt / 64))
static __global__ void __launch_bounds__(1024) mc_summary_kernel(McArgs a, int S, int32_t* info) {
  __shared__ int64_t scan[1024];
  __shared__ int smax[1024];
  __shared__ int64_t carry;
  const int t = threadIdx.x;
  int mx = 0;
  if (t == 0) carry = 0;
  for (int c0 = 0; c0 < S; c0 += 1024) {
    const int s = c0 + t;
    const int64_t n = s < S ? a.cnt[s] : 0;
    mx = max(mx, (int)n);
    const int64_t nb = (n + 63) / 64;
    scan[t] = nb * (nb + 1) / 2;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
      const int64_t v = t >= d ? scan[t - d] : 0;
      __syncthreads();
      scan[t] += v;
      __syncthreads();
    }
    const int64_t excl = carry + (t ? scan[t - 1] : 0);
    if (s < S) a.seg_base[s] = excl;
    __syncthreads();
    if (t == 1023) carry += scan[1023];
    __syncthreads();
  }
  smax[t] = mx;
  __syncthreads();
  for (int d = 512; d > 0; d >>= 1) {
    if (t < d) smax[t] = max(smax[t], smax[t + d]);
    __syncthreads();
  }
  if (t == 0) {
    int neg = 0;
    for (int b = 0; b < a.B; ++b) neg |= a.negk[b] != 0u;
    a.seg_base[S] = carry;
    info[0] = smax[0];
    info[1] = neg;
    info[2] = (int32_t)(uint32_t)(carry & 0xffffffffll);
    info[3] = (int32_t)(uint32_t)(carry >> 32);
  }
}

struct McMerge {
  McArgs a;
  const int32_t* keep;  // [S][P]
  const int32_t* kcnt;  // [S]
  int P;
  int max_num;          // <= 0: no cut
  int64_t out_cap;
  float* out_boxes;     // [B][out_cap][4]
  float* out_scores;    // [B][out_cap]
  int64_t* out_labels;  // [B][out_cap]
  int32_t* out_counts;  // [B]
};

__device__ __forceinline__ uint64_t mc_kept_key(const McMerge& m, int seg, int j) {
  const int64_t o = (int64_t)seg * m.a.seg_ld + m.keep[(int64_t)seg * m.P + j];
  return ((uint64_t)float_key(m.a.ssc[o]) << 32) | (uint32_t)~(uint32_t)m.a.scand[o];
}

// grid (kept chunks of 256, segments per image, images)
static __global__ void __launch_bounds__(256) mc_merge_kernel(McMerge m) {
  const int b = blockIdx.z, c = blockIdx.y, G = m.a.by_class ? m.a.C : 1;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int seg = b * G + c;
  if (blockIdx.x == 0 && c == 0 && threadIdx.x == 0) {
    int total = 0;
    for (int q = 0; q < G; ++q) total += m.kcnt[b * G + q];
    m.out_counts[b] = (m.max_num > 0 && total > m.max_num) ? m.max_num : total;
  }
  if (j >= m.kcnt[seg]) return;
  const uint64_t key = mc_kept_key(m, seg, j);
  int rank = j;
  for (int q = 0; q < G; ++q) {
    if (q == c) continue;
    const int oseg = b * G + q;
    int lo = 0, hi = m.kcnt[oseg];  // kept pairs of class q ordered before this one
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (mc_kept_key(m, oseg, mid) > key)
        lo = mid + 1;
      else
        hi = mid;
    }
    rank += lo;
  }
  if (m.max_num > 0 && rank >= m.max_num) return;
  const int64_t o = (int64_t)seg * m.a.seg_ld + m.keep[(int64_t)seg * m.P + j];
  int label;
  const int64_t i = mc_row(m.a, b, (uint32_t)m.a.scand[o], &label);
  float* ob = m.out_boxes + ((int64_t)b * m.out_cap + rank) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) ob[q] = mc_coord(m.a, b, i, q, label);
  m.out_scores[(int64_t)b * m.out_cap + rank] = m.a.ssc[o];
  m.out_labels[(int64_t)b * m.out_cap + rank] = label;
}

static size_t al(size_t v) { return (v + 255) & ~(size_t)255; }

struct McLayout {
  size_t cnt, maxk, negk, seg_base, rec, rows, ssc, scand, total;
};

static McLayout mc_layout(int B, int C, int64_t n_max) {
  McLayout z{};
  const size_t S = (size_t)B * C, n = (size_t)(n_max > 0 ? n_max : 1);
  z.cnt = 0;
  z.maxk = z.cnt + S * sizeof(int32_t);  // cnt + maxk + negk contiguous: one memset
  z.negk = z.maxk + (size_t)B * sizeof(uint32_t);
  z.seg_base = al(z.negk + (size_t)B * sizeof(uint32_t));
  z.rec = al(z.seg_base + (S + 1) * sizeof(int64_t));
  z.rows = z.rec + al(S * n * sizeof(uint64_t));
  z.ssc = z.rows + al(S * n * sizeof(float4));
  z.scand = z.ssc + al(S * n * sizeof(float));
  z.total = z.scand + al(S * n * sizeof(int32_t));
  return z;
}

static void mc_bind(McArgs& a, char* ws, int B, int C, int64_t n_max, int strict, int by_class) {
  const McLayout z = mc_layout(B, C, n_max);
  a.n_max = n_max;
  a.by_class = by_class;
  a.seg_ld = (by_class || strict) ? n_max : n_max * C;
  a.cnt = reinterpret_cast<int32_t*>(ws + z.cnt);
  a.maxk = reinterpret_cast<uint32_t*>(ws + z.maxk);
  a.negk = reinterpret_cast<uint32_t*>(ws + z.negk);
  a.seg_base = reinterpret_cast<int64_t*>(ws + z.seg_base);
  a.rec = reinterpret_cast<uint64_t*>(ws + z.rec);
  a.rows = reinterpret_cast<float4*>(ws + z.rows);
  a.ssc = reinterpret_cast<float*>(ws + z.ssc);
  a.scand = reinterpret_cast<int32_t*>(ws + z.scand);
}

}  // namespace frh

using namespace frh;

extern "C" size_t frh_mcnms_workspace(int32_t num_imgs, int32_t num_classes, int64_t n_max) {
  if (num_imgs <= 0 || num_classes <= 0 || n_max < 0) return 0;
  return mc_layout(num_imgs, num_classes, n_max).total;
}

extern "C" int32_t frh_mcnms_prepare(int32_t num_imgs, int32_t num_classes, int64_t n_max, const int32_t* num_rows,
                                     const float* boxes, int64_t box_img_stride, int32_t box_per_class,
                                     const float* scores, int64_t score_img_stride, const float* score_factor,
                                     int64_t sf_img_stride, int32_t sf_per_class, const uint8_t* row_valid,
                                     int64_t valid_img_stride,
                                     const uint8_t* channel_mask, int32_t mode, int32_t by_class, float min_score,
                                     void* workspace, size_t ws_bytes, int32_t* info, void* stream) {
  FRH_REQUIRE(num_imgs >= 1 && num_classes >= 1 && n_max >= 0, "bad sizes");
  FRH_REQUIRE(mode == 0 || mode == 1, "mode must be 0 (official) or 1 (strict)");
  FRH_REQUIRE(num_rows && boxes && scores && channel_mask && info, "null pointer argument");
  FRH_REQUIRE(n_max * num_classes < INT32_MAX, "candidate index overflow");
  FRH_REQUIRE(workspace && ws_bytes >= frh_mcnms_workspace(num_imgs, num_classes, n_max), "workspace too small");
  FRH_REQUIRE(!(mode == 1 && sf_per_class), "strict mode takes a per-row score factor");
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  McArgs a{};
  a.B = num_imgs;
  a.C = num_classes;
  a.num_rows = num_rows;
  a.boxes = boxes;
  a.box_ld = box_img_stride;
  a.per_class = box_per_class;
  a.scores = scores;
  a.score_ld = score_img_stride;
  a.sf = score_factor;
  a.sf_ld = sf_img_stride;
  a.sf_per_class = sf_per_class;
  a.valid = row_valid;
  a.valid_ld = valid_img_stride;
  a.chan = channel_mask;
  a.strict = mode;
  a.min_score = min_score;
  mc_bind(a, ws, num_imgs, num_classes, n_max > 0 ? n_max : 1, mode, by_class);
  const int S = by_class ? num_imgs * num_classes : num_imgs;
  FRH_HIP(hipMemsetAsync(ws, 0, mc_layout(num_imgs, num_classes, a.n_max).seg_base, st));
  if (n_max > 0) {
    const int64_t per_img = mode ? n_max : n_max * num_classes;
    hipLaunchKernelGGL(mc_candidates_kernel, dim3((unsigned)((per_img + 255) / 256), (unsigned)num_imgs), dim3(256),
                       0, st, a);
  }
  hipLaunchKernelGGL(mc_summary_kernel, dim3(1), dim3(1024), 0, st, a, S, info);
  return check_launch("frh_mcnms_prepare");
}

extern "C" size_t frh_mcnms_nms_workspace(int32_t num_imgs, int32_t num_classes, int32_t max_count,
                                         int64_t mask_tiles) {
  if (num_imgs <= 0 || num_classes <= 0 || max_count <= 0 || mask_tiles < 0) return 0;
  const size_t S = (size_t)num_imgs * num_classes;  // enough for either segmentation
  return al((size_t)mask_tiles * 64 * sizeof(uint64_t)) + al(S * (size_t)max_count * sizeof(int32_t)) +
         al(S * sizeof(int32_t));
}

extern "C" int32_t frh_mcnms_finish(int32_t num_imgs, int32_t num_classes, int64_t n_max, int32_t max_count,
                                    int64_t mask_tiles, const float* boxes, int64_t box_img_stride,
                                    int32_t box_per_class, const float* scores, int64_t score_img_stride,
                                    int32_t mode, int32_t by_class, double nms_iou, int32_t max_num,
                                    float* out_boxes, float* out_scores, int64_t* out_labels, int32_t* out_counts,
                                    int64_t out_cap, void* workspace, size_t ws_bytes, void* nms_ws,
                                    size_t nms_ws_bytes, void* stream) {
  FRH_REQUIRE(num_imgs >= 1 && num_classes >= 1 && n_max >= 0 && max_count >= 0 && mask_tiles >= 0, "bad sizes");
  FRH_REQUIRE(boxes && out_counts, "null pointer argument");
  FRH_REQUIRE(workspace && ws_bytes >= frh_mcnms_workspace(num_imgs, num_classes, n_max), "workspace too small");
  FRH_REQUIRE(max_count <= kMcMaxSeg, "a segment has %d candidates (limit %d): raise min_score / pre_nms", max_count,
              kMcMaxSeg);
  hipStream_t st = as_stream(stream);
  const int S = by_class ? num_imgs * num_classes : num_imgs;
  if (max_count == 0) return hipMemsetAsync(out_counts, 0, (size_t)num_imgs * sizeof(int32_t), st) == hipSuccess
                                 ? FRH_OK
                                 : FRH_ELAUNCH;
  FRH_REQUIRE(out_boxes && out_scores && out_labels, "null output");
  const int64_t per_img = (int64_t)(S / num_imgs) * max_count;
  FRH_REQUIRE(out_cap >= (max_num > 0 ? std::min<int64_t>(max_num, per_img) : per_img), "out_cap too small");
  FRH_REQUIRE(!mode || scores, "strict mode needs the scores (labels)");
  FRH_REQUIRE(nms_ws && nms_ws_bytes >= frh_mcnms_nms_workspace(num_imgs, num_classes, max_count, mask_tiles),
              "nms workspace too small");
  McArgs a{};
  a.B = num_imgs;
  a.C = num_classes;
  a.boxes = boxes;
  a.box_ld = box_img_stride;
  a.per_class = box_per_class;
  a.scores = scores;
  a.score_ld = score_img_stride;
  a.strict = mode;
  mc_bind(a, reinterpret_cast<char*>(workspace), num_imgs, num_classes, n_max > 0 ? n_max : 1, mode, by_class);
  // sort: one workgroup per (segment, chunk of 16384 records), then a rank merge if chunked
  const int nq = (max_count + kMcSortChunk - 1) / kMcSortChunk;
  const size_t lds = (size_t)next_pow2(std::min(max_count, kMcSortChunk)) * sizeof(uint64_t);
  if (lds > 65536)
    FRH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(mc_sort_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(mc_sort_kernel, dim3((unsigned)S, (unsigned)nq), dim3(1024), lds, st, a, (int)(nq > 1));
  if (nq > 1)
    hipLaunchKernelGGL(mc_rank_kernel, dim3((unsigned)((max_count + 255) / 256), (unsigned)S), dim3(256), 0, st, a);
  int32_t r = check_launch("mcnms sort");
  if (r) return r;
  char* nw = reinterpret_cast<char*>(nms_ws);
  uint64_t* mask = reinterpret_cast<uint64_t*>(nw);
  const size_t mask_b = al((size_t)mask_tiles * 64 * sizeof(uint64_t));
  int32_t* keep = reinterpret_cast<int32_t*>(nw + mask_b);
  int32_t* kcnt = reinterpret_cast<int32_t*>(nw + mask_b + al((size_t)S * max_count * sizeof(int32_t)));
  r = launch_nms_sorted(S, reinterpret_cast<const float*>(a.rows), a.seg_ld * 4, a.cnt, max_count, nms_iou,
                        max_num > 0 ? max_num : -1, keep, max_count, kcnt, mask, a.seg_base, st);
  if (r) return r;
  McMerge m{a, keep, kcnt, max_count, max_num, out_cap, out_boxes, out_scores, out_labels, out_counts};
  const int kmax = max_num > 0 ? std::min(max_num, max_count) : max_count;
  hipLaunchKernelGGL(mc_merge_kernel, dim3((unsigned)((kmax + 255) / 256), (unsigned)(S / num_imgs), (unsigned)num_imgs),
                     dim3(256), 0, st, m);
  return check_launch("frh_mcnms_finish");
}
