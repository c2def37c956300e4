// a9: RPN proposals for all (image, level) segments at once.
// Reference: lib/heads/rpn_head.py:68-120 (predict_single_image), decode from
// lib/utils.py:83-144, NMS = torchvision.ops.nms semantics (nms.hip).
//
//  1. keys (score = sigmoid or 2-way softmax of the logits -> ordered u32)
//     + first-level histogram, then refine + collect (seg_topk.h: one
//     workgroup per 4096 anchors; a selected anchor is decoded + clamped by
//     the workgroup that selects it), then rank: each selection's position in
//     (score desc, index asc) order after the min-size compaction, by counting.
//  2. NMS mask + scan over all segments in one launch (nms.hip, nms_fused_kernel),
//     keep <= post_nms.
//  3. merge   (1 block per image): concatenate the levels' survivors and, if
//     more than max_num, keep the best max_num by (score desc, concat order).
#include "seg_topk.h"

namespace frh {

int32_t launch_nms_sorted(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                          double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                          uint64_t* mask, const int64_t* seg_base, hipStream_t st, int64_t* stamps = nullptr);
size_t nms_mask_bytes(int32_t S, int32_t n_max);
bool nms_fused_fits(int32_t S, int32_t n_max);
size_t nms_fused_flag_bytes(int32_t S, int32_t n_max);
int32_t launch_nms_fused(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                         double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                         uint64_t* mask, uint32_t* flags, int32_t* status, hipStream_t st,
                         int64_t* stamps = nullptr, const float* row_scores = nullptr, uint32_t* kscore = nullptr);

constexpr int kPropThreads = 1024;
constexpr int kMaxSort = 16384;

struct PropArgs {
  const float* cls[FRH_MAX_LEVELS];
  const float* reg[FRH_MAX_LEVELS];
  int64_t cst[FRH_MAX_LEVELS][4], rst[FRH_MAX_LEVELS][4];  // element strides (b, c, y, x)
  int nchw;  // every level contiguous [B, C*A, H, W]: flat indexing
  int nhwc_cls;  // every level's cls output packed channels-last: anchor (a, cell) at cell * C*A + a
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
  uint64_t* sel_keys;  // [S][P] selection records (RpnPol)
  float4* stage;       // [S][kRpnSelFused] boxes decoded at selection (fused path)
  int32_t* sel_count; // [S]
  int64_t* stamps;    // tools timing only (null in the product): rpn_select_kernel phase times
  int32_t* status;    // the caller's device status word (include/frcnn_amd.h FRH_DEVERR_*)
};

struct ImgArgs {
  float hw[2 * 64];
  float min_size[64];
};

// score from the logit(s) of one anchor: sigmoid, or channel 1 of a 2-way softmax
__device__ __forceinline__ float score_of2(float x0, float x1, int C) {
  if (C == 1) return 1.0f / (1.0f + expf(-x0));
  float mx = fmaxf(x0, x1);
  float e0 = expf(x0 - mx), e1 = expf(x1 - mx);
  return e1 / (e0 + e1);
}

// element (image b, row c, level-local anchor i = a*H*W + y*W + x) of a [B, R*A, H, W]
// head output viewed per image as [R, A*H*W] (anchor_head.py:82; rpn_head.py:72): tensor
// channel c*A + a, whatever the strides (NCHW or channels-last)
__device__ __forceinline__ int64_t rpn_elem(const int64_t (&st)[4], int A, int H, int W, int b, int c, int64_t i) {
  const uint32_t hw = (uint32_t)H * (uint32_t)W, u = (uint32_t)i, a = u / hw, sp = u - a * hw;
  const uint32_t y = sp / (uint32_t)W, x = sp - y * (uint32_t)W;
  return (int64_t)b * st[0] + (int64_t)(c * A + (int)a) * st[1] + (int64_t)y * st[2] + (int64_t)x * st[3];
}

// logit c (0, or 1 for the second softmax channel; 0 when C == 1) of anchor i of level l,
// image b, any layout (the degenerate tie path's keys, recomputed)
__device__ __forceinline__ float rpn_logit(const PropArgs& p, int l, int b, int c, int i) {
  if (c >= p.C) return 0.0f;
  return p.cls[l][rpn_elem(p.cst[l], p.A, p.h[l], p.w[l], b, c, i)];
}

constexpr int kRpnHistBits = 12;
constexpr int kRpnSelFused = 2048;  // selections decoded at selection time, ordered by rpn_rank_kernel

// keys = order-preserving u32 of the score (never 0: scores are >= 0) and the
// first-level top-k histogram of their top 12 bits; also seeds the state words
// read by the large-k sort kernel.  Grid (chunks of 4096, segments).
static __global__ void __launch_bounds__(kTkThreads) rpn_keys_kernel(PropArgs p, TkBufs b) {
  __shared__ uint32_t h[1 << kRpnHistBits];
  const int seg = blockIdx.y;
  const int bi = seg / p.L, l = seg % p.L;
  const int64_t hwa = (int64_t)p.A * p.h[l] * p.w[l];
  const int64_t base = (int64_t)blockIdx.x * kTkChunk;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int n = (int)hwa;
    b.state[seg * TK_WORDS + TK_N] = n;
    b.state[seg * TK_WORDS + TK_K] = (p.pre_nms > 0 && p.pre_nms < n) ? p.pre_nms : n;
  }
  if (base >= hwa) return;
  tk_hist1_clear(h, 1 << kRpnHistBits);
  uint32_t* kk = const_cast<uint32_t*>(b.keys) + (int64_t)seg * b.ld;
  float x0[kTkPerThread], x1[kTkPerThread];  // every logit load in flight at once
  if (p.nhwc_cls) {  // memory order (cell-major), keys stored at their anchor index
    const float* cls = p.cls[l] + (int64_t)bi * p.cst[l][0];
    const int CA = p.C * p.A, hw = p.h[l] * p.w[l];
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      const int m = (int)base + r * kTkThreads + threadIdx.x;
      const int cell = (int)((uint32_t)m / (uint32_t)p.A), a = m - cell * p.A;
      x0[r] = m < hwa ? cls[(int64_t)cell * CA + a] : 0.0f;
      x1[r] = (p.C == 2 && m < hwa) ? cls[(int64_t)cell * CA + p.A + a] : 0.0f;
    }
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      const int m = (int)base + r * kTkThreads + threadIdx.x;
      const int cell = (int)((uint32_t)m / (uint32_t)p.A), a = m - cell * p.A;
      uint32_t key = 0u;
      if (m < hwa) {
        key = float_key(score_of2(x0[r], x1[r], p.C));
        kk[a * hw + cell] = key;
      }
      tk_hist_add(h, m < hwa, key >> (32 - kRpnHistBits));
    }
    tk_hist1_flush(h, 1 << kRpnHistBits, b.hist1 + (int64_t)seg * (1 << kRpnHistBits));
    return;
  }
  if (p.nchw) {
    const float* cls = p.cls[l] + (int64_t)bi * p.C * hwa;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      const int64_t i = base + r * kTkThreads + threadIdx.x;
      x0[r] = i < hwa ? cls[i] : 0.0f;
      x1[r] = (p.C == 2 && i < hwa) ? cls[hwa + i] : 0.0f;
    }
  } else {
    const float* cls = p.cls[l];
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      const int64_t i = base + r * kTkThreads + threadIdx.x;
      x0[r] = i < hwa ? cls[rpn_elem(p.cst[l], p.A, p.h[l], p.w[l], bi, 0, i)] : 0.0f;
      x1[r] = (p.C == 2 && i < hwa) ? cls[rpn_elem(p.cst[l], p.A, p.h[l], p.w[l], bi, 1, i)] : 0.0f;
    }
  }
#pragma unroll
  for (int r = 0; r < kTkPerThread; ++r) {
    const int64_t i = base + r * kTkThreads + threadIdx.x;
    uint32_t key = 0u;
    if (i < hwa) {
      key = float_key(score_of2(x0[r], x1[r], p.C));
      kk[i] = key;
    }
    tk_hist_add(h, i < hwa, key >> (32 - kRpnHistBits));
  }
  tk_hist1_flush(h, 1 << kRpnHistBits, b.hist1 + (int64_t)seg * (1 << kRpnHistBits));
}

// Decode + clamp of anchor i of segment seg (utils.py:83-144).
__device__ __forceinline__ float4 rpn_decode_one(const PropArgs& p, const ImgArgs& ia, int seg, int i) {
  const int b = seg / p.L, l = seg % p.L;
  const int64_t hwa = (int64_t)p.A * p.h[l] * p.w[l];
  const float img_h = ia.hw[2 * b], img_w = ia.hw[2 * b + 1];
  const int64_t ai = p.off[l] + i;
  const float* an = p.anchors;
  const int64_t ld = p.anchor_ld;
  float ax1 = an[ai], ay1 = an[ld + ai], ax2 = an[2 * ld + ai], ay2 = an[3 * ld + ai];
  float d[4];
  if (p.nchw) {
    const float* reg = p.reg[l] + (int64_t)b * 4 * hwa;
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = reg[q * hwa + i];
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = p.reg[l][rpn_elem(p.rst[l], p.A, p.h[l], p.w[l], b, q, i)];
  }
  float tx = d[0] * p.sd[0] + p.m[0];
  float ty = d[1] * p.sd[1] + p.m[1];
  float tw = d[2] * p.sd[2] + p.m[2];
  float th = d[3] * p.sd[3] + p.m[3];
  float bw = (ax2 - ax1) + 1.0f, bh = (ay2 - ay1) + 1.0f;
  float bcx = (ax2 + ax1) / 2.0f, bcy = (ay2 + ay1) / 2.0f;
  float cx = tx * bw + bcx, cy = ty * bh + bcy;
  float ww = expf(tw) * bw, hh = expf(th) * bh;
  float hw2 = ww / 2.0f, hh2 = hh / 2.0f;
  float v[4] = {cx - hw2, cy - hh2, cx + hw2, cy + hh2};
  float hi[4] = {img_w - 1.0f, img_h - 1.0f, img_w - 1.0f, img_h - 1.0f};
  float box[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float y = (v[q] < 0.0f) ? 0.0f : v[q];
    box[q] = (y > hi[q]) ? hi[q] : y;
  }
  return make_float4(box[0], box[1], box[2], box[3]);
}

// min-size filter (rpn_head.py:86-90)
__device__ __forceinline__ bool rpn_big_enough(float4 b, float min_size) {
  return min_size <= 0.0f || ((((b.z - b.x) + 1.0f) >= min_size) && (((b.w - b.y) + 1.0f) >= min_size));
}

__device__ __forceinline__ int rpn_k(const PropArgs& p, int n) { return (p.pre_nms > 0 && p.pre_nms < n) ? p.pre_nms : n; }

// RPN policy of the segmented top-k.  Fused (selection <= kRpnSelFused,
// anchors < 2^20): the workgroup that selects anchor i decodes it at once into
// stage[slot] and records key << 32 | (~i & 0xfffff) << 12 | big-enough << 11 |
// slot; rpn_rank_kernel then orders the records.  Otherwise the record is
// key << 32 | ~i and rpn_sort_decode_kernel follows.  Records and staged boxes
// cross workgroups and launches (xwg_store, seg_topk.h).
struct RpnPol {
  const PropArgs& p;
  const ImgArgs& ia;
  const TkBufs& b;
  int seg;
  bool fused;
  __device__ void select(int i, uint32_t key, int slot) {
    uint64_t* rec = p.sel_keys + (int64_t)seg * p.P + slot;
    if (!fused) {
      xwg_store(rec, ((uint64_t)key << 32) | (uint32_t)~(uint32_t)i);
      return;
    }
    const float4 bx = rpn_decode_one(p, ia, seg, i);
    const bool live = rpn_big_enough(bx, ia.min_size[seg / p.L]);
    uint64_t* sb = reinterpret_cast<uint64_t*>(p.stage + ((int64_t)seg * kRpnSelFused + slot));
    xwg_store(sb, ((uint64_t)__float_as_uint(bx.y) << 32) | __float_as_uint(bx.x));
    xwg_store(sb + 1, ((uint64_t)__float_as_uint(bx.w) << 32) | __float_as_uint(bx.z));
    xwg_store(rec, ((uint64_t)key << 32) | ((~(uint32_t)i & 0xfffffu) << 12) | (live ? 0x800u : 0u) |
                       (uint32_t)slot);
  }
  __device__ void finish(int kv) {
    if (threadIdx.x == 0) b.state[seg * TK_WORDS + TK_K] = kv;  // the sort launch's count
  }
};

// Fused path, after collect: the order of the kv <= kRpnSelFused records of a
// segment by (score desc, index asc) without a sort.  Every workgroup holds all
// records in LDS; 8 threads per record count the big-enough records above it
// -- its output position after the min-size compaction -- and the first of them
// moves the staged box and score there.  Grid (kRpnSelFused / 32, segments).
constexpr int kRankPer = 32;  // records per workgroup
static __global__ void __launch_bounds__(256) rpn_rank_kernel(PropArgs p, const int32_t* state) {
  __shared__ uint64_t rec[kRpnSelFused];
  __shared__ int part[4];
  const int seg = blockIdx.y, t = threadIdx.x;
  const int cap = p.P < kRpnSelFused ? p.P : kRpnSelFused;
  const uint64_t* src = p.sel_keys + (int64_t)seg * p.P;
  uint64_t r[kRpnSelFused / 256];  // the whole row in flight at once, beside the count
#pragma unroll
  for (int e = 0; e < kRpnSelFused / 256; ++e) r[e] = e * 256 + t < cap ? src[e * 256 + t] : 0ull;
  const int kv = state[seg * TK_WORDS + TK_K];
#pragma unroll
  for (int e = 0; e < kRpnSelFused / 256; ++e) rec[e * 256 + t] = e * 256 + t < kv ? r[e] : 0ull;
  __syncthreads();
  const int first = blockIdx.x * kRankPer;
  if (blockIdx.x == 0) {  // the segment's kept count
    int c = 0;
    for (int j = t; j < kv; j += 256) c += (int)((rec[j] >> 11) & 1u);
    c = block_sum(c, part);
    if (t == 0) p.sel_count[seg] = c;
  }
  if (first >= kv) return;
  const int q = first + (t >> 3), lane8 = t & 7;
  const uint64_t x = q < kv ? rec[q] : ~0ull;
  int above = 0;
  const int kv8 = (kv + 7) & ~7;  // padding records are 0: never above
#pragma unroll 8
  for (int j = lane8; j < kv8; j += 8) {
    const uint64_t y = rec[j];
    above += (y > x && ((y >> 11) & 1u)) ? 1 : 0;
  }
  above += __shfl_xor(above, 1, kWave);
  above += __shfl_xor(above, 2, kWave);
  above += __shfl_xor(above, 4, kWave);
  if (lane8 == 0 && q < kv && ((x >> 11) & 1u)) {
    const float4 bx = p.stage[(int64_t)seg * kRpnSelFused + (int)(x & 0x7ffu)];
    reinterpret_cast<float4*>(p.sel_boxes)[(int64_t)seg * p.P + above] = bx;
    p.sel_scores[(int64_t)seg * p.P + above] = key_float((uint32_t)(x >> 32));
  }
}

// Top-k launches: grid (chunks of 4096, segments), 256 threads (seg_topk.h).
static __global__ void __launch_bounds__(kTkThreads) rpn_refine_kernel(PropArgs p, TkBufs b) {
  __shared__ TkSmem sm;
  const int seg = blockIdx.y;
  const int l = seg % p.L;
  const int n = p.A * p.h[l] * p.w[l];
  tk_refine_chunk(b, seg, n, rpn_k(p, n), sm);
}

static __global__ void __launch_bounds__(kTkThreads) rpn_collect_kernel(PropArgs p, ImgArgs ia, TkBufs b, bool fused) {
  __shared__ TkSmem sm;
  const int seg = blockIdx.y;
  const int l = seg % p.L;
  const int n = p.A * p.h[l] * p.w[l];
  RpnPol pol{p, ia, b, seg, fused};
  tk_collect_chunk(b, seg, n, tk_plan_refined(b, seg), pol, sm);
}

// ---------------------------------------------------------------------------
// Fused selection: keys -> two-level histogram -> collect + decode -> order, in ONE
// launch whose phases are separated by in-launch segment barriers (seg_topk.h,
// seg_barrier) instead of the four kernel boundaries of rpn_keys / refine / collect
// / rank.  The keys stay in registers from the logit load to the collect (no key
// re-reads); every workgroup of a segment reads the segment's histograms after the
// barrier and finds the same buckets (no last-workgroup publish hop).  Workgroup x
// of segment seg owns key chunk x (x < nch) and the records [64x, 64x + 64) of the
// final order; G(seg) = max(1, nch, ceil(k / 64)) workgroups take part, the rest of
// the grid row returns at once.  Selection rule, record layout and the order are
// those of the four-launch path (bit-identical outputs).
constexpr int kSelRankPer = 64;    // records ordered per workgroup
constexpr int kRpnTieCap = 2048;   // prefix ties sorted in LDS; more: workgroup 0's radix select

__host__ __device__ __forceinline__ int rpn_sel_groups(int n, int pre_nms) {
  const int nch = (n + kTkChunk - 1) / kTkChunk, k = (pre_nms > 0 && pre_nms < n) ? pre_nms : n;
  const int r = (k + kSelRankPer - 1) / kSelRankPer;
  return nch > r ? (nch > 1 ? nch : 1) : (r > 1 ? r : 1);
}

__device__ __forceinline__ uint64_t rpn_record(uint32_t key, int i, bool live, int slot) {
  return ((uint64_t)key << 32) | ((~(uint32_t)i & 0xfffffu) << 12) | (live ? 0x800u : 0u) | (uint32_t)slot;
}

static __global__ void __launch_bounds__(kTkThreads) rpn_select_kernel(PropArgs p, ImgArgs ia, TkBufs b) {
  __shared__ TkSmem sm;
  static_assert(kRpnTieCap + kRpnSelFused <= kTkCandCap, "ties + records share the candidate area");
  const int seg = blockIdx.y, x = blockIdx.x, t = threadIdx.x;
  const int bi = seg / p.L, l = seg % p.L;
  const int n = p.A * p.h[l] * p.w[l];
  const int G = rpn_sel_groups(n, p.pre_nms);
  if (x >= G) return;
  // tools timing build (p.stamps non-null): 16 int64 per workgroup, s_memrealtime at the phases
  auto stamp = [&](int q) {
    if (p.stamps && t == 0)
      p.stamps[((int64_t)seg * gridDim.x + x) * 16 + q] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const int k = rpn_k(p, n);
  int32_t* st = b.state + seg * TK_WORDS;
  int32_t* bar = b.state + tk_bars_offset((int)gridDim.y) + seg * kBarWords;  // its own line
  const int64_t base = (int64_t)x * kTkChunk;
  const bool has_keys = base < n;
  const uint32_t* gh1 = b.hist1 + (int64_t)seg * (1 << kRpnHistBits);
  uint32_t* gh2 = b.hist2 + (int64_t)seg * kTkBins2;
  constexpr int sh1 = 32 - kRpnHistBits, sh2 = sh1 - 12;

  // ---- phase 1: keys (registers only: the degenerate tie path recomputes them) + first-level histogram.
  // Register r of thread t holds memory position m = base + 256 r + t of the level: anchor m
  // itself, or, for packed channels-last outputs (cell-major: m = cell * A + a), anchor
  // a * H * W + cell -- coalesced logit loads; the anchor index rides along for the ties.
  const int hw = p.h[l] * p.w[l];
  auto anchor = [&](int r) -> int {
    const int m = (int)base + r * kTkThreads + t;
    if (!p.nhwc_cls) return m;
    const int cell = (int)((uint32_t)m / (uint32_t)p.A);
    return (m - cell * p.A) * hw + cell;
  };
  uint32_t key[kTkPerThread];
  tk_hist1_clear(sm.h1, 1 << kRpnHistBits);
  if (has_keys) {
    float x0[kTkPerThread], x1[kTkPerThread];  // every logit load in flight at once
    const int64_t hwa = n;
    if (p.nhwc_cls) {
      const float* cls = p.cls[l] + (int64_t)bi * p.cst[l][0];
      const int CA = p.C * p.A;
#pragma unroll
      for (int r = 0; r < kTkPerThread; ++r) {
        const int m = (int)base + r * kTkThreads + t;
        const int cell = (int)((uint32_t)m / (uint32_t)p.A), a = m - cell * p.A;
        x0[r] = m < n ? cls[(int64_t)cell * CA + a] : 0.0f;
        x1[r] = (p.C == 2 && m < n) ? cls[(int64_t)cell * CA + p.A + a] : 0.0f;
      }
    } else if (p.nchw) {
      const float* cls = p.cls[l] + (int64_t)bi * p.C * hwa;
#pragma unroll
      for (int r = 0; r < kTkPerThread; ++r) {
        const int64_t i = base + r * kTkThreads + t;
        x0[r] = i < hwa ? cls[i] : 0.0f;
        x1[r] = (p.C == 2 && i < hwa) ? cls[hwa + i] : 0.0f;
      }
    } else {
      const float* cls = p.cls[l];
#pragma unroll
      for (int r = 0; r < kTkPerThread; ++r) {
        const int64_t i = base + r * kTkThreads + t;
        x0[r] = i < hwa ? cls[rpn_elem(p.cst[l], p.A, p.h[l], p.w[l], bi, 0, i)] : 0.0f;
        x1[r] = (p.C == 2 && i < hwa) ? cls[rpn_elem(p.cst[l], p.A, p.h[l], p.w[l], bi, 1, i)] : 0.0f;
      }
    }
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      const int64_t m = base + r * kTkThreads + t;
      key[r] = m < hwa ? float_key(score_of2(x0[r], x1[r], p.C)) : 0u;
      tk_hist_add(sm.h1, m < hwa, key[r] >> sh1);
    }
    tk_hist1_flush(sm.h1, 1 << kRpnHistBits, const_cast<uint32_t*>(gh1));
  } else {
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) key[r] = 0u;
  }
  stamp(1);
  if (!seg_barrier(bar + 0, G, p.status, FRH_DEVERR_SELECT_BARRIER)) return;
  stamp(2);

  // ---- phase 2: bucket b1 (every workgroup reads the same final histogram), then b2
  tk_find(sm, 1 << kRpnHistBits, k > 0 ? k : 1, [&](int i) { return xwg_load(gh1 + i); });
  const bool all = k <= 0 || sm.tot <= k;
  TkPlan plan{all, k <= 0 ? 0 : (all ? sm.tot : k), 0u, sh2, 0};
  stamp(3);
  if (!all) {
    const uint32_t b1 = (uint32_t)sm.bin;
    const int k1 = k - sm.above;
    for (int i = t; i < kTkBins2; i += kTkThreads) sm.h2[i] = 0u;
    __syncthreads();
    if (has_keys) {
#pragma unroll
      for (int r = 0; r < kTkPerThread; ++r)
        tk_hist_add(sm.h2, key[r] != 0u && (key[r] >> sh1) == b1, (key[r] >> sh2) & 0xfffu);
      __syncthreads();
      for (int i = t; i < kTkBins2; i += kTkThreads) {
        const uint32_t c = sm.h2[i];
        if (c) atomicAdd(&gh2[i], c);
      }
    }
    stamp(4);
    if (!seg_barrier(bar + 1, G, p.status, FRH_DEVERR_SELECT_BARRIER)) return;
    stamp(5);
    tk_find(sm, kTkBins2, k1, [&](int i) { return xwg_load(gh2 + i); });
    plan.P = (b1 << 12) | (uint32_t)sm.bin;
    plan.k2 = k1 - sm.above;
  }
  const int kv = plan.kv, k2 = all ? 0 : plan.k2, nabove = kv - k2;
  stamp(6);

  // ---- phase 3: collect from the registers; selections decoded by the selecting workgroup
  RpnPol pol{p, ia, b, seg, true};
  uint64_t* cand = b.cand + (int64_t)seg * b.ld;
  if (kv > 0 && has_keys) {
    uint32_t sel = 0u, eq = 0u;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r) {
      const uint32_t pre = key[r] >> plan.sh;
      sel |= (key[r] != 0u && (all || pre > plan.P)) ? 1u << r : 0u;
      eq |= (key[r] != 0u && !all && pre == plan.P) ? 1u << r : 0u;
    }
    const int2 slots = block_reserve2(__popc(sel), __popc(eq), &st[TK_OUT], sm.part, &sm.base, &sm.cbase);
    stamp(7);
    int c = slots.y;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r)
      if (eq & (1u << r)) xwg_store(cand + c++, ((uint64_t)key[r] << 32) | (uint32_t)~(uint32_t)anchor(r));
    int s = slots.x;
    const int gbase = sm.base, nsel = sm.tot_sel;
#pragma unroll
    for (int r = 0; r < kTkPerThread; ++r)
      if (sel & (1u << r)) sm.cand[s++ - gbase] = ((uint64_t)key[r] << 32) | (uint32_t)anchor(r);
    __syncthreads();
    for (int j = t; j < nsel; j += kTkThreads) {
      const uint64_t e = sm.cand[j];
      pol.select((int)(uint32_t)e, (uint32_t)(e >> 32), gbase + j);
    }
  }
  stamp(8);
  if (!seg_barrier(bar + 2, G, p.status, FRH_DEVERR_SELECT_BARRIER)) return;
  stamp(9);

  // ---- phase 4: every record of the segment in LDS (the prefix ties ordered here)
  uint64_t* tie = sm.cand;                 // [kRpnTieCap], later the live-masked records
  uint64_t* rec = sm.cand + kRpnTieCap;    // [kRpnSelFused]
  const uint64_t* grec = p.sel_keys + (int64_t)seg * p.P;
  const int ncand = k2 > 0 ? xwg_load(st + TK_CAND) : 0;
  if (k2 > 0 && ncand > kRpnTieCap) {
    // degenerate key set: workgroup 0 takes the k2 ties by an exact radix select over the
    // prefix (lowest index first among equal keys), then one more barrier
    if (x == 0) {
      int32_t* idx = reinterpret_cast<int32_t*>(cand);  // the consumed candidate row
      auto key_at = [&](int i) -> uint32_t { return float_key(score_of2(rpn_logit(p, l, bi, 0, i),
                                                                        rpn_logit(p, l, bi, 1, i), p.C)); };
      auto key_of = [&](int i) -> uint32_t {
        const uint32_t kq = key_at(i);
        return (kq >> plan.sh) == plan.P ? kq : 0u;
      };
      block_topk_select(key_of, n, k2, idx, sm.fb);
      for (int j = t; j < k2; j += kTkThreads) {
        const int i = idx[j];
        const float4 bx = rpn_decode_one(p, ia, seg, i);
        xwg_store(const_cast<uint64_t*>(grec) + nabove + j,
                  rpn_record(key_at(i), i, rpn_big_enough(bx, ia.min_size[bi]), nabove + j));
      }
    }
    if (!seg_barrier(bar + 3, G, p.status, FRH_DEVERR_SELECT_BARRIER)) return;
    for (int j = t; j < kv; j += kTkThreads) rec[j] = xwg_load(grec + j);
  } else {
    {  // every record load of this thread in flight at once (<= kRpnSelFused / 256 = 8)
      uint64_t rv[kRpnSelFused / kTkThreads];
#pragma unroll
      for (int u = 0; u < kRpnSelFused / kTkThreads; ++u) {
        const int j = u * kTkThreads + t;
        rv[u] = j < nabove ? xwg_load(grec + j) : 0ull;
      }
#pragma unroll
      for (int u = 0; u < kRpnSelFused / kTkThreads; ++u) {
        const int j = u * kTkThreads + t;
        if (j < nabove) rec[j] = rv[u];
      }
    }
    if (k2 > 0) {
      const int P2 = next_pow2(ncand > 1 ? ncand : 1);
      for (int j = t; j < P2; j += kTkThreads) tie[j] = j < ncand ? xwg_load(cand + j) : 0ull;
      __syncthreads();
      stamp(10);
      block_bitonic_sort_desc(tie, P2);
      stamp(11);
      for (int j = t; j < k2; j += kTkThreads) {
        const uint64_t e = tie[j];
        const int i = (int)~(uint32_t)e;
        const float4 bx = rpn_decode_one(p, ia, seg, i);
        rec[nabove + j] = rpn_record((uint32_t)(e >> 32), i, rpn_big_enough(bx, ia.min_size[bi]), nabove + j);
      }
    }
  }
  __syncthreads();

  // ---- phase 5: order by counting (rpn_rank_kernel's rule) over the live-masked records
  stamp(12);
  const int kv32 = (kv + 31) & ~31;  // padding records are 0: never above
  for (int j = t; j < kv32; j += kTkThreads) {
    const uint64_t r = j < kv ? rec[j] : 0ull;
    tie[j] = ((r >> 11) & 1u) ? r : 0ull;
  }
  __syncthreads();
  if (x == 0) {  // the segment's kept count
    int c = 0;
    for (int j = t; j < kv; j += kTkThreads) c += (int)((rec[j] >> 11) & 1u);
    c = block_sum(c, sm.part);
    if (t == 0) p.sel_count[seg] = c;
  }
  // register-blocked count: thread (group g = t / 16, slice q = t % 16) holds this workgroup's
  // records 4g .. 4g + 3 and counts them against every 16th record pair of the segment (16-B
  // LDS reads, each compared with four records: a quarter of the LDS traffic of one record per
  // thread); the 16 slices of a group are lanes of one wave, summed by shuffles.  Lane q < 4 of
  // the group then writes record 4g + q, whose box it fetched before the count.
  static_assert(kSelRankPer == 4 * (kTkThreads / 16), "one pass");
  const int grp = t >> 4, slc = t & 15;
  const uint64_t* stage = reinterpret_cast<const uint64_t*>(p.stage + (int64_t)seg * kRpnSelFused);
  if (x * kSelRankPer < kv) {
    const int q0 = x * kSelRankPer + 4 * grp;
    uint64_t me[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) me[i] = q0 + i < kv ? rec[q0 + i] : ~0ull;
    // the written record's box, in flight during the count
    const int qw = q0 + (slc & 3);
    const uint64_t mw = qw < kv ? rec[qw] : 0ull;
    const bool writes = slc < 4 && qw < kv && ((mw >> 11) & 1u);
    const int wslot = (int)(mw & 0x7ffu);
    float4 bx = make_float4(0.f, 0.f, 0.f, 0.f);
    uint64_t blo = 0ull, bhi = 0ull;
    if (writes) {
      if (wslot < nabove) {
        blo = xwg_load(stage + 2 * wslot);
        bhi = xwg_load(stage + 2 * wslot + 1);
      } else {
        bx = rpn_decode_one(p, ia, seg, (int)(~(uint32_t)(mw >> 12) & 0xfffffu));
      }
    }
    const ulonglong2* tv = reinterpret_cast<const ulonglong2*>(tie);
    int a[4] = {0, 0, 0, 0};
    const int np = kv32 / 2;  // record pairs, a multiple of 16
    for (int j = slc; j < np; j += 64) {
      ulonglong2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = j + 16 * u < np ? tv[j + 16 * u] : make_ulonglong2(0ull, 0ull);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] += (v[u].x > me[i] ? 1 : 0) + (v[u].y > me[i] ? 1 : 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] += __shfl_xor(a[i], 1, kWave);
      a[i] += __shfl_xor(a[i], 2, kWave);
      a[i] += __shfl_xor(a[i], 4, kWave);
      a[i] += __shfl_xor(a[i], 8, kWave);
    }
    if (writes) {
      const int i = slc & 3;
      const int above = i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
      if (wslot < nabove)
        bx = make_float4(__uint_as_float((uint32_t)blo), __uint_as_float((uint32_t)(blo >> 32)),
                         __uint_as_float((uint32_t)bhi), __uint_as_float((uint32_t)(bhi >> 32)));
      reinterpret_cast<float4*>(p.sel_boxes)[(int64_t)seg * p.P + above] = bx;
      p.sel_scores[(int64_t)seg * p.P + above] = key_float((uint32_t)(mw >> 32));
    }
  }
  stamp(13);
}

// ... and one 1024-thread block per segment orders them by (score desc, index
// asc) in LDS (up to kMaxSort) and decodes
static __global__ void __launch_bounds__(kPropThreads) rpn_sort_decode_kernel(PropArgs p, ImgArgs ia, const int32_t* state) {
  extern __shared__ uint64_t skeys[];
  __shared__ int wave_tot[kPropThreads / 64];
  const int seg = blockIdx.x;
  const int m = state[seg * TK_WORDS + TK_K];
  const int P2 = next_pow2(m > 1 ? m : 1);
  const uint64_t* sl = p.sel_keys + (int64_t)seg * p.P;
  for (int j = threadIdx.x; j < P2; j += blockDim.x) skeys[j] = j < m ? sl[j] : 0ull;
  __syncthreads();
  block_bitonic_sort_desc(skeys, P2);
  const float min_size = ia.min_size[seg / p.L];
  float* ob = p.sel_boxes + (int64_t)seg * p.P * 4;
  float* os = p.sel_scores + (int64_t)seg * p.P;
  int written = 0;
  for (int base = 0; base < m; base += blockDim.x) {
    const int j = base + threadIdx.x;
    bool live = j < m;
    float4 bx = make_float4(0.f, 0.f, 0.f, 0.f);
    if (live) {
      bx = rpn_decode_one(p, ia, seg, (int)~(uint32_t)skeys[j]);
      live = rpn_big_enough(bx, min_size);
    }
    int tot;
    const int r = block_rank(live, wave_tot, &tot);
    if (live) {
      reinterpret_cast<float4*>(ob)[written + r] = bx;
      os[written + r] = key_float((uint32_t)(skeys[j] >> 32));
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
// a binary search (upper bound for earlier levels, lower bound for later).  No sort.
__device__ __forceinline__ float kept_score(const MergeArgs& p, int seg, int j) {
  return p.sel_scores[(int64_t)seg * p.P + p.keep[(int64_t)seg * p.P + j]];
}

__device__ __forceinline__ void merge_write(const MergeArgs& p, int b, int seg, int pos, int rank, float s) {
  float4 bx = reinterpret_cast<const float4*>(p.sel_boxes)[(int64_t)seg * p.P + pos];
  float* ob = p.out_boxes + (int64_t)b * 4 * p.out_cap;
  ob[rank] = bx.x;
  ob[p.out_cap + rank] = bx.y;
  ob[2 * p.out_cap + rank] = bx.z;
  ob[3 * p.out_cap + rank] = bx.w;
  p.out_scores[(int64_t)b * p.out_cap + rank] = s;
}

// One 1024-thread workgroup per (level, image): the image's survivor scores of every
// level are gathered into LDS first (L * P floats; each thread's keep-index loads in
// flight together, then its score gathers), so the searches are LDS reads, not chains
// of dependent global loads.  The workgroup's own survivors (j = t, t + 1024) are loaded
// by the threads that rank them -- keep index, then score and box together -- so their
// outputs need no further loads.
constexpr int kMergeThreads = 1024;
constexpr int kMergePer = 16;  // gathered scores per thread and batch
constexpr int kMergeOwn = 2;   // own survivors per thread (post_nms <= 2048)

static __global__ void __launch_bounds__(kMergeThreads) rpn_merge_lds_kernel(MergeArgs p) {
  extern __shared__ float ms[];  // [L][P] survivor scores of image b
  __shared__ int cnt_s[FRH_MAX_LEVELS + 1];
  const int l = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  if (t < p.L) cnt_s[t] = p.keep_count[b * p.L + t];
  __syncthreads();
  int total = 0, base = 0;
  for (int q = 0; q < p.L; ++q) {
    base += q < l ? cnt_s[q] : 0;
    total += cnt_s[q];
  }
  const bool cut = p.max_num > 0 && total > p.max_num;
  if (l == 0 && t == 0) p.out_counts[b] = cut ? p.max_num : total;
  const int seg = b * p.L + l, cnt = cnt_s[l];
  // own survivors: keep index, then score + box (in flight with the staging gathers below)
  int own_pos[kMergeOwn];
#pragma unroll
  for (int u = 0; u < kMergeOwn; ++u) {
    const int j = t + u * kMergeThreads;
    own_pos[u] = j < cnt ? p.keep[(int64_t)seg * p.P + j] : -1;
  }
  float own_s[kMergeOwn];
  float4 own_bx[kMergeOwn];
#pragma unroll
  for (int u = 0; u < kMergeOwn; ++u) {
    if (own_pos[u] >= 0) {
      own_s[u] = p.sel_scores[(int64_t)seg * p.P + own_pos[u]];
      own_bx[u] = reinterpret_cast<const float4*>(p.sel_boxes)[(int64_t)seg * p.P + own_pos[u]];
    }
  }
  if (cut) {
    // flat index e over (level, survivor), e = q * P + i
    for (int e0 = 0; e0 < p.L * p.P; e0 += kMergeThreads * kMergePer) {
      int kidx[kMergePer];
#pragma unroll
      for (int u = 0; u < kMergePer; ++u) {
        const int e = e0 + u * kMergeThreads + t, q = e / p.P, i = e - q * p.P;
        kidx[u] = (q < p.L && i < cnt_s[q]) ? p.keep[(int64_t)(b * p.L + q) * p.P + i] : -1;
      }
#pragma unroll
      for (int u = 0; u < kMergePer; ++u) {
        const int e = e0 + u * kMergeThreads + t, q = e / p.P;
        if (kidx[u] >= 0) ms[e] = p.sel_scores[(int64_t)(b * p.L + q) * p.P + kidx[u]];
      }
    }
    __syncthreads();
  }
  float* ob = p.out_boxes + (int64_t)b * 4 * p.out_cap;
#pragma unroll
  for (int u = 0; u < kMergeOwn; ++u) {
    const int j = t + u * kMergeThreads;
    if (own_pos[u] < 0) continue;
    const float s = own_s[u];
    int rank = base + j;
    if (cut) {
      rank = j;
      for (int q = 0; q < p.L; ++q) {
        if (q == l) continue;
        int lo = 0, hi = cnt_s[q];
        // count of survivors of level q ordered before (s, this level)
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const float o = ms[q * p.P + mid];
          const bool before = q < l ? (o >= s) : (o > s);
          if (before)
            lo = mid + 1;
          else
            hi = mid;
        }
        rank += lo;
      }
      if (rank >= p.max_num) continue;
    }
    ob[rank] = own_bx[u].x;
    ob[p.out_cap + rank] = own_bx[u].y;
    ob[2 * p.out_cap + rank] = own_bx[u].z;
    ob[3 * p.out_cap + rank] = own_bx[u].w;
    p.out_scores[(int64_t)b * p.out_cap + rank] = s;
  }
}

// The same with the searches in global memory (levels x survivors beyond the LDS):
// grid (survivor chunks of 256, level, image).
static __global__ void __launch_bounds__(256) rpn_merge_kernel(MergeArgs p) {
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
  merge_write(p, b, seg, pos, rank, s);
}

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

static __global__ void __launch_bounds__(kMwThreads) rpn_merge_wide_kernel(MergeArgs p,
                                                                           const uint32_t* __restrict__ kscore) {
  extern __shared__ float ms[];  // image b's other levels' kept scores, packed in level order
  __shared__ int cnt_s[FRH_MAX_LEVELS], beg_s[FRH_MAX_LEVELS];
  const int L = p.L, l = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const int seg = b * L + l, j = blockIdx.x * kMwThreads + t, jc = min(j, p.P - 1);
  const int cv = t < L ? p.keep_count[b * L + t] : 0;  // in flight together with the own survivor
  const int pos_raw = p.keep[(int64_t)seg * p.P + jc];
  const uint32_t scb = kscore[(int64_t)seg * p.P + jc];
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
  if (blockIdx.x == 0 && l == 0 && t == 0) p.out_counts[b] = cut ? p.max_num : total;
  if ((int)blockIdx.x * kMwThreads >= own_n) return;  // workgroup-uniform
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
        v[u] = e < n_other ? kscore[(int64_t)(b * L + q) * p.P + (e - beg_s[q])] : 0u;
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

static size_t al(size_t v) { return (v + 255) & ~(size_t)255; }

int32_t rpn_proposals_impl(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                           const float* const* reg_ptrs, const int64_t* cls_strides, const int64_t* reg_strides,
                           const int32_t* grid_hw, int32_t num_anchors, int32_t cls_channels, const float* anchors,
                           int64_t anchor_ld, const float* means, const float* stds, const float* img_hw,
                           const float* min_size, int32_t pre_nms, int32_t post_nms, int32_t max_num, double nms_iou,
                           float* out_boxes, float* out_scores, int32_t* out_counts, int32_t* status,
                           void* workspace, size_t ws_bytes, void* stream, bool select_launches,
                           int64_t* select_stamps = nullptr, bool nms_launches = false, bool merge_launch = false,
                           int64_t* nms_stamps = nullptr);

struct PropLayout {
  int P;
  size_t boxes, scores, idx, stage, cnt, keep, kcnt, kscore, mask, keys, mem, zero, nflags, zero_bytes, total;
  int64_t nmax, kld;
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
  z.kld = nmax;
  const size_t S = (size_t)B * L;
  z.boxes = 0;
  z.scores = z.boxes + al(S * P * 4 * sizeof(float));
  z.idx = z.scores + al(S * P * sizeof(float));
  z.stage = z.idx + al(S * P * sizeof(uint64_t));
  z.cnt = z.stage + al(S * kRpnSelFused * sizeof(float4));
  z.keep = z.cnt + al(S * sizeof(int32_t));
  z.kcnt = z.keep + al(S * P * sizeof(int32_t));
  z.kscore = z.kcnt + al(S * sizeof(int32_t));
  z.mask = z.kscore + al(S * P * sizeof(float));
  z.keys = z.mask + al(nms_mask_bytes((int32_t)S, P));
  z.mem = z.keys + al(S * (size_t)z.kld * sizeof(uint32_t));
  z.zero = z.mem + al(S * (size_t)z.kld * sizeof(uint64_t));
  // zeroed by one memset per call: the selection's histograms / state / barriers, then the
  // one-launch NMS's tile flags
  z.nflags = z.zero + al(tk_zero_bytes((int)S, kRpnHistBits));
  z.zero_bytes = z.nflags - z.zero + nms_fused_flag_bytes((int32_t)S, P);
  z.total = z.zero + al(z.zero_bytes);
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

extern "C" int32_t frh_rpn_proposals_strided(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                             const float* const* reg_ptrs, const int64_t* cls_strides,
                                             const int64_t* reg_strides, const int32_t* grid_hw,
                                             int32_t num_anchors, int32_t cls_channels, const float* anchors,
                                             int64_t anchor_ld, const float* means, const float* stds,
                                             const float* img_hw, const float* min_size, int32_t pre_nms,
                                             int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                             float* out_scores, int32_t* out_counts, int32_t* status,
                                             void* workspace, size_t ws_bytes, void* stream);

extern "C" int32_t frh_rpn_proposals(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                     const float* const* reg_ptrs, const int32_t* grid_hw, int32_t num_anchors,
                                     int32_t cls_channels, const float* anchors, int64_t anchor_ld,
                                     const float* means, const float* stds, const float* img_hw,
                                     const float* min_size, int32_t pre_nms, int32_t post_nms, int32_t max_num,
                                     double nms_iou, float* out_boxes, float* out_scores, int32_t* out_counts,
                                     int32_t* status, void* workspace, size_t ws_bytes, void* stream) {
  FRH_REQUIRE(num_levels >= 1 && num_levels <= FRH_MAX_LEVELS && grid_hw, "bad level count %d", num_levels);
  int64_t cs[4 * FRH_MAX_LEVELS], rs[4 * FRH_MAX_LEVELS];
  for (int l = 0; l < num_levels; ++l) {  // contiguous [B, R*A, H, W]
    const int64_t hw = (int64_t)grid_hw[2 * l] * grid_hw[2 * l + 1];
    cs[4 * l] = (int64_t)cls_channels * num_anchors * hw, cs[4 * l + 1] = hw, cs[4 * l + 2] = grid_hw[2 * l + 1],
    cs[4 * l + 3] = 1;
    rs[4 * l] = (int64_t)4 * num_anchors * hw, rs[4 * l + 1] = hw, rs[4 * l + 2] = grid_hw[2 * l + 1], rs[4 * l + 3] = 1;
  }
  return frh_rpn_proposals_strided(num_imgs, num_levels, cls_ptrs, reg_ptrs, cs, rs, grid_hw, num_anchors,
                                   cls_channels, anchors, anchor_ld, means, stds, img_hw, min_size, pre_nms, post_nms,
                                   max_num, nms_iou, out_boxes, out_scores, out_counts, status, workspace, ws_bytes,
                                   stream);
}

extern "C" int32_t frh_rpn_proposals_strided(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                             const float* const* reg_ptrs, const int64_t* cls_strides,
                                             const int64_t* reg_strides, const int32_t* grid_hw,
                                             int32_t num_anchors, int32_t cls_channels, const float* anchors,
                                             int64_t anchor_ld, const float* means, const float* stds,
                                             const float* img_hw, const float* min_size, int32_t pre_nms,
                                             int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                             float* out_scores, int32_t* out_counts, int32_t* status,
                                             void* workspace, size_t ws_bytes, void* stream) {
  return frh::rpn_proposals_impl(num_imgs, num_levels, cls_ptrs, reg_ptrs, cls_strides, reg_strides, grid_hw,
                                 num_anchors, cls_channels, anchors, anchor_ld, means, stds, img_hw, min_size, pre_nms,
                                 post_nms, max_num, nms_iou, out_boxes, out_scores, out_counts, status, workspace,
                                 ws_bytes, stream, false);
}

// select_launches: the four-launch selection even where the one-launch one applies
// (tools: A/B measurement and equality tests of the two)
int32_t frh::rpn_proposals_impl(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                const float* const* reg_ptrs, const int64_t* cls_strides, const int64_t* reg_strides,
                                const int32_t* grid_hw, int32_t num_anchors, int32_t cls_channels,
                                const float* anchors, int64_t anchor_ld, const float* means, const float* stds,
                                const float* img_hw, const float* min_size, int32_t pre_nms, int32_t post_nms,
                                int32_t max_num, double nms_iou, float* out_boxes, float* out_scores,
                                int32_t* out_counts, int32_t* status, void* workspace, size_t ws_bytes, void* stream,
                                bool select_launches, int64_t* select_stamps, bool nms_launches, bool merge_launch,
                                int64_t* nms_stamps) {
  FRH_REQUIRE(cls_strides && reg_strides, "null stride arrays");
  FRH_REQUIRE(num_imgs >= 1 && num_imgs <= 64, "num_imgs %d must be in [1, 64]", num_imgs);
  FRH_REQUIRE(num_levels >= 1 && num_levels <= FRH_MAX_LEVELS, "bad level count %d", num_levels);
  FRH_REQUIRE(cls_channels == 1 || cls_channels == 2, "cls_channels must be 1 (sigmoid) or 2 (softmax)");
  FRH_REQUIRE(cls_ptrs && reg_ptrs && grid_hw && anchors && img_hw && min_size && out_boxes && out_scores &&
                  out_counts && means && stds && status,
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
  p.nchw = 1;
  for (int l = 0; l < num_levels; ++l) {
    p.cls[l] = cls_ptrs[l];
    p.reg[l] = reg_ptrs[l];
    p.h[l] = grid_hw[2 * l];
    p.w[l] = grid_hw[2 * l + 1];
    p.off[l] = off;
    const int64_t hw = (int64_t)p.h[l] * p.w[l];
    off += (int64_t)num_anchors * hw;
    for (int q = 0; q < 4; ++q) p.cst[l][q] = cls_strides[4 * l + q], p.rst[l][q] = reg_strides[4 * l + q];
    p.nhwc_cls = (l == 0 || p.nhwc_cls) && p.cst[l][1] == 1 && p.cst[l][3] == (int64_t)cls_channels * num_anchors &&
                 p.cst[l][2] == (int64_t)p.w[l] * cls_channels * num_anchors;
    p.nchw = p.nchw && p.cst[l][0] == (int64_t)cls_channels * num_anchors * hw && p.cst[l][1] == hw &&
             p.cst[l][2] == p.w[l] && p.cst[l][3] == 1 && p.rst[l][0] == (int64_t)4 * num_anchors * hw &&
             p.rst[l][1] == hw && p.rst[l][2] == p.w[l] && p.rst[l][3] == 1;
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
  p.sel_keys = reinterpret_cast<uint64_t*>(ws + z.idx);
  p.stage = reinterpret_cast<float4*>(ws + z.stage);
  p.sel_count = reinterpret_cast<int32_t*>(ws + z.cnt);
  p.stamps = select_stamps;
  p.status = status;
  // per-image sizes travel by value in the kernel arguments
  ImgArgs ia{};
  for (int b = 0; b < num_imgs; ++b) {
    ia.hw[2 * b] = img_hw[2 * b];
    ia.hw[2 * b + 1] = img_hw[2 * b + 1];
    ia.min_size[b] = min_size[b];
  }
  const int S = num_imgs * num_levels;
  // 1. keys + first-level histogram, 2. top-k + order + decode + min-size
  // (sort + decode fused into the collect launch when the selection is <= kRpnSelFused)
  char* zb = ws + z.zero;
  TkBufs tb{reinterpret_cast<uint32_t*>(ws + z.keys), z.kld, reinterpret_cast<uint32_t*>(zb), kRpnHistBits,
            reinterpret_cast<uint32_t*>(zb + (size_t)S * (1 << kRpnHistBits) * sizeof(uint32_t)),
            reinterpret_cast<int32_t*>(zb + (size_t)S * ((1 << kRpnHistBits) + kTkBins2) * sizeof(uint32_t)),
            reinterpret_cast<uint64_t*>(ws + z.mem)};
  FRH_HIP(hipMemsetAsync(zb, 0, z.zero_bytes, st));
  const dim3 grid((unsigned)((z.nmax + kTkChunk - 1) / kTkChunk), (unsigned)S);
  const bool fused = z.P <= kRpnSelFused && z.nmax < (1 << 20);  // record layout limits
  // one-launch selection: every segment's workgroups resident together (seg_barrier): the
  // grid's live workgroups stay within 3/4 of what the device holds of this kernel (CU
  // count x occupancy; TkSmem ~35 KB of LDS: 4 per CU on a whole MI355X = 1024)
  int gx = 1, live_wgs = 0;
  for (int l = 0; l < num_levels; ++l) {
    const int g = rpn_sel_groups(num_anchors * p.h[l] * p.w[l], pre_nms);
    gx = g > gx ? g : gx;
    live_wgs += g * num_imgs;
  }
  if (fused && live_wgs <= resident_capacity(reinterpret_cast<const void*>(rpn_select_kernel), kTkThreads) * 3 / 4 &&
      !select_launches) {
    hipLaunchKernelGGL(rpn_select_kernel, dim3((unsigned)gx, (unsigned)S), dim3(kTkThreads), 0, st, p, ia, tb);
  } else {
  hipLaunchKernelGGL(rpn_keys_kernel, grid, dim3(kTkThreads), 0, st, p, tb);
  hipLaunchKernelGGL(rpn_refine_kernel, grid, dim3(kTkThreads), 0, st, p, tb);
  hipLaunchKernelGGL(rpn_collect_kernel, grid, dim3(kTkThreads), 0, st, p, ia, tb, fused);
  if (fused) {
    hipLaunchKernelGGL(rpn_rank_kernel, dim3(kRpnSelFused / kRankPer, (unsigned)S), dim3(256), 0, st, p, tb.state);
  } else {
    const size_t lds_sel = (size_t)next_pow2(z.P) * sizeof(uint64_t);
    if (lds_sel > 65536)
      FRH_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(rpn_sort_decode_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sel));
    hipLaunchKernelGGL(rpn_sort_decode_kernel, dim3(S), dim3(kPropThreads), lds_sel, st, p, ia, tb.state);
  }
  }
  int32_t r = check_launch("rpn_select");
  if (r) return r;
  int32_t* keep = reinterpret_cast<int32_t*>(ws + z.keep);
  int32_t* kcnt = reinterpret_cast<int32_t*>(ws + z.kcnt);
  uint64_t* nmask = reinterpret_cast<uint64_t*>(ws + z.mask);
  const int64_t out_cap = max_num > 0 ? max_num : post * num_levels;
  const bool nms_fused = !nms_launches && nms_fused_fits(S, z.P);
  // 4. the cross-level merge: the wide form over the one-launch NMS's compact kept scores
  const size_t wide_lds = (size_t)(num_levels - 1) * z.P * sizeof(float);
  const bool wide = nms_fused && !merge_launch && wide_lds <= 65536 - 256;
  uint32_t* kscore = wide ? reinterpret_cast<uint32_t*>(ws + z.kscore) : nullptr;
  if (nms_fused)  // 3. NMS
    r = launch_nms_fused(S, p.sel_boxes, (int64_t)z.P * 4, p.sel_count, z.P, nms_iou, (post_nms > 0) ? post_nms : -1,
                         keep, z.P, kcnt, nmask, reinterpret_cast<uint32_t*>(ws + z.nflags), status, st, nms_stamps,
                         p.sel_scores, kscore);
  else
    r = launch_nms_sorted(S, p.sel_boxes, (int64_t)z.P * 4, p.sel_count, z.P, nms_iou,
                          (post_nms > 0) ? post_nms : -1, keep, z.P, kcnt, nmask, nullptr, st);
  if (r) return r;
  MergeArgs mp{p.sel_boxes, p.sel_scores, keep, kcnt, num_levels, z.P, max_num, out_cap, out_boxes, out_scores,
               out_counts};
  const size_t merge_lds = (size_t)num_levels * z.P * sizeof(float);
  if (wide) {
    const dim3 mg((unsigned)((post + kMwThreads - 1) / kMwThreads), (unsigned)num_levels, (unsigned)num_imgs);
    hipLaunchKernelGGL(rpn_merge_wide_kernel, mg, dim3(kMwThreads), wide_lds, st, mp, kscore);
  } else if (merge_lds <= 65536 - 256 && z.P <= kMergeThreads * kMergeOwn) {  // + the kernel's static counts
    hipLaunchKernelGGL(rpn_merge_lds_kernel, dim3((unsigned)num_levels, (unsigned)num_imgs), dim3(kMergeThreads),
                       merge_lds, st, mp);
  } else {
    dim3 mg((unsigned)((post + 255) / 256), (unsigned)num_levels, (unsigned)num_imgs);
    hipLaunchKernelGGL(rpn_merge_kernel, mg, dim3(256), 0, st, mp);
  }
  return check_launch("rpn_merge");
}
