// a16: ATSS target assignment with LTRB targets and centerness, all images in
// three launches.
// Reference: lib/heads/fcos_head.py:283-368 (FCOSHead.single_image_targets_atss)
// and its helpers topk_by_center (:106-116), bbox2ltrb (:78-87),
// positive_ltrb (:51-53), centerness (:56-59), paint_value (:90-94);
// calc_iou (lib/utils.py:151-172).
//
// The reference walks gts in order and, per gt, its 9 nearest cells on every
// level; a candidate cell is written when iou > mean + std of the gt's 45
// candidate IoUs, its centre lies inside the gt (ltrb > 0) and iou >= the IoU
// already stored at the cell.  That sequential fold has a closed form used
// here: candidate (g, c) is accepted iff it is valid and its IoU is >= every
// valid candidate of an earlier gt at the same cell (a rejected candidate is
// below the running maximum, so it never changes it), and the cell's final
// owner is its accepted candidate with the largest g.  So:
//   atss_fill      paint: cls 0 inside round(img / stride), else -1; reg -1; owner -1
//   atss_topk      block per (gt, level, image): the k nearest cell centres,
//                  (distance, cell index) ascending, and their calc_iou
//   atss_resolve   block per image: per-gt threshold (mean + unbiased std, in
//                  double), validity, acceptance by the closed form, owner =
//                  atomicMax(g), then the owners write label / ltrb / centerness.
#include <math.h>

#include "common.h"

namespace frh {

constexpr int kAtssMaxLevels = 16;
constexpr int kAtssMaxK = 16;
constexpr int kAtssThreads = 256;

struct AtssArgs {
  int B, L, K, Gmax;
  int64_t N;
  int64_t off[kAtssMaxLevels + 1];
  int gh[kAtssMaxLevels], gw[kAtssMaxLevels];
  float stride[kAtssMaxLevels];
  const float* anchors;
  int64_t ald;
  const float* gts;
  int64_t gseg;
  const int32_t* ngt;
  const int64_t* labels;
  const int32_t* img_hw;
  int64_t* cls;
  float* reg;
  float* ctr;
  // workspace
  int32_t* cand;   // [B][Gmax][L*K] global cell index or -1
  float* ciou;     // [B][Gmax][L*K]
  uint8_t* valid;  // [B][Gmax][L*K]
  float* thr;      // [B][Gmax]
  int32_t* owner;  // [B][N]
};

__device__ __forceinline__ int level_of(const AtssArgs& a, int64_t c) {
  int l = 0;
  while (l + 1 < a.L && c >= a.off[l + 1]) ++l;
  return l;
}

__global__ void atss_fill_kernel(AtssArgs a) {
  const int b = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.N) return;
  const int l = level_of(a, c);
  const int64_t i = c - a.off[l];
  const int y = (int)(i / a.gw[l]), x = (int)(i - (int64_t)y * a.gw[l]);
  // paint_value: [0, 0, img_w, img_h] * (1 / stride) in f32, round half-even, inclusive slice
  const float sc = (float)(1.0 / (double)a.stride[l]);
  const int x2 = (int)rintf((float)a.img_hw[2 * b + 1] * sc), y2 = (int)rintf((float)a.img_hw[2 * b] * sc);
  const bool in = y <= y2 && x <= x2;
  const int64_t o = (int64_t)b * a.N + c;
  a.cls[o] = in ? 0 : -1;
  a.ctr[o] = in ? 0.0f : -1.0f;
  reinterpret_cast<float4*>(a.reg)[o] = make_float4(-1.0f, -1.0f, -1.0f, -1.0f);
  a.owner[o] = -1;
}

__device__ __forceinline__ void gt_box(const AtssArgs& a, int b, int g, float* bx) {
  const float* G = a.gts + (int64_t)b * a.gseg;
#pragma unroll
  for (int q = 0; q < 4; ++q) bx[q] = G[(int64_t)q * a.Gmax + g];
}

// keep the 16 smallest keys, ascending (branch-free insertion)
__device__ __forceinline__ void push16(uint64_t (&best)[kAtssMaxK], uint64_t key) {
#pragma unroll
  for (int j = 0; j < kAtssMaxK; ++j) {
    const uint64_t lo = best[j] < key ? best[j] : key;
    key = best[j] < key ? key : best[j];
    best[j] = lo;
  }
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t w = ((uint64_t)(uint32_t)__shfl_xor((int)(v >> 32), o, kWave) << 32) |
                       (uint32_t)__shfl_xor((int)(uint32_t)v, o, kWave);
    v = w < v ? w : v;
  }
  return v;
}

__global__ void __launch_bounds__(kAtssThreads) atss_topk_kernel(AtssArgs a) {
  __shared__ uint64_t s_keys[kAtssThreads * kAtssMaxK];
  __shared__ uint64_t s_top[kAtssMaxK];
  const int g = blockIdx.x, l = blockIdx.y, b = blockIdx.z;
  if (g >= a.ngt[b]) return;
  float bx[4];
  gt_box(a, b, g, bx);
  // topk_by_center: centre_of(anchor) - centre_of(gt), L2 norm, k smallest
  const float bcx = (bx[2] + bx[0]) / 2.0f, bcy = (bx[3] + bx[1]) / 2.0f;
  const int64_t hw = (int64_t)a.gh[l] * a.gw[l];
  const int64_t c0 = a.off[l];
  const float* A = a.anchors;
  const int64_t ld = a.ald;
  uint64_t best[kAtssMaxK];
#pragma unroll
  for (int j = 0; j < kAtssMaxK; ++j) best[j] = ~0ull;
  for (int64_t i = threadIdx.x; i < hw; i += blockDim.x) {
    const int64_t c = c0 + i;
    const float acx = (A[2 * ld + c] + A[c]) / 2.0f, acy = (A[3 * ld + c] + A[ld + c]) / 2.0f;
    const float dx = acx - bcx, dy = acy - bcy;
    const float d = sqrtf(dx * dx + dy * dy);
    push16(best, ((uint64_t)float_key(d) << 32) | (uint64_t)i);
  }
#pragma unroll
  for (int j = 0; j < kAtssMaxK; ++j) s_keys[threadIdx.x * kAtssMaxK + j] = best[j];
  __syncthreads();
  if (threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    uint64_t m[kAtssMaxK];
#pragma unroll
    for (int j = 0; j < kAtssMaxK; ++j) m[j] = ~0ull;
    for (int t = lane; t < kAtssThreads; t += kWave)
#pragma unroll
      for (int j = 0; j < kAtssMaxK; ++j) push16(m, s_keys[t * kAtssMaxK + j]);
    for (int r = 0; r < a.K; ++r) {
      const uint64_t w = wave_min_u64(m[0]);
      const bool mine = m[0] == w;  // keys are unique (cell index in the low bits)
      if (mine) {
#pragma unroll
        for (int j = 0; j + 1 < kAtssMaxK; ++j) m[j] = m[j + 1];
        m[kAtssMaxK - 1] = ~0ull;
      }
      if (lane == 0) s_top[r] = w;
    }
  }
  __syncthreads();
  const int LK = a.L * a.K;
  const int64_t base = ((int64_t)b * a.Gmax + g) * LK + (int64_t)l * a.K;
  for (int j = threadIdx.x; j < a.K; j += blockDim.x) {
    const uint64_t key = s_top[j];
    if (j < hw && key != ~0ull) {
      const int64_t c = c0 + (int64_t)(uint32_t)key;
      a.cand[base + j] = (int32_t)c;
      a.ciou[base + j] = iou_plus1(A[c], A[ld + c], A[2 * ld + c], A[3 * ld + c], bx[0], bx[1], bx[2], bx[3]);
    } else {
      a.cand[base + j] = -1;
      a.ciou[base + j] = 0.0f;
    }
  }
}

__device__ __forceinline__ void cell_ltrb(const AtssArgs& a, int64_t c, const float* bx, float* lt) {
  const int l = level_of(a, c);
  const int64_t i = c - a.off[l];
  const int y = (int)(i / a.gw[l]), x = (int)(i - (int64_t)y * a.gw[l]);
  const float s = a.stride[l];
  const float cx = (float)x * s + s / 2.0f, cy = (float)y * s + s / 2.0f;
  lt[0] = cx - bx[0];
  lt[1] = cy - bx[1];
  lt[2] = bx[2] - cx;
  lt[3] = bx[3] - cy;
}

__global__ void __launch_bounds__(kAtssThreads) atss_resolve_kernel(AtssArgs a) {
  const int b = blockIdx.x;
  const int G = a.ngt[b];
  const int LK = a.L * a.K;
  const int64_t cb = (int64_t)b * a.Gmax * LK;
  const int32_t* cand = a.cand + cb;
  const float* ciou = a.ciou + cb;
  uint8_t* valid = a.valid + cb;
  float* thr = a.thr + (int64_t)b * a.Gmax;
  // per-gt threshold: mean + unbiased std of its candidate IoUs
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    double s = 0.0, ss = 0.0;
    int n = 0;
    for (int j = 0; j < LK; ++j)
      if (cand[g * LK + j] >= 0) {
        s += ciou[g * LK + j];
        ++n;
      }
    const double mean = s / n;
    for (int j = 0; j < LK; ++j)
      if (cand[g * LK + j] >= 0) {
        const double d = (double)ciou[g * LK + j] - mean;
        ss += d * d;
      }
    thr[g] = (float)mean + (float)sqrt(ss / (n - 1));
  }
  __syncthreads();
  for (int e = threadIdx.x; e < G * LK; e += blockDim.x) {
    const int g = e / LK;
    const int32_t c = cand[e];
    uint8_t v = 0;
    if (c >= 0 && ciou[e] > thr[g]) {
      float bx[4], lt[4];
      gt_box(a, b, g, bx);
      cell_ltrb(a, c, bx, lt);
      v = lt[0] > 0.0f && lt[1] > 0.0f && lt[2] > 0.0f && lt[3] > 0.0f;
    }
    valid[e] = v;
  }
  __syncthreads();
  int32_t* owner = a.owner + (int64_t)b * a.N;
  for (int e = threadIdx.x; e < G * LK; e += blockDim.x) {
    if (!valid[e]) continue;
    const int g = e / LK, j = e - g * LK, lb = (j / a.K) * a.K;
    const int32_t c = cand[e];
    const float iou = ciou[e];
    float exist = 0.0f;
    for (int h = 0; h < g; ++h)
      for (int q = lb; q < lb + a.K; ++q) {
        const int eq = h * LK + q;
        if (cand[eq] == c && valid[eq]) exist = fmaxf(exist, ciou[eq]);
      }
    if (iou >= exist) atomicMax(&owner[c], g);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < G * LK; e += blockDim.x) {
    if (!valid[e]) continue;
    const int g = e / LK;
    const int32_t c = cand[e];
    if (__hip_atomic_load(&owner[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != g) continue;
    float bx[4], lt[4];
    gt_box(a, b, g, bx);
    cell_ltrb(a, c, bx, lt);
    const int64_t o = (int64_t)b * a.N + c;
    a.cls[o] = a.labels[(int64_t)b * a.Gmax + g];
    reinterpret_cast<float4*>(a.reg)[o] = make_float4(lt[0], lt[1], lt[2], lt[3]);
    // centerness on ltrb + 1e-6
    const float l = lt[0] + 1e-6f, t = lt[1] + 1e-6f, r = lt[2] + 1e-6f, bb = lt[3] + 1e-6f;
    a.ctr[o] = sqrtf((fminf(l, r) / fmaxf(l, r)) * (fminf(t, bb) / fmaxf(t, bb)));
  }
}

struct AtssLayout {
  size_t cand, ciou, valid, thr, owner, total;
};

static AtssLayout atss_layout(int32_t B, int32_t G, int32_t L, int32_t K, int64_t N) {
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  AtssLayout w;
  const size_t nc = (size_t)B * (size_t)(G > 0 ? G : 1) * (size_t)L * (size_t)K;
  size_t o = 0;
  w.cand = o;
  o += up(nc * 4);
  w.ciou = o;
  o += up(nc * 4);
  w.valid = o;
  o += up(nc);
  w.thr = o;
  o += up((size_t)B * (size_t)(G > 0 ? G : 1) * 4);
  w.owner = o;
  o += up((size_t)B * (size_t)N * 4);
  w.total = o;
  return w;
}

}  // namespace frh

using namespace frh;

extern "C" size_t frh_atss_workspace(int32_t batch, int32_t max_gts, int32_t num_levels, int32_t topk,
                                     int64_t num_cells) {
  if (batch <= 0 || num_levels <= 0 || topk <= 0 || num_cells < 0) return 0;
  return atss_layout(batch, max_gts, num_levels, topk, num_cells).total;
}

extern "C" int32_t frh_atss_assign(int32_t batch, int32_t num_levels, const int32_t* grid_hw, const float* strides,
                                   const float* anchors, int64_t anchor_ld, const float* gts, int64_t gt_seg_stride,
                                   const int32_t* num_gts, const int64_t* gt_labels, int32_t max_gts,
                                   const int32_t* img_hw, int32_t topk, int64_t* cls, float* reg, float* ctr,
                                   void* workspace, size_t ws_bytes, void* stream) {
  FRH_REQUIRE(batch >= 0 && max_gts >= 0, "negative sizes");
  FRH_REQUIRE(num_levels >= 1 && num_levels <= kAtssMaxLevels, "num_levels %d not in [1, %d]", num_levels,
              kAtssMaxLevels);
  FRH_REQUIRE(topk >= 1 && topk <= kAtssMaxK, "topk %d not in [1, %d]", topk, kAtssMaxK);
  FRH_REQUIRE(grid_hw && strides, "null host array");
  if (batch == 0) return FRH_OK;
  AtssArgs a{};
  a.B = batch;
  a.L = num_levels;
  a.K = topk;
  a.Gmax = max_gts;
  int64_t n = 0;
  for (int l = 0; l < num_levels; ++l) {
    FRH_REQUIRE(grid_hw[2 * l] >= 1 && grid_hw[2 * l + 1] >= 1, "empty grid at level %d", l);
    FRH_REQUIRE(strides[l] > 0.0f, "stride must be positive");
    a.off[l] = n;
    a.gh[l] = grid_hw[2 * l];
    a.gw[l] = grid_hw[2 * l + 1];
    a.stride[l] = strides[l];
    n += (int64_t)a.gh[l] * a.gw[l];
  }
  a.off[num_levels] = n;
  FRH_REQUIRE(n < ((int64_t)1 << 31), "too many cells");
  FRH_REQUIRE(anchor_ld >= n, "anchor_ld %lld < cells %lld", (long long)anchor_ld, (long long)n);
  a.N = n;
  FRH_REQUIRE(anchors && num_gts && img_hw && cls && reg && ctr, "null pointer argument");
  FRH_REQUIRE(max_gts == 0 || (gts && gt_labels), "null gt pointer");
  const AtssLayout w = atss_layout(batch, max_gts, num_levels, topk, n);
  FRH_REQUIRE(workspace && ws_bytes >= w.total, "workspace too small (%zu < %zu)", ws_bytes, w.total);
  char* ws = reinterpret_cast<char*>(workspace);
  a.anchors = anchors;
  a.ald = anchor_ld;
  a.gts = gts;
  a.gseg = gt_seg_stride;
  a.ngt = num_gts;
  a.labels = gt_labels;
  a.img_hw = img_hw;
  a.cls = cls;
  a.reg = reg;
  a.ctr = ctr;
  a.cand = reinterpret_cast<int32_t*>(ws + w.cand);
  a.ciou = reinterpret_cast<float*>(ws + w.ciou);
  a.valid = reinterpret_cast<uint8_t*>(ws + w.valid);
  a.thr = reinterpret_cast<float*>(ws + w.thr);
  a.owner = reinterpret_cast<int32_t*>(ws + w.owner);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(atss_fill_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)batch), dim3(256), 0, st, a);
  if (max_gts > 0) {
    hipLaunchKernelGGL(atss_topk_kernel, dim3((unsigned)max_gts, (unsigned)num_levels, (unsigned)batch),
                       dim3(kAtssThreads), 0, st, a);
    hipLaunchKernelGGL(atss_resolve_kernel, dim3((unsigned)batch), dim3(kAtssThreads), 0, st, a);
  }
  return check_launch("frh_atss_assign");
}
