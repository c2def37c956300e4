// a3/a4: IoU tables and MaxIoU assignment, batched over segments (images).
// Reference: lib/utils.py:151-182 (calc_iou/elem_iou), lib/region.py:60-107 (MaxIoUAssigner).
//
// Assignment is ONE launch, one thread per box, gts in LDS:
//   every workgroup computes its boxes' row maxima (first argmax, NaN wins like
//   torch.max) and threshold labels, and its own per-gt maxima (wave max + LDS
//   atomicMax on order-preserving u32 keys), which it folds into the segment's
//   per-gt maxima with a device atomicMax (skipped when the value there is
//   already as large).  A box can take the "tied at a gt's maximum" rule
//   (region.py:95-106) only if it ties its own workgroup's maximum of that gt
//   (the segment maximum is >= the workgroup's): such candidate boxes, found by
//   re-evaluating only the gts whose workgroup maximum reaches min_pos_iou, are
//   appended to a per-segment list instead of being labelled; every other box
//   is final.  The workgroup then arrives at the segment's counter; the last to
//   arrive labels the candidates against the final maxima and resets the
//   counters.  Hand-off (MI355X_MICROARCH.md hand-off table, row 1): list
//   entries stored write-through (agent-scope relaxed stores) and drained before
//   the arrival, maxima by device atomics, all read with agent-scope loads.
// The IoU expression is identical everywhere, so the equality tests see exactly
// the values the maxima were reduced from.
#include "common.h"

namespace frh {

constexpr int kMaxGts = 1024;  // gts staged in LDS per block
constexpr int kAssignThreads = 256;

__global__ void iou_table_kernel(const float* __restrict__ a, int64_t lda, int64_t n,
                                 const float* __restrict__ b, int64_t ldb, int64_t k,
                                 float* __restrict__ out) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * k) return;
  int64_t i = idx / k, j = idx - i * k;
  out[idx] = iou_plus1(a[i], a[lda + i], a[2 * lda + i], a[3 * lda + i], b[j], b[ldb + j],
                       b[2 * ldb + j], b[3 * ldb + j]);
}

__global__ void elem_iou_kernel(const float* __restrict__ a, int64_t lda, const float* __restrict__ b,
                                int64_t ldb, int64_t n, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float ax1 = a[i], ay1 = a[lda + i], ax2 = a[2 * lda + i], ay2 = a[3 * lda + i];
  float bx1 = b[i], by1 = b[ldb + i], bx2 = b[2 * ldb + i], by2 = b[3 * ldb + i];
  float tlx = fmaxf(ax1, bx1), tly = fmaxf(ay1, by1), brx = fminf(ax2, bx2), bry = fminf(ay2, by2);
  float area_i = (brx - tlx) * (bry - tly);
  area_i = area_i * ((tlx < brx && tly < bry) ? 1.0f : 0.0f);
  float area_a = (ax2 - ax1) * (ay2 - ay1);
  float area_b = (bx2 - bx1) * (by2 - by1);
  out[i] = area_i / ((area_a + area_b) - area_i);
}

struct AssignArgs {
  const float* boxes;
  int64_t box_ld, box_seg_stride;
  const int32_t* num_boxes;
  const uint8_t* valid;
  int64_t valid_seg_stride;
  const float* gts;
  int64_t gt_ld, gt_seg_stride;
  const int32_t* num_gts;
  float pos_iou, neg_iou, min_pos_iou;
  int64_t* labels;
  int64_t label_seg_stride;
  float* max_iou;
  int64_t iou_seg_stride;
  uint32_t* colmax;  // [S, max_gts] order-preserving keys; zero between calls
  int32_t* state;    // [S, 4]: arrivals, candidates; zero between calls
  int32_t* cand;     // [S, cand_ld] candidate box indices
  int64_t cand_ld;
  int32_t max_gts;
};

__device__ __forceinline__ void load_gts(const AssignArgs& p, int s, int G, float4* sg) {
  const float* g = p.gts + (int64_t)s * p.gt_seg_stride;
  for (int j = threadIdx.x; j < G; j += blockDim.x)
    sg[j] = make_float4(g[j], g[p.gt_ld + j], g[2 * p.gt_ld + j], g[3 * p.gt_ld + j]);
}

__device__ __forceinline__ float4 load_box(const AssignArgs& p, int s, int64_t i) {
  const float* b = p.boxes + (int64_t)s * p.box_seg_stride;
  return make_float4(b[i], b[p.box_ld + i], b[2 * p.box_ld + i], b[3 * p.box_ld + i]);
}

__device__ __forceinline__ float iou_box(const float4& a, const float4& g) {
  return iou_plus1(a.x, a.y, a.z, a.w, g.x, g.y, g.z, g.w);
}

// row max / first argmax with NaN winning like torch.max (region.py:88)
__device__ __forceinline__ void row_step(int j, float v, float& m, int& arg) {
  if (j == 0) {
    m = v;
  } else if (!(v <= m) && !isnan(m)) {
    m = v;
    arg = j;
  }
}

// thresholds (region.py:90-92) on the row maximum
__device__ __forceinline__ int64_t threshold_label(const AssignArgs& p, float m, int arg) {
  int64_t lab = -1;
  if (m < p.neg_iou) lab = 0;
  if (m >= p.pos_iou) lab = (int64_t)arg + 1;
  return lab;
}

// The last workgroup of segment s: every candidate box gets its full label -- the
// first gt whose final maximum it ties (>= min_pos_iou) overrides the thresholds
// (region.py:95-106).  scm: the final maxima as floats (NaN where no valid box
// reached the gt: never equal).
__device__ void label_candidates(const AssignArgs& p, int s, int G, const float4* sg, float* scm) {
  for (int j = threadIdx.x; j < G; j += blockDim.x) {
    const uint32_t k = __hip_atomic_load(p.colmax + (int64_t)s * p.max_gts + j, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    scm[j] = k ? key_float(k) : __uint_as_float(0x7fc00000u);
  }
  int32_t* st = p.state + 4 * s;
  const int ncand = __hip_atomic_load(st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  int64_t* lab_out = p.labels + (int64_t)s * p.label_seg_stride;
  float* iou_out = p.max_iou ? p.max_iou + (int64_t)s * p.iou_seg_stride : nullptr;
  for (int t = threadIdx.x; t < ncand; t += blockDim.x) {
    const int64_t i = __hip_atomic_load(p.cand + (int64_t)s * p.cand_ld + t, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    const float4 a = load_box(p, s, i);
    float m = 0.f, m_eq = 0.f;
    int arg = 0, eq = -1;
    for (int j = 0; j < G; ++j) {
      const float v = iou_box(a, sg[j]);
      row_step(j, v, m, arg);
      if (eq < 0 && v == scm[j] && scm[j] >= p.min_pos_iou) {
        eq = j;
        m_eq = v;
      }
    }
    int64_t lab = threshold_label(p, m, arg);
    float out_iou = m;
    if (eq >= 0) {
      lab = (int64_t)eq + 1;
      out_iou = m_eq;
    }
    lab_out[i] = lab;
    if (iou_out) iou_out[i] = out_iou;
  }
  __syncthreads();  // every read of the maxima and the list is done: reset for the next call
  for (int j = threadIdx.x; j < G; j += blockDim.x)
    __hip_atomic_store(p.colmax + (int64_t)s * p.max_gts + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0) {
    __hip_atomic_store(st + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(st + 0, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// R boxes per thread (box base + r * 256 + tid: coalesced): 4 for anchor sets, so a
// workgroup pays its gt staging and its arrival once per 1024 boxes; 1 for a few
// thousand proposals, which need the workgroups more
template <int R>
__global__ void __launch_bounds__(kAssignThreads) maxiou_assign_kernel(AssignArgs p) {
  __shared__ float4 sg[kMaxGts];
  __shared__ uint32_t scol[kMaxGts];  // this workgroup's per-gt maxima (keys); later the final maxima
  __shared__ int snear[kMaxGts];      // gts whose workgroup maximum reaches min_pos_iou
  __shared__ int nnear, last;
  const int s = blockIdx.y;
  const int n = p.num_boxes[s];
  const int G = p.num_gts[s];
  const int64_t base = (int64_t)blockIdx.x * (kAssignThreads * R) + threadIdx.x;
  const bool any = (int64_t)blockIdx.x * (kAssignThreads * R) < n && G > 0;  // uniform per block
  if (any) {
    load_gts(p, s, G, sg);
    for (int j = threadIdx.x; j < G; j += blockDim.x) scol[j] = 0u;
  }
  if (threadIdx.x == 0) nnear = 0;
  bool live[R];
  float4 a[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = base + r * kAssignThreads;
    live[r] = i < n;
    if (live[r] && p.valid) live[r] = p.valid[(int64_t)s * p.valid_seg_stride + i] != 0;
    a[r] = live[r] ? load_box(p, s, i) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  float m[R];
  int arg[R];
#pragma unroll
  for (int r = 0; r < R; ++r) m[r] = 0.f, arg[r] = 0;
  if (any) {
    for (int j = 0; j < G; ++j) {
      const float4 g = sg[j];
      uint32_t key = 0u;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float v = iou_box(a[r], g);
        if (live[r]) {
          row_step(j, v, m[r], arg[r]);
          key = max(key, float_key(v));
        }
      }
      key = wave_max_u32(key);
      if (lane_id() == 0 && key) atomicMax(&scol[j], key);
    }
  }
  __syncthreads();
  if (any) {
    uint32_t* cm = p.colmax + (int64_t)s * p.max_gts;
    for (int j = threadIdx.x; j < G; j += blockDim.x) {
      const uint32_t k = scol[j];
      if (!k) continue;
      atomicMax(cm + j, k);
      if (key_float(k) >= p.min_pos_iou) snear[atomicAdd(&nnear, 1)] = j;
    }
  }
  __syncthreads();
  // candidates: ties of this workgroup's maximum of a gt that reaches min_pos_iou
  bool cand[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    cand[r] = false;
    if (live[r])
      for (int t = 0; t < nnear && !cand[r]; ++t) {
        const int j = snear[t];
        cand[r] = iou_box(a[r], sg[j]) == key_float(scol[j]);
      }
    const int slot = wave_append(cand[r], p.state + 4 * s + 1);
    if (cand[r])
      __hip_atomic_store(p.cand + (int64_t)s * p.cand_ld + slot, (int32_t)(base + r * kAssignThreads),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // arrival: every wave drains its list entries and maxima, then one lane adds for the
  // workgroup; the labels of the other boxes (which no other workgroup touches) go after it
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(p.state + 4 * s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (int)gridDim.x - 1;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = base + r * kAssignThreads;
    if (cand[r] || i >= p.cand_ld) continue;  // cand_ld = max_boxes: rows past the count are padding
    const bool lab = live[r] && G > 0;  // padding rows (i >= n) and masked boxes: label -1, IoU 0
    p.labels[(int64_t)s * p.label_seg_stride + i] = lab ? threshold_label(p, m[r], arg[r]) : -1;
    if (p.max_iou) p.max_iou[(int64_t)s * p.iou_seg_stride + i] = lab ? m[r] : 0.0f;
  }
  __syncthreads();
  if (!last) return;
  if (!any && G > 0) load_gts(p, s, G, sg);  // the last workgroup may be one past the boxes
  __syncthreads();
  if (G > 0) label_candidates(p, s, G, sg, reinterpret_cast<float*>(scol));
  else if (threadIdx.x == 0) __hip_atomic_store(p.state + 4 * s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace frh

using namespace frh;

extern "C" int32_t frh_iou_table(const float* a, int64_t lda, int64_t n, const float* b, int64_t ldb,
                                 int64_t k, float* out, void* stream) {
  FRH_REQUIRE(n >= 0 && k >= 0, "negative sizes");
  if (n == 0 || k == 0) return FRH_OK;
  FRH_REQUIRE(a && b && out, "null pointer argument");
  int64_t total = n * k;
  hipLaunchKernelGGL(iou_table_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     as_stream(stream), a, lda, n, b, ldb, k, out);
  return check_launch("frh_iou_table");
}

extern "C" int32_t frh_elem_iou(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t n,
                                float* out, void* stream) {
  FRH_REQUIRE(n >= 0, "negative size");
  if (n == 0) return FRH_OK;
  FRH_REQUIRE(a && b && out, "null pointer argument");
  hipLaunchKernelGGL(elem_iou_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), a, lda, b, ldb, n, out);
  return check_launch("frh_elem_iou");
}

static size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

// [zeroed: state S x 4 int32 | colmax S x max_gts u32] [candidates S x max_boxes int32]
static size_t assign_zero_bytes(int32_t num_segs, int32_t max_gts) {
  return al256((size_t)num_segs * 16) + al256((size_t)num_segs * (size_t)(max_gts > 0 ? max_gts : 1) * 4);
}

extern "C" size_t frh_maxiou_assign_zero_bytes(int32_t num_segs, int32_t max_gts) {
  return assign_zero_bytes(num_segs, max_gts);
}

extern "C" size_t frh_maxiou_assign_workspace(int32_t num_segs, int32_t max_gts, int64_t max_boxes) {
  return assign_zero_bytes(num_segs, max_gts) + al256((size_t)num_segs * (size_t)(max_boxes > 0 ? max_boxes : 1) * 4);
}

extern "C" int32_t frh_maxiou_assign(int32_t num_segs, const float* boxes, int64_t box_ld,
                                     int64_t box_seg_stride, const int32_t* num_boxes,
                                     const uint8_t* valid, int64_t valid_seg_stride,
                                     const float* gts, int64_t gt_ld, int64_t gt_seg_stride,
                                     const int32_t* num_gts, float pos_iou, float neg_iou,
                                     float min_pos_iou, int64_t* labels, int64_t label_seg_stride,
                                     float* max_iou, int64_t iou_seg_stride, int64_t max_boxes,
                                     int32_t max_gts, void* workspace, size_t ws_bytes, void* stream) {
  FRH_REQUIRE(num_segs >= 0 && max_boxes >= 0, "negative sizes");
  if (num_segs == 0 || max_boxes == 0) return FRH_OK;
  FRH_REQUIRE(boxes && num_boxes && gts && num_gts && labels, "null pointer argument");
  FRH_REQUIRE(max_gts <= kMaxGts, "max_gts %d exceeds %d", max_gts, kMaxGts);
  FRH_REQUIRE(max_boxes <= (int64_t)0x7fffffff, "too many boxes");
  int32_t mg = max_gts > 0 ? max_gts : 1;
  FRH_REQUIRE(workspace && ws_bytes >= frh_maxiou_assign_workspace(num_segs, mg, max_boxes), "workspace too small");
  char* ws = static_cast<char*>(workspace);
  const size_t zs = al256((size_t)num_segs * 16);
  AssignArgs p{boxes, box_ld, box_seg_stride, num_boxes, valid, valid_seg_stride, gts, gt_ld,
               gt_seg_stride, num_gts, pos_iou, neg_iou, min_pos_iou, labels, label_seg_stride,
               max_iou, iou_seg_stride, reinterpret_cast<uint32_t*>(ws + zs), reinterpret_cast<int32_t*>(ws),
               reinterpret_cast<int32_t*>(ws + assign_zero_bytes(num_segs, mg)), max_boxes, mg};
  if (max_boxes >= 32768) {
    const dim3 grid((unsigned)((max_boxes + 4 * kAssignThreads - 1) / (4 * kAssignThreads)), (unsigned)num_segs);
    hipLaunchKernelGGL(maxiou_assign_kernel<4>, grid, dim3(kAssignThreads), 0, as_stream(stream), p);
  } else {
    const dim3 grid((unsigned)((max_boxes + kAssignThreads - 1) / kAssignThreads), (unsigned)num_segs);
    hipLaunchKernelGGL(maxiou_assign_kernel<1>, grid, dim3(kAssignThreads), 0, as_stream(stream), p);
  }
  return check_launch("frh_maxiou_assign");
}
