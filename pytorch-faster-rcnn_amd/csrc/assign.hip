// a3/a4: IoU tables and MaxIoU assignment, batched over segments (images).
// Reference: lib/utils.py:151-182 (calc_iou/elem_iou), lib/region.py:60-107 (MaxIoUAssigner).
//
// Assignment runs in two passes over the boxes of every segment:
//   pass 1: per-gt max IoU over all valid boxes (wave max-reduce + one
//           atomicMax per wave on an order-preserving u32 key),
//   pass 2: recompute the box's G IoUs (cheaper than storing the N x G
//           table), apply the neg/pos thresholds on the row max and the
//           "every box tied at a gt's max" rule with the first tied gt.
// The IoU expression is identical in both passes, so the equality test of
// pass 2 sees exactly the values pass 1 reduced.
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
  uint32_t* colmax;  // [S, max_gts] order-preserving keys
  int32_t max_gts;
};

__device__ __forceinline__ void load_gts(const AssignArgs& p, int s, int G, float4* sg) {
  const float* g = p.gts + (int64_t)s * p.gt_seg_stride;
  for (int j = threadIdx.x; j < G; j += blockDim.x)
    sg[j] = make_float4(g[j], g[p.gt_ld + j], g[2 * p.gt_ld + j], g[3 * p.gt_ld + j]);
}

__global__ void __launch_bounds__(kAssignThreads) assign_colmax_kernel(AssignArgs p) {
  __shared__ float4 sg[kMaxGts];
  __shared__ uint32_t scol[kMaxGts];
  const int s = blockIdx.y;
  const int n = p.num_boxes[s];
  const int G = p.num_gts[s];
  if ((int64_t)blockIdx.x * blockDim.x >= n || G <= 0) return;  // uniform per block
  load_gts(p, s, G, sg);
  for (int j = threadIdx.x; j < G; j += blockDim.x) scol[j] = 0u;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool live = i < n;
  if (live && p.valid) live = p.valid[(int64_t)s * p.valid_seg_stride + i] != 0;
  float x1 = 0.f, y1 = 0.f, x2 = 0.f, y2 = 0.f;
  if (live) {
    const float* b = p.boxes + (int64_t)s * p.box_seg_stride;
    x1 = b[i];
    y1 = b[p.box_ld + i];
    x2 = b[2 * p.box_ld + i];
    y2 = b[3 * p.box_ld + i];
  }
  for (int j = 0; j < G; ++j) {
    float4 g = sg[j];
    uint32_t key = live ? float_key(iou_plus1(x1, y1, x2, y2, g.x, g.y, g.z, g.w)) : 0u;
    key = wave_max_u32(key);
    if (lane_id() == 0 && key) atomicMax(&scol[j], key);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < G; j += blockDim.x)
    if (scol[j]) atomicMax(&p.colmax[(int64_t)s * p.max_gts + j], scol[j]);
}

__global__ void __launch_bounds__(kAssignThreads) assign_label_kernel(AssignArgs p) {
  __shared__ float4 sg[kMaxGts];
  __shared__ float scm[kMaxGts];
  const int s = blockIdx.y;
  const int n = p.num_boxes[s];
  const int G = p.num_gts[s];
  if ((int64_t)blockIdx.x * blockDim.x >= n) return;
  load_gts(p, s, G, sg);
  for (int j = threadIdx.x; j < G; j += blockDim.x) {
    uint32_t k = p.colmax[(int64_t)s * p.max_gts + j];
    // a gt that no valid box reached keeps key 0: never equal to any IoU
    scm[j] = k ? key_float(k) : __uint_as_float(0x7fc00000u);
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t* lab_out = p.labels + (int64_t)s * p.label_seg_stride;
  float* iou_out = p.max_iou ? p.max_iou + (int64_t)s * p.iou_seg_stride : nullptr;
  bool live = !p.valid || p.valid[(int64_t)s * p.valid_seg_stride + i] != 0;
  if (!live || G <= 0) {
    lab_out[i] = -1;
    if (iou_out) iou_out[i] = 0.0f;
    return;
  }
  const float* b = p.boxes + (int64_t)s * p.box_seg_stride;
  float x1 = b[i], y1 = b[p.box_ld + i], x2 = b[2 * p.box_ld + i], y2 = b[3 * p.box_ld + i];
  // row max / first argmax, NaN wins like torch.max (region.py:88)
  float m = 0.f, m_eq = 0.f;
  int arg = 0, eq = -1;
  for (int j = 0; j < G; ++j) {
    float4 g = sg[j];
    float v = iou_plus1(x1, y1, x2, y2, g.x, g.y, g.z, g.w);
    if (j == 0) {
      m = v;
    } else if (!(v <= m) && !isnan(m)) {
      m = v;
      arg = j;
    }
    if (eq < 0 && v == scm[j] && scm[j] >= p.min_pos_iou) {  // region.py:95-101
      eq = j;
      m_eq = v;
    }
  }
  int64_t lab = -1;
  if (m < p.neg_iou) lab = 0;                    // region.py:90
  if (m >= p.pos_iou) lab = (int64_t)arg + 1;    // region.py:92,106
  float out_iou = m;
  if (eq >= 0) {                                 // region.py:101-106
    lab = (int64_t)eq + 1;
    out_iou = m_eq;
  }
  lab_out[i] = lab;
  if (iou_out) iou_out[i] = out_iou;
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

extern "C" size_t frh_maxiou_assign_workspace(int32_t num_segs, int32_t max_gts) {
  return (size_t)num_segs * (size_t)(max_gts > 0 ? max_gts : 1) * sizeof(uint32_t);
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
  FRH_REQUIRE(workspace && ws_bytes >= frh_maxiou_assign_workspace(num_segs, mg), "workspace too small");
  AssignArgs p{boxes, box_ld, box_seg_stride, num_boxes, valid, valid_seg_stride, gts, gt_ld,
               gt_seg_stride, num_gts, pos_iou, neg_iou, min_pos_iou, labels, label_seg_stride,
               max_iou, iou_seg_stride, reinterpret_cast<uint32_t*>(workspace), mg};
  FRH_HIP(hipMemsetAsync(workspace, 0, frh_maxiou_assign_workspace(num_segs, mg), as_stream(stream)));
  dim3 grid((unsigned)((max_boxes + kAssignThreads - 1) / kAssignThreads), (unsigned)num_segs);
  if (max_gts > 0)
    hipLaunchKernelGGL(assign_colmax_kernel, grid, dim3(kAssignThreads), 0, as_stream(stream), p);
  hipLaunchKernelGGL(assign_label_kernel, grid, dim3(kAssignThreads), 0, as_stream(stream), p);
  return check_launch("frh_maxiou_assign");
}
