// a10: greedy NMS with torchvision.ops.nms semantics on pre-sorted segments
// (call sites lib/heads/rpn_head.py:103, lib/utils.py:220).
//
// Two launches:
//  mask: one wave per (segment, 64-row block, 64-col block >= row block);
//        lane i sets bit j when IoU(row i, col j) > thr (j after i), the
//        64 column boxes staged in LDS.  Rows are 64-bit words per col block.
//  scan: one workgroup per segment walks the row blocks in score order.
//        Wave 0 resolves the block's 64 candidates sequentially with
//        readlane'd diagonal words (pure register/SALU work), then all
//        waves OR the kept rows' words into the LDS suppression bitmap with
//        8 independent loads per lane in flight.
#include "block_ops.h"

namespace frh {

constexpr int kMaxNmsWords = 256;  // n <= 16384 boxes per segment

__global__ void __launch_bounds__(64) nms_mask_kernel(const float* __restrict__ boxes, int64_t seg_stride,
                                                      const int32_t* __restrict__ counts, int64_t n_max, int nbw,
                                                      double thr, uint64_t* __restrict__ mask) {
  __shared__ float4 cb_box[64];
  __shared__ float cb_area[64];
  const int s = blockIdx.z, rb = blockIdx.y, cb = blockIdx.x;
  if (cb < rb) return;
  const int n = counts[s];
  if (rb * 64 >= n || cb * 64 >= n) return;
  const float4* bx = reinterpret_cast<const float4*>(boxes + (int64_t)s * seg_stride);
  const int t = threadIdx.x;
  const int col = cb * 64 + t;
  if (col < n) {
    float4 c = bx[col];
    cb_box[t] = c;
    cb_area[t] = (c.z - c.x) * (c.w - c.y);
  }
  __syncthreads();
  const int row = rb * 64 + t;
  if (row >= n) return;
  const float4 a = bx[row];
  const float aa = (a.z - a.x) * (a.w - a.y);
  const int ncols = min(64, n - cb * 64);
  const int start = (cb == rb) ? t + 1 : 0;
  uint64_t bits = 0;
  for (int j = start; j < ncols; ++j) {
    float v = iou_tv(a, aa, cb_box[j], cb_area[j]);
    if ((double)v > thr) bits |= 1ull << j;
  }
  mask[((int64_t)s * n_max + row) * nbw + cb] = bits;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

__global__ void __launch_bounds__(256) nms_scan_kernel(const uint64_t* __restrict__ mask,
                                                       const int32_t* __restrict__ counts, int64_t n_max, int nbw,
                                                       int max_keep, int32_t* __restrict__ keep, int64_t kstride,
                                                       int32_t* __restrict__ kcounts) {
  __shared__ uint64_t remv[kMaxNmsWords];
  __shared__ uint64_t s_kb;
  __shared__ int s_nkeep;
  const int s = blockIdx.x, tid = threadIdx.x;
  const int n = counts[s];
  const int nb = (n + 63) >> 6;
  for (int w = tid; w < nb; w += blockDim.x) remv[w] = 0;
  if (tid == 0) s_nkeep = 0;
  __syncthreads();
  const uint64_t* M = mask + (int64_t)s * n_max * nbw;
  int32_t* K = keep + (int64_t)s * kstride;
  const int q = tid & 31, rg = tid >> 5;  // word offset / row group of 8 for the OR phase
  for (int b = 0; b < nb; ++b) {
    const int nk = s_nkeep;
    if (max_keep >= 0 && nk >= max_keep) break;
    if (tid < 64) {
      const int row = b * 64 + tid;
      const uint64_t diag = row < n ? M[(int64_t)row * nbw + b] : 0ull;
      uint64_t r = remv[b];
      const int valid = n - b * 64;
      if (valid < 64) r |= (~0ull) << valid;
      uint64_t kb = 0;
      for (int i = 0; i < 64; ++i) {
        uint64_t di = readlane64(diag, i);
        if (!((r >> i) & 1ull)) {
          kb |= 1ull << i;
          r |= di;
        }
      }
      if (max_keep >= 0) {
        int room = max_keep - nk;
        while (__popcll(kb) > room) kb &= ~(1ull << (63 - __clzll(kb)));  // drop lowest-score extras
      }
      if ((kb >> tid) & 1ull) K[nk + __popcll(kb & lanemask_lt())] = row;
      if (tid == 0) {
        s_kb = kb;
        s_nkeep = nk + __popcll(kb);
      }
    }
    __syncthreads();
    const uint64_t kb = s_kb;
    if (kb) {
      for (int w0 = b + 1; w0 < nb; w0 += 32) {
        const int w = w0 + q;
        if (w < nb) {
          uint64_t v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            int row = b * 64 + rg * 8 + j;
            row = row < n ? row : n - 1;
            v[j] = M[(int64_t)row * nbw + w];
          }
          uint64_t acc = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc |= ((kb >> (rg * 8 + j)) & 1ull) ? v[j] : 0ull;
          if (acc) atomicOr((unsigned long long*)&remv[w], (unsigned long long)acc);
        }
      }
    }
    __syncthreads();
  }
  if (tid == 0) kcounts[s] = s_nkeep;
}

int32_t launch_nms_sorted(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                          double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                          uint64_t* mask, hipStream_t st) {
  const int nbw = (n_max + 63) / 64;
  dim3 g(nbw, nbw, S);
  hipLaunchKernelGGL(nms_mask_kernel, g, dim3(64), 0, st, boxes, seg_stride, counts, (int64_t)n_max, nbw, thr, mask);
  hipLaunchKernelGGL(nms_scan_kernel, dim3(S), dim3(256), 0, st, mask, counts, (int64_t)n_max, nbw, max_keep, keep,
                     kstride, kcounts);
  return check_launch("nms");
}

size_t nms_mask_bytes(int32_t S, int32_t n_max) {
  const size_t nbw = (size_t)((n_max + 63) / 64);
  return (size_t)S * (size_t)n_max * nbw * sizeof(uint64_t);
}

}  // namespace frh

using namespace frh;

extern "C" size_t frh_nms_workspace(int32_t num_segs, int32_t n_max) {
  return nms_mask_bytes(num_segs, n_max > 0 ? n_max : 1);
}

extern "C" int32_t frh_nms_sorted(int32_t num_segs, const float* boxes, int64_t seg_stride, const int32_t* counts,
                                  int32_t n_max, double iou_thr, int32_t max_keep, int32_t* keep,
                                  int64_t keep_seg_stride, int32_t* keep_counts, void* workspace, size_t ws_bytes,
                                  void* stream) {
  FRH_REQUIRE(num_segs >= 0 && n_max >= 0, "negative sizes");
  if (num_segs == 0) return FRH_OK;
  FRH_REQUIRE(n_max <= 64 * kMaxNmsWords, "n_max %d exceeds %d", n_max, 64 * kMaxNmsWords);
  FRH_REQUIRE(boxes && counts && keep && keep_counts, "null pointer argument");
  FRH_REQUIRE(workspace && ws_bytes >= frh_nms_workspace(num_segs, n_max), "workspace too small");
  if (n_max == 0) {
    FRH_HIP(hipMemsetAsync(keep_counts, 0, sizeof(int32_t) * num_segs, as_stream(stream)));
    return FRH_OK;
  }
  return launch_nms_sorted(num_segs, boxes, seg_stride, counts, n_max, iou_thr, max_keep, keep, keep_seg_stride,
                           keep_counts, reinterpret_cast<uint64_t*>(workspace), as_stream(stream));
}
