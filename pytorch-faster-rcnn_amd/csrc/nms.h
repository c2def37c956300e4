// NMS launch shared by the proposal, multiclass-NMS and tools code (definitions: nms.hip).
#pragma once
#include "common.h"

namespace frh {

// Greedy NMS over S pre-sorted segments (mask + scan).  colcnt: [S][ceil(n_max / 64)]
// int32 column-block counters, ZERO at launch -> one fused launch (S <= 256); nullptr ->
// separate mask and scan launches.  stamps: tools-only per-block timestamps.
int32_t launch_nms_sorted(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                          double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                          uint64_t* mask, const int64_t* seg_base, hipStream_t st, int64_t* stamps = nullptr,
                          int32_t* colcnt = nullptr);
size_t nms_mask_bytes(int32_t S, int32_t n_max);
inline size_t nms_colcnt_bytes(int32_t S, int32_t n_max) {
  return (size_t)S * (size_t)((n_max + 63) / 64) * sizeof(int32_t);
}

}  // namespace frh
