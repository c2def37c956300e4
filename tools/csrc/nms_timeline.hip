// TOOLS ONLY: the product NMS (pytorch-faster-rcnn_amd/csrc/nms.hip) recompiled with
// per-block resolver timestamps (FRH_NMS_TIMELINE), under renamed symbols so it links
// beside the product objects in libfrcnn_tools.so.  tools/bench_nms.py --timeline.
#define FRH_NMS_TIMELINE 1
#define launch_nms_sorted tl_launch_nms_sorted
#define nms_mask_bytes tl_nms_mask_bytes
#define nms_mask_kernel tl_nms_mask_kernel
#define nms_scan_kernel tl_nms_scan_kernel
#define frh_nms_workspace frh_tl_nms_workspace
#define frh_nms_sorted frh_tl_nms_sorted
#include "../../pytorch-faster-rcnn_amd/csrc/nms.hip"

extern "C" int32_t frh_tl_nms_timeline(void* stamps) {
  uint64_t* p = reinterpret_cast<uint64_t*>(stamps);
  return hipMemcpyToSymbol(HIP_SYMBOL(frh::g_nms_tl), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
