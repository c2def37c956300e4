// TOOLS ONLY: the exact-test NMS mask (tools/csrc/nms_exact_mask.inc) under renamed
// symbols, linked beside the product objects; tools/bench_nms.py --ab times it against
// the product's float-filtered mask on the same segments.
#define launch_nms_sorted ex_launch_nms_sorted
#define nms_mask_bytes ex_nms_mask_bytes
#define nms_mask_kernel ex_nms_mask_kernel
#define nms_scan_kernel ex_nms_scan_kernel
#define frh_nms_workspace frh_ex_nms_workspace
#define frh_nms_sorted frh_ex_nms_sorted
#include "nms_exact_mask.inc"
