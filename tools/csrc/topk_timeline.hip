// TOOLS ONLY: the product RPN proposals (pytorch-faster-rcnn_amd/csrc/proposals.hip,
// segmented top-k of seg_topk.h) recompiled with segment-0 timestamps (FRH_TK_TIMELINE),
// under renamed entry points so it links beside the product objects in
// libfrcnn_tools.so.  tools/bench_topk.py.
#define FRH_TK_TIMELINE 1
#define frh_rpn_proposals_workspace frh_tl_rpn_proposals_workspace
#define frh_rpn_proposals_nms_view frh_tl_rpn_proposals_nms_view
#define frh_rpn_proposals frh_tl_rpn_proposals
#include "../../pytorch-faster-rcnn_amd/csrc/proposals.hip"

extern "C" int32_t frh_tl_topk_timeline(void* stamps) {
  uint64_t* p = reinterpret_cast<uint64_t*>(stamps);
  return hipMemcpyToSymbol(HIP_SYMBOL(frh::g_tk_tl), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
