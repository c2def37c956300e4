"""Timeline of the RPN segmented top-k (seg_topk.h) on a real cfg2 forward pass.

    python tools/bench_topk.py
Runs the bench model's forward_train with frh_rpn_proposals redirected to the tools
build of proposals.hip (tools/csrc/topk_timeline.hip, FRH_TK_TIMELINE): segment 0's
collect workgroups stamp entry / selections done / check-in, and its last workgroup
stamps the candidate sort, the tie selections and the fused sort + decode
(wall_clock64, 100 MHz).  Prints the phases in microseconds."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tools'), REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import toolslib  # noqa: E402
from frcnn_amd import ops, _lib, set_sampler_mode  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    set_sampler_mode('device', seed=1)
    model, batch = bench.make_model_and_batch(dev, batch=2)
    tl = toolslib.load()
    prod_call, prod_query = ops.call, _lib.query

    def call(name, *args):
        if name.startswith('frh_rpn_proposals'):
            return toolslib.call(name.replace('frh_', 'frh_tl_', 1), *args)
        return prod_call(name, *args)

    def query(name, *args):
        if name.startswith('frh_rpn_proposals'):
            return getattr(tl, name.replace('frh_', 'frh_tl_', 1))(*args)
        return prod_query(name, *args)

    ops.call, _lib.query = call, query
    stamps = torch.zeros(2048, dtype=torch.int64, device=dev)
    with torch.no_grad():
        for it in range(4):
            stamps.zero_()
            toolslib.call('frh_tl_topk_timeline', _lib.ptr(stamps))
            model.forward_train(*batch)
            torch.cuda.synchronize()
            toolslib.call('frh_tl_topk_timeline', None)
            s = stamps.cpu().numpy()
            wg = s[:1024].reshape(-1, 4)
            wg = wg[wg[:, 0] > 0]
            t0 = wg[:, 0].min()
            us = lambda v: (v - t0) / 100.0  # noqa: E731
            print('iter {}: {} workgroups of segment 0; entry p50/max {:.1f}/{:.1f}  selections done p50/max '
                  '{:.1f}/{:.1f}  check-in p50/max {:.1f}/{:.1f} us'.format(
                      it, len(wg), np.median(us(wg[:, 0])), us(wg[:, 0]).max(), np.median(us(wg[:, 1])),
                      us(wg[:, 1]).max(), np.median(us(wg[wg[:, 2] > 0, 2])) if (wg[:, 2] > 0).any() else -1,
                      us(wg[wg[:, 2] > 0, 2]).max() if (wg[:, 2] > 0).any() else -1), flush=True)
            names = ['cand loaded', 'cand sorted', 'ties selected', 'records read', 'records sorted',
                     'boxes gathered', '-', 'end']
            last = [(n, us(s[1024 + i])) for i, n in enumerate(names) if s[1024 + i] > 0]
            print('   last workgroup: ' + '  '.join('{} {:.1f}'.format(n, v) for n, v in last), flush=True)


if __name__ == '__main__':
    main()
