"""Per-dispatch RoIAlign forward durations, four clocks on the SAME dispatches (profiles/r04).

Run (one process, under rocprofv3's kernel trace):
    rocprofv3 --kernel-trace -d OUT/trace -o run --output-format csv -- \\
        python tools/roi_dispatch_table.py --out OUT/launches.json [--tracer]
then join:
    python tools/roi_dispatch_table.py --join OUT --out profiles/r04/roi_dispatch_table.json

The run is bench.py's cfg2 forward_train step (graphed trunk, device sampler, MIOpen search
off so the warmup stays short).  After the warmup, each RoIAlign forward launch of the
measured steps goes through frh_roi_align_fwd_strided_timed: a HIP event pair bound to the
dispatch's own start / end (hipExtLaunchKernel) and the kernel's in-launch span (first wave
start to last wave end, s_memrealtime).  With --tracer the measured steps also run under
torch.profiler (the ROCm kernel tracer bench.py's kernel lines use).  ops counts every
RoIAlign forward launch of the process, so launch n is the n-th RoIAlign dispatch in
rocprofv3's trace: the join lists, per dispatch, rocprofv3's begin / end and duration, the
event pair's duration, the in-kernel span and the tracer's duration, and their medians.
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def run(args):
    sys.path.insert(0, REPO)
    import torch
    import bench
    from frcnn_amd import ops, set_sampler_mode
    from frcnn_amd.graphs import capture_trunk
    dev = torch.device('cuda', 0)
    torch.backends.cudnn.benchmark = False
    set_sampler_mode('device', seed=1234)
    model, _ = bench.make_model(dev, seed=0)
    batch = bench.make_batch(dev, 2, seed=0)

    def step():
        return sum(model.forward_train(*batch).values())

    for _ in range(args.warmup):
        step()
    capture_trunk(model, batch[0])
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    pool = []
    spans = bench.span_slots(4 * args.steps, dev)
    for i in range(4 * args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        e1.record()
        pool.append((e0, e1, spans[i]))
    torch.cuda.synchronize()
    ops.ROI_ALIGN_PROFILE['event_pool'] = pool
    ops.ROI_ALIGN_PROFILE['timed'] = timed = []
    first = ops.ROI_ALIGN_PROFILE['launches']  # 0-based index of the first measured launch
    tracer = []
    if args.tracer:
        from torch.profiler import profile, ProfilerActivity
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
        evs = sorted((e.time_range.start, e.name, e.time_range.elapsed_us()) for e in prof.events()
                     if e.name and 'roi_align_fwd' in e.name)
        tracer = [float(us) for _, _, us in evs]
    else:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    ops.ROI_ALIGN_PROFILE['timed'] = None
    out = {'first_launch_index': first, 'launches': []}
    for i, (e0, e1, sp) in enumerate(timed):
        out['launches'].append({'index': first + i, 'event_us': 1e3 * e0.elapsed_time(e1),
                                'span_us': bench.span_of(sp),
                                'tracer_us': tracer[i] if i < len(tracer) else None})
    out['total_launches'] = ops.ROI_ALIGN_PROFILE['launches']
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(out, open(args.out, 'w'), indent=1)
    print('measured launches', len(timed), 'first index', first, flush=True)


def join(args):
    run_out = json.load(open(os.path.join(args.join, 'launches.json')))
    paths = glob.glob(os.path.join(args.join, 'trace', '**', '*kernel_trace.csv'), recursive=True)
    if not paths:
        raise SystemExit('no kernel_trace.csv under {}'.format(args.join))
    rows = [r for p in paths for r in csv.DictReader(open(p))]
    rows = sorted((r for r in rows if 'roi_align_fwd' in r['Kernel_Name']), key=lambda r: int(r['Start_Timestamp']))
    if len(rows) != run_out['total_launches']:
        raise SystemExit('{} RoIAlign dispatches traced, {} launched'.format(len(rows), run_out['total_launches']))
    table = []
    for L in run_out['launches']:
        r = rows[L['index']]
        b, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        table.append({'dispatch_id': int(r['Dispatch_Id']), 'kernel': r['Kernel_Name'].split('(')[0],
                      'rocprof_begin_ns': b, 'rocprof_end_ns': e, 'rocprof_us': (e - b) / 1e3,
                      'event_us': round(L['event_us'], 3), 'span_us': round(L['span_us'], 3),
                      'tracer_us': L['tracer_us']})

    def med(k):
        v = [t[k] for t in table if t[k] is not None]
        return round(float(np.median(v)), 3) if v else None
    summary = {k: med(k) for k in ('rocprof_us', 'event_us', 'span_us', 'tracer_us')}
    res = {'what': 'RoIAlign forward dispatches of the measured cfg2 steps (B=2), the same dispatches '
                   'under four clocks: rocprofv3 kernel trace, dispatch-bound HIP event pair '
                   '(hipExtLaunchKernel), in-kernel span (first wave start .. last wave end, '
                   's_memrealtime 100 MHz), torch.profiler kernel tracer',
           'median': summary, 'dispatches': table}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(res, open(args.out, 'w'), indent=1)
    print(json.dumps(summary))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--tracer', action='store_true')
    ap.add_argument('--join', help='directory holding launches.json and trace/ (rocprofv3 output)')
    ap.add_argument('--out', required=True)
    args = ap.parse_args()
    join(args) if args.join else run(args)


if __name__ == '__main__':
    main()
