"""Per-step kernel breakdown of a profiled bench run, restricted to the timed steps.

rocprofv3's --stats summary also counts the warmup, where MIOpen's algorithm search
launches naive reference convolutions and every candidate kernel.  This reads the kernel
trace instead: each bench step launches the RoIAlign forward exactly once, so the
timed region is the window between the end of launch W-1 and the end of launch W+K-1
(the launches after it are the bench's replay).  Kernels are grouped by class.

    python tools/step_breakdown.py <rocprof dir with run_kernel_trace.csv> --warmup 3 --steps 10
"""
import argparse
import collections
import csv
import json
import os

CLASSES = [
    ('RoIAlign forward', ('roi_align_fwd',)),
    ('RoIAlign backward', ('roi_align_bwd',)),
    ('NMS', ('nms_',)),
    ('segmented top-k (+ fused sort/decode, label apply)', ('tk_', 'rpn_select', 'sampler_select')),
    ('RPN select/decode/merge', ('rpn_',)),
    ('assignment', ('assign_',)),
    ('sampler compaction', ('chunk_',)),
    ('fused losses', ('cls_loss', 'smooth_l1', 'loss_finalize')),
    ('frozen-BN/residual/ReLU bn_act', ('bn_act',)),
    ('FPN merge (+ lateral bias), RPN conv bias + ReLU', ('fpn_merge', 'bias_act')),
    ('other frcnn_amd kernels', ('frh::',)),
    ('MIOpen convolutions', ('miopenSp3AsmConv', 'igemm_', 'naive_conv', 'kernel_grouped_conv', 'conv_', 'Im2d2Col')),
    ('MIOpen layout transposes', ('batched_transpose', 'transpose_')),
    ('GEMMs (Tensile / hipBLASLt)', ('Cijk_',)),
    ('torch elementwise / reductions', ('at::native',)),
]


def kernel_class(name):
    for cls, keys in CLASSES:
        if any(k in name for k in keys):
            return cls
    return 'other'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace_dir')
    ap.add_argument('--warmup', type=int, required=True)
    ap.add_argument('--steps', type=int, required=True)
    ap.add_argument('--marker', default='roi_align_fwd')
    ap.add_argument('--out', default=None)
    args = ap.parse_args()

    rows = list(csv.DictReader(open(os.path.join(args.trace_dir, 'run_kernel_trace.csv'))))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [r for r in rows if args.marker in r['Kernel_Name']]
    if len(marks) < args.warmup + args.steps:
        raise SystemExit('only {} marker launches'.format(len(marks)))
    t0 = int(marks[args.warmup - 1]['End_Timestamp'])
    t1 = int(marks[args.warmup + args.steps - 1]['End_Timestamp'])
    per_name = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if s >= t0 and e <= t1:
            per_name[r['Kernel_Name']][0] += 1
            per_name[r['Kernel_Name']][1] += e - s
    per_class = collections.defaultdict(float)
    for n, (_, ns) in per_name.items():
        per_class[kernel_class(n)] += ns
    busy = sum(per_class.values())
    k = args.steps
    out = {'window_ms_per_step': (t1 - t0) / 1e6 / k, 'gpu_busy_ms_per_step': busy / 1e6 / k,
           'classes_us_per_step': {c: round(v / 1e3 / k, 1) for c, v in sorted(per_class.items(), key=lambda x: -x[1])},
           'top_kernels_us_per_step': [(n[:90], c // k, round(ns / 1e3 / k, 1)) for n, (c, ns) in
                                       sorted(per_name.items(), key=lambda x: -x[1][1])[:30]],
           'frh_kernels_us_per_step': [(n[:90], c // k, round(ns / 1e3 / k, 1)) for n, (c, ns) in
                                       sorted(per_name.items(), key=lambda x: -x[1][1]) if 'frh::' in n]}
    txt = json.dumps(out, indent=1)
    if args.out:
        open(args.out, 'w').write(txt + '\n')
    print(txt)


if __name__ == '__main__':
    main()
