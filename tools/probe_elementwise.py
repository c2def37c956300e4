"""Which torch ops launch the non-frcnn_amd elementwise kernels of the cfg2 bench step.

    python tools/probe_elementwise.py

torch.profiler over a few steps of bench.py's cfg2 forward_train (graphed trunk off, so the
launching ops are visible): per CPU op, the device kernels it launched (name, count, µs per
step), for the at::native elementwise / copy kernels and MIOpen's OpTensor kernels.
"""
import collections
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import bench
    from frcnn_amd import set_sampler_mode
    from torch.profiler import profile, ProfilerActivity
    dev = torch.device('cuda', 0)
    torch.backends.cudnn.benchmark = False
    set_sampler_mode('device', seed=3)
    model, _ = bench.make_model(dev, seed=0)
    batch = bench.make_batch(dev, 2, seed=0)
    for _ in range(3):
        sum(model.forward_train(*batch).values())
    torch.cuda.synchronize()
    steps = 3
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(steps):
            sum(model.forward_train(*batch).values())
        torch.cuda.synchronize()
    # kernel -> launching CPU op through the correlation links of the trace events
    evs = prof.events()
    by_id = {}
    for e in evs:
        by_id[e.id] = e
    agg = collections.defaultdict(lambda: [0, 0.0])
    for e in evs:
        if e.device_type == torch.autograd.DeviceType.CPU:
            for k in e.kernels:
                name = k.name
                if 'frh::' in name:
                    continue
                if not any(s in name for s in ('at::native', 'OpTensor', 'SubTensor', 'transpose', 'Transpose')):
                    continue
                key = (e.name, str(e.input_shapes)[:120], name[:90])
                agg[key][0] += 1
                agg[key][1] += k.duration
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    out = [{'op': k[0], 'shapes': k[1], 'kernel': k[2], 'launches_per_step': v[0] / steps,
            'us_per_step': round(v[1] / steps, 1)} for k, v in rows[:40]]
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
