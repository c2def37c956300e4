"""Attribute the bench step's GPU kernels to the torch ops that launched them
(torch.profiler, one cfg2 forward_train step after warmup; graphed trunk as in bench.py).

    python tools/op_profile.py [--graphs on|off] > gpurun_out/op_profile.txt
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--graphs', default='on', choices=['on', 'off'])
    ap.add_argument('--rows', type=int, default=40)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    import frcnn_amd
    frcnn_amd.set_sampler_mode('device', seed=1234)
    torch.backends.cudnn.benchmark = True
    model, _ = bench.make_model(dev, seed=0)
    batch = bench.make_batch(dev, 2, seed=0)
    for _ in range(3):
        model.forward_train(*batch)
    if args.graphs == 'on':
        from frcnn_amd.graphs import capture_trunk
        capture_trunk(model, batch[0])
        model.forward_train(*batch)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        for _ in range(2):
            sum(model.forward_train(*batch).values())
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by='cuda_time_total', row_limit=args.rows,
                                                             max_name_column_width=60, max_shapes_column_width=70))


if __name__ == '__main__':
    main()
