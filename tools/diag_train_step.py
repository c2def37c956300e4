"""Where does a cfg2 TrainStep spend its time?  ms per step of the train iteration with the
optimizer forms TrainStep can use (foreach SGD, fused SGD, fused SGD + found_inf), and the
optimizer step alone, on the GPU.   python tools/diag_train_step.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd'), os.path.join(REPO, 'tests', 'golden')]
import torch  # noqa: E402

import bench  # noqa: E402
from frcnn_amd import set_sampler_mode, ops  # noqa: E402
from frcnn_amd.train import TrainStep  # noqa: E402


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / n


def main():
    dev = torch.device('cuda', 0)
    set_sampler_mode('device', seed=3)
    model, cfg = bench.make_model(dev, seed=0)
    batch = bench.make_batch(dev, 2, seed=0)
    clip = cfg.optimizer_config.get('grad_clip')
    for name in ('guard', 'fused', 'foreach'):
        step = TrainStep(model, cfg.optimizer, clip)
        if name != 'guard':
            step._guard = False
            if hasattr(step.optimizer, 'found_inf'):
                del step.optimizer.found_inf
        if name == 'foreach':
            for g in step.optimizer.param_groups:
                g['fused'] = False
                g['foreach'] = True
        print(name, 'train step ms', round(timed(lambda: step(*batch)), 2), flush=True)
        print(name, 'optimizer.step ms', round(timed(step.optimizer.step, 10), 3), flush=True)
    ops.check_device_status(dev)


if __name__ == '__main__':
    main()
