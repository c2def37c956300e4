"""Do two processes compute the same trunk outputs?  (the cross-process
DDP difference was attributed to MIOpen choosing different convolution solutions per process,
without a record of two processes' outputs differing.)

Each child builds the cfg4 Cascade R-CNN model of tests/test_gpu_ddp.py (bench.make_model, seed
0) and its 2-image batch (seed 0), runs the backbone + FPN + RPN head forward (no grad) with
cudnn.benchmark off, then forward_train + backward on the device sampler (seed 1234: the DDP
test's per-rank quantity), and writes the outputs, losses and per-parameter gradient norms to an
npz.  Children run one after the other
(sequential) and two at a time on the one GPU (concurrent: the DDP test's situation), with
torch.use_deterministic_algorithms (cudnn.deterministic + the fixed-point RoIAlign backward)
on and off.  The parent reports, per pair, whether every output is
bit-identical and the largest difference.

    python tools/diag_trunk_processes.py [--out gpurun_out/diag_trunk]"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(path, deterministic):
    sys.path[:0] = [REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
    import numpy as np
    import torch
    import bench
    dev = torch.device('cuda', 0)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = deterministic
    torch.use_deterministic_algorithms(deterministic, warn_only=True)  # + the fixed-point RoIAlign backward
    model, _ = bench.make_model(dev, seed=0, config=os.path.join(bench.CONFIG_DIR, 'cascade_rcnn_r50_fpn.py'))
    imgs = bench.make_batch(dev, 2, seed=0)[0]
    with torch.no_grad():
        feats = model.extract_feat(imgs)
        cls, reg = model.rpn_head(feats)
    torch.cuda.synchronize()
    arrs = {}
    for name, ts in (('feat', feats), ('cls', cls), ('reg', reg)):
        for i, t in enumerate(ts):
            arrs['{}{}'.format(name, i)] = t.float().cpu().numpy()
    # the DDP test's quantity: forward_train's losses and their gradients, device sampler seeded
    from frcnn_amd import set_sampler_mode
    set_sampler_mode('device', seed=1234)
    batch = bench.make_batch(dev, 2, seed=0)
    losses = model.forward_train(*batch)
    total = sum(losses.values())
    total.backward()
    torch.cuda.synchronize()
    for k, v in losses.items():
        arrs['loss_' + k] = v.detach().float().cpu().numpy()
    grads = [p.grad for p in model.parameters() if p.grad is not None]
    arrs['grad_norms'] = torch.stack([g.float().norm() for g in grads]).cpu().numpy()
    np.savez(path, **arrs)


def compare(a, b):
    import numpy as np
    za, zb = np.load(a), np.load(b)
    diff = {k: float(np.abs(za[k] - zb[k]).max()) for k in za.files if not np.array_equal(za[k], zb[k])}
    return not diff, diff


def main():
    if len(sys.argv) > 2 and sys.argv[1] == '--child':
        return child(sys.argv[2], sys.argv[3] == '1')
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', default=os.path.join(REPO, 'gpurun_out', 'diag_trunk'))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    res = {}
    for det in (1, 0):
        paths = [os.path.join(args.out, 'seq{}_{}.npz'.format(det, i)) for i in range(2)]
        for p in paths:  # one after the other
            subprocess.run([sys.executable, __file__, '--child', p, str(det)], check=True, timeout=300)
        cpaths = [os.path.join(args.out, 'con{}_{}.npz'.format(det, i)) for i in range(2)]
        procs = [subprocess.Popen([sys.executable, __file__, '--child', p, str(det)]) for p in cpaths]
        for q in procs:  # two at a time on the one GPU
            assert q.wait(timeout=300) == 0
        res['deterministic={}'.format(det)] = {
            'sequential': dict(zip(('bit_identical', 'differing_outputs_max_abs_diff'), compare(*paths))),
            'concurrent': dict(zip(('bit_identical', 'differing_outputs_max_abs_diff'), compare(*cpaths))),
            'sequential_vs_concurrent': dict(zip(('bit_identical', 'differing_outputs_max_abs_diff'), compare(paths[0], cpaths[0])))}
        print(json.dumps(res), flush=True)
    json.dump(res, open(os.path.join(args.out, 'summary.json'), 'w'), indent=1)


if __name__ == '__main__':
    main()
