#!/usr/bin/env python
"""Benchmark: FasterRCNN_R50_FPN forward+loss img/s (BASELINE.json metric, config 2).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU, 2 images per GPU (imgs_per_gpu=2), synthetic 600x1000
images padded to 608x1024, VOC ground-truth boxes (tests/golden/voc_gts.npz),
random-init weights.  A step = CascadeRCNN(1 stage).forward_train on the
GPU's batch: backbone+FPN+RPN convs (PyTorch-ROCm), then the HIP detection
path (anchor targets, proposals+NMS, RCNN targets, RoIAlign) and the losses.
Images are independent units: ranks share nothing on the data path
("scaling": "weak"); the forward+loss metric has no collective.

The JSON line carries the RoIAlign forward roofline (the timed region's launches
replayed back to back between one HIP event pair on their stream, algorithmic
bytes per SURVEY §8(d), PMC traffic from profiles/roi_align_pmc.json) and a CPU
baseline: the same forward+loss on the host, with the hot path run by the
oracle's C restatement (oracle/pipeline.py), on a bounded 1-image sample.
"""
import argparse
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'pytorch-faster-rcnn_amd'))
sys.path.insert(0, os.path.join(REPO, 'tests', 'golden'))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIG_DIR = os.path.join(REPO, 'pytorch-faster-rcnn_amd', 'configs')
CONFIG = os.path.join(CONFIG_DIR, 'faster_rcnn_r50_fpn.py')
# --config choices (BASELINE configs 1-5) -> model name used in the metric string
CONFIG_NAMES = {'faster_rcnn_r50_fpn': 'FasterRCNN_R50_FPN', 'faster_rcnn_r50': 'FasterRCNN_R50_C4',
                'retinanet_r50_fpn': 'RetinaNet_R50_FPN', 'cascade_rcnn_r50_fpn': 'CascadeRCNN_R50_FPN',
                'fcos_r50_fpn_atss': 'ATSS_R50_FPN'}
IMG_SHAPE, PAD_SHAPE = (600, 1000), (608, 1024)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def img_meta():
    return {'img_shape': IMG_SHAPE + (3,), 'pad_shape': PAD_SHAPE + (3,), 'scale_factor': 1.6,
            'ori_shape': (375, 625, 3)}


def voc_gts():
    z = np.load(os.path.join(REPO, 'tests', 'golden', 'voc_gts.npz'))
    return [(z['boxes_{}'.format(i)], z['labels_{}'.format(i)]) for i in range(int(z['n']))]


def make_batch(dev, batch, seed, rank=0):
    g = torch.Generator(device='cpu').manual_seed(seed + 1000 * rank)
    imgs = torch.randn(batch, 3, PAD_SHAPE[0], PAD_SHAPE[1], generator=g).to(dev)
    gts = voc_gts()
    sel = [gts[i] for i in shard_images(None, rank, batch)]
    boxes = [torch.from_numpy(b).to(dev) for b, _ in sel]
    labels = [torch.from_numpy(l).to(dev) for _, l in sel]
    return imgs, boxes, labels, [img_meta() for _ in range(batch)]


def make_model(dev, seed=0, config=CONFIG):
    from frcnn_amd.config import Config
    from frcnn_amd.builder import build_module
    cfg = Config.fromfile(config)
    torch.manual_seed(seed)
    model = build_module(cfg.model, train_cfg=cfg.train_cfg, test_cfg=cfg.test_cfg)
    model.init_weights()
    model.train()
    return model.to(dev), cfg


def make_model_and_batch(dev, batch=2, seed=0, rank=0):
    model, _ = make_model(dev, seed)
    return model, make_batch(dev, batch, seed, rank)


def roi_align_bytes(rec):
    """Algorithmic bytes of one RoIAlign forward launch:
    4*C*(sum_K ph*pw + sum_img sum_{levels with >=1 roi} H_l*W_l) + 20*K."""
    _, _, rois, levels, shapes, (ph, pw) = rec[:6]
    K = rois.shape[0]
    C = shapes[0][1]
    bidx = rois[:, 0].long()
    lv = levels if levels is not None else torch.zeros_like(bidx)
    used = torch.unique(bidx * 64 + lv).cpu().tolist()
    feat_elems = sum(shapes[u % 64][2] * shapes[u % 64][3] for u in used)
    return 4 * C * (K * ph * pw + feat_elems) + 20 * K


def nms_roofline(recs, dev):
    """The timed steps' RPN NMS calls (all images x levels per call: mask + scan kernels)
    replayed back to back between one HIP event pair on their stream, with preallocated
    outputs; algorithmic bytes per ops.nms_bytes.  NMS at RPN sizes is
    latency-bound (greedy scan), so the fraction is reported next to the microseconds."""
    if not recs:
        return None
    from frcnn_amd import ops, _lib
    outs = []
    for ws, rows, cnt, P, thr, max_keep in recs:
        S = rows.shape[0]
        keep = torch.empty(S, P, dtype=torch.int32, device=dev)
        kc = torch.empty(S, dtype=torch.int32, device=dev)
        nws = _lib.workspace(_lib.query('frh_nms_workspace', S, P), dev)
        outs.append((rows, cnt, P, thr, max_keep, keep, kc, nws))

    def launch(o):
        rows, cnt, P, thr, max_keep, keep, kc, nws = o
        _lib.call('frh_nms_sorted', rows.shape[0], _lib.ptr(rows), rows.stride(0), _lib.ptr(cnt), P, thr, max_keep,
                  _lib.ptr(keep), keep.stride(0), _lib.ptr(kc), _lib.ptr(nws), nws.numel(), _lib.stream_of(rows))
    for o in outs[:2]:
        launch(o)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for o in outs:
        launch(o)
    e1.record()
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / len(outs)
    nbytes = float(np.mean([ops.nms_bytes(o[1], o[6]) for o in outs]))
    achieved = nbytes / (us * 1e-6) / 1e9
    segs = outs[0][0].shape[0]
    return {'kernel': 'nms_mask_kernel + nms_scan_kernel (RPN, {} segments of <= {} boxes)'.format(
                segs, outs[0][2]),
            'bound': 'latency (greedy scan); hbm for the mask', 'achieved': achieved, 'peak': HBM_PEAK_GBS,
            'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'avg_call_us': us,
            'algorithmic_bytes_per_call': nbytes, 'calls': len(outs),
            'timing': 'the timed steps\' RPN NMS calls replayed back to back between one HIP event pair'}


def cpu_baseline(seed, max_s):
    """Same forward+loss on the host: torch CPU convs + the oracle's C hot path, 1 image."""
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    import pipeline  # oracle/pipeline.py (test infrastructure)
    threads = torch.get_num_threads()
    model, cfg = make_model(torch.device('cpu'), seed)
    imgs, boxes, labels, metas = make_batch(torch.device('cpu'), 1, seed)
    t0 = time.time()
    n = 0
    while True:
        pipeline.forward_train_cpu(model, cfg, imgs, boxes, labels, metas)
        n += 1
        if time.time() - t0 > max_s or n >= 3:
            break
    dt = time.time() - t0
    return {'value': n / dt, 'unit': 'img/s', 'cores': threads, 'kind': 'port',
            'sample': '{} x 1-image forward+loss of the cfg2 model on CPU (torch CPU convs + oracle C hot path, '
                      '{} threads)'.format(n, threads)}


def max_over_ranks(elapsed, dev, world):
    """Job time = the slowest rank's (weak scaling: every rank has its own shard)."""
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_images(world, rank, batch):
    """VOC gt indices of this rank's images: disjoint per rank, ranks x batch in total."""
    n = len(voc_gts())
    return [(rank * batch + i) % n for i in range(batch)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=2, help='images per GPU (imgs_per_gpu=2 in cfg2)')
    ap.add_argument('--sampler', default='device', choices=['device', 'numpy'])
    ap.add_argument('--cpu-baseline-seconds', type=float, default=20.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--mode', default='fwd', choices=['fwd', 'train'],
                    help='fwd: forward+loss (the BASELINE metric); train: forward+loss+backward with the '
                         'DDP gradient all-reduce (RCCL) + grad clip + SGD step (frcnn_amd.train)')
    ap.add_argument('--config', default='faster_rcnn_r50_fpn', choices=sorted(CONFIG_NAMES),
                    help='model config (the BASELINE metric is faster_rcnn_r50_fpn; others are extra lines)')
    ap.add_argument('--bucket-mb', type=float, default=None, help='DDP all-reduce bucket size (train mode)')
    ap.add_argument('--conv-search', default='auto', choices=['auto', 'on', 'off'],
                    help='benchmark MIOpen convolution algorithms in the warmup (torch.backends.cudnn.benchmark; '
                         '+5.8%% img/s on cfg2 fwd, ~1 min of search).  auto = on for fwd, off for train (the '
                         'backward-convolution search takes several minutes)')
    ap.add_argument('--no-conv-search', dest='conv_search', action='store_const', const='off')
    ap.add_argument('--graphs', default='auto', choices=['auto', 'on', 'off'],
                    help='replay backbone + neck + RPN head convs as one captured hipGraph (frcnn_amd.graphs) '
                         'after the warmup.  auto = on for fwd with a two-stage detector, off for train')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    import frcnn_amd
    from frcnn_amd import ops
    frcnn_amd.set_sampler_mode(args.sampler, seed=1234 + rank)
    np.random.seed(rank)

    if args.conv_search == 'auto':
        args.conv_search = 'on' if args.mode == 'fwd' else 'off'
    args.conv_search = args.conv_search == 'on'
    torch.backends.cudnn.benchmark = args.conv_search
    model, cfg = make_model(dev, seed=0, config=os.path.join(CONFIG_DIR, args.config + '.py'))
    batch = make_batch(dev, args.batch, seed=0, rank=rank)

    if args.mode == 'train':
        from frcnn_amd.train import TrainStep, DEFAULT_BUCKET_MB
        opt_cfg = cfg.get('optimizer_config', None) or {}
        train_step = TrainStep(model, cfg.get('optimizer', None), opt_cfg.get('grad_clip', None), world, dev,
                               args.bucket_mb or DEFAULT_BUCKET_MB)

        def step():
            return train_step(*batch)
    else:
        def step():
            losses = model.forward_train(*batch)
            return sum(losses.values())

    # Warmup (MIOpen's algorithm search runs here): a heartbeat on stderr keeps long
    # searches visibly alive (train mode searches the backward convolutions too).
    hb_stop = threading.Event()

    def heartbeat(t_start=time.perf_counter()):
        while not hb_stop.wait(30.0):
            if rank == 0:
                print('bench: warmup running, {:.0f} s'.format(time.perf_counter() - t_start), file=sys.stderr,
                      flush=True)

    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    for w in range(args.warmup):
        step()
        if rank == 0:
            print('bench: warmup step {}/{} done'.format(w + 1, args.warmup), file=sys.stderr, flush=True)
    hb_stop.set()

    graphed = False
    if args.graphs == 'auto':
        args.graphs = 'on' if args.mode == 'fwd' and hasattr(model, 'graphed_trunk') else 'off'
    if args.graphs == 'on':
        from frcnn_amd.graphs import capture_trunk
        if not hasattr(model, 'graphed_trunk'):
            raise SystemExit('--graphs on: {} has no graphed trunk'.format(type(model).__name__))
        capture_trunk(model, batch[0])
        graphed = True
        for _ in range(2):
            step()
        if rank == 0:
            print('bench: trunk captured as a hipGraph', file=sys.stderr, flush=True)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    ops.ROI_ALIGN_PROFILE['records'].clear()
    ops.ROI_ALIGN_PROFILE['on'] = True
    ops.NMS_PROFILE['records'].clear()
    ops.NMS_PROFILE['on'] = True
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    barrier()
    elapsed = time.perf_counter() - t0
    ops.ROI_ALIGN_PROFILE['on'] = False
    ops.NMS_PROFILE['on'] = False
    assert torch.isfinite(loss).all()

    t_max = max_over_ranks(elapsed, dev, world)

    recs = ops.ROI_ALIGN_PROFILE['records']
    ms = [r[0].elapsed_time(r[1]) for r in recs]  # per-launch event pairs inside the steps
    bytes_per = [roi_align_bytes(r) for r in recs]
    # Kernel duration: the timed region's launches replayed back to back on their stream
    # between one HIP event pair (per-launch pairs add the event packets' own latency).
    avg_ms = float('nan')
    if recs:
        for r in recs[:2]:
            ops.roi_align_replay(r)  # warm
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record()
        for r in recs:
            ops.roi_align_replay(r)
        r1.record()
        torch.cuda.synchronize(dev)
        avg_ms = r0.elapsed_time(r1) / len(recs)
    avg_bytes = float(np.mean(bytes_per)) if bytes_per else float('nan')
    achieved = avg_bytes / (avg_ms * 1e-3) / 1e9 if ms else None

    nms_line = nms_roofline(ops.NMS_PROFILE['records'], dev)
    ops.NMS_PROFILE['records'].clear()

    traffic = None
    pmc = os.path.join(REPO, 'profiles', 'roi_align_pmc.json')
    if os.path.exists(pmc):
        traffic = json.load(open(pmc)).get('hbm_bytes_per_launch')

    if rank == 0:
        imgs_total = world * args.batch * args.steps
        out = {
            'metric': 'img/s ' + CONFIG_NAMES[args.config] + ' 1000x600 ' + ('fwd+loss' if args.mode == 'fwd' else
                                                               'train step (fwd+loss+bwd+allreduce+SGD)'),
            'value': imgs_total / t_max,
            'unit': 'img/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': 1e3 * t_max / args.steps,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': 'synthetic images N(0,1) [B,3,608,1024], VOC07 trainval gt boxes, random-init weights',
            'config': {'workload': 'configs/{}.py{} forward_train'.format(
                           args.config, ' (BASELINE config 2)' if args.config == 'faster_rcnn_r50_fpn' else ''),
                       'conv_algorithms': 'MIOpen benchmarked (warmup)' if args.conv_search else 'MIOpen heuristic',
                       'trunk': 'hipGraph replay (backbone + neck + RPN head convs)' if graphed else 'eager',
                       'global_batch': world * args.batch, 'imgs_per_gpu': args.batch,
                       'image': '600x1000 padded 608x1024', 'parallelism': 'dp{}'.format(world),
                       'sampler': args.sampler, 'mode': args.mode},
            'roofline': {'kernel': 'roi_align_fwd_pair_kernel<8, 1664, 1, 2, 0, false, true, 1, true, 1, true> (single slab buffer, nt stores, lean tap state)', 'bound': 'hbm',
                         'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': (achieved / HBM_PEAK_GBS) if achieved else None, 'traffic': traffic,
                         'avg_launch_us': avg_ms * 1e3, 'algorithmic_bytes_per_launch': avg_bytes,
                         'launches': len(ms), 'avg_launch_us_in_step_events': float(np.mean(ms)) * 1e3,
                         'timing': 'the timed steps\' RoIAlign launches replayed back to back between one HIP event '
                                   'pair on their stream; traffic = PMC FETCH_SIZE (x2 calibrated) + WRITE_SIZE per '
                                   'launch, profiles/roi_align_pmc.json'},
        }
        if not recs:
            out['roofline'] = None  # no RoIAlign on this model's path
        if nms_line:
            out['nms'] = nms_line
            if recs:  # the two kernels the north star names, as one HBM fraction per step
                b = avg_bytes + nms_line['algorithmic_bytes_per_call']
                t = avg_ms * 1e-3 + nms_line['avg_call_us'] * 1e-6
                out['roi_align_nms_combined'] = {'bytes': b, 'us': t * 1e6, 'achieved': b / t / 1e9,
                                                 'frac': b / t / 1e9 / HBM_PEAK_GBS, 'unit': 'GB/s'}
        if not args.no_cpu_baseline and world == 1 and args.config == 'faster_rcnn_r50_fpn':
            try:
                out['cpu_baseline'] = cpu_baseline(0, args.cpu_baseline_seconds)
            except Exception as e:  # the baseline must never hide the GPU number
                out['cpu_baseline'] = {'value': None, 'error': repr(e)[:200]}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
