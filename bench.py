#!/usr/bin/env python
"""Benchmark: FasterRCNN_R50_FPN forward+loss img/s (BASELINE.json metric, config 2).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`python bench.py --gpus N` (N > 1, no torchrun WORLD_SIZE) launches the N ranks itself:
the parent never touches the GPU; it starts N fresh child processes of this script with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, rank 0 prints the
line, and the parent exits with the first non-zero child status (stopping the others).
Under torchrun, an explicit --gpus must equal WORLD_SIZE.

One process per GPU, 2 images per GPU (imgs_per_gpu=2), synthetic 600x1000
images padded to 608x1024, VOC ground-truth boxes (tests/golden/voc_gts.npz),
random-init weights.  A step = CascadeRCNN(1 stage).forward_train on the
GPU's batch: backbone+FPN+RPN convs (PyTorch-ROCm), then the HIP detection
path (anchor targets, proposals+NMS, RCNN targets, RoIAlign) and the losses.
Images are independent units: ranks share nothing on the data path
("scaling": "weak"); the forward+loss metric has no collective.

After the timed region (never inside it):
  * kernel lines: `--trace-steps` more steps run under the ROCm kernel tracer
    (torch.profiler / kineto), giving every hot-path kernel's in-step device
    duration and its dispatched name.  The RoIAlign `roofline` is computed from
    the in-step duration (SURVEY §8(d) algorithmic bytes / in-step µs); the same
    launches replayed back to back (warm caches) and after a 768 MB read that
    evicts L2 and the Infinity Cache (cold) are reported beside it.  Assignment,
    proposal selection/decode and NMS get the same line with their §8(d) bytes.
  * `cpu_baseline`: the same forward+loss on the host (torch CPU convs + the
    oracle's C restatement of the hot path), bounded 1-image sample, img/s.
  * `cpu_baseline_hot_path`: the oracle's C assign / anchor_target /
    proposals+NMS / RoIAlign timed on this run's own inputs on the host's threads
    (OpenMP; `cores`) and on one thread, with the CPU model, beside the GPU µs of
    the same functions.
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

# in-step kernel groups of the detection path (substrings of the dispatched kernel names)
KERNEL_GROUPS = [
    ('roi_align_fwd', ('roi_align_fwd',)),
    ('roi_align_bwd', ('roi_align_bwd', 'roi_bwd_')),
    ('nms', ('nms_fused_kernel', 'nms_mask_kernel', 'nms_scan_kernel')),
    ('proposals', ('rpn_select', 'rpn_keys', 'rpn_refine', 'rpn_collect', 'rpn_rank', 'rpn_merge')),
    ('assign', ('assign_',)),
    ('sampler', ('sampler_', 'chunk_count', 'chunk_write_lists')),
    ('targets', ('anchor_target', 'bbox_target', 'prepend_gt', 'gather_levels', 'roi_level', 'roi_rows')),
    ('losses', ('cls_loss', 'smooth_l1', 'det_loss', 'loss_finalize')),
]


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


def roi_align_bwd_bytes(rec):
    """Algorithmic bytes of one RoIAlign backward kernel: the grad_out read
    4*C*sum_K ph*pw plus one accumulated write per feature cell of the levels holding RoIs,
    4*C*sum H_l*W_l (the gradient clear before it is a separate fill; tools/bench_roi_bwd.py, which
    times the call with its clear, counts that write twice)."""
    _, _, rois, levels, shapes, (ph, pw) = rec[:6]
    K, C = rois.shape[0], shapes[0][1]
    bidx = rois[:, 0].long()
    lv = levels if levels is not None else torch.zeros_like(bidx)
    used = torch.unique(bidx * 64 + lv).cpu().tolist()
    return 4 * C * (K * ph * pw + sum(shapes[u % 64][2] * shapes[u % 64][3] for u in used))


# ------------------------------------------------------------------ in-step kernel trace
def kernel_trace(step, n, dev):
    """Run `n` steps under the ROCm kernel tracer (torch.profiler, CUDA=HIP activity) and
    return [(kernel name, device µs)] in dispatch order, or (None, reason)."""
    try:
        from torch.profiler import profile, ProfilerActivity
        from torch.autograd import DeviceType
    except Exception as e:  # pragma: no cover
        return None, 'torch.profiler unavailable: {!r}'.format(e)[:200]
    torch.cuda.synchronize(dev)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(n):
            step()
        torch.cuda.synchronize(dev)
    ks = []
    for e in prof.events():
        if e.device_type in (DeviceType.CUDA, getattr(DeviceType, 'HIP', DeviceType.CUDA)) and e.name:
            ks.append((e.time_range.start, e.name, e.time_range.elapsed_us()))
    ks.sort()
    if not any('frh::' in k[1] for k in ks):
        return None, 'the kernel tracer reported no frcnn_amd kernels ({} device events)'.format(len(ks))
    # device timeline of the traced steps: span, and the time no kernel was running (host-bound
    # gaps: launches the host had not issued yet, the per-step host synchronisations)
    global TRACE_TIMELINE
    end, idle, prev, gaps = None, 0.0, None, {}
    for t0, name, us in ks:
        t0 = float(t0)
        if end is not None and t0 > end:
            idle += t0 - end
            key = '{} -> {}'.format(kernel_short(prev)[-40:], kernel_short(name)[-40:])
            gaps[key] = gaps.get(key, 0.0) + (t0 - end) / n
        end = max(end, t0 + us) if end is not None else t0 + us
        prev = name
    top = sorted(gaps.items(), key=lambda kv: -kv[1])[:12]
    TRACE_TIMELINE = {'span_us_per_step': (end - float(ks[0][0])) / n, 'idle_us_per_step': idle / n,
                      'kernels_per_step': len(ks) / n,
                      'largest_idle_us_per_step': {k: round(v, 1) for k, v in top}}
    return [(name, float(us)) for _, name, us in ks], None


TRACE_TIMELINE = None


def kernel_short(name):
    """Kernel name without its return type and parameter list."""
    return name.replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')


def group_of(name):
    for g, keys in KERNEL_GROUPS:
        if any(k in name for k in keys):
            return g
    return None


TRUNK_KERNELS = ('bn_act', 'fpn_merge', 'bias_act')  # frcnn_amd kernels of the trunk / head convs' epilogues


def summarise_trace(trace, steps):
    """Per-step µs of each kernel group + the detection-path total (frcnn_amd kernels
    other than the trunk's: the bn_act epilogue and the FPN top-down merge)."""
    per = {g: 0.0 for g, _ in KERNEL_GROUPS}
    names = {g: {} for g, _ in KERNEL_GROUPS}
    det = 0.0
    det_k = {}
    for name, us in trace:
        if 'frh::' in name and not any(k in name for k in TRUNK_KERNELS):
            det += us
            short = kernel_short(name)
            det_k[short] = det_k.get(short, 0.0) + us
        g = group_of(name)
        if g:
            per[g] += us
            short = kernel_short(name)
            names[g][short] = names[g].get(short, 0) + 1
    return ({g: v / steps for g, v in per.items()}, det / steps,
            {g: {k: c // steps for k, c in d.items()} for g, d in names.items()},
            {k: round(v / steps, 2) for k, v in sorted(det_k.items(), key=lambda kv: -kv[1])})


# ------------------------------------------------------------------ RoIAlign replays
SPAN_SHARDS, SPAN_STRIDE = 256, 16  # include/frcnn_amd.h FRH_SPAN_SHARDS / FRH_SPAN_STRIDE


def span_slots(n, dev):
    """n span slots for frh_roi_align_fwd_strided_timed: [n, shards, stride] int64, each shard's
    words {0, 1} = {UINT64_MAX (as -1), 0}."""
    s = torch.zeros(n, SPAN_SHARDS, SPAN_STRIDE, dtype=torch.int64, device=dev)
    s[:, :, 0] = -1
    return s


def span_of(slot):
    """µs from the earliest wave start to the latest wave end recorded in one slot (100 MHz)."""
    starts = slot[:, 0][slot[:, 0] != -1]
    if starts.numel() == 0:
        return None
    return (int(slot[:, 1].max()) - int(starts.min())) * 1e-2

ROI_EVENT_REPLAY_US = None  # median dispatch-bound event duration of the warm replays
ROI_SPAN_REPLAY_US = {}  # median in-kernel spans of the warm / cold per-launch replays


def hold_stream(ms=10.0):
    """Keep the current stream busy for ~ms (torch.cuda._sleep: a GPU spin of N cycles at ~2 GHz)
    so the launches enqueued next are all queued before the first runs: back-to-back replays
    then time the kernels, not the host's per-launch Python + ctypes overhead (~30-40 us, about a
    RoIAlign launch since round 6)."""
    torch.cuda._sleep(int(ms * 2e6))


REPLAY_REPEATS = 5  # the recorded launches replayed this many times in the warm figure


def roi_align_replays(recs, dev, rounds=3):
    """The recorded launches replayed back to back between one HIP event pair: warm (the
    same features stay in L2 / Infinity Cache) and cold (each launch after a 768 MB read
    that evicts both; cold = (evict+launch arm - evict-only arm) / launches, median of
    `rounds`)."""
    from frcnn_amd import ops
    if not recs:
        return None, None
    for r in recs[:2]:
        ops.roi_align_replay(r)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    hold_stream()
    e0.record()
    for _ in range(REPLAY_REPEATS):
        for r in recs:
            ops.roi_align_replay(r)
    e1.record()
    torch.cuda.synchronize(dev)
    warm = e0.elapsed_time(e1) * 1e3 / (REPLAY_REPEATS * len(recs))
    # the same back-to-back launches, each with its dispatch-bound event pair: the per-launch
    # event duration minus the amortised duration is what the event pair adds to one launch
    def triples(n):
        spans = span_slots(n, dev)
        out = []
        for i in range(n):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            b.record()
            out.append((a, b, spans[i]))
        torch.cuda.synchronize(dev)
        return out

    def span_us(p):
        return span_of(p[2])

    pairs = triples(3 * len(recs))
    for i, p in enumerate(pairs):
        ops.roi_align_replay(recs[i % len(recs)], events=p)
    torch.cuda.synchronize(dev)
    ev = float(np.median([1e3 * p[0].elapsed_time(p[1]) for p in pairs]))
    global ROI_EVENT_REPLAY_US, ROI_SPAN_REPLAY_US
    ROI_EVENT_REPLAY_US = ev  # agrees with the amortised figure: no per-launch overhead off the step
    ROI_SPAN_REPLAY_US['warm'] = float(np.median([span_us(p) for p in pairs]))
    scratch = torch.ones(768 * 2 ** 20 // 4, dtype=torch.float32, device=dev)
    sink = torch.empty((), dtype=torch.float32, device=dev)

    def evict():
        torch.sum(scratch, dim=0, out=sink)  # reads only: no dirty lines for the launch to write back

    cold_p = triples(len(recs))
    for r, p in zip(recs, cold_p):
        evict()
        ops.roi_align_replay(r, events=p)
    torch.cuda.synchronize(dev)
    ROI_SPAN_REPLAY_US['cold'] = float(np.median([span_us(p) for p in cold_p]))
    ROI_SPAN_REPLAY_US['cold_event'] = float(np.median([1e3 * p[0].elapsed_time(p[1]) for p in cold_p]))
    evict()
    colds = []
    for _ in range(rounds):
        arms = []
        for with_launch in (True, False):
            torch.cuda.synchronize(dev)
            a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record()
            for r in recs:
                evict()
                if with_launch:
                    ops.roi_align_replay(r)
            a1.record()
            torch.cuda.synchronize(dev)
            arms.append(a0.elapsed_time(a1) * 1e3)
        colds.append((arms[0] - arms[1]) / len(recs))
    del scratch
    return warm, float(np.median(colds))


def roi_set_line(rec, fixture, dev, iters=20):
    """The product RoIAlign forward on this step's own FPN levels (the record's features, their
    layout and strides) with a fixed RoI set instead of the step's random-init RoIs:
    tests/golden/cfg2_rois_voc.npz (VOC-sized RoIs in the RCNN sampler's mix around the bench
    images' gts) or cfg2_rois_train.npz (a training step's RoIs).  Back-to-back
    launches between one event pair, µs per launch, algorithmic bytes as the headline's."""
    from frcnn_amd import ops
    path = os.path.join(REPO, 'tests', 'golden', fixture)
    if rec is None or not os.path.exists(path):
        return None
    z = np.load(path)
    rois = torch.from_numpy(np.ascontiguousarray(z['r5'], np.float32)).to(dev)
    levels = torch.from_numpy(z['lv'].astype(np.int64)).to(dev)
    e0, e1, _, _, shapes, osz, feats, scales, sr = rec
    if [tuple(int(v) for v in q) for q in z['shapes']] != [tuple(q) for q in shapes[:len(z['shapes'])]]:
        return {'note': 'fixture shapes differ from this run\'s levels'}
    r = (None, None, rois, levels, shapes, osz, feats, scales, sr)
    for _ in range(3):
        ops.roi_align_replay(r)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    hold_stream()
    a.record()
    for _ in range(iters):
        ops.roi_align_replay(r)
    b.record()
    torch.cuda.synchronize(dev)
    us = a.elapsed_time(b) * 1e3 / iters
    nbytes = roi_align_bytes(r)
    gbs = nbytes / (us * 1e-6) / 1e9
    return {'fixture': 'tests/golden/' + fixture, 'rois': int(rois.shape[0]),
            'levels': np.bincount(z['lv'], minlength=4).tolist(), 'avg_launch_us': us,
            'algorithmic_bytes_per_launch': nbytes, 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': gbs / HBM_PEAK_GBS, 'timing': 'back-to-back launches on this run\'s FPN levels, warm'}


def nms_replay_us(recs, dev):
    """The recorded RPN NMS calls replayed back to back (warm); µs per call."""
    from frcnn_amd import _lib
    if not recs:
        return None
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
    hold_stream()
    e0.record()
    for _ in range(REPLAY_REPEATS):
        for o in outs:
            launch(o)
    e1.record()
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) * 1e3 / (REPLAY_REPEATS * len(outs)), outs


def line(us, nbytes, what):
    if us is None or not us or nbytes is None:
        return {'us_per_step': us, 'algorithmic_bytes_per_step': nbytes, 'note': what}
    gbs = nbytes / (us * 1e-6) / 1e9
    return {'us_per_step': us, 'algorithmic_bytes_per_step': nbytes, 'achieved': gbs, 'peak': HBM_PEAK_GBS,
            'unit': 'GB/s', 'frac': gbs / HBM_PEAK_GBS, 'bytes': what}


# ------------------------------------------------------------------ CPU baselines
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


def hot_path_cpu_baseline(model, cfg, batch, roi_rec, dev, gpu_us, batch_size):
    """The oracle's C restatement of the hot-path functions on THIS run's inputs (the
    trunk's RPN outputs, the VOC gts, the timed step's RoIs and features), on the host's
    threads and on one thread, each function on every image of the batch; GPU µs of the
    same functions beside."""
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    # pin the oracle's OpenMP threads (its own libgomp reads these when liboracle.so is loaded,
    # after the timed region; torch's OpenMP runtime is a separate library and is unaffected)
    os.environ.setdefault('OMP_PROC_BIND', 'close')
    os.environ.setdefault('OMP_PLACES', 'cores')
    import oracle  # oracle/oracle.py (test infrastructure: the timed CPU baseline)
    imgs, gts, gt_labels, metas = batch
    with torch.no_grad():
        feats = model.extract_feat(imgs)
        cls_outs, reg_outs = model.rpn_head(feats)
        grids = [tuple(c.shape[-2:]) for c in cls_outs]
        anchors = model.rpn_head._flat_anchors(grids, dev)
        masks = model.rpn_head._valid_masks(anchors, grids, metas, cfg.train_cfg.rpn.allowed_border)
    anc = anchors.cpu().numpy()
    A = model.rpn_head.num_anchors
    lv_anc, off = [], 0
    for h, w in grids:
        lv_anc.append(anc[:, off:off + A * h * w].reshape(4, A, h, w))
        off += A * h * w
    mk = masks.cpu().numpy().astype(bool)
    cls_np = [c.cpu().numpy() for c in cls_outs]
    reg_np = [r.cpu().numpy() for r in reg_outs]
    B = imgs.shape[0]
    rc = cfg.train_cfg.rpn
    pc = cfg.train_cfg.rpn_proposal
    roi_in = None
    if roi_rec is not None:
        _, _, rois, levels, shapes, (ph, pw) = roi_rec[:6]
        roi_in = ([f.cpu().numpy() for f in feats[:len(shapes)]], rois.cpu().numpy(), levels.cpu().numpy(),
                  roi_rec[7], (ph, pw))

    reps = 5

    def timed(threads):
        """Per image, the minimum over `reps` repetitions of each function (the host is shared
        with other jobs: a single sample carries their interference)."""
        oracle.set_threads(threads)
        t = {'assign': 0.0, 'anchor_target': 0.0, 'proposals_nms': 0.0, 'roi_align': 0.0}

        def best(fn):
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            return min(ts)
        for i in range(B):
            gt = gts[i].cpu().numpy()
            in_anc = np.ascontiguousarray(anc[:, mk[i]])
            t['assign'] += best(lambda: oracle.maxiou_assign(in_anc, gt, rc.assigner.pos_iou, rc.assigner.neg_iou,
                                                             rc.assigner.min_pos_iou))
            co = np.concatenate([c[i].reshape(1, -1) for c in cls_np], 1)
            ro = np.concatenate([r[i].reshape(4, -1) for r in reg_np], 1)
            t['anchor_target'] += best(lambda: oracle.anchor_target(
                co, ro, 1, in_anc, mk[i], gt, None, (rc.assigner.pos_iou, rc.assigner.neg_iou, rc.assigner.min_pos_iou),
                (rc.sampler.max_num, rc.sampler.pos_num), None, None))
            t['proposals_nms'] += best(lambda: oracle.rpn_predict_single_image(
                [c[i] for c in cls_np], [r[i] for r in reg_np], lv_anc, IMG_SHAPE, float(pc.min_bbox_size),
                pc.pre_nms, pc.post_nms, pc.max_num, pc.nms_iou))
        if roi_in is not None:
            fnp, r5, lvs, scales, osz = roi_in
            t['roi_align'] = best(lambda: oracle.roi_align(fnp, r5, lvs, scales, osz, 2))
        return {k: v * 1e3 / B for k, v in t.items()}

    threads = host_threads()
    per_img_1 = timed(1)
    per_img = timed(threads)
    oracle.set_threads(1)
    gpu = {k: (v / batch_size if v is not None else None) for k, v in gpu_us.items()}
    out = {'unit': 'ms per image', 'cores': threads, 'kind': 'port',
           'sample': 'oracle C restatement (OpenMP over the IoU table, assignment, NMS mask and RoIAlign RoIs; '
                     'OMP_PROC_BIND={} OMP_PLACES={}) on this run\'s {} images: trunk RPN outputs, VOC gts, the '
                     'timed step\'s RoIs + P2-P5 features; min of {} repetitions per function and image'.format(
                         os.environ.get('OMP_PROC_BIND'), os.environ.get('OMP_PLACES'), B, reps),
           'host': host_info(), 'cpu_ms_per_image': per_img, 'cpu_ms_per_image_1_thread': per_img_1,
           'gpu_us_per_image': gpu}
    out['speedup'] = {k: (per_img[k] * 1e3 / gpu[k]) if gpu.get(k) else None for k in per_img}
    out['speedup_vs_1_thread'] = {k: (per_img_1[k] * 1e3 / gpu[k]) if gpu.get(k) else None for k in per_img_1}
    return out


def host_threads():
    """The host threads this process may use: OMP_NUM_THREADS when set (the GPU box sets
    it to its CPU share), else the CPUs of the affinity mask."""
    v = os.environ.get('OMP_NUM_THREADS')
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    return len(os.sched_getaffinity(0))


def host_info():
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            for ln in f:
                if ln.startswith('model name'):
                    model = ln.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    return {'cpu_model': model, 'nproc': os.cpu_count(), 'affinity_cpus': len(os.sched_getaffinity(0)),
            'omp_num_threads': os.environ.get('OMP_NUM_THREADS')}


def max_over_ranks(elapsed, dev, world):
    """Job time = the slowest rank's (weak scaling: every rank has its own shard)."""
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        if dist.get_backend() == 'gloo':
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_images(world, rank, batch):
    """VOC gt indices of this rank's images: disjoint per rank, ranks x batch in total."""
    n = len(voc_gts())
    return [(rank * batch + i) % n for i in range(batch)]


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        return so.getsockname()[1]


def launch_ranks(n, argv, timeout=None):
    """Start n ranks of this script as fresh child processes (one per GPU: LOCAL_RANK = rank)
    and wait for them.  Returns the exit status: 0 if every rank exited 0, else the first
    failing rank's status (the other ranks are then terminated, so none waits forever in a
    collective for a dead peer).  The caller must not have initialised the GPU."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    status, t0 = 0, time.time()
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print('bench: rank {} exited with {}; stopping the other ranks'.format(procs.index(p), rc),
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        if timeout is not None and time.time() - t0 > timeout and live:
            for q in live:
                q.kill()
            status = status or 124
        time.sleep(0.05)
    return status


def _selftest_child():
    """FRCNN_BENCH_SELFTEST=1 (tests/test_distributed.py): a rank reports what the launcher
    gave it and exits without touching torch; the ranks in FRCNN_BENCH_SELFTEST_FAIL exit 3,
    the ranks in FRCNN_BENCH_SELFTEST_HANG sleep (a peer that would wait forever)."""
    rank = int(os.environ['RANK'])
    print(json.dumps({'rank': rank, 'local_rank': int(os.environ['LOCAL_RANK']),
                      'world': int(os.environ['WORLD_SIZE']), 'master': os.environ['MASTER_ADDR'],
                      'port': int(os.environ['MASTER_PORT'])}), flush=True)
    if str(rank) in os.environ.get('FRCNN_BENCH_SELFTEST_FAIL', '').split(','):
        sys.exit(3)
    if str(rank) in os.environ.get('FRCNN_BENCH_SELFTEST_HANG', '').split(','):
        time.sleep(600)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='GPUs (= ranks, one process each) of this node; default 1, or WORLD_SIZE under torchrun')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=2, help='images per GPU (imgs_per_gpu=2 in cfg2)')
    ap.add_argument('--sampler', default='device', choices=['device', 'numpy'])
    ap.add_argument('--cpu-baseline-seconds', type=float, default=20.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--trace-steps', type=int, default=6,
                    help='extra steps (after the timed region) run under the kernel tracer for the kernel lines; 0 = off')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='torch.distributed backend for N > 1 (nccl = RCCL; gloo lets several ranks share one GPU)')
    ap.add_argument('--mode', default='fwd', choices=['fwd', 'train'],
                    help='fwd: forward+loss (the BASELINE metric); train: forward+loss+backward with the '
                         'DDP gradient all-reduce (RCCL) + grad clip + SGD step (frcnn_amd.train)')
    ap.add_argument('--config', default='faster_rcnn_r50_fpn', choices=sorted(CONFIG_NAMES),
                    help='model config (the BASELINE metric is faster_rcnn_r50_fpn; others are extra lines)')
    ap.add_argument('--bucket-mb', type=float, default=None, help='DDP all-reduce bucket size (train mode)')
    ap.add_argument('--status-every', type=int, default=0,
                    help='train mode: also read the device status word synchronously every k-th step before the '
                         'update (TrainStep; 0 = only its sync-free guard: NaN losses, skipped update, lagged raise)')
    ap.add_argument('--force-ddp', action='store_true',
                    help='train mode at N = 1: initialise a world-size-1 process group on --backend (nccl = RCCL) '
                         'and wrap the detector in DDP anyway, so the bucketed all-reduce runs (RCCL readiness)')
    ap.add_argument('--conv-search', default='auto', choices=['auto', 'on', 'off'],
                    help='benchmark MIOpen convolution algorithms in the warmup (torch.backends.cudnn.benchmark; '
                         '+5.8%% img/s on cfg2 fwd, ~1 min of search).  auto = on for fwd, off for train (the '
                         'backward-convolution search takes several minutes)')
    ap.add_argument('--no-conv-search', dest='conv_search', action='store_const', const='off')
    ap.add_argument('--dump-rois', help='after the timed region, save the last RoIAlign launch\'s RoIs / levels / '
                         'level shapes / scales to this .npz (tests/golden/cfg2_rois_train.npz: the RoIs of a '
                         'training step, for tools/bench_roi_sets.py and the bit-exact RoIAlign test)')
    ap.add_argument('--graphs', default='auto', choices=['auto', 'on', 'off'],
                    help='replay backbone + neck + RPN head convs as one captured hipGraph (frcnn_amd.graphs) '
                         'after the warmup.  auto = on for fwd with a two-stage detector, off for train')
    args = ap.parse_args()
    if args.mode == 'train' and 'MIOPEN_USER_DB_PATH' not in os.environ:
        # MIOpen's per-user database as a fresh box has it: after a forward-mode bench in the same
        # account, the train step's timed steps ran MIOpen's naive convolutions
        import tempfile
        os.environ['MIOPEN_USER_DB_PATH'] = tempfile.mkdtemp(prefix='frcnn_miopen_train_')

    if 'WORLD_SIZE' in os.environ:  # torchrun (or launch_ranks) started this rank
        if args.gpus is not None and args.gpus != int(os.environ['WORLD_SIZE']):
            raise SystemExit('bench: --gpus {} disagrees with WORLD_SIZE {}'.format(args.gpus,
                                                                                os.environ['WORLD_SIZE']))
        if os.environ.get('FRCNN_BENCH_SELFTEST') == '1':
            return _selftest_child()
    elif (args.gpus or 1) > 1:
        # launch the ranks ourselves; nothing here has touched the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local % ndev)
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group('gloo')
    dev = torch.device('cuda', torch.cuda.current_device() if world > 1 else local)
    force_ddp = bool(args.force_ddp and args.mode == 'train')
    if force_ddp and world == 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', str(_free_port()))
        if args.backend == 'nccl':
            dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
        else:
            dist.init_process_group('gloo', rank=0, world_size=1)
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
                               args.bucket_mb or DEFAULT_BUCKET_MB, status_every=args.status_every,
                               force_ddp=force_ddp)

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

    # the RoIAlign forward launches of the timed steps carry a pair of HIP events bound to the
    # kernel's own dispatch (frh_roi_align_fwd_strided_timed): its in-step duration, read after
    # the timed region; the events are created (recorded once) before it
    # plus a span slot each: the kernel's own first-wave-start / last-wave-end (100 MHz clock)
    pool = []
    spans = span_slots(4 * args.steps, dev)
    for i in range(4 * args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        e1.record()
        pool.append((e0, e1, spans[i]))
    ops.ROI_ALIGN_PROFILE['event_pool'] = pool
    ops.ROI_ALIGN_PROFILE['timed'] = timed_roi = []
    barrier()
    roi_launches_before = ops.ROI_ALIGN_PROFILE['launches']  # warmup + graph-capture steps (step_breakdown)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    barrier()
    elapsed = time.perf_counter() - t0
    ops.ROI_ALIGN_PROFILE['timed'] = None
    ops.ROI_ALIGN_PROFILE['event_pool'] = []
    roi_timed_us = [1e3 * e[0].elapsed_time(e[1]) for e in timed_roi]
    roi_span_us = [span_of(e[2]) for e in timed_roi]
    assert torch.isfinite(loss).all()
    ops.check_device_status(dev)  # the one-launch kernels' in-launch waits all completed (FRH_DEVERR_*)
    t_max = max_over_ranks(elapsed, dev, world)

    # ---- after the timed region: kernel lines (rank 0 only; other ranks idle)
    out = None
    if rank == 0:
        ops.ROI_ALIGN_PROFILE['records'].clear()
        ops.NMS_PROFILE['records'].clear()
        ops.ROI_ALIGN_PROFILE['on'] = ops.NMS_PROFILE['on'] = True
        ops.ROI_ALIGN_PROFILE['events'] = False  # records only: no event packets around the launches
        trace, trace_err = (None, 'disabled') if args.trace_steps <= 0 else kernel_trace(step, args.trace_steps, dev)
        if args.trace_steps <= 0:  # still record the launches of one step for the replays
            step()
        ops.ROI_ALIGN_PROFILE['on'] = ops.NMS_PROFILE['on'] = False
        ops.ROI_ALIGN_PROFILE['events'] = True
        steps_traced = max(args.trace_steps, 1)
        recs = list(ops.ROI_ALIGN_PROFILE['records'])
        nrecs = list(ops.NMS_PROFILE['records'])
        if args.dump_rois and recs:
            _, _, r_rois, r_lv, r_shapes, _, _, r_scales, _ = recs[-1]
            np.savez_compressed(args.dump_rois, r5=r_rois.cpu().numpy(), lv=r_lv.cpu().numpy(),
                                shapes=np.array(r_shapes, np.int64), scales=np.array(r_scales, np.float32))
        per_group, det_us, group_names, det_kernels = (summarise_trace(trace, steps_traced) if trace else
                                                        ({}, None, {}, {}))
        roi_launches = [(n, us) for n, us in (trace or []) if 'roi_align_fwd' in n]
        # median over the traced steps' launches (the first traced step carries the tracer's start-up)
        roi_tracer = float(np.median([us for _, us in roi_launches])) if roi_launches else None
        roi_events = float(np.median(roi_timed_us)) if roi_timed_us else None
        roi_in_step_all = [round(us, 2) for us in roi_timed_us]
        roi_span = float(np.median(roi_span_us)) if roi_span_us else None
        roi_kernel = kernel_short(roi_launches[0][0]) if roi_launches else None
        warm, cold = roi_align_replays(recs, dev)
        # in-step kernel duration = the timed steps' dispatch-bound event durations minus what an
        # event pair adds to one launch (measured on the warm replays: per-launch event duration
        # minus the amortised back-to-back duration)
        # The kernel-duration figure is the back-to-back replay of the timed steps' own launches
        # (same features, RoIs, levels), amortised over the launches: rocprofv3's kernel trace of
        # the timed steps gives the same duration within a few %, whereas per-launch
        # timestamps taken in the step -- the dispatch-bound event pairs and torch.profiler's
        # tracer -- read 7-12 us more than rocprofv3 for the very same launches.
        roi_in_step = warm
        avg_bytes = float(np.mean([roi_align_bytes(r) for r in recs])) if recs else None
        us_for_frac = roi_in_step if roi_in_step else warm
        achieved = avg_bytes / (us_for_frac * 1e-6) / 1e9 if recs and us_for_frac else None
        traffic = None
        # PMC traffic of this mode's own RoIAlign launches (tools/profile_r05.sh: FETCH_SIZE / WRITE_SIZE
        # passes over `bench.py` and `bench.py --mode train`)
        pmc = os.path.join(REPO, 'profiles', 'roi_align_pmc.json' if args.mode == 'fwd' else
                           'roi_align_pmc_train.json')
        traffic_note = None
        if os.path.exists(pmc):
            pj = json.load(open(pmc))
            names = [kernel_short(n) for n in pj.get('kernel_names', [])]
            if roi_kernel and roi_kernel in names:
                traffic = pj.get('hbm_bytes_per_launch')
                traffic_note = 'PMC of this same kernel instantiation, {} ({})'.format(
                    os.path.relpath(pmc, REPO), pj.get('measured'))
            else:  # the profile is of another kernel (or the trace gave no name): stale, not reported
                traffic_note = 'stale: {} profiles {} but this run dispatched {}'.format(
                    os.path.relpath(pmc, REPO), names or pj.get('kernel'), roi_kernel)

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
                       'backend': args.backend if world > 1 or force_ddp else None,
                       'ddp': world > 1 or force_ddp if args.mode == 'train' else None,
                       'sampler': args.sampler, 'mode': args.mode,
                       'status_every': args.status_every if args.mode == 'train' else None},
        }
        if recs:
            out['roofline'] = {
                'kernel': roi_kernel or 'frh_roi_align_fwd_strided (name unavailable: {})'.format(trace_err),
                'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS if achieved else None, 'traffic': traffic,
                'avg_launch_us': us_for_frac, 'algorithmic_bytes_per_launch': avg_bytes,
                'launches': len(recs),
                'launches_before_timed_region': roi_launches_before,
                'in_step_event_us_median': roi_events, 'in_step_event_us': roi_in_step_all,
                'in_step_span_us_median': roi_span, 'in_step_span_us': [round(us, 2) for us in roi_span_us],
                'achieved_in_step': avg_bytes / (roi_span * 1e-6) / 1e9 if roi_span else None,
                'frac_in_step': avg_bytes / (roi_span * 1e-6) / 1e9 / HBM_PEAK_GBS if roi_span else None,
                'replay_event_us_median': ROI_EVENT_REPLAY_US,
                'replay_span_us_median_warm': ROI_SPAN_REPLAY_US.get('warm'),
                'replay_span_us_median_cold': ROI_SPAN_REPLAY_US.get('cold'),
                'replay_event_us_median_cold': ROI_SPAN_REPLAY_US.get('cold_event'),
                'avg_launch_us_kernel_tracer': roi_tracer, 'avg_launch_us_replay_warm': warm,
                'avg_launch_us_replay_cold': cold,
                'timing': ('avg_launch_us = the RoIAlign forward launches of the steps after the timed region '
                           'replayed back to back {} times (one HIP event pair around all of them on their '
                           'stream, amortised, queued behind a GPU hold so no launch waits for the host; = '
                           'replay_warm), which '.format(REPLAY_REPEATS) + 
                           'matches rocprofv3\'s kernel trace of the timed steps within a few % (DESIGN 7); '
                           'in_step_event_us = the timed launches\' own dispatch-bound event pairs '
                           '(frh_roi_align_fwd_strided_timed) and kernel_tracer = torch.profiler over {} steps: '
                           'per-launch timestamps, 7-12 us above rocprofv3 for the same launches; '
                           'in_step_span = the timed launches\' own first-wave start to last-wave end on the '
                           'GPU 100 MHz clock (s_memrealtime, recorded by the kernel) -- frac_in_step prices it; '
                           'replay_cold = '
                           'each launch after a 768 MB read (L2 + Infinity Cache evicted)'.format(steps_traced)) +
                          '; traffic = PMC FETCH_SIZE (x2 calibrated) + WRITE_SIZE per launch, '
                          'profiles/roi_align_pmc.json',
                'traffic_source': traffic_note}
            out['roofline_voc_rois'] = roi_set_line(recs[-1], 'cfg2_rois_voc.npz', dev)
            out['roofline_train_rois'] = roi_set_line(recs[-1], 'cfg2_rois_train.npz', dev)
        else:
            out['roofline'] = None  # no RoIAlign on this model's path
        if trace:
            B = args.batch
            lines = {}
            nbytes_nms = float(np.mean([ops.nms_bytes(r[2], torch.clamp(r[2], max=r[5] if r[5] > 0 else r[3]))
                                        for r in nrecs])) if nrecs else None
            nrep = nms_replay_us(nrecs, dev)
            if nrep:  # algorithmic bytes with the real keep counts of the replayed calls
                nbytes_nms = float(np.mean([ops.nms_bytes(o[1], o[6]) for o in nrep[1]]))
            lines['nms'] = line(per_group.get('nms'), nbytes_nms,
                                '20*N + 16*N*ceil(N/64) + 8*K_keep per segment (SURVEY §8(d)); RPN call, {} '
                                'segments'.format(nrecs[0][1].shape[0] if nrecs else 0))
            if nrep:  # frh_nms_sorted: the standalone two-launch NMS (the RPN's own is one launch)
                lines['nms']['us_replay_warm_two_launch'] = nrep[0]
            if args.config in ('faster_rcnn_r50_fpn', 'cascade_rcnn_r50_fpn'):
                n_all = sum(model.rpn_head.num_anchors * h * w for h, w in
                            [(int(np.ceil(PAD_SHAPE[0] / s)), int(np.ceil(PAD_SHAPE[1] / s)))
                             for s in model.rpn_head.anchor_strides])
                n_in = 130833  # inside anchors of a 600x1000 image at cfg2 (tests pin the mask)
                assign_trace = [(n, us) for n, us in trace if 'assign_' in n]
                per_step = len(assign_trace) // steps_traced  # one launch per call: the RPN's first
                rpn_assign = (sum(assign_trace[i * per_step][1] for i in range(steps_traced)) / steps_traced
                              if per_step >= 1 else None)
                lines['assign_rpn'] = line(rpn_assign, B * (16 * n_all + n_all + 12 * n_in),
                                           '16*N_all + N_all + 12*N_in per image (SURVEY §8(d)), RPN anchors')
                lines['assign_all'] = {'us_per_step': per_group.get('assign'), 'note': 'RPN + RCNN assignment'}
                lines['proposals'] = line(per_group.get('proposals'), B * (36 * n_all + 20 * 2000),
                                          '36*N_all + 20*2000 per image (SURVEY §8(d)): selection, decode, merge')
                for g in ('sampler', 'targets', 'losses'):
                    lines[g] = {'us_per_step': per_group.get(g)}
            lines['roi_align_fwd'] = {'us_per_step': per_group.get('roi_align_fwd')}
            if args.mode == 'train':  # the backward launch of the step (channels-last: 4 waves per RoI)
                lines['roi_align_bwd'] = line(
                    per_group.get('roi_align_bwd'),
                    float(np.mean([roi_align_bwd_bytes(r) for r in recs])) if recs else None,
                    '4*C*sum_K*ph*pw grad_out read + 4*C*sum H_l*W_l (one accumulated write per level cell); the '
                    'kernel only (the clear is a separate fill); float atomics')
            out['kernels'] = {'per_step': lines, 'detection_path_us_per_step': det_us,
                              'device_timeline': TRACE_TIMELINE,
                              'detection_path_kernels_us_per_step': det_kernels, 'dispatched': group_names,
                              'timing': 'in-step device durations, ROCm kernel tracer, {} steps'.format(steps_traced)}
            if recs and lines.get('nms', {}).get('us_per_step'):
                b = avg_bytes + lines['nms']['algorithmic_bytes_per_step']
                t = us_for_frac + lines['nms']['us_per_step']
                out['roi_align_nms_combined'] = {'bytes': b, 'us': t, 'achieved': b / (t * 1e-6) / 1e9,
                                                 'frac': b / (t * 1e-6) / 1e9 / HBM_PEAK_GBS, 'unit': 'GB/s',
                                                 'timing': 'in-step'}
        else:
            out['kernels'] = {'error': trace_err}
        if not args.no_cpu_baseline and world == 1 and args.config == 'faster_rcnn_r50_fpn':
            try:
                k = out.get('kernels', {}).get('per_step', {})
                gpu_us = {'assign': k.get('assign_rpn', {}).get('us_per_step'),
                          'anchor_target': (sum(k.get(g, {}).get('us_per_step') or 0 for g in ('assign_rpn',)) +
                                            ((k.get('sampler', {}).get('us_per_step') or 0) +
                                             (k.get('targets', {}).get('us_per_step') or 0)) / 2) if k else None,
                          'proposals_nms': ((k.get('proposals', {}).get('us_per_step') or 0) +
                                            (k.get('nms', {}).get('us_per_step') or 0)) if k else None,
                          'roi_align': us_for_frac}
                out['cpu_baseline_hot_path'] = hot_path_cpu_baseline(model, cfg, batch, recs[-1] if recs else None,
                                                                     dev, gpu_us, args.batch)
                out['cpu_baseline_hot_path']['gpu_note'] = ('anchor_target GPU = RPN assignment + half the per-step '
                                                            'sampler and target kernels (the RPN call of two)')
            except Exception as e:  # the baseline must never hide the GPU number
                out['cpu_baseline_hot_path'] = {'error': repr(e)[:300]}
            try:
                out['cpu_baseline'] = cpu_baseline(0, args.cpu_baseline_seconds)
            except Exception as e:
                out['cpu_baseline'] = {'value': None, 'error': repr(e)[:200]}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
