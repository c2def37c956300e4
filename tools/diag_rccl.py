"""RCCL on the one-GPU box: a world-size-1 `nccl` process group (RCCL on ROCm)
with `device_id`, then one of each collective the data-parallel path uses or could use, on
device tensors, each checked against its exact single-rank result.  Run it under
`rocprofv3 --kernel-trace` (tools/profile_r06.sh) to list the kernels RCCL itself launches, and
with NCCL_DEBUG=INFO for RCCL's own init log (version, device, channels).

    python tools/diag_rccl.py          (prints one JSON line)
A world of one rank makes RCCL's all-reduce SUM in place a no-op copy (no kernel); AVG is the
pre-multiplied sum, which RCCL runs as a one-rank reduce kernel; out-of-place all-gather /
reduce-scatter are device copies."""
import json
import os
import socket

import torch
import torch.distributed as dist


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1')
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    out = {'backend': dist.get_backend(), 'nccl_version': '.'.join(map(str, torch.cuda.nccl.version()))}
    n = 25 * 2 ** 20 // 4  # one 25-MB DDP bucket of f32
    x = torch.randn(n, device=dev)
    ok = {}
    t = x.clone()
    dist.all_reduce(t)  # SUM
    ok['all_reduce_sum'] = bool(torch.equal(t, x))
    t = x.clone()
    dist.all_reduce(t, op=dist.ReduceOp.AVG)
    ok['all_reduce_avg'] = bool(torch.equal(t, x))
    t = x.clone()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok['all_reduce_max'] = bool(torch.equal(t, x))
    g = torch.empty_like(x)
    dist.all_gather_into_tensor(g, x)
    ok['all_gather'] = bool(torch.equal(g, x))
    r = torch.empty_like(x)
    dist.reduce_scatter_tensor(r, x)
    ok['reduce_scatter'] = bool(torch.equal(r, x))
    t = x.clone()
    dist.broadcast(t, 0)
    ok['broadcast'] = bool(torch.equal(t, x))
    torch.cuda.synchronize()
    # timing of the bucket-sized all-reduce over the one rank (the per-bucket floor of DDP's exchange)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        dist.all_reduce(t, op=dist.ReduceOp.AVG)
    e1.record()
    torch.cuda.synchronize()
    out['avg_allreduce_25MB_us'] = e0.elapsed_time(e1) * 1e3 / 20
    out['ok'] = ok
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    assert all(ok.values()), ok


if __name__ == '__main__':
    main()
