"""The N>1 bench path on CPU: world_size-2 `gloo` process group (the GPU run uses the same
code over RCCL).  Ranks own disjoint image shards, meet only at the barrier and the
max-time all-reduce, and rank 0's value = all ranks' images / slowest rank's time."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import bench
    shard = bench.shard_images(world, rank, 2)
    imgs, boxes, labels, metas = bench.make_batch(torch.device('cpu'), 2, seed=0, rank=rank)
    elapsed = 0.5 + rank  # rank 1 is the slow one
    dist.barrier()
    t = bench.max_over_ranks(elapsed, torch.device('cpu'), world)
    q.put((rank, shard, [b.shape[1] for b in boxes], float(imgs.sum()), t))
    dist.destroy_process_group()


def test_two_rank_gloo_shards_and_max_time():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, n0, x0, t0), (r1, s1, n1, x1, t1) = out
    assert set(s0).isdisjoint(s1) and len(s0) == len(s1) == 2
    assert x0 != x1  # different synthetic images per rank
    assert t0 == t1 == 1.5  # both ranks report the slowest rank's time
