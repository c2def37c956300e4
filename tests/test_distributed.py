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


def _run_bench(args, env_extra, timeout=120):
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    env.update(env_extra)
    r = subprocess.run([sys.executable, os.path.join(repo, 'bench.py')] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith('{')]
    return r.returncode, lines, r.stderr


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus N` without torchrun starts N rank processes itself (RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set, one port for all), SURVEY §8(e)."""
    rc, lines, err = _run_bench(['--gpus', '3'], {'FRCNN_BENCH_SELFTEST': '1'})
    assert rc == 0, err
    assert sorted(d['rank'] for d in lines) == [0, 1, 2]
    assert all(d['world'] == 3 and d['local_rank'] == d['rank'] and d['master'] == '127.0.0.1' for d in lines)
    assert len({d['port'] for d in lines}) == 1


def test_bench_launcher_fails_loudly_and_stops_peers():
    """A rank that fails makes the parent exit non-zero; a peer that would wait forever for
    it is stopped instead of hanging the launch."""
    rc, lines, err = _run_bench(['--gpus', '2'], {'FRCNN_BENCH_SELFTEST': '1', 'FRCNN_BENCH_SELFTEST_FAIL': '1',
                                                  'FRCNN_BENCH_SELFTEST_HANG': '0'}, timeout=60)
    assert rc == 3, (rc, err)
    assert 'rank 1 exited with 3' in err


def test_bench_gpus_must_match_torchrun_world():
    rc, lines, err = _run_bench(['--gpus', '4'], {'WORLD_SIZE': '2', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert rc != 0 and 'disagrees with WORLD_SIZE 2' in err
