"""bench.py's own N-rank launch on the GPU box: `bench.py --gpus 2 --backend gloo` starts two
rank processes on the one GPU (gloo lets two ranks share it), each runs the real cfg2
forward+loss step, and rank 0's line reports both ranks (the driver's 1..8
scaling run calls bench.py the same way on an 8-GPU node, over RCCL)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(400)
def test_bench_gpus_2_gloo_reports_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '2', '--backend', 'gloo',
                        '--steps', '3', '--warmup', '2', '--trace-steps', '0', '--no-cpu-baseline',
                        '--conv-search', 'off'], env=env, capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = lines[0]
    assert d['n_gpus'] == 2 and d['config']['global_batch'] == 4 and d['config']['parallelism'] == 'dp2'
    assert d['value'] > 0 and d['steps'] == 3
