import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
sys.path.insert(0, os.path.join(REPO, 'tools', 'probe'))
from probe_roi import timeit
pl = ctypes.CDLL(os.path.join(REPO, 'tools', 'probe', 'libprobe.so'))
dev = torch.device('cuda', 0)
K, C = 1024, 256
out = torch.empty(K * C * 49, device=dev)
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for contig in (0, 1):
    for nch in (16, 64):
        us = timeit(lambda: pl.probe_store(ctypes.c_void_p(out.data_ptr()), K, C, nch, contig, s))
        print('store contig={} nch/wave={}: {:6.1f} us ({:.2f} TB/s)'.format(contig, nch, us, out.numel() * 4 / us / 1e6), flush=True)
