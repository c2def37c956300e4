"""Build libfrcnn_amd.so (gfx950) from csrc/*.hip with hipcc, in-tree.

Each translation unit is compiled separately (parallel, incremental on
mtime) and linked into frcnn_amd/libfrcnn_amd.so so the shared library travels
with the source tree to the GPU box.  Numerics flags: -ffp-contract=off (no
FMA contraction; the reference's IoU/assignment is reproduced bit-exactly)
and HIP's default correctly-rounded f32 divide/sqrt.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OBJ = os.path.join(HERE, 'build', 'obj')
OUT = os.path.join(HERE, 'frcnn_amd', 'libfrcnn_amd.so')
INCLUDE = os.path.join(os.path.dirname(HERE), 'include')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off',
         '-fhip-fp32-correctly-rounded-divide-sqrt', '-Wall', '-Wno-unused-function',
         '-I' + CSRC, '-I' + INCLUDE]


def _deps_mtime():
    hdrs = glob.glob(os.path.join(CSRC, '*.h')) + glob.glob(os.path.join(INCLUDE, '*.h'))
    return max([os.path.getmtime(h) for h in hdrs] + [0])


def _compile(src, hdr_mtime, verbose):
    obj = os.path.join(OBJ, os.path.basename(src) + '.o')
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
        return obj
    cmd = [HIPCC] + FLAGS + ['-c', src, '-o', obj]
    if verbose:
        print(' '.join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('hipcc failed for {}:\n{}{}'.format(src, r.stdout, r.stderr))
    return obj


def build(verbose=False, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    hm = _deps_mtime()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hm, verbose), srcs))
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(o) for o in objs):
        return OUT
    cmd = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', OUT] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('link failed:\n{}{}'.format(r.stdout, r.stderr))
    return OUT


if __name__ == '__main__':
    print(build(verbose='-v' in sys.argv))
