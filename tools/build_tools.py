"""Build the TOOLS-ONLY library tools/lib/libfrcnn_tools.so (never used by the product).

    python tools/build_tools.py
It links the product objects (pytorch-faster-rcnn_amd/build/obj, built first by
build_lib.build()) with tools/csrc/*.hip: the RoIAlign laboratory (the product default
kernel, a stamped build of it and candidates under measurement), entry points declared
in tools/csrc/frcnn_tools.h.  tools/bench_roi_align.py loads it through tools/toolslib.py.
Not part of __graft_entry__.build(): run it by hand before a measurement.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, 'pytorch-faster-rcnn_amd')
sys.path.insert(0, PKG)
import build_lib  # noqa: E402

SRC = os.path.join(HERE, 'csrc')
OBJ = os.path.join(HERE, 'lib', 'obj')
OUT = os.path.join(HERE, 'lib', 'libfrcnn_tools.so')
FLAGS = build_lib.FLAGS + ['-I' + SRC]


def _compile(src, hdr_mtime):
    obj = os.path.join(OBJ, os.path.basename(src) + '.o')
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
        return obj
    r = subprocess.run([build_lib.HIPCC] + FLAGS + ['-c', src, '-o', obj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('hipcc failed for {}:\n{}{}'.format(src, r.stdout, r.stderr))
    return obj


def build():
    build_lib.build()
    os.makedirs(OBJ, exist_ok=True)
    # any product header / source or tools header / include can change a tools object
    deps = glob.glob(os.path.join(SRC, '*.h')) + glob.glob(os.path.join(SRC, '*.inc')) + \
        glob.glob(os.path.join(build_lib.CSRC, '*.hip'))
    hm = max([build_lib._deps_mtime()] + [os.path.getmtime(h) for h in deps])
    srcs = sorted(glob.glob(os.path.join(SRC, '*.hip')))
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(lambda s: _compile(s, hm), srcs))
    prod = sorted(glob.glob(os.path.join(build_lib.OBJ, '*.o')))
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(o) for o in objs + prod):
        return OUT
    r = subprocess.run([build_lib.HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', OUT] + prod + objs,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('link failed:\n{}{}'.format(r.stdout, r.stderr))
    return OUT


if __name__ == '__main__':
    print(build())
