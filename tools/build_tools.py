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


SPIN_OBJ = os.path.join(HERE, 'lib', 'obj_spin')
SPIN_OUT = os.path.join(HERE, 'lib', 'libfrcnn_spin.so')


def build_spin():
    """tools/lib/libfrcnn_spin.so: the product library rebuilt with FRH_SPIN_TICKS=0, so every
    in-launch wait of the one-launch kernels that is not met at its first poll runs out at
    once -- the failure path of the device status word (tests/test_gpu_status.py)."""
    os.makedirs(SPIN_OBJ, exist_ok=True)
    hm = build_lib._deps_mtime()
    srcs = sorted(glob.glob(os.path.join(build_lib.CSRC, '*.hip'))) + [os.path.join(SRC, 'nms_lab.hip')]

    def one(src):
        obj = os.path.join(SPIN_OBJ, os.path.basename(src) + '.o')
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hm):
            return obj
        r = subprocess.run([build_lib.HIPCC] + FLAGS + ['-DFRH_SPIN_TICKS=0ull', '-c', src, '-o', obj],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('hipcc failed for {}:\n{}{}'.format(src, r.stdout, r.stderr))
        return obj
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(one, srcs))
    if os.path.exists(SPIN_OUT) and os.path.getmtime(SPIN_OUT) >= max(os.path.getmtime(o) for o in objs):
        return SPIN_OUT
    r = subprocess.run([build_lib.HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', SPIN_OUT] + objs,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('link failed:\n{}{}'.format(r.stdout, r.stderr))
    return SPIN_OUT


def build():
    build_lib.build()
    build_spin()
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
