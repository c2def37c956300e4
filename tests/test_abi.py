"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
symbol include/frcnn_amd.h declares, and the ctypes table matches the header
(argument counts).  No compute calls (no GPU here)."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, 'include', 'frcnn_amd.h')


def header_decls():
    txt = open(HEADER).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    out = {}
    for m in re.finditer(r'\b(?:int32_t|size_t|const char\*)\s+(frh_\w+)\s*\(([^;]*?)\)\s*;', txt, flags=re.S):
        args = m.group(2).strip()
        n = 0 if args in ('', 'void') else args.count(',') + 1
        out[m.group(1)] = n
    return out


def test_header_parses():
    d = header_decls()
    assert len(d) >= 30
    assert 'frh_roi_align_fwd' in d and 'frh_rpn_proposals' in d


def test_library_exports_every_header_symbol():
    from frcnn_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail('libfrcnn_amd.so not built (run __graft_entry__.build())')
    lib = _lib.load()
    for name in header_decls():
        assert hasattr(lib, name), name
    assert lib.frh_abi_version() == _lib.ABI_VERSION


def test_ctypes_table_matches_header():
    from frcnn_amd import _lib
    d = header_decls()
    assert set(d) == set(_lib.SIGNATURES), set(d) ^ set(_lib.SIGNATURES)
    for name, n in d.items():
        assert len(_lib.SIGNATURES[name][1]) == n, name


def test_product_refuses_cpu_tensors():
    import torch
    from frcnn_amd import ops
    a = torch.zeros(4, 3)
    with pytest.raises(RuntimeError):
        ops.iou_table(a, a)


def test_errors_are_reported():
    """A bad argument returns a status and a message, never crashes (no device needed)."""
    from frcnn_amd import _lib
    with pytest.raises(RuntimeError, match='num_levels'):
        _lib.call('frh_anchor_grid', 0, None, None, None, None, 3, 0, None, 0, None)


def test_product_exports_only_the_header():
    """Every exported frh_* symbol of the product library is declared in the product
    header: diagnostics and losing variants live in the tools-only library
    (tools/csrc, tools/lib/libfrcnn_tools.so)."""
    import subprocess
    from frcnn_amd import _lib
    out = subprocess.run(['nm', '-D', '--defined-only', _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.split()[-1].startswith('frh_')}
    assert exported == set(header_decls()) | {'frh_abi_version', 'frh_last_error'}, exported ^ set(header_decls())


def test_tools_header_matches_tools_table():
    import sys
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    import toolslib
    txt = re.sub(r'/\*.*?\*/', '', open(os.path.join(REPO, 'tools', 'csrc', 'frcnn_tools.h')).read(), flags=re.S)
    d = {}
    for m in re.finditer(r'\b(?:int32_t|size_t)\s+(frh_\w+)\s*\(([^;]*?)\)\s*;', txt, flags=re.S):
        d[m.group(1)] = m.group(2).count(',') + 1
    assert set(d) == set(toolslib.TOOL_SIGNATURES)
    for name, n in d.items():
        assert len(toolslib.TOOL_SIGNATURES[name][1]) == n, name
    assert not set(d) & set(header_decls())
