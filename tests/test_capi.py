"""CPU-side checks of the C-ABI library: it loads without a GPU and exports exactly the
entry points include/lbwn.h declares (no compute calls here)."""
import os
import re

from tests.conftest import ROOT


def header_functions():
    txt = open(os.path.join(ROOT, 'include', 'lbwn.h')).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(lbwn_[a-z0-9_]+)\s*\(', txt)))


def test_library_loads_and_exports_header_symbols():
    from lbwn import _lib
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), 'liblbwn.so does not export %s' % n
    assert set(names) == set(_lib.EXPORTED), 'ctypes table and header disagree: %s' % (
        set(names) ^ set(_lib.EXPORTED))
    assert lib.lbwn_abi_version() == _lib.ABI_VERSION


def test_recep_field_via_capi():
    from lbwn import _lib
    import ctypes
    lib = _lib.load()
    a = _lib.Arch()
    a.n_blocks, a.n_block_layers = 5, 10
    assert lib.lbwn_recep_field_sz(ctypes.byref(a)) == 5115


def test_plan_rejects_bad_arch_without_gpu():
    import ctypes
    from lbwn import _lib
    lib = _lib.load()
    a = _lib.Arch()
    a.n_blocks, a.n_block_layers, a.n_quant, a.n_res, a.n_dil, a.n_skip, a.n_post = 5, 10, 256, 64, 32, 512, 512
    h = ctypes.c_void_p()
    assert lib.lbwn_plan_create(ctypes.byref(a), 8, 4096, ctypes.byref(h)) == 22
    assert b'n_res' in lib.lbwn_last_error()
    a.n_res = 32
    assert lib.lbwn_plan_create(ctypes.byref(a), 8, 4096, ctypes.byref(h)) == 0
    assert lib.lbwn_plan_workspace_bytes(h) > 500 * 2 ** 20
    lib.lbwn_plan_destroy(h)
    # par/arch2.json widths (n_res 3, n_dil 4, n_skip 8, n_post 6): accepted, head padded inside
    a.n_res, a.n_dil, a.n_skip, a.n_post = 3, 4, 8, 6
    assert lib.lbwn_plan_create(ctypes.byref(a), 2, 512, ctypes.byref(h)) == 0
    lib.lbwn_plan_destroy(h)
