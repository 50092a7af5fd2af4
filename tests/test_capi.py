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


def test_torch_ops_registered_device_only():
    """lbwn::dilconv_gate / lbwn::dilconv_gate_bwd are torch.library ops with autograd; they have
    no CPU kernel (the oracle is never a fallback), so CPU tensors fail loudly."""
    import pytest
    import torch
    from lbwn import torch_ops  # noqa: F401  (registers the ops)
    assert hasattr(torch.ops.lbwn, 'dilconv_gate') and hasattr(torch.ops.lbwn, 'dilconv_gate_bwd')
    x = torch.zeros(1, 10, 32)
    w = torch.zeros(2, 32, 32)
    b = torch.zeros(32)
    with pytest.raises((NotImplementedError, RuntimeError)):
        torch.ops.lbwn.dilconv_gate(x, w, w, b, b, torch.zeros(32, 32), b, 2, 4)
    # shapes through the fake (meta) kernels
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        xf = torch.empty(2, 4 + 100, 32, device='cuda')
        wf = torch.empty(2, 32, 16, device='cuda')
        z, xo = torch.ops.lbwn.dilconv_gate(xf, wf, wf, torch.empty(16, device='cuda'), torch.empty(16, device='cuda'),
                                            torch.empty(16, 32, device='cuda'), torch.empty(32, device='cuda'), 4, 4)
        assert tuple(z.shape) == (2, 100, 16) and tuple(xo.shape) == (2, 100, 32)


def test_plan_chain_tile_env(monkeypatch):
    """LBWN_CHAIN_TILE = <fwd>[:<bwd>] (each 128 / 64 / w32) selects the chains' form at plan
    creation; anything else is refused there (EINVAL), before any device work."""
    import ctypes
    from lbwn import _lib
    lib = _lib.load()
    a = _lib.Arch()
    a.n_blocks, a.n_block_layers, a.n_quant, a.n_res, a.n_dil, a.n_skip, a.n_post = 5, 10, 256, 32, 32, 512, 512
    h = ctypes.c_void_p()
    for v in ('128', '64', 'w32', '128:w32', 'w32:64', ''):
        monkeypatch.setenv('LBWN_CHAIN_TILE', v)
        assert lib.lbwn_plan_create(ctypes.byref(a), 8, 4096, ctypes.byref(h)) == 0, v
        lib.lbwn_plan_destroy(h)
    for v in ('96', '128:', ':64', '128:64:w32', 'w16'):
        monkeypatch.setenv('LBWN_CHAIN_TILE', v)
        assert lib.lbwn_plan_create(ctypes.byref(a), 8, 4096, ctypes.byref(h)) == 22, v
        assert b'LBWN_CHAIN_TILE' in lib.lbwn_last_error()


def test_plan_bwd_wgrad_env(monkeypatch):
    """LBWN_BWD_WGRAD=1 (read at plan creation) takes the residual stack's weight gradients out
    of the backward chain: the plan then carves the chain's DV and G exports (the workspace grows
    by 3 x 128 B per position and layer, rounded to 32-row blocks); 0 keeps them in the chain."""
    import ctypes
    from lbwn import _lib
    lib = _lib.load()
    lib.lbwn_plan_workspace_bytes.restype = ctypes.c_size_t
    a = _lib.Arch()
    a.n_blocks, a.n_block_layers, a.n_quant, a.n_res, a.n_dil, a.n_skip, a.n_post = 5, 10, 256, 32, 32, 512, 512
    sizes = {}
    for v in ('0', '1'):
        monkeypatch.setenv('LBWN_BWD_WGRAD', v)
        h = ctypes.c_void_p()
        assert lib.lbwn_plan_create(ctypes.byref(a), 8, 4096, ctypes.byref(h)) == 0, v
        sizes[v] = lib.lbwn_plan_workspace_bytes(h)
        lib.lbwn_plan_destroy(h)
    grow = sizes['1'] - sizes['0']
    assert 3 * 128 * 50 * 8 * 4096 <= grow <= 3 * 128 * 50 * 8 * 4096 + 3 * 4096 * 50, grow


def test_gemm_mode_env_selects_f32_mfma():
    """LBWN_GEMM=f32 (read once, at the first GEMM or mode query) selects the f32-MFMA GEMMs
    (mode 0); unset or anything else keeps the bf16-split form (mode 1).  Fresh processes: the
    mode is process state."""
    import subprocess
    import sys
    code = ('import sys; sys.path.insert(0, %r); from lbwn import _lib; print(_lib.load().lbwn_gemm_get_mode())'
            % os.path.join(ROOT, 'lb-wavenet_amd'))
    for val, want in (('f32', '0'), ('', '1'), ('bf16', '1')):
        env = dict(os.environ, LBWN_GEMM=val)
        out = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-2000:]
        assert out.stdout.strip().splitlines()[-1] == want, (val, out.stdout)


def test_product_loads_only_the_in_tree_library(monkeypatch):
    """The product path has no library override: lbwn._lib loads lb-wavenet_amd/lbwn/liblbwn.so
    (variant builds are for tools/with_lib.py A/B runs only)."""
    from lbwn import _lib
    assert _lib.LIB_PATH == os.path.join(ROOT, 'lb-wavenet_amd', 'lbwn', 'liblbwn.so')
    src = open(os.path.join(ROOT, 'lb-wavenet_amd', 'lbwn', '_lib.py')).read()
    assert 'environ' not in src


def test_env_switches_are_all_tested():
    """Every LBWN_* switch the product library reads is set by some test."""
    import glob
    src = ''.join(open(f).read() for f in glob.glob(os.path.join(ROOT, 'lb-wavenet_amd', 'csrc', '*.[hc]*')))
    read = set(re.findall(r'getenv\("(LBWN_[A-Z0-9_]+)"\)', src))
    assert read, 'no switches found'
    tests = ''.join(open(f).read() for f in glob.glob(os.path.join(ROOT, 'tests', 'test_*.py')))
    untested = sorted(v for v in read if not re.search(r"(['\"]%s['\"]|\b%s=)" % (v, v), tests))
    assert not untested, 'read by the library but set by no test: %s' % untested


def test_side_stream_kernels_fit_beside_dskip():
    """The backward's side stream (dPRE, the slab reduction, the GC gradients) runs beside dSKIP's
    A-in-registers GEMM only while its kernels fit in the VGPRs that GEMM's two waves per SIMD leave
    free (512 - 2 x 240): a kernel past that budget waits for dSKIP's blocks instead, with nothing
    failing (round 6: the GEMM at 242 VGPRs put dPRE 74 -> 306 us at C2).  Read from the gfx950
    code objects of the built library (tools/kernel_regs.py), no GPU."""
    import importlib.util
    import pytest
    if not os.path.exists('/opt/rocm/lib/llvm/bin/llvm-readelf'):
        pytest.skip('llvm-readelf not installed')
    spec = importlib.util.spec_from_file_location('kernel_regs', os.path.join(ROOT, 'tools', 'kernel_regs.py'))
    kr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(kr)
    res = kr.kernel_resources()
    assert res, 'no gfx950 code objects found in liblbwn.so'

    def regs(pattern):
        hits = {k: v['vgpr'] + v['agpr'] for k, v in res.items() if re.search(pattern, k)}
        assert hits, pattern
        return hits
    amn = regs(r'gemm_x3q_kernelILi8ELb1E')
    assert max(amn.values()) <= 240, amn
    for k in ('pre_grad_part_kernel', 'pre_grad_reduce_kernel', 'layer_reduce_all_kernel', 'gc_tile_sum_kernel',
              'gc_wgrad_kernel', 'gc_egrad_part_kernel', 'gc_egrad_sum_kernel'):
        for name, n in regs(k).items():
            assert n <= 32, (name, n)
