"""ctypes binding of liblbwn.so (include/lbwn.h).

The library is the product: there is no CPU fallback.  ``load()`` raises if the .so is
missing or was built for another ABI, and every wrapper raises ``LbwnError`` with the
library's message on a non-zero return.  torch is imported first so the process has ONE
HIP runtime (torch's bundled libamdhip64.so.7 satisfies the .so's NEEDED entry).
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the .so: shared HIP runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'liblbwn.so')   # the in-tree build only (tools/with_lib.py loads variants)
ABI_VERSION = 2

c_int, c_int64, c_float, c_void_p, c_size_t = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
c_fp = ctypes.c_void_p   # device pointers are passed as integers


class LbwnError(RuntimeError):
    pass


class Arch(ctypes.Structure):
    _fields_ = [('n_blocks', c_int), ('n_block_layers', c_int), ('n_quant', c_int), ('n_res', c_int),
                ('n_dil', c_int), ('n_skip', c_int), ('n_post', c_int), ('n_gc_embed', c_int),
                ('n_gc_category', c_int), ('n_lc_in', c_int), ('n_lc_out', c_int),
                ('n_lc_upsample', c_int), ('lc_upsample', c_int * 8), ('use_bias', c_int)]


class Params(ctypes.Structure):
    _fields_ = [(n, c_fp) for n in (
        'pre', 'pre_b', 'sig', 'sig_b', 'gate', 'gate_b', 'res', 'res_b', 'skip', 'skip_b',
        'gc_embed', 'gc_sig', 'gc_gate', 'lc_sig', 'lc_gate')] + [('lc_up', c_fp * 8)] + [
        (n, c_fp) for n in ('post1', 'post1_b', 'post2', 'post2_b')]


_SIGS = {
    'lbwn_last_error': (ctypes.c_char_p, []),
    'lbwn_abi_version': (c_int, []),
    'lbwn_recep_field_sz': (c_int, [ctypes.POINTER(Arch)]),
    'lbwn_plan_create': (c_int, [ctypes.POINTER(Arch), c_int, c_int, ctypes.POINTER(c_void_p)]),
    'lbwn_plan_destroy': (None, [c_void_p]),
    'lbwn_plan_workspace_bytes': (c_size_t, [c_void_p]),
    'lbwn_plan_probe': (c_int, [c_void_p, ctypes.c_char_p, c_void_p, c_void_p]),
    'lbwn_plan_stream_wait': (c_int, [c_void_p, ctypes.c_char_p, c_void_p, ctypes.POINTER(c_int)]),
    'lbwn_plan_tensor': (c_int, [c_void_p, ctypes.c_char_p, ctypes.POINTER(c_size_t), ctypes.POINTER(c_size_t)]),
    'lbwn_train_forward': (c_int, [c_void_p, ctypes.POINTER(Params), c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_void_p]),
    'lbwn_train_backward': (c_int, [c_void_p, ctypes.POINTER(Params), ctypes.POINTER(Params), c_fp, c_fp, c_fp,
                                    c_fp, c_void_p]),
    'lbwn_adam_tf1': (c_int, [c_fp, c_fp, c_fp, c_fp, c_int64, c_int64, c_float, c_float, c_float, c_float,
                              c_float, c_fp, c_fp, c_fp, c_void_p]),
    'lbwn_gen_plan_create': (c_int, [ctypes.POINTER(Arch), c_int, c_int64, c_int64, ctypes.POINTER(c_void_p)]),
    'lbwn_gen_plan_destroy': (None, [c_void_p]),
    'lbwn_gen_workspace_bytes': (c_size_t, [c_void_p]),
    'lbwn_gen_tensor': (c_int, [c_void_p, ctypes.c_char_p, ctypes.POINTER(c_size_t), ctypes.POINTER(c_size_t)]),
    'lbwn_gen_start': (c_int, [c_void_p, ctypes.POINTER(Params), c_fp, c_fp, c_fp, c_int64, ctypes.c_uint64, c_int,
                               c_void_p]),
    'lbwn_gen_run': (c_int, [c_void_p, ctypes.POINTER(Params), c_fp, c_int, c_void_p]),
    'lbwn_gen_is_persistent': (c_int, [c_void_p]),
    'lbwn_mulaw_encode': (c_int, [c_fp, c_fp, c_int64, c_int, c_int, c_void_p]),
    'lbwn_mulaw_decode': (c_int, [c_fp, c_fp, c_int64, c_int, c_void_p]),
    'lbwn_gemm_f32': (c_int, [c_fp, c_int64, c_int, c_fp, c_int64, c_int, c_fp, c_int64, c_int, c_int, c_int,
                              c_fp, c_int, c_int, c_fp, c_int64, c_int, c_int, c_fp, c_void_p]),
    'lbwn_gemm_f32_presplit': (c_int, [c_fp, c_int64, c_int, c_fp, c_int, c_fp, c_int64, c_int, c_fp, c_int64, c_int,
                                       c_int, c_fp, c_int, c_int, c_fp, c_int64, c_int, c_void_p]),
    'lbwn_split_planes_elems_abi': (c_int64, [c_int, c_int]),
    'lbwn_split_planes': (c_int, [c_fp, c_int64, c_int, c_int, c_int, c_fp, c_void_p]),
    'lbwn_gemm_set_mode': (c_int, [c_int]),
    'lbwn_gemm_get_mode': (c_int, []),
    'lbwn_layer_image_floats_abi': (c_int, []),
    'lbwn_layer_forward': (c_int, [c_fp, c_fp, c_fp, c_int64, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp,
                                   c_fp, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_fp, c_void_p]),
    'lbwn_layer_backward_ws_floats': (c_int64, [c_int, c_int, c_int]),
    'lbwn_layer_backward': (c_int, [c_fp, c_fp, c_int64, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp,
                                    c_int64, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int64, c_fp, c_int,
                                    c_int, c_int, c_int, c_int, c_int, c_fp, c_void_p]),
    'lbwn_dsep_prepend': (c_int, [c_fp, c_int64, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    'lbwn_dsep_save': (c_int, [c_fp, c_int64, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    'lbwn_head_xent': (c_int, [c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_void_p]),
}

EXPORTED = sorted(_SIGS)
_lib = None


def load(path=LIB_PATH):
    """Load liblbwn.so (once).  Raises LbwnError when it is absent: no fallback path."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise LbwnError('liblbwn.so not found at %s — build it with __graft_entry__.build() '
                        '(or `make -C lb-wavenet_amd/csrc`); there is no CPU fallback' % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.lbwn_abi_version() != ABI_VERSION:
        raise LbwnError('liblbwn.so ABI %d != %d' % (lib.lbwn_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def check(ret):
    if ret != 0:
        msg = _lib.lbwn_last_error().decode() if _lib is not None else ''
        raise LbwnError('lbwn error %d: %s' % (ret, msg))
    return ret


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
