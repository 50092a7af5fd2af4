"""torch.library ops ``lbwn::*`` over the C ABI, with autograd (SURVEY §8b host surface).

``lbwn::dilconv_gate`` is one residual layer of tmodel.py:117-184 (dilated causal conv over
``[x[t-d] | x[t]]``, tanh·σ gate, 1×1 residual): the HIP kernels behind ``lbwn_layer_forward``
and ``lbwn_layer_backward``, composable with torch autograd so a caller can build its own stack
(the training plan in ``tmodel.WaveNetTrain`` is the fused, fast path for whole networks).

Layouts are the reference's (arch.py:112-167): ``w_sig``/``w_gate`` [2][n_res][n_dil] (tap 0
= x[t-d]), ``w_res`` [n_dil][n_res], biases [n_dil] / [n_res].  ``x_halo`` is [B][H+T][n_res]
with the layer's SAVE (D-separation state, tmodel.py:122-127) in rows [H-d, H) and x in rows
[H, H+T).  Only device tensors are accepted: there is no CPU implementation (the numpy oracle is
test infrastructure, never a fallback).
"""
from typing import Tuple

import torch

from . import _lib

_LIB = None


def _lib_loaded():
    global _LIB
    if _LIB is None:
        _LIB = _lib.load()
    return _LIB


def _check_inputs(x_halo, w_sig, dilation, H):
    if not x_halo.is_cuda:
        raise RuntimeError('lbwn::dilconv_gate: device tensors only (no CPU implementation)')
    if x_halo.dtype != torch.float32 or x_halo.dim() != 3:
        raise ValueError('lbwn::dilconv_gate: x_halo must be float32 [B][H+T][n_res]')
    if not (1 <= dilation <= H):
        raise ValueError('lbwn::dilconv_gate: need 1 <= dilation <= H')
    B, HT, Cr = x_halo.shape
    if HT <= H:
        raise ValueError('lbwn::dilconv_gate: x_halo has no body rows (H+T <= H)')
    if w_sig.shape[0] != 2 or w_sig.shape[1] != Cr:
        raise ValueError('lbwn::dilconv_gate: w_sig must be [2][n_res][n_dil]')
    return B, HT - H, Cr, w_sig.shape[2]


def _same_device(*ts):
    dev = ts[0].device
    for t in ts[1:]:
        if t.device != dev:
            raise ValueError('lbwn::dilconv_gate: all tensors must be on one device (%s vs %s)' % (dev, t.device))


@torch.library.custom_op('lbwn::dilconv_gate', mutates_args=(), device_types='cuda')
def dilconv_gate(x_halo: torch.Tensor, w_sig: torch.Tensor, w_gate: torch.Tensor, b_sig: torch.Tensor,
                 b_gate: torch.Tensor, w_res: torch.Tensor, b_res: torch.Tensor, dilation: int,
                 H: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (z [B][T][n_dil], x_out [B][T][n_res] = x + z·RES + b_res)."""
    B, T, Cr, Cd = _check_inputs(x_halo, w_sig, dilation, H)
    _same_device(x_halo, w_sig, w_gate, b_sig, b_gate, w_res, b_res)
    lib = _lib_loaded()
    dev = x_halo.device
    with torch.cuda.device(dev):   # the kernels launch on the tensors' device and its current stream
        x_halo = x_halo.contiguous()
        z = torch.empty(B, T, Cd, dtype=torch.float32, device=dev)
        xo = torch.empty(B, H + T, Cr, dtype=torch.float32, device=dev)
        ws = torch.empty(lib.lbwn_layer_image_floats_abi() + 16, dtype=torch.float32, device=dev)
        args = [t.contiguous() for t in (w_sig, w_gate, b_sig, b_gate, w_res, b_res)]
        _lib.check(lib.lbwn_layer_forward(x_halo.data_ptr(), xo.data_ptr(), z.data_ptr(), Cd,
                                          *[t.data_ptr() for t in args], None, None, None, 0,
                                          B, T, H, dilation, Cr, Cd, ws.data_ptr(),
                                          torch.cuda.current_stream(dev).cuda_stream))
        return z, xo[:, H:].contiguous()


@dilconv_gate.register_fake
def _(x_halo, w_sig, w_gate, b_sig, b_gate, w_res, b_res, dilation, H):
    B, HT, Cr = x_halo.shape
    return x_halo.new_empty(B, HT - H, w_sig.shape[2]), x_halo.new_empty(B, HT - H, Cr)


@torch.library.custom_op('lbwn::dilconv_gate_bwd', mutates_args=(), device_types='cuda')
def dilconv_gate_bwd(dz: torch.Tensor, dx_out: torch.Tensor, x_halo: torch.Tensor, w_sig: torch.Tensor,
                     w_gate: torch.Tensor, b_sig: torch.Tensor, b_gate: torch.Tensor, w_res: torch.Tensor,
                     b_res: torch.Tensor, dilation: int, H: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor,
                                                                          torch.Tensor, torch.Tensor, torch.Tensor,
                                                                          torch.Tensor]:
    """lbwn_layer_backward: (dx_halo, dw_sig, dw_gate, db_sig, db_gate, dw_res, db_res)."""
    B, T, Cr, Cd = _check_inputs(x_halo, w_sig, dilation, H)
    _same_device(dz, dx_out, x_halo, w_sig, w_gate, b_sig, b_gate, w_res, b_res)
    lib = _lib_loaded()
    dev = x_halo.device
    f32 = dict(dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):   # the kernels launch on the tensors' device and its current stream
        ws = torch.empty(int(lib.lbwn_layer_backward_ws_floats(B, T, Cr)), **f32)
        dxh = torch.empty(B, H + T, Cr, **f32)
        g = [torch.empty_like(t) for t in (w_sig, w_gate, b_sig, b_gate, w_res, b_res)]
        args = [t.contiguous() for t in (w_sig, w_gate, b_sig, b_gate, w_res, b_res)]
        _lib.check(lib.lbwn_layer_backward(x_halo.contiguous().data_ptr(), dz.contiguous().data_ptr(), Cd,
                                           dx_out.contiguous().data_ptr(), *[t.data_ptr() for t in args],
                                           None, None, None, 0, dxh.data_ptr(), *[t.data_ptr() for t in g],
                                           None, 0, None, B, T, H, dilation, Cr, Cd, ws.data_ptr(),
                                           torch.cuda.current_stream(dev).cuda_stream))
        return (dxh, *g)


@dilconv_gate_bwd.register_fake
def _(dz, dx_out, x_halo, w_sig, w_gate, b_sig, b_gate, w_res, b_res, dilation, H):
    return (torch.empty_like(x_halo), torch.empty_like(w_sig), torch.empty_like(w_gate), torch.empty_like(b_sig),
            torch.empty_like(b_gate), torch.empty_like(w_res), torch.empty_like(b_res))


def _setup_context(ctx, inputs, output):
    x_halo, w_sig, w_gate, b_sig, b_gate, w_res, b_res, dilation, H = inputs
    ctx.save_for_backward(x_halo, w_sig, w_gate, b_sig, b_gate, w_res, b_res)
    ctx.dilation, ctx.H = dilation, H


def _backward(ctx, dz, dx_out):
    x_halo, w_sig, w_gate, b_sig, b_gate, w_res, b_res = ctx.saved_tensors
    B, HT, Cr = x_halo.shape
    T, Cd = HT - ctx.H, w_sig.shape[2]
    if dz is None:
        dz = x_halo.new_zeros(B, T, Cd)
    if dx_out is None:
        dx_out = x_halo.new_zeros(B, T, Cr)
    gx, gws, gwg, gbs, gbg, gwr, gbr = dilconv_gate_bwd(dz, dx_out, x_halo, w_sig, w_gate, b_sig, b_gate, w_res,
                                                        b_res, ctx.dilation, ctx.H)
    return gx, gws, gwg, gbs, gbg, gwr, gbr, None, None


dilconv_gate.register_autograd(_backward, setup_context=_setup_context)


class DilatedResidualLayer(torch.nn.Module):
    """One residual block layer as an nn.Module over ``lbwn::dilconv_gate`` (weights in the
    reference layouts; SAVE kept in a buffer and updated with the last d input rows, as
    tmodel.py:165 assigns prev_z_save)."""

    def __init__(self, n_res, n_dil, dilation, batch_sz, H=None):
        super().__init__()
        self.dilation, self.H = dilation, H or dilation
        self.w_sig = torch.nn.Parameter(torch.empty(2, n_res, n_dil))
        self.w_gate = torch.nn.Parameter(torch.empty(2, n_res, n_dil))
        self.b_sig = torch.nn.Parameter(torch.zeros(n_dil))
        self.b_gate = torch.nn.Parameter(torch.zeros(n_dil))
        self.w_res = torch.nn.Parameter(torch.empty(n_dil, n_res))
        self.b_res = torch.nn.Parameter(torch.zeros(n_res))
        for w in (self.w_sig, self.w_gate, self.w_res):
            torch.nn.init.xavier_uniform_(w.view(-1, w.shape[-1]))
        self.register_buffer('save', torch.zeros(batch_sz, dilation, n_res))

    def forward(self, x):
        """x [B][T][n_res] -> (z [B][T][n_dil], x_out [B][T][n_res]); SAVE <- last d rows of [SAVE ++ x]."""
        B, T, Cr = x.shape
        H, d = self.H, self.dilation
        x_halo = torch.cat([x.new_zeros(B, H - d, Cr), self.save, x], dim=1)
        z, xo = torch.ops.lbwn.dilconv_gate(x_halo, self.w_sig, self.w_gate, self.b_sig, self.b_gate, self.w_res,
                                            self.b_res, d, H)
        with torch.no_grad():
            self.save.copy_(x_halo[:, H + T - d:H + T])
        return z, xo
