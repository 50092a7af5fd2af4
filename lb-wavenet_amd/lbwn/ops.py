"""µ-law codec (ops.py:4-39).  Device variants run the HIP kernels (lbwn_mulaw_*); the
numpy variants are the host-side data-preparation path the reference also runs on the CPU
(mu_encode_np / mu_decode_np)."""
import numpy as np
import torch

from . import _lib


def mu_encode_np(x, n_quanta):
    """ops.py:23-28."""
    mu = n_quanta - 1
    amp = np.sign(x) * np.log1p(mu * np.abs(x)) / np.log1p(mu)
    quant = (amp + 1) * 0.5 * mu + 0.5
    return quant.astype(np.int32)


def mu_decode_np(quant, n_quanta):
    """ops.py:31-39."""
    mu = n_quanta - 1
    qf = np.asarray(quant).astype(np.float32)
    inv_mu = 1.0 / mu
    a = (2 * qf - 1) * inv_mu - 1
    return np.sign(a) * ((1 + mu) ** np.fabs(a) - 1) * inv_mu


def mu_encode(x, n_quanta, tf32=True, stream=None):
    """ops.py:4-9 on device: float32 tensor -> int32 codes (tf32=False: numpy-variant math)."""
    lib = _lib.load()
    x = x.to(torch.float32).contiguous()
    q = torch.empty(x.shape, dtype=torch.int32, device=x.device)
    _lib.check(lib.lbwn_mulaw_encode(x.data_ptr(), q.data_ptr(), x.numel(), n_quanta, int(tf32),
                                     _lib.stream_ptr(stream)))
    return q


def mu_decode(q, n_quanta, stream=None):
    """ops.py:12-20 on device: int32 codes -> float32 amplitudes."""
    lib = _lib.load()
    q = q.to(torch.int32).contiguous()
    x = torch.empty(q.shape, dtype=torch.float32, device=q.device)
    _lib.check(lib.lbwn_mulaw_decode(q.data_ptr(), x.data_ptr(), q.numel(), n_quanta, _lib.stream_ptr(stream)))
    return x
