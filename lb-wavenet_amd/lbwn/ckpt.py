"""Checkpoints — drop-in for ckpt.Checkpoint (ckpt.py:13-81).

The reference writes TF V2 ``<ckpt_path>-<step>.{index,meta,data-00000-of-00001}`` through
a tf.train.Saver over the model's serial-named variables (tmodel.py:330, names built at
arch.py:142: ``SIGNAL_2_7``, ``SAVE_128_2_7``, ``GLOBAL_STEP``, ...).  TF cannot run here,
so the same variables are written as ONE safetensors file ``<ckpt_path>-<step>.safetensors``
with identical keys; the optimizer's TF1 Adam slots may ride along under TF's slot names
(``<var>/Adam``, ``<var>/Adam_1``) so a resume is exact.  ``max_to_keep`` rotation follows
tf.train.Saver (oldest files deleted beyond n_keep_checkpoints).  Loading never unpickles:
safetensors only.  A reference-written TF V2 bundle (``<pfx>-<step>.index`` +
``.data-00000-of-00001``) at the same prefix is read when no safetensors file is there
(lbwn/tfckpt.py), and ``export_tf_bundle`` writes one the reference's Saver can restore.
"""
import os
import sys

import numpy as np
import torch
from safetensors.torch import load_file, save_file

from . import tfckpt

SUFFIX = '.safetensors'


def ckpt_file(path_pfx, step=None):
    """'<pfx>-<step>.safetensors' (or '<pfx>.safetensors' / an existing file path as given)."""
    if step is not None:
        return '{}-{}{}'.format(path_pfx, step, SUFFIX)
    return path_pfx if path_pfx.endswith(SUFFIX) else path_pfx + SUFFIX


def save_tensors(path, tensors):
    """tensors: {name: tensor/array}; written contiguous on the host."""
    out = {}
    for k, v in tensors.items():
        t = v.detach() if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
        out[k] = t.to('cpu').contiguous().clone()
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + '.tmp'
    save_file(out, tmp)
    os.replace(tmp, path)     # a crash mid-write never leaves a truncated checkpoint
    return path


def load_tensors(path):
    """{name: cpu tensor} from '<pfx>-<step>' prefixes or a .safetensors path; a TF V2 bundle
    at the prefix when there is no safetensors file (the reference's own checkpoints)."""
    f = ckpt_file(path)
    if not os.access(f, os.R_OK) and not path.endswith(SUFFIX) and tfckpt.exists(path):
        return {k: torch.from_numpy(np.array(v)) for k, v in tfckpt.read_bundle(path).items()}
    if not os.access(f, os.R_OK):
        print("Couldn't find checkpoint file {}".format(f), file=sys.stderr)   # ckpt.py:71-75
        sys.exit(1)
    return load_file(f)


class Checkpoint:
    """ckpt.Checkpoint's contract: add_saveable_objects(dict), save(step) -> path prefix,
    restore() from '<ckpt_path>-<resume_step>'."""

    def __init__(self, ckpt_path, n_keep_checkpoints, resume_step):
        self.ckpt_path = ckpt_path
        self.n_keep_checkpoints = n_keep_checkpoints
        self.resume_step = resume_step
        self.saveable_objects = {}
        self._written = []

    def add_saveable_objects(self, objs):
        self.saveable_objects.update(objs)

    def save(self, step, extra=None):
        if self.ckpt_path is None:
            raise ValueError('save: no ckpt_path')
        tensors = dict(self.saveable_objects)
        if extra:
            tensors.update(extra)
        path_pfx = '{}-{}'.format(self.ckpt_path, step)
        save_tensors(ckpt_file(path_pfx), tensors)
        self._written.append(path_pfx)
        while self.n_keep_checkpoints and len(self._written) > self.n_keep_checkpoints:
            old = self._written.pop(0)
            try:
                os.remove(ckpt_file(old))
            except OSError:
                pass
        return path_pfx

    def restore(self, select=None):
        """``select(name, tensor) -> tensor`` picks the part of a stored tensor this
        process owns (data-parallel SAVE rows); identity by default."""
        f = '{}-{}'.format(self.ckpt_path, self.resume_step)
        print('Restoring from {}'.format(f))
        loaded = load_tensors(f)
        if select is not None:
            loaded = {k: select(k, v) for k, v in loaded.items()}
        missing = [k for k in self.saveable_objects if k not in loaded]
        if missing:
            print('Checkpoint {} lacks {} variables (first: {})'.format(f, len(missing), missing[0]), file=sys.stderr)
            sys.exit(1)
        with torch.no_grad():
            for k, dst in self.saveable_objects.items():
                src = loaded[k]
                if src.dim() == 0 and dst.numel() == 1:   # TF's scalar GLOBAL_STEP / VALID_SAMPLES
                    src = src.reshape(dst.shape)
                if tuple(src.shape) != tuple(dst.shape):
                    print('Checkpoint {}: {} has shape {}, model expects {}'.format(
                        f, k, tuple(src.shape), tuple(dst.shape)), file=sys.stderr)
                    sys.exit(1)
                dst.copy_(src.to(dst.dtype))
        return loaded


# the reference's scalar int32 counters (tmodel.py:223-226, arch.py:101-102); the rest keep dtype/shape
_TF_SCALARS = ('GLOBAL_STEP', 'VALID_SAMPLES')


def export_tf_bundle(tensors, prefix):
    """Write {name: tensor} as a TF V2 bundle at ``prefix`` in the reference's variable forms
    (GLOBAL_STEP / VALID_SAMPLES as int32 scalars); returns the prefix."""
    out = {}
    for k, v in tensors.items():
        a = (v.detach().to('cpu') if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))).numpy()
        if k in _TF_SCALARS:
            a = np.asarray(a.reshape(()), dtype=np.int32)
        out[k] = a
    return tfckpt.write_bundle(prefix, out)
