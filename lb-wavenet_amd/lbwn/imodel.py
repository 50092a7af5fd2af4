"""WaveNetGen — drop-in for imodel.WaveNetGen (imodel.py:7-303) on MI355X.

Same constructor arguments as the reference (imodel.py:9-23: n_blocks, n_block_layers,
n_quant, n_res, n_dil, n_skip, n_post1, n_gc_embed, n_gc_category, use_bias, batch_sz,
chunk_sz, teacher_vec).  The TF while_loop becomes lbwn_gen_run: the whole step is HIP
kernels with device-resident state, optionally captured as a hipGraph of ``chunk_sz``
steps and replayed.  The reference's generation path does not run as shipped;
this class implements its stated intent (tests.py:1: tmodel and imodel are equivalent
functions), adding PRE_BIAS to the input embedding by default (``pre_bias=False``
reproduces imodel.py:75-77 literally).
"""
import ctypes
import sys

import numpy as np
import torch

from . import _lib
from .arch import ParamLayout, normalize_arch


class WaveNetGen:
    def __init__(self, n_blocks, n_block_layers, n_quant, n_res, n_dil, n_skip, n_post1, n_gc_embed,
                 n_gc_category, use_bias, batch_sz, chunk_sz, teacher_vec=None, *, pre_bias=True, seed=0,
                 device='cuda', graph=True):
        self.arch = normalize_arch(dict(n_blocks=n_blocks, n_block_layers=n_block_layers, n_quant=n_quant,
                                        n_res=n_res, n_dil=n_dil, n_skip=n_skip, n_post=n_post1,
                                        n_gc_embed=n_gc_embed, n_gc_category=n_gc_category, use_bias=use_bias))
        self.batch_sz = batch_sz
        self.chunk_sz = chunk_sz
        self.pre_bias = bool(pre_bias)
        self.seed = int(seed)
        self.device = torch.device(device)
        self.use_graph = graph
        self.lib = _lib.load()
        self.layout = ParamLayout(self.arch)
        self.flat = torch.zeros(self.layout.n_total, dtype=torch.float32, device=self.device)
        self.vars = self.layout.views(self.flat)
        self.teacher_vec = teacher_vec
        self.teacher_mu = None
        if teacher_vec is not None:
            from .ops import mu_encode
            self.teacher_mu = mu_encode(torch.as_tensor(np.asarray(teacher_vec), dtype=torch.float32,
                                                        device=self.device), n_quant)   # imodel.py:46
            print('Teacher vec is {} samples long.'.format(len(teacher_vec)), file=sys.stderr)
        self._plan = None
        self._ws = None
        self._graph = None

    # ---- parameters -------------------------------------------------------------------------
    def load_params(self, src):
        """src: WaveNetTrain, {serial name: tensor/array}, or a flat tensor of this layout."""
        with torch.no_grad():
            if hasattr(src, 'vars'):
                src = src.vars
            if isinstance(src, torch.Tensor):
                self.flat.copy_(src)
                return
            for name, v in self.vars.items():
                v.copy_(torch.as_tensor(np.asarray(src[name]) if not isinstance(src[name], torch.Tensor)
                                        else src[name], dtype=torch.float32))

    def restore(self, path):
        from .ckpt import load_tensors
        self.load_params(load_tensors(path))

    # ---- graph ------------------------------------------------------------------------------
    def build_graph(self, max_steps):
        """Allocate the generation plan for up to max_steps samples (imodel.py:279-303)."""
        a = _lib.Arch()
        for k in ('n_blocks', 'n_block_layers', 'n_quant', 'n_res', 'n_dil', 'n_skip', 'n_post',
                  'n_gc_embed', 'n_gc_category', 'n_lc_in', 'n_lc_out'):
            setattr(a, k, int(self.arch[k]))
        a.use_bias = int(self.arch['use_bias'])
        self._arch_c = a
        h = ctypes.c_void_p()
        n_teach = 0 if self.teacher_mu is None else self.teacher_mu.numel()
        _lib.check(self.lib.lbwn_gen_plan_create(ctypes.byref(a), self.batch_sz, int(max_steps), int(n_teach),
                                                 ctypes.byref(h)))
        self._plan = h
        self.max_steps = int(max_steps)
        nbytes = self.lib.lbwn_gen_workspace_bytes(h)
        self._ws = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
        P = _lib.Params()
        base = self.flat.data_ptr()
        for field, off in self.layout.kind_base.items():
            if field.startswith('lc_up'):
                continue
            setattr(P, field, base + 4 * off)
        self._params_c = P
        self._graph = None
        return self

    @property
    def persistent(self):
        """True when the plan runs each gen_run as one persistent launch (stream groups of <= 16,
        B <= 80 on 256 CUs)."""
        return bool(self._plan is not None and self.lib.lbwn_gen_is_persistent(self._plan))

    def tensor(self, name, dtype=torch.float32):
        off, nb = _lib.c_size_t(), _lib.c_size_t()
        _lib.check(self.lib.lbwn_gen_tensor(self._plan, name.encode(), ctypes.byref(off), ctypes.byref(nb)))
        return self._ws[off.value:off.value + nb.value].view(dtype)

    def init_buffers(self, gc_ids=None):
        """imodel.init_buffers: zero the lookback/loop buffers, load teacher + GC ids."""
        self._gc = None
        if self.arch['n_gc_embed'] > 0:
            if gc_ids is None:
                raise ValueError('GC arch: gc_ids [batch_sz] required (generate.py:94)')
            ids = np.asarray(gc_ids, np.int32).reshape(-1)
            if ids.size != self.batch_sz:
                raise ValueError('gc_ids has %d entries, batch_sz is %d' % (ids.size, self.batch_sz))
            self._gc = torch.as_tensor(ids, device=self.device)
        t = self.teacher_mu
        _lib.check(self.lib.lbwn_gen_start(self._plan, ctypes.byref(self._params_c), self._ws.data_ptr(),
                                           _lib.ptr(self._gc), _lib.ptr(t), 0 if t is None else t.numel(),
                                           self.seed, int(self.pre_bias), _lib.stream_ptr()))

    def _launch(self, n):
        _lib.check(self.lib.lbwn_gen_run(self._plan, ctypes.byref(self._params_c), self._ws.data_ptr(), n,
                                         _lib.stream_ptr()))

    def step(self, n_steps):
        """Advance every stream by n_steps samples (graph replay of chunk_sz-step chunks)."""
        chunk = self.chunk_sz
        done = 0
        if self.use_graph and n_steps >= chunk:
            if self._graph is None:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        self._launch(chunk)
                torch.cuda.current_stream().wait_stream(s)
                self._graph = g
                done += chunk           # capture does not execute; replay below covers it
                self._graph.replay()
            while n_steps - done >= chunk:
                self._graph.replay()
                done += chunk
        if n_steps - done > 0:
            self._launch(n_steps - done)

    def run(self, gen_sz, gc_ids=None):
        """The reference's sess.run(wave_ops) (generate.py:110): generate gen_sz steps from a
        fresh state; the returned waveform holds whole chunks only (imodel.py:256-258)."""
        if self._plan is None or self.max_steps < gen_sz:
            self.build_graph(gen_sz)
        self.init_buffers(gc_ids)
        self.step(int(gen_sz))
        self.check_status()
        n_out = (int(gen_sz) // self.chunk_sz) * self.chunk_sz
        wav = self.tensor('wav').view(self.batch_sz, self.max_steps)[:, :n_out]
        return int(gen_sz), wav, int(gen_sz) % self.chunk_sz

    def check_status(self):
        """Raise if a skip helper's granule poll timed out (status 5): the step's skip sum, and
        every draw after it, would be wrong."""
        s = int(self.tensor('status', torch.int32).item())
        if s != 0:
            raise RuntimeError('generation status %d: a skip-helper hand-off timed out' % s)

    def samples(self):
        return self.tensor('samples', torch.int32).view(self.batch_sz, self.max_steps)

    def logits(self):
        return self.tensor('logits').view(self.batch_sz, self.arch['n_quant'])
