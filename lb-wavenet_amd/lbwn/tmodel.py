"""WaveNetTrain — drop-in for tmodel.WaveNetTrain (tmodel.py:6-358) on MI355X.

Same constructor arguments and methods as the reference; the TF graph is replaced by an
lbwn plan (liblbwn.so) that runs the whole forward/loss/backward as a fixed sequence of
HIP launches on the current torch stream.  The reference's TF-eager flow (train.py:219-222)

    grads_and_vars, loss = net.build(wav_input, mel_input, id_mask)
    optimizer.apply_gradients(grads_and_vars)

is reproduced literally (lbwn.optim.AdamOptimizer).
"""
import ctypes
import sys
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .ckpt import Checkpoint
from .arch import ParamLayout, layer_iter, n_layers, recep_field_sz, save_layout, xavier_limit


def _i32(x, dev):
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=torch.int32).contiguous()
    return torch.as_tensor(np.asarray(x), dtype=torch.int32, device=dev).contiguous()


class GradsAndVars(list):
    """list of (grad view, serial name) like TF's compute_gradients output; carries the
    flat buffers so the optimizer applies one fused update."""

    def __init__(self, net, pairs):
        super().__init__(pairs)
        self.net = net


class WaveNetTrain:
    def __init__(self, n_blocks, n_block_layers, n_quant, n_res, n_dil, n_skip, n_post, n_gc_embed,
                 n_gc_category, n_lc_in, n_lc_out, lc_upsample, use_bias, wav_input_type, batch_sz,
                 l2_factor, add_summary=False, n_keep_checkpoints=10, ckpt_path=None, resume_step=0,
                 n_valid_total=0, sess=None, print_interval=10, device='cuda', seed=0):
        self.arch = dict(n_blocks=n_blocks, n_block_layers=n_block_layers, n_quant=n_quant, n_res=n_res,
                         n_dil=n_dil, n_skip=n_skip, n_post=n_post, n_gc_embed=n_gc_embed,
                         n_gc_category=n_gc_category, n_lc_in=n_lc_in, n_lc_out=n_lc_out,
                         lc_upsample=list(lc_upsample), use_bias=bool(use_bias), wav_input_type=wav_input_type)
        for k, v in self.arch.items():
            setattr(self, k, v)
        self.batch_sz = batch_sz
        self.l2_factor = float(l2_factor)
        self.add_summary = add_summary
        self.n_keep_checkpoints = n_keep_checkpoints
        self.ckpt_path = ckpt_path
        self.resume_step = resume_step
        self.n_valid_total = n_valid_total
        self.print_interval = print_interval
        self.dp = None      # lbwn.dist.DPContext when training data-parallel (set by train.py)
        self.device = torch.device(device)
        self.lib = _lib.load()
        self.layout = ParamLayout(self.arch)
        self.save_index, n_save = save_layout(self.arch, batch_sz)
        dev = self.device
        self.flat = torch.zeros(self.layout.n_total, dtype=torch.float32, device=dev)
        self.grad_flat = torch.zeros_like(self.flat)
        self.save_flat = torch.zeros(n_save, dtype=torch.float32, device=dev)
        self.stats = torch.zeros(4, dtype=torch.float32, device=dev)
        self.counters = torch.zeros(4, dtype=torch.int64, device=dev)   # GLOBAL_STEP, VALID_SAMPLES, adam t-1, status
        self.vars = self.layout.views(self.flat)
        self.grads = self.layout.views(self.grad_flat)
        self.save_vars = OrderedDict((n, self.save_flat[o:o + int(np.prod(s))].view(*s))
                                     for n, (o, s) in self.save_index.items())
        self._arch_c = self._make_arch_struct()
        self._params_c = self._make_params_struct(self.flat)
        self._grads_c = self._make_params_struct(self.grad_flat)
        self._plans = {}
        self._ws = None
        self._last = None
        self._sp_cache = None
        self.init_vars(seed)
        # host mirror of GLOBAL_STEP: counts the optimizer calls (attempted steps) so the print
        # cadence needs no sync; re-read from counters[0] by check_status, since a step skipped
        # on the device (chain timeout) does not advance GLOBAL_STEP
        self.global_step_host = 0
        # checkpoint surface (ckpt.py:13-81; the saveables are self.vars, tmodel.py:330)
        self.ckpt = Checkpoint(ckpt_path, n_keep_checkpoints, resume_step)
        self.ckpt.add_saveable_objects(self.state_tensors())

    # ---- reference API -------------------------------------------------------------------
    def get_recep_field_sz(self):
        return recep_field_sz(self.arch)

    def has_global_cond(self):
        return self.n_gc_embed > 0

    def use_lc_input(self):
        return self.n_lc_out > 0

    def init_vars(self, seed=0, bias_scale=0.0):
        """Xavier-uniform weights (arch.py:63), zero biases (arch.py:64), Xavier SAVE
        (tmodel.py:123-124 passes no initializer)."""
        g = torch.Generator(device='cpu').manual_seed(seed)
        with torch.no_grad():
            for name, e in self.layout.entries.items():
                if e.is_bias:
                    if bias_scale:
                        v = (torch.rand(e.shape, generator=g) * 2 - 1) * bias_scale
                    else:
                        v = torch.zeros(e.shape)
                else:
                    lim = xavier_limit(e.shape)
                    v = (torch.rand(e.shape, generator=g) * 2 - 1) * lim
                self.vars[name].copy_(v)
            for name, t in self.save_vars.items():
                lim = xavier_limit(list(t.shape))
                t.copy_((torch.rand(t.shape, generator=g) * 2 - 1) * lim)
        self.counters.zero_()

    def build(self, wav_input, lc_input, id_mask):
        """Forward + loss + backward of one slice (tmodel.py:292-340).  Returns
        (grads_and_vars, loss) with loss a 0-d device tensor (total = mean xent + l2)."""
        self.forward(wav_input, lc_input, id_mask, backward=True)
        gv = GradsAndVars(self, [(self.grads[n], n) for n in self.layout.names()])
        return gv, self.total_loss()

    # ---- engine ------------------------------------------------------------------------------
    def _make_arch_struct(self):
        a = _lib.Arch()
        for k in ('n_blocks', 'n_block_layers', 'n_quant', 'n_res', 'n_dil', 'n_skip', 'n_post',
                  'n_gc_embed', 'n_gc_category', 'n_lc_in', 'n_lc_out'):
            setattr(a, k, int(self.arch[k]))
        ups = self.arch['lc_upsample'] if self.arch['n_lc_out'] > 0 else []
        a.n_lc_upsample = len(ups)
        for i, s in enumerate(ups):
            a.lc_upsample[i] = int(s)
        a.use_bias = int(self.arch['use_bias'])
        return a

    def _make_params_struct(self, flat):
        P = _lib.Params()
        base = flat.data_ptr()
        kb = self.layout.kind_base
        for field in ('pre', 'pre_b', 'sig', 'sig_b', 'gate', 'gate_b', 'res', 'res_b', 'skip', 'skip_b',
                      'gc_embed', 'gc_sig', 'gc_gate', 'lc_sig', 'lc_gate', 'post1', 'post1_b', 'post2',
                      'post2_b'):
            setattr(P, field, base + 4 * kb[field] if field in kb else None)
        for i in range(8):
            k = 'lc_up%d' % i
            P.lc_up[i] = base + 4 * kb[k] if k in kb else None
        return P

    def _plan(self, T):
        if T not in self._plans:
            h = ctypes.c_void_p()
            _lib.check(self.lib.lbwn_plan_create(ctypes.byref(self._arch_c), self.batch_sz, T, ctypes.byref(h)))
            nbytes = self.lib.lbwn_plan_workspace_bytes(h)
            self._plans[T] = (h, nbytes)
        h, nbytes = self._plans[T]
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return h

    def plan_tensor(self, T, name):
        """fp32 view of a named plan workspace tensor (debug/parity)."""
        h = self._plan(T)
        off, nb = _lib.c_size_t(), _lib.c_size_t()
        _lib.check(self.lib.lbwn_plan_tensor(h, name.encode(), ctypes.byref(off), ctypes.byref(nb)))
        return self._ws[off.value:off.value + nb.value].view(torch.float32)

    def workspace_bytes(self, T):
        self._plan(T)
        return self._plans[T][1]

    def forward(self, wav_input, lc_input, id_mask, backward=True, stream=None):
        """Run the plan on one slice; wav_input int [B,T] mu-law codes (raw floats are
        mu_encode'd first when wav_input_type == 'raw', tmodel.py:58-62)."""
        dev = self.device
        if self.wav_input_type == 'raw':
            from .ops import mu_encode
            wav_input = mu_encode(torch.as_tensor(wav_input, dtype=torch.float32, device=dev), self.n_quant)
        q = _i32(wav_input, dev)
        ids = _i32(id_mask, dev)
        B, T = q.shape
        if B != self.batch_sz:
            raise ValueError('batch %d != batch_sz %d' % (B, self.batch_sz))
        mel = None
        if self.use_lc_input():
            mel = torch.as_tensor(lc_input, dtype=torch.float32, device=dev).contiguous()
        h = self._plan(T)
        sp = _lib.stream_ptr(stream)
        self._last = (q, ids, mel)   # keep inputs alive until the stream consumed them
        _lib.check(self.lib.lbwn_train_forward(h, ctypes.byref(self._params_c), self._ws.data_ptr(), q.data_ptr(),
                                               ids.data_ptr(), _lib.ptr(mel), self.save_flat.data_ptr(),
                                               self.stats.data_ptr(), sp))
        if backward:
            _lib.check(self.lib.lbwn_train_backward(h, ctypes.byref(self._params_c), ctypes.byref(self._grads_c),
                                                    self._ws.data_ptr(), q.data_ptr(), ids.data_ptr(),
                                                    _lib.ptr(mel), sp))
        return self.stats

    def status_word(self, T=None):
        """int32 view of the plan's per-step status word (zeroed at each forward; the chains
        OR their timeout codes in: bit 0 forward chain, bit 1 backward chain)."""
        T = T if T is not None else self._last[0].shape[1]
        return self.plan_tensor(T, 'status')[:1].view(torch.int32)

    def status_ptr(self):
        """Device pointer of the last step's status word (None before any step)."""
        if self._last is None:
            return None
        key = (self._last[0].shape[1], self._ws.data_ptr())
        if self._sp_cache is None or self._sp_cache[0] != key:
            self._sp_cache = (key, self.status_word().data_ptr())
        return self._sp_cache[1]

    def wait_point(self, point, stream):
        """Make a torch stream wait for a point of the last backward (lbwn_plan_stream_wait);
        False if the plan has no such point."""
        if self._last is None:
            return False
        waited = ctypes.c_int(0)
        _lib.check(self.lib.lbwn_plan_stream_wait(self._plan(self._last[0].shape[1]), point.encode(),
                                                  stream.cuda_stream, ctypes.byref(waited)))
        return bool(waited.value)

    def status(self, T=None):
        """Cumulative status (synchronises): every applied step's status word is ORed into
        counters[3] by the optimizer kernel (which skips a failed step's update on the
        device), plus the current step's word for a step not yet applied.  0 = ok; bit 0 = a
        forward-chain hand-off timed out, bit 1 = a backward-chain one."""
        return int(self.counters[3].item()) | int(self.status_word(T).item())

    def check_status(self, T=None):
        st = self.status(T)
        self.global_step_host = int(self.counters[0].item())
        if st:
            raise RuntimeError('lbwn: chain hand-off timed out (status word %#x): the failed steps were '
                               'not applied' % st)

    def l2_loss(self):
        """tmodel.py:250-261: Σ_{trainable, non-BIAS} Σv²/2 (the weight region of the flat buffer)."""
        w = self.flat[:self.layout.n_weights]
        return 0.5 * torch.dot(w, w)

    def total_loss(self):
        nv = self.stats[1]
        mean = torch.where(nv > 0, self.stats[0] / torch.clamp(nv, min=1.0), torch.zeros_like(nv))
        return mean + self.l2_factor * self.l2_loss()

    def progress_line(self):
        """tmodel.py:263-267 columns: step, total, mean xent, l2, avg_diff, n_valid,
        n_valid_cumul, n_valid_total, %."""
        st = self.stats.tolist()
        cnt = self.counters.tolist()
        nv = int(st[1])
        mean = st[0] / nv if nv else 0.0
        l2 = float(self.l2_loss())
        total = mean + self.l2_factor * l2
        B, T = self._last[0].shape
        world = self.dp.world if self.dp is not None else 1     # stats[2] is summed over ranks
        avg_diff = int(st[2]) // (world * B * (T - 1))
        pct = cnt[1] * 100.0 / self.n_valid_total if self.n_valid_total else 0.0
        return ('{:5d}\t{:8.4f}\t{:8.4f}\t{:7.2f}\t{:5.0f}\t{:5.0f}\t{:10d}\t{:14d}\t{:5.2f}'.format(
            cnt[0], total, mean, l2, avg_diff, nv, cnt[1], int(self.n_valid_total), pct))

    def maybe_print(self, file=None):
        """The in-graph progress print (tmodel.py:272-281): every print_interval steps,
        BEFORE the counters advance.  Uses the host mirror of GLOBAL_STEP, so steps that do
        not print never synchronise with the device."""
        if self.print_interval and self.global_step_host % self.print_interval == 0:
            print(self.progress_line(), file=file or sys.stderr)

    # ---- checkpoints (ckpt.py:53-81) --------------------------------------------------------
    def save(self, step, optimizer=None):
        """Write '<ckpt_path>-<step>.safetensors'; with ``optimizer`` its Adam slots too.
        Data-parallel: a collective (every rank calls it).  The weights are replicated, but
        SAVE is per stream, so the ranks' rows are gathered and rank 0 writes the SAVE of
        the GLOBAL batch [world·B, d, Cr] -- the same file a single process over world·B
        streams writes; the other ranks return None."""
        if self.device.type == 'cuda':
            torch.cuda.synchronize(self.device)
        extra = dict(optimizer.state_tensors(self)) if optimizer is not None else {}
        if self.dp is not None and self.dp.enabled:
            extra.update(self._gather_save())
            if self.dp.rank != 0:
                return None
        return self.ckpt.save(step, extra)

    def _gather_save(self):
        import torch.distributed as dist
        parts = [torch.empty_like(self.save_flat) for _ in range(self.dp.world)]
        dist.all_gather(parts, self.save_flat)
        return OrderedDict((n, torch.cat([p[o:o + int(np.prod(s))].view(*s) for p in parts], 0))
                           for n, (o, s) in self.save_index.items())

    def restore(self, optimizer=None):
        """Load '<ckpt_path>-<resume_step>' into the live buffers (ckpt.py:63-81).  Under
        data parallelism each rank takes its own rows of the global-batch SAVE."""
        select = None
        if self.dp is not None and self.dp.enabled:
            rows = self.dp.rows(self.batch_sz)
            select = lambda name, t: t[rows] if name in self.save_vars else t   # noqa: E731
        loaded = self.ckpt.restore(select)
        if optimizer is not None:
            optimizer.load_state_tensors(self, loaded)
        self.global_step_host = int(self.counters[0])
        return loaded

    # ---- state dicts (checkpoint surface, names as arch.py:142) ----------------------------
    def state_tensors(self):
        out = OrderedDict(self.vars)
        out.update(self.save_vars)
        out['GLOBAL_STEP'] = self.counters[0:1]
        out['VALID_SAMPLES'] = self.counters[1:2]
        return out
