"""Data parallelism over streams: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on ROCm; "gloo" in the CPU tests).

The B·N global slots are independent (data.py:210-224) and each slot's D-separation state
SAVE[b] lives with its rank, so the ONLY exchange per step is one all_reduce(SUM) of the
un-normalised gradient (Σ-xent grads, raw) together with the loss statistics — Adam then
divides by the GLOBAL n_valid (stats[1]) and adds l2·θ on every rank, identically, so the
replicas never drift.  Weights are broadcast from rank 0 once at start.
"""
import os

import torch
import torch.distributed as dist


def _reduce_status(word):
    """MAX over ranks of the int32 step status word, in place: a chain timeout on ANY rank makes
    the word non-zero on every rank, so every rank's optimizer skips the step on the device; the
    word then holds the highest failure code any rank reported (bit 1, the backward chain, over
    bit 0).  One in-place collective on the word itself -- no bit expansion kernels on the device
    path, where every small launch beside dSKIP waits for a CU."""
    dist.all_reduce(word.view(torch.int32), op=dist.ReduceOp.MAX)


class DPContext:
    def __init__(self, world=1, rank=0, local_rank=0, last_on_main=True):
        self.world, self.rank, self.local_rank = world, rank, local_rank
        # the last bucket (after the whole backward) issued from the main stream itself: two
        # cross-stream hops (main -> RCCL's stream -> main) before the optimizer instead of four
        # through the comm stream
        self.last_on_main = last_on_main

    @property
    def enabled(self):
        return self.world > 1

    def rows(self, per_rank):
        """This rank's slot range of a globally dealt batch."""
        return slice(self.rank * per_rank, (self.rank + 1) * per_rank)

    def broadcast_params(self, net):
        if self.enabled:
            dist.broadcast(net.flat, 0)

    def reduce_grads(self, net):
        """Σ over ranks of the raw gradient buffer and of (Σxent, n_valid, Σ|argmax diff|), and
        the MAX of the step status words (a timed-out chain on ANY rank makes every rank's
        optimizer skip the step on the device, so no rank applies garbage gradients;
        _reduce_status).

        Three buckets, each one RCCL group call over in-place views:
          0 "head": POST1, POST2, their biases, SKIP_BIAS + the stats + the status word — final
            once the backward chain has completed (lbwn_plan_stream_wait "head_grads"), so its
            all-reduce runs on a side stream beside the backward's tail (dSKIP, the slab
            reduction, dPRE, the conditioning grads);
          1 "side": PRE, SIGNAL, GATE, RESIDUAL, the GC tables and their biases — final once the
            plan's side stream has run dPRE, the slab reduction and the GC grads ("side_grads"),
            while dSKIP may still run on the main stream;
          2 "rest": SKIP and the LC weights, after the whole backward.
        No collective ever overlaps a persistent chain launch: bucket 0 starts after the backward
        chain, and the current stream waits for both buckets before the optimizer (hence before
        the next step's forward chain).  A chain's tiles assume every block of a round is resident
        (DESIGN §4): an RCCL kernel holding CUs during a chain launch would stall its lock-step
        hand-offs."""
        if not self.enabled:
            return
        plan = _Buckets.of(net)
        if not net.grad_flat.is_cuda:   # gloo (CPU tests): the same buckets, in order
            for k in range(len(plan.ranges)):
                _all_reduce_many(plan.tensors(k, net), cuda=False)
                if k == 0:
                    _reduce_status(net.status_word())
            return
        main = torch.cuda.current_stream(net.grad_flat.device)
        comm = self._comm_stream(net.grad_flat.device)
        # each bucket waits for its point of the backward, or for the whole backward when the
        # plan has no such point (the comm stream's order keeps the buckets' all-reduces serial).
        # Everything is reduced in place -- the gradient ranges, the stats and the status word --
        # one RCCL group call per bucket: no staging copies or conversion kernels, which beside
        # dSKIP wait for CUs its 240-VGPR waves leave only to kernels of <= 32 VGPRs and so ran
        # after it (one-rank RCCL, C2: 144 us per step with staging, tools/dp_overhead.py).
        for k, point in enumerate(('head_grads', 'side_grads', None)):
            if not plan.ranges[k] and k > 0:
                continue
            status = net.status_word() if k == 0 else None
            if point is None and self.last_on_main:
                _all_reduce_many(plan.tensors(k, net), cuda=True, status=status)   # on main, after the backward
                continue
            if point is None or not net.wait_point(point, comm):
                comm.wait_stream(main)
            with torch.cuda.stream(comm):
                _all_reduce_many(plan.tensors(k, net), cuda=True, status=status)
        main.wait_stream(comm)

    def reduce_grads_flat(self, net):
        """The whole gradient + stats as one message after the backward, and the status word's MAX
        (the reference bucketing of tests/test_dropin.py::test_dp_bucketed_equals_flat)."""
        if not self.enabled:
            return
        n = net.grad_flat.numel()
        buf = torch.empty(n + 3, dtype=torch.float32, device=net.grad_flat.device)
        buf[:n].copy_(net.grad_flat)
        buf[n:n + 3].copy_(net.stats[:3])
        dist.all_reduce(buf)
        net.grad_flat.copy_(buf[:n])
        net.stats[:3].copy_(buf[n:n + 3])
        _reduce_status(net.status_word())

    def _comm_stream(self, device):
        s = getattr(self, '_comm', None)
        if s is None:
            s = self._comm = torch.cuda.Stream(device=device)
        return s

    def max_over_ranks(self, value, device):
        if not self.enabled:
            return value
        t = torch.tensor([value], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        if self.enabled:
            dist.barrier()


def _all_reduce_many(ts, cuda, status=None):
    """SUM-all-reduce each tensor in place, as one coalesced RCCL group call on the device path
    (one launch per bucket instead of one per range; a group takes one dtype and op), then MAX
    the status word."""
    if cuda and dist.is_initialized() and len(ts) > 1:
        from torch.distributed.distributed_c10d import _coalescing_manager
        with _coalescing_manager(device=ts[0].device):
            for t in ts:
                dist.all_reduce(t)
    else:
        for t in ts:
            dist.all_reduce(t)
    if status is not None:
        _reduce_status(status)


class _Buckets:
    """Flat ranges of the three all-reduce buckets (lbwn.arch.ParamLayout: weights
    [pre, sig, gate, res, skip, gc.., lc.., post1, post2] then biases [pre_b, sig_b, gate_b,
    res_b, skip_b, post1_b, post2_b]), reduced in place."""

    def __init__(self, net):
        lay = net.layout
        kb = lay.kind_base
        # weights: [pre sig gate res | skip | gc_embed gc_sig gc_gate | lc.. | post1 post2]
        head = [(kb['post1'], lay.n_weights)]
        side = [(0, kb['skip'])]
        after_skip = min([kb[k] for k in kb if k.startswith('lc_up') or k in ('lc_sig', 'gc_embed')] + [kb['post1']])
        rest = [(kb['skip'], after_skip)]
        if 'gc_embed' in kb:
            end_gc = min([kb[k] for k in kb if k.startswith('lc_up') or k == 'lc_sig'] + [kb['post1']])
            side.append((kb['gc_embed'], end_gc))
            if end_gc < kb['post1']:
                rest.append((end_gc, kb['post1']))
        elif after_skip < kb['post1']:
            rest.append((after_skip, kb['post1']))
        if 'skip_b' in kb:   # biases: [pre_b sig_b gate_b res_b | skip_b post1_b post2_b]
            head.append((kb['skip_b'], lay.n_total))
            side.append((lay.n_weights, kb['skip_b']))
        self.ranges = [head, side, rest]
        covered = sorted(r for rs in self.ranges for r in rs)
        assert covered[0][0] == 0 and covered[-1][1] == lay.n_total and all(
            covered[i][1] == covered[i + 1][0] for i in range(len(covered) - 1)), ('buckets must tile the buffer', covered)
        self.device = net.grad_flat.device

    @staticmethod
    def of(net):
        b = getattr(net, '_dp_buckets', None)
        if b is None or b.device != net.grad_flat.device:
            b = _Buckets(net)
            net._dp_buckets = b
        return b

    def tensors(self, k, net):
        """Bucket k's in-place views: its gradient ranges, and for bucket 0 the loss stats (built
        once per buffer pair: the step's host time is the DP path's budget too)."""
        key = (k, net.grad_flat.data_ptr(), net.stats.data_ptr())
        views = getattr(self, '_views', None)
        if views is None:
            views = self._views = {}
        ts = views.get(key)
        if ts is None:
            ts = [net.grad_flat[a:b] for a, b in self.ranges[k]]
            if k == 0:
                ts.append(net.stats[:3])
            views[key] = ts
        return ts


def init(backend=None, device_type='cuda'):
    """Read RANK / LOCAL_RANK / WORLD_SIZE (torch.distributed.run), bind the GPU, and join
    the process group when WORLD_SIZE > 1."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if device_type == 'cuda':
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        backend = backend or ('nccl' if device_type == 'cuda' else 'gloo')
        if backend == 'nccl':
            dist.init_process_group(backend, device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    return DPContext(world, rank, local)
