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


STATUS_BITS = 8     # the plan's status word uses bits 0-1 (lbwn.h); 8 leave room


def status_to_bits(word, out):
    """int32 status word [1] -> one float per bit [STATUS_BITS], so that the all_reduce SUM of
    the ranks' words is an OR per bit once thresholded (a SUM of the words themselves would
    turn two ranks' bit 0 into bit 1 and blame the wrong chain)."""
    sh = torch.arange(STATUS_BITS, dtype=torch.int32, device=word.device)
    out.copy_(((word.view(torch.int32) >> sh) & 1).to(torch.float32))


def bits_to_status(bits, word):
    """Inverse of status_to_bits after the reduction: bit k set if any rank set it."""
    sh = torch.arange(STATUS_BITS, dtype=torch.int32, device=word.device)
    word.view(torch.int32).copy_(((bits > 0).to(torch.int32) << sh).sum(dtype=torch.int32).view(1))


class DPContext:
    def __init__(self, world=1, rank=0, local_rank=0):
        self.world, self.rank, self.local_rank = world, rank, local_rank

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
        the OR of the step status words (a timed-out chain on ANY rank makes every rank's
        optimizer skip the step on the device, so no rank applies garbage gradients; the bits
        travel as per-bit counts, status_to_bits).

        Three buckets, each ONE message (a staging copy of its flat ranges):
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
                plan.pack(k, net)
                dist.all_reduce(plan.buf[k])
                plan.unpack(k, net)
            return
        main = torch.cuda.current_stream(net.grad_flat.device)
        comm = self._comm_stream(net.grad_flat.device)
        # each bucket waits for its point of the backward, or for the whole backward when the
        # plan has no such point (the comm stream's order keeps the buckets' all-reduces serial)
        for k, point in enumerate(('head_grads', 'side_grads', None)):
            if not plan.ranges[k] and k > 0:
                continue
            if point is None or not net.wait_point(point, comm):
                comm.wait_stream(main)
            with torch.cuda.stream(comm):
                plan.pack(k, net)
                dist.all_reduce(plan.buf[k])
                plan.unpack(k, net)
        main.wait_stream(comm)

    def reduce_grads_flat(self, net):
        """The whole gradient + stats + status as one message after the backward (the reference
        bucketing of tests/test_dropin.py::test_dp_bucketed_equals_flat)."""
        if not self.enabled:
            return
        n = net.grad_flat.numel()
        buf = torch.empty(n + 3 + STATUS_BITS, dtype=torch.float32, device=net.grad_flat.device)
        sw = net.status_word()
        buf[:n].copy_(net.grad_flat)
        buf[n:n + 3].copy_(net.stats[:3])
        status_to_bits(sw, buf[n + 3:])
        dist.all_reduce(buf)
        net.grad_flat.copy_(buf[:n])
        net.stats[:3].copy_(buf[n:n + 3])
        bits_to_status(buf[n + 3:], sw)

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


class _Buckets:
    """Flat ranges of the two all-reduce buckets (lbwn.arch.ParamLayout: weights
    [pre, sig, gate, res, skip, gc.., lc.., post1, post2] then biases [pre_b, sig_b, gate_b,
    res_b, skip_b, post1_b, post2_b]) and their staging buffers."""

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
        sizes = [sum(b - a for a, b in head) + 3 + STATUS_BITS] + [sum(b - a for a, b in r) for r in (side, rest)]
        self.buf = [torch.empty(n, dtype=torch.float32, device=net.grad_flat.device) for n in sizes]

    @staticmethod
    def of(net):
        b = getattr(net, '_dp_buckets', None)
        if b is None or b.buf[0].device != net.grad_flat.device:
            b = _Buckets(net)
            net._dp_buckets = b
        return b

    def pack(self, k, net):
        o = 0
        for a, b in self.ranges[k]:
            self.buf[k][o:o + b - a].copy_(net.grad_flat[a:b])
            o += b - a
        if k == 0:
            self.buf[0][o:o + 3].copy_(net.stats[:3])
            status_to_bits(net.status_word(), self.buf[0][o + 3:])

    def unpack(self, k, net):
        o = 0
        for a, b in self.ranges[k]:
            net.grad_flat[a:b].copy_(self.buf[k][o:o + b - a])
            o += b - a
        if k == 0:
            net.stats[:3].copy_(self.buf[0][o:o + 3])
            bits_to_status(self.buf[0][o + 3:], net.status_word())


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
