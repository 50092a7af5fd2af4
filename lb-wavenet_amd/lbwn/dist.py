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
        """Σ over ranks of the raw gradient buffer and of (Σxent, n_valid, Σ|argmax diff|).
        stats and grads go as ONE flat message (6–8 MB for arch3/arch5: a single ring
        all_reduce is ≤0.1 ms on xGMI, so no bucketing is needed at this size)."""
        if not self.enabled:
            return
        n = net.grad_flat.numel()
        buf = self._buf(net)
        buf[:n].copy_(net.grad_flat)
        buf[n:n + 3].copy_(net.stats[:3])
        dist.all_reduce(buf)
        net.grad_flat.copy_(buf[:n])
        net.stats[:3].copy_(buf[n:n + 3])

    def _buf(self, net):
        key = '_dp_buf'
        b = getattr(net, key, None)
        if b is None or b.numel() != net.grad_flat.numel() + 4:
            b = torch.empty(net.grad_flat.numel() + 4, dtype=torch.float32, device=net.grad_flat.device)
            setattr(net, key, b)
        return b

    def max_over_ranks(self, value, device):
        if not self.enabled:
            return value
        t = torch.tensor([value], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        if self.enabled:
            dist.barrier()


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
