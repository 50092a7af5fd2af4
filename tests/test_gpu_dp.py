"""The data-parallel reduction's device path (lbwn/dist.py DPContext.reduce_grads)
on the real training plan, on one GPU.

The CUDA branch reduces the head bucket in place on a comm stream that waits on the plan's "head_grads"
point (lbwn_plan_stream_wait) while the backward's tail (dSKIP, the slab reduction, dPRE, the
conditioning gradients) still runs on the main and side streams, and the side bucket (PRE,
SIGNAL, GATE, RESIDUAL, GC and their biases) at "side_grads" while dSKIP may still run.  An early event, or a tail
kernel writing into a head range, would corrupt the gradients silently; so would a missing wait
before Adam.  The collective itself is replaced by an exact stand-in (x2 on the stream it is
called on: the ring's SUM over two identical ranks), so the test needs no second GPU and every
comparison is bitwise.  Basis: the independent slots of data.py:210-224."""
import os

import numpy as np
import pytest
import torch

from lbwn import dist as lbdist
from lbwn.arch import load_arch
from lbwn.optim import AdamOptimizer
from tests.conftest import ROOT
from tests.test_gpu_configs import _batch as _batch_mixed
from tests.test_gpu_parity import make_net

pytestmark = pytest.mark.gpu


def _batch(arch, B, T, seed):
    """As the configs tests' batch, but with voice ids constant over every 128-position tile
    (file boundaries and masked runs on tile edges): the GC gradient of a mixed tile is
    scattered with float atomics, whose order -- and so the last bits of GC_EMBED's
    gradient -- differs run to run, which a bitwise comparison must not see."""
    q, ids, mel = _batch_mixed(arch, B, T, seed)
    ids = np.repeat(ids[:, ::128], 128, axis=1)[:, :T]
    return q, ids, mel


def _diff_names(net, a, b):
    """Parameter names whose gradient bits differ between flat buffers a and b."""
    return [n for n, e in net.layout.entries.items()
            if np.any(a[e.offset:e.offset + e.numel] != b[e.offset:e.offset + e.numel])]


def _fake_all_reduce(t, op=None, group=None, async_op=False):
    """SUM (x2) or MAX (identity) over two identical ranks, enqueued on the current stream (as RCCL
    would be)."""
    assert t.is_cuda
    if op is None or op == lbdist.dist.ReduceOp.SUM:
        t.mul_(2.0)
    else:
        assert op == lbdist.dist.ReduceOp.MAX


def _bits(t):
    return t.detach().contiguous().view(torch.int32).cpu().numpy()


@pytest.fixture
def dp2(monkeypatch):
    monkeypatch.setattr(lbdist.dist, 'all_reduce', _fake_all_reduce)
    return lbdist.DPContext(world=2, rank=0, local_rank=0)


@pytest.mark.parametrize('name,B,T', [('arch3', 4, 4096), ('arch5', 4, 4096)])
def test_dp_device_path_bucketed_equals_flat(name, B, T, dp2, monkeypatch):
    """Per step: the bucketed reduction (comm stream, head bucket after the backward chain, side
    bucket after the side stream's gradient kernels) == the flat one-message reduction after a
    full synchronize, bitwise, for the gradients, the loss stats and the status word;
    "head_grads" and "side_grads" are real wait points for arch3 and arch5."""
    arch = load_arch(os.path.join(ROOT, 'par', name + '.json'))
    net = make_net(arch, B, seed=2)
    q, ids, mel = _batch(arch, B, T, 5)
    waits = []
    real_wait = net.wait_point
    monkeypatch.setattr(net, 'wait_point', lambda p, s: waits.append(real_wait(p, s)) or waits[-1])
    save0 = net.save_flat.clone()

    net.forward(q, mel, ids)
    dp2.reduce_grads(net)
    torch.cuda.synchronize()
    assert waits == [True, True], 'head_grads and side_grads must be wait points of the %s chain plan' % name
    g_a, s_a, w_a = _bits(net.grad_flat), net.stats[:3].cpu().numpy(), _bits(net.status_word())

    net.save_flat.copy_(save0)                    # same D-sep state -> the same step again
    net.forward(q, mel, ids)
    torch.cuda.synchronize()
    g_raw = net.grad_flat.clone()
    s_raw = net.stats[:3].clone()
    dp2.reduce_grads_flat(net)
    torch.cuda.synchronize()
    assert np.array_equal(_bits(g_raw * 2.0), _bits(net.grad_flat)), 'flat reduction is not exact x2'
    assert np.array_equal(g_a, _bits(net.grad_flat)), 'bucketed != flat (a head range raced the tail): %s' % (
        _diff_names(net, g_a, _bits(net.grad_flat))[:12],)
    assert np.array_equal(s_a, net.stats[:3].cpu().numpy())
    assert np.array_equal(s_a, (s_raw * 2.0).cpu().numpy())
    assert w_a[0] == _bits(net.status_word())[0] == 0


@pytest.mark.parametrize('name,B,T', [('arch3', 4, 4096), ('arch5', 4, 4096)])
def test_dp_device_path_steps_match_single_process(name, B, T, dp2):
    """Three training steps through reduce_grads + TF1 Adam with the x2 stand-in equal three
    plain single-process steps bitwise: Adam divides the doubled gradient by the doubled
    n_valid, (2g)/(2n) == g/n exactly, so any ordering fault (Adam reading a bucket before its
    unpack, a pack reading a gradient before the tail wrote it) shows as a bit difference."""
    arch = load_arch(os.path.join(ROOT, 'par', name + '.json'))
    batches = [_batch(arch, B, T, 10 + k) for k in range(3)]
    out = []
    for use_dp in (False, True):
        net = make_net(arch, B, seed=4)
        opt = AdamOptimizer(1e-3)
        for q, ids, mel in batches:
            net.forward(q, mel, ids)
            if use_dp:
                dp2.reduce_grads(net)
            opt.apply(net)
        torch.cuda.synchronize()
        net.check_status()
        out.append((_bits(net.flat), _bits(net.save_flat), net.counters.cpu().numpy()))
    (w0, s0, c0), (w1, s1, c1) = out
    assert np.array_equal(w0, w1), '%d weights differ' % int((w0 != w1).sum())
    assert np.array_equal(s0, s1)
    assert c0[0] == c1[0] == 3 and c0[3] == c1[3] == 0
    assert c1[1] == 2 * c0[1]                      # VALID_SAMPLES counts the global n_valid


def test_dp_device_path_real_rccl_one_rank(monkeypatch):
    """The CUDA branch of reduce_grads through the real RCCL collective (a one-rank "nccl" process
    group on 127.0.0.1; SUM over one rank is the identity): the comm stream, the head_grads /
    side_grads wait points, the three buckets' pack -> all_reduce -> unpack with RCCL's own kernels
    on the device, and the main stream's wait before the optimizer.  Gradients, stats and the status
    word equal the un-reduced step's bitwise, and three steps with it equal three plain steps."""
    import socket
    import torch.distributed as tdist
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    tdist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1,
                             device_id=torch.device('cuda', 0))
    try:
        monkeypatch.setattr(lbdist.DPContext, 'enabled', property(lambda self: True))
        ctx = lbdist.DPContext(world=1, rank=0, local_rank=0)
        arch = load_arch(os.path.join(ROOT, 'par', 'arch5.json'))
        B, T = 2, 4096
        net = make_net(arch, B, seed=3)
        q, ids, mel = _batch(arch, B, T, 9)
        save0 = net.save_flat.clone()
        net.forward(q, mel, ids)
        torch.cuda.synchronize()
        g_raw, s_raw, w_raw = _bits(net.grad_flat), net.stats[:3].cpu().numpy(), _bits(net.status_word())
        net.save_flat.copy_(save0)
        net.forward(q, mel, ids)
        ctx.reduce_grads(net)
        torch.cuda.synchronize()
        assert np.array_equal(g_raw, _bits(net.grad_flat)), _diff_names(net, g_raw, _bits(net.grad_flat))[:12]
        assert np.array_equal(s_raw, net.stats[:3].cpu().numpy())
        assert w_raw[0] == _bits(net.status_word())[0] == 0
        out = []
        for use_dp in (False, True):
            net = make_net(arch, B, seed=4)
            opt = AdamOptimizer(1e-3)
            for k in range(3):
                q, ids, mel = _batch(arch, B, T, 20 + k)
                net.forward(q, mel, ids)
                if use_dp:
                    ctx.reduce_grads(net)
                opt.apply(net)
            torch.cuda.synchronize()
            net.check_status()
            out.append(_bits(net.flat))
        assert np.array_equal(out[0], out[1]), '%d weights differ' % int((out[0] != out[1]).sum())
    finally:
        tdist.destroy_process_group()
