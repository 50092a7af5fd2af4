"""The shipped configurations through the HIP path at their real dimensions (BASELINE.json
configs): arch5 (LC 80->80 upsampled x[4,4,4,4] = hop 256, GC 16/376,
tmodel.py:68-83, :150-160, par/arch5.json:2-15) and arch1 (n_post1 key, GC 17/377,
par/arch1.json:2-10), forward + loss + backward against the float64 oracle.

Bars as tests/test_gpu_parity.py: z within 1e-5 absolute on identical inputs (north_star),
5e-5 end to end through 50 layers, SAVE 1e-5, n_valid exact, gradients 2e-4 of scale."""
import os

import numpy as np
import pytest
import torch

from lbwn.arch import load_arch
from oracle import wavenet_ref as R
from tests.conftest import ROOT
from tests.test_gpu_parity import close, make_net, oracle_params

pytestmark = pytest.mark.gpu


def _arch(name, gc=None):
    return load_arch(os.path.join(ROOT, 'par', name + '.json'), num_global_cond=gc)


def _batch(arch, B, T, seed):
    """Voice ids change at 'file' boundaries with F-1 masked samples after each, like the
    dealer's output (data.py:133, :156-159)."""
    rng = np.random.default_rng(seed)
    q = rng.integers(0, arch['n_quant'], size=(B, T)).astype(np.int32)
    ncat = max(1, arch['n_gc_category'])
    ids = np.empty((B, T), np.int32)
    for b in range(B):
        cuts = np.sort(rng.choice(np.arange(64, T - 64), 3, replace=False))
        v = rng.integers(1, ncat + 1, 4)
        ids[b] = np.repeat(v, np.diff(np.r_[0, cuts, T]))
        ids[b, :37] = 0
        ids[b, cuts[1]:cuts[1] + 50] = 0
    hop = int(np.prod(arch['lc_upsample'])) if arch['n_lc_out'] else 0
    mel = rng.standard_normal((B, T // hop, arch['n_lc_in'])).astype(np.float32) if hop else None
    return q, ids, mel


def _check_config(arch, B, T, seed=0, grads=True, z_identical=True):
    net = make_net(arch, B, seed=seed)
    q, ids, mel = _batch(arch, B, T, seed)
    P, S = oracle_params(net)
    lg, cache, new_save = R.forward(arch, P, q, ids, S, mel=mel)
    st, dlog = R.loss_fcn(arch, P, lg, q, ids, 0.0)
    net.forward(q, mel, ids, backward=grads)
    torch.cuda.synchronize()
    assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0, 'chain hand-off timed out'
    stats = net.stats.cpu().numpy()
    assert int(stats[1]) == st['n_valid']
    # Σ|argmax diff|: exact except where the top two logits are within fp32 noise (narrow heads
    # such as arch2's n_post 6 give near-flat logits): each such position may move by <= Q-1
    lgv = lg[:, :-1]
    srt = np.sort(lgv, axis=2)
    amb = ((srt[..., -1] - srt[..., -2]) <= 1e-5 * max(1.0, np.abs(lgv).max())) & (ids[:, 1:] != 0)
    assert abs(int(stats[2]) - st['sum_absdiff']) <= (arch['n_quant'] - 1) * int(amb.sum()), int(amb.sum())
    if not amb.any():
        assert int(stats[2]) // (B * (T - 1)) == st['avg_diff']
    np.testing.assert_allclose(stats[0] / st['n_valid'], st['mean_xent'], rtol=1e-5)
    for k, v in new_save.items():
        close(net.save_vars[k].cpu().numpy(), v, 1e-5, k)
    if grads:
        G = R.backward(arch, P, cache, dlog, 0.0)
        inv = 1.0 / st['n_valid']
        for name in net.layout.names():
            close(net.grads[name].cpu().double().numpy() * inv, G[name], 2e-4, name)
    if not z_identical:
        return
    # fresh forward from the original SAVE: every layer's z on identical inputs (the GPU's own
    # x_l, halo = SAVE; GC rows and the upsampled LC from the oracle), then end to end
    net2 = make_net(arch, B, seed=seed)
    net2.forward(q, mel, ids, backward=False)
    torch.cuda.synchronize()
    L, Cd, Cr = R.n_layers(arch), arch['n_dil'], arch['n_res']
    H, M = 2 ** (arch['n_block_layers'] - 1), B * T
    z = net2.plan_tensor(T, 'z').view(M, L * Cd).cpu().numpy()
    xs = net2.plan_tensor(T, 'x')
    stride = xs.numel() // L
    emb, lc = cache['emb'], cache['lc']
    for l, b, bl, d in ((l,) + R.layer_index(arch, l) for l in range(L)):
        xb = xs[l * stride:l * stride + B * (H + T) * Cr].view(B, H + T, Cr).cpu().double().numpy()
        sfx = '_%d_%d' % (b, bl)
        prev, x = xb[:, H - d:H - d + T], xb[:, H:]
        v = {}
        for nm in ('SIGNAL', 'GATE'):
            v[nm] = prev @ P[nm + sfx][0] + x @ P[nm + sfx][1] + P[nm + '_BIAS' + sfx]
            if emb is not None:
                v[nm] = v[nm] + emb @ P['GC_' + nm + sfx]
            if lc is not None:
                v[nm] = v[nm] + lc @ P['LC_' + nm + sfx]
        zl = np.tanh(v['SIGNAL']) * R._sigmoid(v['GATE'])
        np.testing.assert_allclose(z[:, l * Cd:(l + 1) * Cd], zl.reshape(M, Cd), rtol=0, atol=1e-5,
                                   err_msg='z layer %d (identical inputs)' % l)
        np.testing.assert_allclose(z[:, l * Cd:(l + 1) * Cd], cache['z'][l].reshape(M, Cd), rtol=0, atol=5e-5,
                                   err_msg='z layer %d (end to end)' % l)
    s = net2.plan_tensor(T, 's').view(M, -1).cpu().numpy()
    close(s, cache['S'].reshape(M, -1), 1e-5, 'skip sum')


def test_arch5_deep_stack(chain_tile):
    """C4 dims at B=2, T=1024: 4 mel frames per stream through the 4-stage upsample."""
    arch = _arch('arch5')
    assert arch['n_lc_in'] == arch['n_lc_out'] == 80 and arch['lc_upsample'] == [4, 4, 4, 4]
    assert arch['n_gc_embed'] == 16 and arch['n_gc_category'] == 376
    _check_config(arch, 2, 1024)


def test_arch5_one_mel_hop(chain_tile):
    """arch5 at T = 256 = one mel hop per stream (B=2): every d >= 256 layer (d = 256, 512 in
    each of the 5 blocks) reads only SAVE through its dilated tap and keeps old SAVE rows
    (tmodel.py:122-127, :163-166), with the LC term of a single upsampled frame."""
    _check_config(_arch('arch5'), 2, 256, seed=2)


def test_arch5_tile_rounds(chain_tile):
    """arch5 with more 128-position tiles (4 x 66 = 264) than CUs, so the persistent chains
    run in rounds, at T = 8448 = 33 mel hops."""
    _check_config(_arch('arch5'), 4, 8448, seed=1, z_identical=False)


def test_arch1_forward_loss(chain_tile):
    """C1: arch1 (par/arch1.json, n_post1 normalised to n_post, GC 17/377, no use_bias key
    -> True), B=2, T=512 forward + loss + gradients."""
    arch = _arch('arch1')
    assert arch['n_post'] == 512 and arch['n_gc_embed'] == 17 and arch['n_gc_category'] == 377
    _check_config(arch, 2, 512)


def test_arch4_with_gc_override():
    """par/arch4.json lacks n_gc_category: -gc supplies it (train.py:77-80, :138-146)."""
    arch = _arch('arch4', gc=10)
    _check_config(arch, 2, 512, z_identical=False)


def test_arch2_tiny_stack():
    """par/arch2.json (n_res 3, n_dil 4, n_skip 8, n_post 6, GC 16 with -gc; par/arch2.json:5-8):
    odd channel counts on the per-layer kernels, n_post 6 through the zero-padded head."""
    arch = _arch('arch2', gc=10)
    assert (arch['n_res'], arch['n_dil'], arch['n_skip'], arch['n_post']) == (3, 4, 8, 6)
    _check_config(arch, 2, 512)
