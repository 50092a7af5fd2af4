"""Full-size parity for the configurations the oracle tests run scaled down: C4 = arch5 B=32
T=4096 (BASELINE configs[3]; tests/test_gpu_configs.py runs it at B <= 4) and C2 = arch3 B=8
T=4096, against a float64 restatement of the oracle's forward and loss (oracle/wavenet_ref.py
forward / loss_fcn: tmodel.py:68-83, :117-215, :228-249) written in torch so that it finishes in
seconds at full size on the GPU, with torch autograd as the backward (TF's autodiff of the same
graph, tmodel.py:354-358).  The numpy oracle pins this restatement at small sizes
(test_restatement_matches_oracle).  Torch is only the checker here: every value under test comes
from the HIP path (lbwn_train_forward / lbwn_train_backward).

Bars as tests/test_gpu_parity.py: z within 1e-5 on identical inputs (north_star), 5e-5 end to end,
SAVE 1e-5, n_valid exact, mean xent 1e-5, gradients 2e-4 of scale."""
import numpy as np
import pytest
import torch

from oracle import wavenet_ref as R
from tests.test_gpu_configs import _arch, _batch
from tests.test_gpu_parity import close, make_net, oracle_params

pytestmark = pytest.mark.gpu


def torch_forward(arch, P, q, ids, S, mel, keep_x=False):
    """oracle/wavenet_ref.py forward (tmodel.py:292-327) in float64 torch; P, S: {name: tensor}
    (requires_grad where gradients are wanted).  Returns logits [B,T,Q], the per-layer z, the
    skip sum, the new SAVE rows and (keep_x) each layer's input x."""
    B, T = q.shape
    L = R.n_layers(arch)
    ub = arch['use_bias']
    x = P['PRE'][q]
    if ub:
        x = x + P['PRE_BIAS']
    lc = None
    if arch['n_lc_out'] > 0:
        lc = mel
        for i, s in enumerate(arch['lc_upsample']):      # tmodel.py:68-83, non-overlapping transpose conv
            F = P['LC_UPSAMPLE_%d' % i]                   # [s, O, I]
            b_, t_, _ = lc.shape
            lc = torch.einsum('bti,joi->btjo', lc, F).reshape(b_, t_ * s, F.shape[1])
    emb = P['GC_EMBED'][ids] if arch['n_gc_embed'] > 0 else None
    Ssum = 0
    zs, xs, new_save = [], [], {}
    for l in range(L):
        b, bl, d = R.layer_index(arch, l)
        sfx = '_%d_%d' % (b, bl)
        full = torch.cat([S['SAVE_%d%s' % (d, sfx)], x], dim=1)
        prev = full[:, :T]
        v = {}
        for nm in ('SIGNAL', 'GATE'):
            W = P[nm + sfx]
            v[nm] = prev @ W[0] + x @ W[1]
            if ub:
                v[nm] = v[nm] + P[nm + '_BIAS' + sfx]
            if emb is not None:
                v[nm] = v[nm] + emb @ P['GC_' + nm + sfx]
            if lc is not None:
                v[nm] = v[nm] + lc @ P['LC_' + nm + sfx]
        new_save['SAVE_%d%s' % (d, sfx)] = full[:, -d:].detach()
        z = torch.tanh(v['SIGNAL']) * torch.sigmoid(v['GATE'])
        res = z @ P['RESIDUAL' + sfx]
        skp = z @ P['SKIP' + sfx]
        if ub:
            res = res + P['RESIDUAL_BIAS' + sfx]
            skp = skp + P['SKIP_BIAS' + sfx]
        zs.append(z.detach())
        if keep_x:
            xs.append(x.detach())
        Ssum = Ssum + skp
        x = x + res
    h1 = torch.relu(Ssum) @ P['POST1']
    if ub:
        h1 = h1 + P['POST1_BIAS']
    logits = torch.relu(h1) @ P['POST2']
    if ub:
        logits = logits + P['POST2_BIAS']
    return logits, zs, Ssum.detach(), new_save, xs


def torch_sum_xent(logits, q, ids):
    """Σ over valid positions of softmax cross-entropy (tmodel.py:228-249; the HIP path's
    gradients are of this sum, the oracle's of the mean)."""
    lg = logits[:, :-1]
    tgt = q[:, 1:].long()
    mask = (ids[:, 1:] != 0)
    xent = torch.logsumexp(lg, dim=2) - torch.gather(lg, 2, tgt[..., None])[..., 0]
    return (xent * mask).sum(), int(mask.sum())


def _grad(p):
    return p.grad.cpu().numpy() if p.grad is not None else np.zeros(tuple(p.shape))


def _tensors(net, q, ids, mel, dev, grad):
    P0, S0 = oracle_params(net)
    P = {k: torch.tensor(v, device=dev, requires_grad=grad) for k, v in P0.items()}
    S = {k: torch.tensor(v, device=dev) for k, v in S0.items()}
    qt = torch.tensor(q, device=dev, dtype=torch.long)
    it = torch.tensor(ids, device=dev, dtype=torch.long)
    mt = torch.tensor(mel, device=dev, dtype=torch.float64) if mel is not None else None
    return P0, S0, P, S, qt, it, mt


def test_restatement_matches_oracle():
    """The torch restatement equals the numpy oracle (forward, loss, gradients) on a small
    arch5 case, so the full-size comparisons below inherit the oracle's pinning."""
    arch = _arch('arch5')
    B, T = 2, 512
    net = make_net(arch, B, seed=3)
    q, ids, mel = _batch(arch, B, T, 3)
    P0, S0, P, S, qt, it, mt = _tensors(net, q, ids, mel, 'cuda', True)
    lg, cache, new_save = R.forward(arch, P0, q, ids, S0, mel=mel)
    st, dlog = R.loss_fcn(arch, P0, lg, q, ids, 0.0)
    G = R.backward(arch, P0, cache, dlog, 0.0)
    tl, zs, Ss, ns, _ = torch_forward(arch, P, qt, it, S, mt)
    np.testing.assert_allclose(tl.detach().cpu().numpy(), lg, rtol=0, atol=1e-10)
    for k, v in new_save.items():
        np.testing.assert_allclose(ns[k].cpu().numpy(), v, rtol=1e-12, atol=1e-12)
    sx, nv = torch_sum_xent(tl, qt, it)
    assert nv == st['n_valid']
    (sx / nv).backward()
    for k, g in G.items():   # (the last layer's RESIDUAL feeds nothing: no autograd edge, zero gradient)
        close(_grad(P[k]), g, 1e-10, k)


@pytest.mark.parametrize('arch_name,B', [('arch5', 32), ('arch3', 8)])
def test_full_size_forward_backward(arch_name, B, chain_tile):
    """C4 (arch5, B=32) and C2 (arch3, B=8) at T=4096: every layer's z on the HIP path's own
    inputs, z end to end, the skip sum, SAVE, n_valid, mean xent and every gradient."""
    _full_size(arch_name, B)


def test_full_size_c5_per_gpu():
    """C5's per-GPU share (arch5, B=8, T=4096: the shape each rank of the 8-GPU data-parallel
    config trains) at full size, default chain form: its LC backward takes the fused upsample
    backward (128 mel frames; C4's 512 run the per-stage GEMMs) and dlc's deferred split-K
    partials, which C4 does not exercise."""
    _full_size('arch5', 8)


def _full_size(arch_name, B):
    arch = _arch(arch_name)
    T = 4096
    q, ids, mel = _batch(arch, B, T, 11)
    net = make_net(arch, B, seed=11)
    P0, S0, P, S, qt, it, mt = _tensors(net, q, ids, mel, 'cuda', True)
    tl, zs, Ss, ns, _ = torch_forward(arch, P, qt, it, S, mt)
    sx, nv = torch_sum_xent(tl, qt, it)
    sx.backward()
    del tl

    # forward only: z on identical inputs (the plan's own layer inputs x_l, halo = SAVE, through
    # a float64 dilated conv + gate), z end to end, the skip sum, SAVE, n_valid, mean xent
    net.forward(q, mel, ids, backward=False)
    torch.cuda.synchronize()
    assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0, 'chain hand-off timed out'
    stats = net.stats.cpu().numpy()
    assert int(stats[1]) == nv
    np.testing.assert_allclose(stats[0] / nv, float(sx) / nv, rtol=1e-5)
    for k, v in ns.items():
        close(net.save_vars[k].cpu().numpy(), v.cpu().numpy(), 1e-5, k)
    L, Cd, Cr = R.n_layers(arch), arch['n_dil'], arch['n_res']
    H, M = 2 ** (arch['n_block_layers'] - 1), B * T
    z = net.plan_tensor(T, 'z').view(M, L * Cd).double()
    xall = net.plan_tensor(T, 'x')
    stride = xall.numel() // L
    with torch.no_grad():
        Pd = {k: v.detach() for k, v in P.items()}
        emb = Pd['GC_EMBED'][it] if arch['n_gc_embed'] > 0 else None
        lc = None
        if arch['n_lc_out'] > 0:
            lc = mt
            for i, s in enumerate(arch['lc_upsample']):
                F = Pd['LC_UPSAMPLE_%d' % i]
                b_, t_, _ = lc.shape
                lc = torch.einsum('bti,joi->btjo', lc, F).reshape(b_, t_ * s, F.shape[1])
        for l in range(L):
            b, bl, d = R.layer_index(arch, l)
            sfx = '_%d_%d' % (b, bl)
            xb = xall[l * stride:l * stride + B * (H + T) * Cr].view(B, H + T, Cr).double()
            prev, x = xb[:, H - d:H - d + T], xb[:, H:]
            v = {}
            for nm in ('SIGNAL', 'GATE'):
                v[nm] = prev @ Pd[nm + sfx][0] + x @ Pd[nm + sfx][1] + Pd[nm + '_BIAS' + sfx]
                if emb is not None:
                    v[nm] = v[nm] + emb @ Pd['GC_' + nm + sfx]
                if lc is not None:
                    v[nm] = v[nm] + lc @ Pd['LC_' + nm + sfx]
            zl = (torch.tanh(v['SIGNAL']) * torch.sigmoid(v['GATE'])).reshape(M, Cd)
            zg = z[:, l * Cd:(l + 1) * Cd]
            e1 = float((zg - zl).abs().max())
            e2 = float((zg - zs[l].reshape(M, Cd)).abs().max())
            assert e1 <= 1e-5, 'z layer %d (identical inputs): %.3g' % (l, e1)
            assert e2 <= 5e-5, 'z layer %d (end to end): %.3g' % (l, e2)
        s = net.plan_tensor(T, 's').view(M, -1).double()
        close(s.cpu().numpy(), Ss.reshape(M, -1).cpu().numpy(), 1e-5, 'skip sum')
    del net, z, xall, s

    # forward + backward from the same initial state: every gradient of the summed xent
    net = make_net(arch, B, seed=11)
    net.forward(q, mel, ids, backward=True)
    torch.cuda.synchronize()
    assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0, 'chain hand-off timed out'
    scale = 1.0 / nv
    for name in net.layout.names():
        close(net.grads[name].double().cpu().numpy() * scale, _grad(P[name]) * scale, 2e-4, name)
