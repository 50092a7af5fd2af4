"""HIP path vs the CPU oracle (float64), through the C-ABI.  Tolerances: 1e-5 absolute on
conv activations z (north_star), relative 1e-4 (scaled by the tensor's max) on deeper
quantities that accumulate 50 layers of fp32 rounding; bit-exact on integer/mask work."""
import ctypes
import os

import numpy as np
import pytest
import torch

from lbwn import _lib
from lbwn.arch import load_arch, normalize_arch
from lbwn.optim import AdamOptimizer
from lbwn.tmodel import WaveNetTrain
from oracle import wavenet_ref as R
from tests.conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def arch3():
    return load_arch(os.path.join(ROOT, 'par', 'arch3.json'))


def small_arch(nb=2, nbl=4, Cr=32, Cd=32, Cs=64, Cp=32, Q=256):
    return normalize_arch(dict(n_blocks=nb, n_block_layers=nbl, n_quant=Q, n_res=Cr, n_dil=Cd, n_skip=Cs,
                               n_post=Cp, n_gc_embed=0, n_gc_category=0, use_bias=True))


def make_net(arch, B, seed=0, bias_scale=0.1, l2=1e-3):
    net = WaveNetTrain(**arch, batch_sz=B, l2_factor=l2, print_interval=0, seed=seed)
    net.init_vars(seed, bias_scale=bias_scale)
    return net


def oracle_params(net):
    P = {n: v.detach().cpu().double().numpy() for n, v in net.vars.items()}
    S = {n: v.detach().cpu().double().numpy() for n, v in net.save_vars.items()}
    return P, S


def rand_batch(arch, B, T, seed=0, invalid=37):
    rng = np.random.default_rng(seed)
    q = rng.integers(0, arch['n_quant'], size=(B, T)).astype(np.int32)
    ids = np.ones((B, T), np.int32)
    ids[:, :invalid] = 0
    if B > 1:
        ids[1, T // 2:T // 2 + 11] = 0
    return q, ids


def close(a, b, rel, name=''):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(1.0, float(np.max(np.abs(b))))
    err = float(np.max(np.abs(a - b))) if a.size else 0.0
    assert err <= rel * scale, '%s: max err %.3g > %.3g (scale %.3g)' % (name, err, rel * scale, scale)


# ---- GEMM ------------------------------------------------------------------------------

@pytest.fixture
def gemm_mode(lib):
    """Set the GEMM arithmetic for one test (1 = bf16 split, 0 = f32 MFMA), then restore it."""
    old = lib.lbwn_gemm_get_mode()
    yield lambda m: _lib.check(lib.lbwn_gemm_set_mode(m))
    _lib.check(lib.lbwn_gemm_set_mode(old))


@pytest.mark.parametrize('akc,bkc', [(1, 0), (1, 1), (0, 0), (0, 1)])
@pytest.mark.parametrize('split', [1, 3])
@pytest.mark.parametrize('mode', [1, 0])
def test_gemm_layouts(lib, gemm_mode, akc, bkc, split, mode):
    gemm_mode(mode)
    M, N, K = 300, 136, 200
    g = torch.Generator().manual_seed(1)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    Bm = torch.randn(K, N, generator=g, dtype=torch.float64)
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    mask = (torch.rand(M, N, generator=g) > 0.3).double()
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    ref = torch.relu(torch.relu(A) @ Bm + bias) * mask + C0
    Ad = (A if akc else A.t()).contiguous().float().to(DEV)
    Bd = (Bm.t() if bkc else Bm).contiguous().float().to(DEV)
    Cd = C0.float().to(DEV).contiguous()
    md = mask.float().to(DEV)
    bd = bias.float().to(DEV)
    ws = torch.empty(split * M * N, device=DEV)
    _lib.check(lib.lbwn_gemm_f32(Ad.data_ptr(), K if akc else M, akc, Bd.data_ptr(), K if bkc else N, bkc,
                                 Cd.data_ptr(), N, M, N, K, bd.data_ptr(), 1, 1, md.data_ptr(), N, 1, split,
                                 ws.data_ptr(), None))
    torch.cuda.synchronize()
    close(Cd.cpu().numpy(), ref.numpy(), 1e-5, 'gemm')


@pytest.mark.parametrize('mode', [1, 0])
def test_gemm_large_skip_shape(lib, gemm_mode, mode):
    """The skip GEMM shape (K = 1600, N = 512) against torch fp64."""
    gemm_mode(mode)
    M, N, K = 1024, 512, 1600
    g = torch.Generator().manual_seed(2)
    A = torch.rand(M, K, generator=g, dtype=torch.float64) * 2 - 1
    Bm = (torch.rand(K, N, generator=g, dtype=torch.float64) * 2 - 1) * 0.05
    C = torch.empty(M, N, device=DEV)
    Ad, Bd = A.float().to(DEV), Bm.float().to(DEV)
    _lib.check(lib.lbwn_gemm_f32(Ad.data_ptr(), K, 1, Bd.data_ptr(), N, 0, C.data_ptr(), N, M, N, K, None, 0, 0,
                                 None, 0, 0, 1, None, None))
    torch.cuda.synchronize()
    close(C.cpu().numpy(), (A @ Bm).numpy(), 1e-5, 'gemm_skip')


@pytest.mark.parametrize('M,N,K,bkc,epi', [(8192, 512, 1600, 0, 0), (8200, 136, 96, 1, 1), (8192, 1600, 512, 1, 2),
                                           (9000, 256, 512, 0, 1)])
def test_gemm_presplit_tall(lib, gemm_mode, M, N, K, bkc, epi):
    """The tall products of the training step (M >= 8192, A k-contiguous, B pre-split: the
    A-in-registers kernel) against torch fp64: epi 0 plain, 1 bias + relu(A) + relu + mask +
    accumulate, 2 bias only; ragged M / N tiles included."""
    gemm_mode(1)
    g = torch.Generator().manual_seed(11)
    A = torch.randn(M, K, generator=g, dtype=torch.float64)
    Bm = torch.randn(K, N, generator=g, dtype=torch.float64) * 0.05
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    mask = (torch.rand(M, N, generator=g) > 0.3).double()
    C0 = torch.randn(M, N, generator=g, dtype=torch.float64)
    if epi == 1:
        ref = torch.relu(torch.relu(A) @ Bm + bias) * mask + C0
    elif epi == 2:
        ref = A @ Bm + bias
    else:
        ref = A @ Bm
    Ad = A.float().to(DEV).contiguous()
    Bd = (Bm.t() if bkc else Bm).contiguous().float().to(DEV)
    b3 = torch.empty(int(lib.lbwn_split_planes_elems_abi(N, K)), dtype=torch.int16, device=DEV)
    _lib.check(lib.lbwn_split_planes(Bd.data_ptr(), K if bkc else N, N, K, 0 if bkc else 1, b3.data_ptr(), None))
    Cd = C0.float().to(DEV).contiguous() if epi == 1 else torch.empty(M, N, device=DEV)
    md, bd = mask.float().to(DEV), bias.float().to(DEV)
    _lib.check(lib.lbwn_gemm_f32_presplit(Ad.data_ptr(), K, 1, b3.data_ptr(), N, Bd.data_ptr(), K if bkc else N, bkc,
                                          Cd.data_ptr(), N, M, K, bd.data_ptr() if epi else None, int(epi == 1),
                                          int(epi == 1), md.data_ptr() if epi == 1 else None, N, int(epi == 1), None))
    torch.cuda.synchronize()
    close(Cd.cpu().numpy(), ref.numpy(), 1e-5, 'gemm_presplit')


def _gemm_err(lib, A, Bm, akc, bkc, split):
    M, K = A.shape
    N = Bm.shape[1]
    Ad = (A if akc else A.t()).contiguous().float().to(DEV)
    Bd = (Bm.t() if bkc else Bm).contiguous().float().to(DEV)
    C = torch.empty(M, N, device=DEV)
    ws = torch.empty(split * M * N, device=DEV)
    _lib.check(lib.lbwn_gemm_f32(Ad.data_ptr(), K if akc else M, akc, Bd.data_ptr(), K if bkc else N, bkc,
                                 C.data_ptr(), N, M, N, K, None, 0, 0, None, 0, 0, split, ws.data_ptr(), None))
    torch.cuda.synchronize()
    # reference on the f32-rounded operands: only the GEMM's own arithmetic is measured
    ref = A.float().double() @ Bm.float().double()
    scale = torch.abs(A.float().double()) @ torch.abs(Bm.float().double())
    return float(torch.max(torch.abs(C.cpu().double() - ref) / scale))


@pytest.mark.parametrize('shape', [('skip_fwd', 2048, 512, 1600, 1, 0, 1), ('dz', 1024, 1600, 512, 1, 1, 1),
                                   ('dskip', 1600, 512, 32768, 0, 0, 8)])
def test_gemm_split_accuracy(lib, gemm_mode, shape):
    """The bf16-split GEMM is an f32 GEMM: its error against fp64 (relative to Σ|a·b|) is of the
    f32 MFMA's class.  Operands carry a full 24-bit significand (uniform, random exponents over
    2^±4) so that a 1- or 2-term split, or a bf16 product, would fail by orders of magnitude."""
    name, M, N, K, akc, bkc, split = shape
    g = torch.Generator().manual_seed(5)
    A = (torch.rand(M, K, generator=g, dtype=torch.float64) * 2 - 1) * 2.0 ** torch.randint(-4, 5, (M, K), generator=g)
    Bm = (torch.rand(K, N, generator=g, dtype=torch.float64) * 2 - 1) * 2.0 ** torch.randint(-4, 5, (K, N), generator=g)
    gemm_mode(0)
    e32 = _gemm_err(lib, A, Bm, akc, bkc, split)
    gemm_mode(1)
    ex3 = _gemm_err(lib, A, Bm, akc, bkc, split)
    print('%s: max |err|/sum|ab|  f32 MFMA %.3g  bf16-split %.3g' % (name, e32, ex3))
    assert ex3 <= max(2.0 * e32, 1e-7), (name, e32, ex3)


# ---- one layer ---------------------------------------------------------------------------

@pytest.mark.parametrize('d,T', [(1, 128), (2, 200), (64, 256), (512, 300), (256, 100), (8, 1024)])
@pytest.mark.parametrize('C', [32, 5])
def test_layer_forward(lib, d, T, C):
    B, H = 2, 512
    rng = np.random.default_rng(d + T + C)
    xbuf = rng.uniform(-1, 1, size=(B, H + T, C))
    Ws = rng.uniform(-0.3, 0.3, size=(2, C, C))
    Wg = rng.uniform(-0.3, 0.3, size=(2, C, C))
    bs, bg = rng.uniform(-0.1, 0.1, C), rng.uniform(-0.1, 0.1, C)
    Wr, br = rng.uniform(-0.3, 0.3, size=(C, C)), rng.uniform(-0.1, 0.1, C)
    x = xbuf[:, H:]
    prev = xbuf[:, H - d:H - d + T]
    z = np.tanh(prev @ Ws[0] + x @ Ws[1] + bs) * R._sigmoid(prev @ Wg[0] + x @ Wg[1] + bg)
    xo = x + z @ Wr + br
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=DEV).contiguous()
    xin, ws_, wg_, bs_, bg_, wr_, br_ = map(t, (xbuf, Ws, Wg, bs, bg, Wr, br))
    zout = torch.zeros(B * T, C, device=DEV)
    xout = torch.zeros(B, H + T, C, device=DEV)
    wpk = torch.empty(lib.lbwn_layer_image_floats_abi(), device=DEV)
    _lib.check(lib.lbwn_layer_forward(xin.data_ptr(), xout.data_ptr(), zout.data_ptr(), C, ws_.data_ptr(),
                                      wg_.data_ptr(), bs_.data_ptr(), bg_.data_ptr(), wr_.data_ptr(), br_.data_ptr(),
                                      None, None, None, 0, B, T, H, d, C, C, wpk.data_ptr(), None))
    torch.cuda.synchronize()
    np.testing.assert_allclose(zout.cpu().numpy().reshape(B, T, C), z, rtol=0, atol=1e-5)
    np.testing.assert_allclose(xout.cpu().numpy()[:, H:], xo, rtol=0, atol=2e-5)


# ---- head --------------------------------------------------------------------------------

@pytest.mark.parametrize('Q', [256, 100, 512, 520])
def test_head_xent(lib, Q):
    """Softmax xent head: the register-resident kernel (Q <= 256, <= 512, ragged lanes) and the
    generic one (Q > 512)."""
    B, T = 3, 257
    rng = np.random.default_rng(5)
    lg = rng.normal(size=(B, T, Q)) * 3
    q, ids = rand_batch(dict(n_quant=Q), B, T, invalid=20)
    arch = dict(n_quant=Q)
    st, dlog = R.loss_fcn(arch, {}, lg, q, ids, 0.0)
    lgd = torch.tensor(lg, dtype=torch.float32, device=DEV).contiguous()
    qd = torch.tensor(q, device=DEV)
    idd = torch.tensor(ids, device=DEV)
    stats = torch.zeros(4, device=DEV)
    ws = torch.zeros(3 * 2048, device=DEV)
    _lib.check(lib.lbwn_head_xent(lgd.data_ptr(), qd.data_ptr(), idd.data_ptr(), B, T, Q, 1, stats.data_ptr(),
                                  ws.data_ptr(), None))
    s = stats.cpu().numpy()
    assert int(s[1]) == st['n_valid']
    np.testing.assert_allclose(s[0], st['sum_xent'], rtol=1e-5)
    assert int(s[2]) // (B * (T - 1)) == st['avg_diff']
    assert int(s[2]) == st['sum_absdiff']
    np.testing.assert_allclose(lgd.cpu().numpy() / st['n_valid'], dlog, rtol=0, atol=1e-6)


# ---- mu-law --------------------------------------------------------------------------------

def test_mulaw_gpu_golden(lib):
    g = np.load(os.path.join(GOLDEN, 'mulaw.npz'))
    x = torch.tensor(g['mu_x32'], device=DEV)
    q = torch.empty(x.numel(), dtype=torch.int32, device=DEV)
    _lib.check(lib.lbwn_mulaw_encode(x.data_ptr(), q.data_ptr(), x.numel(), 256, 0, None))
    np.testing.assert_array_equal(q.cpu().numpy(), g['mu_enc32_256'])
    qs = torch.arange(256, dtype=torch.int32, device=DEV)
    out = torch.empty(256, device=DEV)
    _lib.check(lib.lbwn_mulaw_decode(qs.data_ptr(), out.data_ptr(), 256, 256, None))
    np.testing.assert_allclose(out.cpu().numpy(), R.mu_decode_tf32(np.arange(256), 256), rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize('nq', [256, 64])
def test_mulaw_tf32_encode(lib, nq):
    """ops.mu_encode (ops.py:4-9, TF float32 graph) on the golden inputs against the oracle's
    float32 restatement.  Bit-exact, except where the exact (float64) pre-truncation value
    (amp+1)·mu/2+0.5 lies within 4 float32 ulps of an integer: there the truncation depends on
    the last bit of log1pf, which TF (Eigen's plog1p), glibc and ROCm's ocml each round
    differently, so either neighbour is the reference's answer.  Such points are counted and
    must be rare."""
    g = np.load(os.path.join(GOLDEN, 'mulaw.npz'))
    xs = np.concatenate([g['mu_x32'], np.linspace(-1, 1, 20001, dtype=np.float32),
                         np.random.default_rng(3).uniform(-1, 1, 20000).astype(np.float32)])
    x = torch.tensor(xs, device=DEV)
    q = torch.empty(x.numel(), dtype=torch.int32, device=DEV)
    _lib.check(lib.lbwn_mulaw_encode(x.data_ptr(), q.data_ptr(), x.numel(), nq, 1, None))
    got = q.cpu().numpy()
    want = R.mu_encode_tf32(xs, nq)
    mu = nq - 1
    x64 = xs.astype(np.float64)
    exact = (np.sign(x64) * np.log1p(mu * np.abs(x64)) / np.log1p(mu) + 1) * 0.5 * mu + 0.5
    frac = exact - np.round(exact)
    tie = np.abs(frac) <= 4 * np.spacing(np.float32(nq), dtype=np.float32)
    bad = (got != want) & ~tie
    assert not bad.any(), 'tf32 encode differs off-boundary at x=%s' % xs[bad][:8]
    assert np.all(np.abs(got.astype(np.int64) - want) <= 1)
    assert int(tie.sum()) <= 0.01 * xs.size, int(tie.sum())
    assert got.min() >= 0 and got.max() <= mu


# ---- full plan -------------------------------------------------------------------------------

def _run_oracle(arch, net, q, ids):
    P, S = oracle_params(net)
    lg, cache, new_save = R.forward(arch, P, q, ids, S)
    st, dlog = R.loss_fcn(arch, P, lg, q, ids, 0.0)
    return P, S, lg, cache, new_save, st, dlog


@pytest.mark.parametrize('which,B,T,mode', [('small', 2, 256, 1), ('small', 3, 200, 1), ('arch3', 2, 512, 1),
                                            ('arch3', 2, 512, 0), ('arch3', 8, 4096, 1)])
def test_plan_forward_backward(lib, gemm_mode, which, B, T, mode, chain_tile):
    """mode 1: GEMMs and the forward chain's conv/residual on the bf16 cores by exact splitting;
    mode 0: every product on the f32 MFMA.  Same bars for both.  ('arch3', 8, 4096) is the
    benchmarked C2 shape itself: 256 tiles of the persistent chains, every gradient vs float64."""
    gemm_mode(mode)
    check_plan(arch3() if which == 'arch3' else small_arch(), B, T)


@pytest.mark.parametrize('T', [40, 96, 200, 384])
def test_plan_slice_shorter_than_dilation(lib, T, chain_tile):
    """Slices shorter than the dilation (T < d; train.py:43-44 --slice-size is free): the
    reference's SAVE update keeps "the last d rows of [SAVE ++ x]" (tmodel.py:122-127,
    :163-166), so for d > T the new SAVE holds old SAVE rows [T, d) and every dilated tap x[t-d]
    is a SAVE row.  arch3 at B=2: T=96 puts d = 128/256/512 past the slice, T=200 d = 256/512,
    T=384 d = 512, T=40 also d = 64 (and a tile shorter than one 64-lane wave).  Exercises
    the SAVE-from-SAVE rows of the flat D-sep copy (prologue.h dsep_flat_body), the chains'
    halo taps with no producer tile, and the backward's truncation of dprev into the halo
    (the gradient into SAVE is dropped).  Forward + backward against the float64 oracle:
    layer-0 SAVE bit-exact, deeper SAVE 1e-5, z on identical inputs 1e-5, gradients 2e-4."""
    check_plan(arch3(), 2, T)


def check_plan(arch, B, T):
    net = make_net(arch, B)
    q, ids = rand_batch(arch, B, T)
    P, S, lg, cache, new_save, st, dlog = _run_oracle(arch, net, q, ids)
    net.forward(q, None, ids, backward=True)
    torch.cuda.synchronize()
    assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0, 'chain hand-off timed out'
    L, Cd = R.n_layers(arch), arch['n_dil']
    # forward activations (z before backward overwrote it is not kept: compare SAVE / stats /
    # logits-derived quantities, then per-layer z via a fresh forward below)
    stats = net.stats.cpu().numpy()
    assert int(stats[1]) == st['n_valid']
    np.testing.assert_allclose(stats[0] / st['n_valid'], st['mean_xent'], rtol=1e-5)
    for i, (k, v) in enumerate(new_save.items()):
        if i == 0:   # layer 0's SAVE is pure data movement of the embedded input: bit-exact
            np.testing.assert_array_equal(net.save_vars[k].cpu().numpy(), v.astype(np.float32), err_msg=k)
        else:        # deeper layers hold fp32-computed residual activations
            close(net.save_vars[k].cpu().numpy(), v, 1e-5, k)
    # gradients: ours are Σxent-grads (raw); the oracle's are of the mean
    G = R.backward(arch, P, cache, dlog, 0.0)
    inv = 1.0 / st['n_valid']
    for name in net.layout.names():
        ours = net.grads[name].cpu().double().numpy() * inv
        close(ours, G[name], 2e-4, name)
    # fresh forward with the original SAVE: z of every layer, skip sum, logits
    net2 = make_net(arch, B)
    net2.forward(q, None, ids, backward=False)
    torch.cuda.synchronize()
    M = B * T
    z = net2.plan_tensor(T, 'z').view(M, L * Cd).cpu().numpy()
    # (a) north_star bar: conv activations within 1e-5 on IDENTICAL inputs -> feed the
    #     oracle's layer the GPU's own x_l (halo = SAVE) and compare z_l.
    H = 2 ** (arch['n_block_layers'] - 1)
    Cr = arch['n_res']
    xs = net2.plan_tensor(T, 'x')
    stride = xs.numel() // L
    for l, b, bl, d in ((l,) + R.layer_index(arch, l) for l in range(L)):
        xb = xs[l * stride:l * stride + B * (H + T) * Cr].view(B, H + T, Cr).cpu().double().numpy()
        sfx = '_%d_%d' % (b, bl)
        prev, x = xb[:, H - d:H - d + T], xb[:, H:]
        v = {nm: prev @ P[nm + sfx][0] + x @ P[nm + sfx][1] + P[nm + '_BIAS' + sfx] for nm in ('SIGNAL', 'GATE')}
        zl = np.tanh(v['SIGNAL']) * R._sigmoid(v['GATE'])
        np.testing.assert_allclose(z[:, l * Cd:(l + 1) * Cd], zl.reshape(M, Cd), rtol=0, atol=1e-5,
                                   err_msg='z layer %d (identical inputs)' % l)
    # (b) end to end through L layers of fp32 residual accumulation vs float64
    for l in range(L):
        np.testing.assert_allclose(z[:, l * Cd:(l + 1) * Cd], cache['z'][l].reshape(M, Cd), rtol=0, atol=5e-5,
                                   err_msg='z layer %d (end to end)' % l)
    s = net2.plan_tensor(T, 's').view(M, -1).cpu().numpy()
    close(s, cache['S'].reshape(M, -1), 1e-5, 'skip sum')
    r2 = net2.plan_tensor(T, 'r2').view(M, -1).cpu().numpy()
    close(r2, cache['r2'].reshape(M, -1), 2e-5, 'relu2')


@pytest.mark.parametrize('B,T,nbl', [(4, 9000, 10), (2, 300, 3)])
def test_chain_matches_per_layer(monkeypatch, B, T, nbl, chain_tile):
    """The persistent chain kernel (tile hand-offs inside one launch) against the one-launch-
    per-layer kernels: same x_l for every layer and same z.  (4, 9000): 284 tiles > 256 CUs,
    so tiles run in rounds, with a ragged last tile; nbl=10 takes d up to the 512-row halo."""
    arch = small_arch(nb=1, nbl=nbl)
    q, ids = rand_batch(arch, B, T)
    out = {}
    for mode in ('chain', 'layers'):
        monkeypatch.setenv('LBWN_NO_CHAIN', '1' if mode == 'layers' else '0')
        net = make_net(arch, B)
        net.forward(q, None, ids, backward=True)
        torch.cuda.synchronize()
        assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0
        out[mode] = {k: net.plan_tensor(T, k).clone() for k in ('x', 'z', 's')}
        out[mode]['save'] = net.save_flat.clone()
        out[mode]['grads'] = {n: g.clone() for n, g in net.grads.items()}
    L, H, Cr = R.n_layers(arch), 2 ** (nbl - 1), arch['n_res']
    stride = out['chain']['x'].numel() // L
    for l in range(L):
        a = out['chain']['x'][l * stride:l * stride + B * (H + T) * Cr].view(B, H + T, Cr)[:, H:]
        b = out['layers']['x'][l * stride:l * stride + B * (H + T) * Cr].view(B, H + T, Cr)[:, H:]
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=0, atol=1e-5, err_msg='x_%d' % l)
    for k in ('z', 's', 'save'):
        np.testing.assert_allclose(out['chain'][k].cpu().numpy(), out['layers'][k].cpu().numpy(), rtol=0,
                                   atol=1e-5, err_msg=k)
    # weight gradients.  Loose on purpose: the two paths' S / relu2 agree to ~1e-6, and at
    # B·T = 36000 a handful of relu masks (S > 0, h1 > 0) sit within that of zero and flip,
    # each moving a gradient by ~1e-3 of its scale (measured; the chain path against the
    # float64 oracle at this size: <= 6e-7 relative when no mask flips).  Element-wise parity
    # is the 1e-5 bar on x/z/s above and the 2e-4 oracle bar in test_plan_forward_backward.
    for n, g in out['chain']['grads'].items():
        close(g.cpu().double().numpy(), out['layers']['grads'][n].cpu().double().numpy(), 5e-3, n)


def cond_arch(gc, lc, C=32):
    a = dict(n_blocks=1, n_block_layers=4, n_quant=256, n_res=C, n_dil=C, n_skip=64, n_post=32,
             n_gc_embed=8 if gc else 0, n_gc_category=5 if gc else 0, use_bias=True)
    if lc:
        a.update(n_lc_in=12, n_lc_out=16, lc_upsample=[2, 4])
    return normalize_arch(a)


@pytest.mark.parametrize('gc,lc,C', [(1, 0, 32), (0, 1, 32), (1, 1, 32), (1, 1, 16)])
def test_plan_conditioning(gc, lc, C, chain_tile):
    """GC (tmodel.py:92-114, :150-154) and LC (tmodel.py:68-83, :155-160) through the plan:
    forward (SAVE, loss) and every gradient against the oracle.  C = 32 runs the persistent
    chain kernels, C = 16 the per-layer kernels."""
    arch = cond_arch(gc, lc, C)
    B, T = 2, 256
    net = make_net(arch, B)
    q, ids = rand_batch(arch, B, T)
    rng = np.random.default_rng(3)
    if gc:   # voice ids change at "file" boundaries; 0 = masked
        for b in range(B):
            cuts = np.sort(rng.choice(np.arange(40, T), 3, replace=False))
            v = rng.integers(1, arch['n_gc_category'] + 1, 4)
            ids[b] = np.repeat(v, np.diff(np.r_[0, cuts, T]))
            ids[b, cuts[1]:cuts[1] + 20] = 0
    mel = rng.standard_normal((B, T // 8, arch['n_lc_in'])).astype(np.float32) if lc else None
    P, S = oracle_params(net)
    lg, cache, new_save = R.forward(arch, P, q, ids, S, mel=mel)
    st, dlog = R.loss_fcn(arch, P, lg, q, ids, 0.0)
    net.forward(q, mel, ids, backward=True)
    torch.cuda.synchronize()
    assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0
    stats = net.stats.cpu().numpy()
    assert int(stats[1]) == st['n_valid']
    np.testing.assert_allclose(stats[0] / st['n_valid'], st['mean_xent'], rtol=1e-5)
    for k, v in new_save.items():
        close(net.save_vars[k].cpu().numpy(), v, 1e-5, k)
    G = R.backward(arch, P, cache, dlog, 0.0)
    inv = 1.0 / st['n_valid']
    names = net.layout.names()
    assert any(n.startswith('GC_') for n in names) == bool(gc)
    assert any(n.startswith('LC_') for n in names) == bool(lc)
    for name in names:
        close(net.grads[name].cpu().double().numpy() * inv, G[name], 2e-4, name)


def test_staged_equals_unstaged_bitwise():
    """README.md:6-21: processing a stream in stages with the saved D-separation state is
    the same function as one long slice.  Position-wise kernels make it bit-exact."""
    arch = small_arch()
    B, T = 2, 512
    q, ids = rand_batch(arch, B, T)
    a = make_net(arch, B)
    a.forward(q, None, ids, backward=False)
    full = a.plan_tensor(T, 'r2').view(B, T, -1).clone()
    save_full = a.save_flat.clone()
    b = make_net(arch, B)
    parts = []
    for lo, hi in ((0, 128), (128, 384), (384, 512)):
        b.forward(q[:, lo:hi], None, ids[:, lo:hi], backward=False)
        parts.append(b.plan_tensor(hi - lo, 'r2').view(B, hi - lo, -1).clone())
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts, 1), full)
    assert torch.equal(b.save_flat, save_full)


def test_staged_equals_unstaged_arch3_bitwise(chain_tile):
    """README.md:6-21 at arch3 through the persistent chains, with stages shorter than the
    deepest dilations (100 and 300 < 512; the 100-row stage is also shorter than d = 128 and
    256): the state carried between stages is SAVE alone, rows [T, d) of it old SAVE rows.
    One 4096-position slice against stages 100 + 300 + 3696: every layer's z, the SAVE state
    after each stage boundary and the post-net output, bit for bit."""
    arch = arch3()
    B, T = 2, 4096
    L, Cd = R.n_layers(arch), arch['n_dil']
    q, ids = rand_batch(arch, B, T)
    a = make_net(arch, B)
    a.forward(q, None, ids, backward=False)
    full_z = a.plan_tensor(T, 'z').view(B, T, L * Cd).clone()
    full_r2 = a.plan_tensor(T, 'r2').view(B, T, -1).clone()
    save_full = a.save_flat.clone()
    b = make_net(arch, B)
    zs, r2s = [], []
    for lo, hi in ((0, 100), (100, 400), (400, 4096)):
        b.forward(q[:, lo:hi], None, ids[:, lo:hi], backward=False)
        assert int(b.plan_tensor(hi - lo, 'status').view(torch.int32)[0]) == 0
        zs.append(b.plan_tensor(hi - lo, 'z').view(B, hi - lo, L * Cd).clone())
        r2s.append(b.plan_tensor(hi - lo, 'r2').view(B, hi - lo, -1).clone())
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(zs, 1), full_z)
    assert torch.equal(b.save_flat, save_full)
    assert torch.equal(torch.cat(r2s, 1), full_r2)


def test_adam_step_matches_oracle():
    arch = small_arch(nb=1, nbl=3)
    B, T = 2, 128
    net = make_net(arch, B, l2=1e-3)
    q, ids = rand_batch(arch, B, T)
    P, S = oracle_params(net)
    opt_o = R.AdamTF1(1e-3)
    opt = AdamOptimizer(1e-3)
    for step in range(3):
        lg, cache, S = R.forward(arch, P, q, ids, S)
        st, dlog = R.loss_fcn(arch, P, lg, q, ids, 1e-3)
        G = R.backward(arch, P, cache, dlog, 1e-3)
        opt_o.step(P, G)
        gv, loss = net.build(q, None, ids)
        np.testing.assert_allclose(float(loss), st['total'], rtol=2e-5)
        opt.apply_gradients(gv)
    torch.cuda.synchronize()
    # Adam normalises each element's step (m/√v): elements whose gradient is ~0 can take a
    # ±lr step on rounding noise, so bound the max by the step size and the bulk tightly.
    for name in net.layout.names():
        d = np.abs(net.vars[name].cpu().double().numpy() - P[name])
        assert d.max() <= 2 * 3 * 1e-3 + 1e-6, name
        assert np.mean(d) <= 2e-6, (name, np.mean(d))
    assert net.counters[0].item() == 3 and net.counters[1].item() == 3 * st['n_valid']


@pytest.mark.parametrize('n,nw', [(1003, 501), (4096, 4096), (7, 3), (1, 0)])
def test_adam_kernel_ragged(lib, n, nw):
    """lbwn_adam_tf1 on lengths that are not multiples of its 4-wide vector step and a weight /
    bias boundary inside a vector: TF1 Adam (training_ops.cc ApplyAdam; oracle AdamTF1) with the
    l2 term on the first nw elements and the gradient scaled by 1 / n_valid, at step t = 5."""
    rng = np.random.default_rng(n)
    p0, g0, m0 = (rng.standard_normal(n).astype(np.float32) for _ in range(3))
    v0 = rng.random(n).astype(np.float32)
    dev = 'cuda'
    p, g, m, v = (torch.tensor(a, device=dev) for a in (p0, g0, m0, v0))
    stats = torch.tensor([0.0, 7.0, 0.0, 0.0], device=dev)
    counters = torch.tensor([4, 0, 4, 0], dtype=torch.int64, device=dev)
    lr, b1, b2, eps, l2 = 1e-3, 0.9, 0.999, 1e-8, 1e-3
    _lib.check(lib.lbwn_adam_tf1(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), nw, n, lr, b1, b2, eps, l2,
                                 stats.data_ptr(), counters.data_ptr(), None, None))
    torch.cuda.synchronize()
    gd = g0.astype(np.float64) / 7.0
    gd[:nw] += l2 * p0[:nw]
    md = b1 * m0 + (1 - b1) * gd
    vd = b2 * v0 + (1 - b2) * gd * gd
    lr_t = lr * np.sqrt(1 - b2 ** 5) / (1 - b1 ** 5)
    pd = p0 - lr_t * md / (np.sqrt(vd) + eps)
    np.testing.assert_allclose(m.cpu().numpy(), md, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(v.cpu().numpy(), vd, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(p.cpu().numpy(), pd, rtol=1e-6, atol=1e-7)


def test_chain_xcd_walk_lc_bitwise(monkeypatch):
    """LC archs walk the chains' tiles XCD-grouped by default (engine.cpp plan creation); the
    block-index walk (LBWN_CHAIN_XCD=0) gives the same outputs and gradients bit for bit (arch5 with
    its LC and GC terms, 64 tiles per chain), except the GC gradients, whose mixed-voice rows are
    float atomics (to f32 rounding)."""
    arch = load_arch(os.path.join(ROOT, 'par', 'arch5.json'))
    B, T = 2, 4096
    q, ids = rand_batch(arch, B, T)
    hop = int(np.prod(arch['lc_upsample']))
    mel = np.random.default_rng(5).standard_normal((B, T // hop, arch['n_lc_in'])).astype(np.float32)
    gid = np.where(ids != 0, 3, 0).astype(np.int32) if arch['n_gc_category'] else ids
    out = []
    for v in (None, '0'):
        if v is None:
            monkeypatch.delenv('LBWN_CHAIN_XCD', raising=False)
        else:
            monkeypatch.setenv('LBWN_CHAIN_XCD', v)
        net = make_net(arch, B)
        net.forward(q, mel, gid, backward=True)
        torch.cuda.synchronize()
        assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0
        out.append((net.stats[:3].cpu().numpy(), net.save_flat.cpu().numpy(),
                    {n: g.cpu().numpy() for n, g in net.grads.items()}))
    (s0, v0, g0), (s1, v1, g1) = out
    assert np.array_equal(s0, s1) and np.array_equal(v0, v1)
    for n in g0:
        if n.startswith('GC_'):   # mixed-voice waves add their GC rows by float atomics (gc_scatter16):
            # the add order follows which CU ran which tile, so these compare to f32 rounding
            np.testing.assert_allclose(g0[n], g1[n], rtol=1e-5, atol=1e-6, err_msg=n)
        else:
            assert np.array_equal(g0[n], g1[n]), n


@pytest.mark.parametrize('env', [{'LBWN_CHAIN_XCD': '1'}, {'LBWN_DZ_XCD': '0'}])
def test_placement_switches_bitwise(monkeypatch, env):
    """The placement-only switches change which block (and so which XCD) computes a tile, never
    the arithmetic of a tile: the XCD-grouped chain walk (layer.hip chain_first) and dZ's 1-D
    tile remap instead of the 2-D XCD blocking (gemm.hip xcd2d_tile) give the default plan's
    outputs and gradients bit for bit (arch3, 128 tiles per chain)."""
    arch = arch3()
    B, T = 4, 4096
    q, ids = rand_batch(arch, B, T)
    out = []
    for use in (False, True):
        for k, v in env.items():
            if use:
                monkeypatch.setenv(k, v)
            else:
                monkeypatch.delenv(k, raising=False)
        net = make_net(arch, B)
        net.forward(q, None, ids, backward=True)
        torch.cuda.synchronize()
        assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0
        out.append((net.stats[:3].cpu().numpy(), net.save_flat.cpu().numpy(),
                    {n: g.cpu().numpy() for n, g in net.grads.items()}))
    (s0, v0, g0), (s1, v1, g1) = out
    assert np.array_equal(s0, s1) and np.array_equal(v0, v1)
    for n in g0:
        assert np.array_equal(g0[n], g1[n]), n


def test_mask_bits_equal_f32_masks(monkeypatch):
    """The relu masks of dS = dH1·POST1ᵀ ⊙ (S > 0) and dH1 = dlogits·POST2ᵀ ⊙ (R2 > 0) travel as
    bits written by the skip / post1 GEMM epilogues (lbwn_gemm_args::mbits_out, read back by the
    same x3q<8> lane layout in dS / dH1); LBWN_GEMM_MBITS=0 (plan creation) makes the backward
    read the f32 S / R2 instead.  The two must agree bit for bit: dS, dH1, the stats, SAVE and
    every gradient (arch3 B=4, T=4096: both ends in the x3q<8> form)."""
    arch = arch3()
    B, T = 4, 4096
    q, ids = rand_batch(arch, B, T)
    out = []
    for mb in ('1', '0'):
        monkeypatch.setenv('LBWN_GEMM_MBITS', mb)
        net = make_net(arch, B)
        net.forward(q, None, ids, backward=True)
        torch.cuda.synchronize()
        assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0
        out.append((net.stats[:3].cpu().numpy(), net.save_flat.cpu().numpy(),
                    {n: g.cpu().numpy() for n, g in net.grads.items()},
                    net.plan_tensor(T, 'ds').cpu().numpy(), net.plan_tensor(T, 'dh').cpu().numpy()))
    (s0, v0, g0, ds0, dh0), (s1, v1, g1, ds1, dh1) = out
    assert np.array_equal(ds0, ds1) and np.array_equal(dh0, dh1)
    assert np.array_equal(s0, s1) and np.array_equal(v0, v1)
    for n in g0:
        assert np.array_equal(g0[n], g1[n]), n


@pytest.mark.parametrize('name,B', [('arch3', 4), ('arch5', 2)])
def test_colsum_side_bitwise(monkeypatch, name, B):
    """The bias gradients' final column sums run on the side stream beside dPOST2 / dPOST1, joined
    before the backward chain (default; LBWN_COLSUM_SIDE=0 at plan creation keeps them in line):
    stats, SAVE and every gradient bit for bit as the in-line order, over two steps (voice ids
    tile-uniform: no GC atomics)."""
    from tests.test_gpu_dp import _batch
    arch = load_arch(os.path.join(ROOT, 'par', name + '.json'))
    T = 4096
    q, ids, mel = _batch(arch, B, T, 7)
    out = []
    for side in ('0', '1'):
        monkeypatch.setenv('LBWN_COLSUM_SIDE', side)
        net = make_net(arch, B)
        for _ in range(2):
            net.forward(q, mel, ids, backward=True)
        torch.cuda.synchronize()
        assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0
        out.append((net.stats[:3].cpu().numpy(), net.save_flat.cpu().numpy(),
                    {n: g.cpu().numpy() for n, g in net.grads.items()}))
    (s0, v0, g0), (s1, v1, g1) = out
    assert np.array_equal(s0, s1) and np.array_equal(v0, v1)
    for n in g0:
        assert np.array_equal(g0[n], g1[n]), n


def test_chain_trace_build_bitwise(monkeypatch):
    """LBWN_CHAIN_TRACE=<block> (read at plan creation: the chains' traced instantiations, whose
    clock stamps feed tools/chain_trace.py and the bench's C4 dilation sweep) computes exactly what
    the untraced chains do: stats, SAVE and every gradient bit for bit, and the stamps are written."""
    arch = arch3()
    B, T = 2, 4096
    q, ids = rand_batch(arch, B, T)
    out = []
    for tr in (None, '1'):
        if tr:
            monkeypatch.setenv('LBWN_CHAIN_TRACE', tr)
        else:
            monkeypatch.delenv('LBWN_CHAIN_TRACE', raising=False)
        net = make_net(arch, B)
        net.forward(q, None, ids, backward=True)
        torch.cuda.synchronize()
        assert int(net.plan_tensor(T, 'status').view(torch.int32)[0]) == 0
        out.append((net.stats[:3].cpu().numpy(), net.save_flat.cpu().numpy(),
                    {n: g.cpu().numpy() for n, g in net.grads.items()},
                    net.plan_tensor(T, 'ctrace').view(torch.int64).cpu().numpy().copy()))
    (s0, v0, g0, _), (s1, v1, g1, tr1) = out
    assert np.array_equal(s0, s1) and np.array_equal(v0, v1)
    for n in g0:
        assert np.array_equal(g0[n], g1[n]), n
    L = R.n_layers(arch)
    st = tr1.reshape(2, L, 16)[:, :, 0]
    assert np.all(st != 0), 'chain stamps missing'
