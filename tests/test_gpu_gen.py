"""Cached generation (imodel.py) on the GPU vs the oracle's restatement.  Draws use the
same counter-based uniforms on both sides, so sample sequences must match exactly (a flip
needs u·Σe to land within fp32 rounding of a CDF boundary: ~1e-6 per draw)."""
import os

import numpy as np
import pytest
import torch

from lbwn.arch import load_arch, normalize_arch
from lbwn.imodel import WaveNetGen
from lbwn.tmodel import WaveNetTrain
from oracle import wavenet_ref as R
from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.fixture(params=['persistent', 'per_step'])
def form(request, monkeypatch):
    """Both execution forms: the persistent one-launch kernel (the default while its blocks fit:
    groups of <= 16 streams, B <= 80 on 256 CUs) and the per-step launches (LBWN_GEN_PERSIST=0:
    vector GEMVs at B <= 16, the head as MFMA GEMMs beyond)."""
    if request.param == 'per_step':
        monkeypatch.setenv('LBWN_GEN_PERSIST', '0')
    else:
        monkeypatch.delenv('LBWN_GEN_PERSIST', raising=False)
    return request.param


def small(gc=0):
    return normalize_arch(dict(n_blocks=2, n_block_layers=4, n_quant=256, n_res=32, n_dil=32, n_skip=64,
                               n_post=32, n_gc_embed=8 if gc else 0, n_gc_category=gc, use_bias=True))


def make_gen(arch, B, chunk, seed=7, teacher=None, pre_bias=True, graph=True):
    tr = WaveNetTrain(**arch, batch_sz=1, l2_factor=0.0, print_interval=0)
    tr.init_vars(3, bias_scale=0.2)
    # sharpen the head so draws are not uniform noise
    with torch.no_grad():
        tr.vars['POST2'].mul_(4.0)
    g = WaveNetGen(arch['n_blocks'], arch['n_block_layers'], arch['n_quant'], arch['n_res'], arch['n_dil'],
                   arch['n_skip'], arch['n_post'], arch['n_gc_embed'], arch['n_gc_category'], arch['use_bias'],
                   B, chunk, None, seed=seed, pre_bias=pre_bias, graph=graph)
    g.load_params(tr)
    P = {n: v.cpu().double().numpy() for n, v in tr.vars.items()}
    return g, P


@pytest.mark.parametrize('pre_bias', [True, False])
def test_gen_free_running_matches_oracle(pre_bias, form):
    arch = small()
    B, n = 3, 48
    g, P = make_gen(arch, B, chunk=16, pre_bias=pre_bias)
    _, wav, _ = g.run(n)
    torch.cuda.synchronize()
    assert g.persistent == (form == 'persistent')
    s_ref, w_ref = R.generate(arch, P, B, n, seed=7, pre_bias=pre_bias)
    assert int(g.tensor('status', torch.int32).item()) == 0     # no hand-off spin timed out
    np.testing.assert_array_equal(g.samples().cpu().numpy()[:, :n], s_ref)
    np.testing.assert_allclose(wav.cpu().numpy(), w_ref[:, :wav.shape[1]], rtol=1e-6, atol=1e-6)


def test_gen_teacher_forced_and_gc(form):
    arch = small(gc=5)
    B, n = 2, 40
    teacher_q = np.random.default_rng(1).integers(0, 256, 25).astype(np.int32)
    g, P = make_gen(arch, B, chunk=10)
    g.teacher_mu = torch.as_tensor(teacher_q, device='cuda')
    g.build_graph(n)
    gc = [2, 5]
    g.run(n, gc_ids=gc)
    torch.cuda.synchronize()
    assert g.persistent == (form == 'persistent')
    assert int(g.tensor('status', torch.int32).item()) == 0
    s_ref, _, lg_ref = R.generate(arch, P, B, n, seed=7, teacher_q=teacher_q, gc_ids=gc, return_logits=True)
    np.testing.assert_array_equal(g.samples().cpu().numpy()[:, :n], s_ref)
    np.testing.assert_allclose(g.logits().cpu().numpy(), lg_ref[:, -1], rtol=0, atol=2e-4 * np.abs(lg_ref).max())


def test_gen_arch3_b10_graph_replay(form):
    arch = load_arch(os.path.join(ROOT, 'par', 'arch3.json'))
    B, n = 10, 300
    g, P = make_gen(arch, B, chunk=100)
    n_out, wav, _ = g.run(n)
    torch.cuda.synchronize()
    assert g.persistent == (form == 'persistent')
    assert wav.shape == (B, 300)
    s_ref, w_ref = R.generate(arch, P, B, n, seed=7)
    got = g.samples().cpu().numpy()[:, :n]
    mism = int((got != s_ref).sum())
    assert mism == 0, '%d / %d draws differ' % (mism, got.size)
    assert int(g.tensor('step', torch.int64).item()) == n
    assert int(g.tensor('status', torch.int32).item()) == 0


def test_gen_rerun_and_large_batch(form):
    """A second run on the same plan restarts the tags with the step counter (stale granules
    from the first run must not be taken); B = 40 > 16 runs as three stream groups (14, 14, 12:
    a ragged last group) of the persistent launch, or with LBWN_GEN_PERSIST=0 the per-step
    GEMM form."""
    arch = small(gc=5)
    B, n = 40, 24
    g, P = make_gen(arch, B, chunk=8)
    gc = [1 + b % 5 for b in range(B)]
    g.run(n, gc_ids=gc)
    g.run(n, gc_ids=gc)
    torch.cuda.synchronize()
    assert g.persistent == (form == 'persistent')
    assert int(g.tensor('status', torch.int32).item()) == 0
    assert int(g.tensor('step', torch.int64).item()) == n
    s_ref, _ = R.generate(arch, P, B, n, seed=7, gc_ids=gc)
    np.testing.assert_array_equal(g.samples().cpu().numpy()[:, :n], s_ref)
    g2, P2 = make_gen(arch, 12, chunk=8)
    g2.run(n, gc_ids=gc[:12])
    g2.run(n, gc_ids=gc[:12])
    torch.cuda.synchronize()
    assert g2.persistent == (form == 'persistent')
    s2, _ = R.generate(arch, P2, 12, n, seed=7, gc_ids=gc[:12])
    np.testing.assert_array_equal(g2.samples().cpu().numpy()[:, :n], s2)
    assert int(g2.tensor('status', torch.int32).item()) == 0


def test_gen_arch3_gemm_form(form):
    """B = 64 (> 16): four stream groups of 16 in one persistent launch (192 blocks), or with
    LBWN_GEN_PERSIST=0 gen_wave per step, then skip / post1 / post2 as bf16-split MFMA GEMMs over
    the 64 streams (split-K, bias + relu epilogues) and the sampler; draws equal the oracle's."""
    arch = load_arch(os.path.join(ROOT, 'par', 'arch3.json'))
    B, n = 64, 60
    g, P = make_gen(arch, B, chunk=20)
    g.run(n)
    torch.cuda.synchronize()
    assert g.persistent == (form == 'persistent')
    assert int(g.tensor('status', torch.int32).item()) == 0
    s_ref, _, lg_ref = R.generate(arch, P, B, n, seed=7, return_logits=True)
    got = g.samples().cpu().numpy()[:, :n]
    mism = int((got != s_ref).sum())
    assert mism == 0, '%d / %d draws differ' % (mism, got.size)
    np.testing.assert_allclose(g.logits().cpu().numpy(), lg_ref[:, -1], rtol=0, atol=1e-4 * np.abs(lg_ref).max())
    assert int(g.tensor('step', torch.int64).item()) == n


def _near_tie(lg_row, u, tol=5e-5):
    """True when the inverse-CDF target u·Σe lies within tol·Σe of a CDF boundary of the
    oracle's float64 logits: an fp32 evaluation of the same logits may then pick the
    neighbouring code (sample_from_logits, oracle/wavenet_ref.py)."""
    e = np.exp(lg_row - lg_row.max())
    c = np.cumsum(e)
    return float(np.min(np.abs(c - u * c[-1]))) <= tol * c[-1]


@pytest.mark.parametrize('B,n', [(10, 2100), (80, 1100)])
def test_gen_arch3_full_ring_depth(B, n, form):
    """C3 at its own chunk size (1000, generate.py:17) and long enough that every lookback ring
    wraps: with d <= 512 each layer's ring (slot t & (d-1)) is rewritten >= 2x (4x at B=10), so
    the d = 512 layers' dilated taps read values this run wrote 512 steps earlier (imodel.py:88-122,
    :190-207), and two chunk boundaries (graph replay -> replay -> a 100-step tail launch) are
    crossed.  B = 80 runs as 5 stream groups of the persistent launch.

    The oracle is evaluated along the GPU's own trajectory (forced_q = the GPU's draws), so
    every one of the B·n draws is checked against the float64 logits it was drawn from; a
    difference is allowed only at a near tie (u·Σe within 5e-5 of a CDF boundary), and at most
    a couple of those.  With no difference, the free-running oracle's draws equal the GPU's
    exactly (each step's input is then the same on both sides)."""
    arch = load_arch(os.path.join(ROOT, 'par', 'arch3.json'))
    g, P = make_gen(arch, B, chunk=1000)
    n_out, wav, rem = g.run(n)
    torch.cuda.synchronize()
    assert g.persistent == (form == 'persistent')
    assert int(g.tensor('status', torch.int32).item()) == 0
    assert int(g.tensor('step', torch.int64).item()) == n
    assert wav.shape == (B, (n // 1000) * 1000) and rem == n % 1000
    got = g.samples().cpu().numpy()[:, :n]
    assert len(np.unique(got)) > 16                      # the draws are not stuck on a few codes
    ref, w_ref, lg = R.generate(arch, P, B, n, seed=7, return_logits=True, forced_q=got)
    bad = np.argwhere(got != ref)
    ties = [(int(b), int(i)) for b, i in bad if _near_tie(lg[b, i], R.philox_uniform(7, int(b), int(i)))]
    assert len(ties) == len(bad), 'draws differ away from a CDF tie at (stream, step) %s' % (
        [tuple(x) for x in bad[:8].tolist()],)
    assert len(bad) <= 2, bad.tolist()
    np.testing.assert_allclose(g.logits().cpu().numpy(), lg[:, -1], rtol=0, atol=1e-4 * np.abs(lg[:, -1]).max())
    if len(bad) == 0:
        np.testing.assert_allclose(wav.cpu().numpy(), w_ref[:, :wav.shape[1]], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('B', [3, 20])
def test_gen_trace_build_same_draws(monkeypatch, B):
    """LBWN_GEN_TRACE=1 (read at gen-plan creation: the persistent kernel's per-phase clock
    stamps, tools/gen_trace.py and the bench's measured_per_layer_us) is the same computation:
    the traced instantiation draws exactly the untraced one's samples (B=20: two stream groups)."""
    arch = small()
    out = []
    for tr in (None, '1'):
        if tr:
            monkeypatch.setenv('LBWN_GEN_TRACE', tr)
        else:
            monkeypatch.delenv('LBWN_GEN_TRACE', raising=False)
        g, _ = make_gen(arch, B, chunk=64)
        g.run(200)
        torch.cuda.synchronize()
        assert int(g.tensor('status', torch.int32).item()) == 0
        out.append(g.samples().cpu().numpy()[:, :200].copy())
    np.testing.assert_array_equal(out[0], out[1])


def test_gen_arch3_c3_length_last_chunk(form):
    """The C3 benchmark's whole run (3 s at 16 kHz = 48,000 steps, B=10, chunk 1000: 48 graph
    replays) checked at its end: after 47,000 steps the device state -- every layer's lookback
    ring and the last draw -- is read back, the last 1,000 steps run on, and the oracle, resumed
    from that state (generate(start=47000, init_rings=, init_q=)), evaluates them along the GPU's
    trajectory: each draw is checked against the float64 logits it was drawn from (near CDF ties
    excepted, as test_gen_arch3_full_ring_depth).  A ring slot, the step counter or the RNG step
    going wrong anywhere in the 47 chunk shifts would show as a draw the state does not explain."""
    arch = load_arch(os.path.join(ROOT, 'par', 'arch3.json'))
    B, n0, n1 = 10, 47000, 1000
    g, P = make_gen(arch, B, chunk=1000)
    g.build_graph(n0 + n1)
    g.init_buffers()
    g.step(n0)
    torch.cuda.synchronize()
    assert int(g.tensor('step', torch.int64).item()) == n0
    rings_flat = g.tensor('rings').cpu().numpy().astype(np.float64)
    L, Cr = R.n_layers(arch), arch['n_res']
    rings, off = [], 0
    for l in range(L):
        d = R.layer_index(arch, l)[2]
        rings.append(rings_flat[off:off + B * d * Cr].reshape(B, d, Cr))
        off += B * d * Cr
    q_last = g.samples().cpu().numpy()[:, n0 - 1].copy()
    g.step(n1)
    torch.cuda.synchronize()
    g.check_status()
    assert g.persistent == (form == 'persistent')
    got = g.samples().cpu().numpy()[:, n0:n0 + n1]
    assert len(np.unique(got)) > 16
    ref, _, lg = R.generate(arch, P, B, n1, seed=7, return_logits=True, forced_q=got, start=n0, init_rings=rings,
                            init_q=q_last)
    bad = np.argwhere(got != ref)
    ties = [(int(b), int(i)) for b, i in bad if _near_tie(lg[b, i], R.philox_uniform(7, int(b), n0 + int(i)))]
    assert len(ties) == len(bad), 'draws differ away from a CDF tie at (stream, step) %s' % (
        [(b, n0 + i) for b, i in bad[:8].tolist()],)
    assert len(bad) <= 2, bad.tolist()
    np.testing.assert_allclose(g.logits().cpu().numpy(), lg[:, -1], rtol=0, atol=1e-4 * np.abs(lg[:, -1]).max())
