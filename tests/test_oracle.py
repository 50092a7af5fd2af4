"""Oracle pinning: golden vectors from the reference's own code, the README KAT,
finite-difference gradients and generation/training equivalence (all CPU)."""
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN
from oracle import wavenet_ref as R
from tests.golden.make_golden import CASES, make_files


def arch_tiny(gc=0, lc=0, nbl=3, nb=2, ub=True):
    """arch2-like tiny dims (par/arch2.json:5-8) so float64 checks run in ms."""
    return dict(n_blocks=nb, n_block_layers=nbl, n_quant=16, n_res=3, n_dil=4, n_skip=8,
                n_post=6, n_gc_embed=5 if gc else 0, n_gc_category=gc, n_lc_in=4 if lc else 0,
                n_lc_out=3 if lc else 0, lc_upsample=[2, 2] if lc else [], use_bias=ub,
                wav_input_type='mu_law_quant')


# ---- A1/A2 ---------------------------------------------------------------------------

def test_mulaw_golden():
    g = np.load(os.path.join(GOLDEN, 'mulaw.npz'))
    for q in (256, 64):
        np.testing.assert_array_equal(R.mu_encode_np(g['mu_x'], q), g['mu_enc_%d' % q])
        np.testing.assert_array_equal(R.mu_decode_np(g['mu_dec_q_%d' % q], q), g['mu_dec_%d' % q])
    np.testing.assert_array_equal(R.mu_encode_np(g['mu_x32'], 256), g['mu_enc32_256'])
    assert g['mu_enc_256'][:9].tolist() == [0, 7, 16, 32, 128, 223, 239, 248, 255]


def test_mulaw_decode_quirk():
    # offset -1/mu: q=128 -> 0.0, q=0 -> -1.0221, q=255 -> +0.9784
    d = R.mu_decode_np(np.array([0, 128, 255]), 256)
    assert d[1] == 0.0 and abs(d[0] + 1.0221) < 1e-3 and abs(d[2] - 0.9784) < 1e-3
    np.testing.assert_allclose(R.mu_decode_tf32(np.arange(256), 256),
                               R.mu_decode_np(np.arange(256), 256), rtol=2e-6, atol=2e-7)


# ---- A3 ------------------------------------------------------------------------------

def _golden_files(name):
    g = np.load(os.path.join(GOLDEN, 'dealer_%s.npz' % name))
    if name == 'small':
        files = [(int(g['file_vid_%d' % i]), g['file_wav_%d' % i], g['file_mel_%d' % i])
                 for i in range(int(g['n_files']))]
    else:
        seed, nf, lo, hi, B, T, F, hop, nmel, mv = CASES[name]
        files = make_files(seed, nf, lo, hi, hop, nmel, mv)
    return g, files


@pytest.mark.parametrize('name', ['small', 'hop4_b3', 'hop256_b4', 'recep5115_b2'])
def test_dealer_golden(name):
    g, files = _golden_files(name)
    B, T, F, hop, nmel = (int(g[k]) for k in ('B', 'T', 'F', 'hop', 'nmel'))
    batches, log = R.deal_batches(files, B, T, F, hop, nmel)
    assert len(batches) == int(g['n_batches'])
    for j, (w, m, ids) in enumerate(batches):
        np.testing.assert_array_equal(ids, g['ids_%d' % j])
        np.testing.assert_array_equal(w.astype(np.int64), g['wav_%d' % j])
        np.testing.assert_array_equal(m.astype(np.int64), g['mel_%d' % j])


def test_dealer_survey_case():
    g, files = _golden_files('small')
    batches, log = R.deal_batches(files, 1, 8, 4, 1, 2)
    assert [b[2][0].tolist() for b in batches] == [[0, 0, 0, 3, 3, 3, 3, 3],
                                                    [3, 3, 0, 0, 0, 5, 5, 5],
                                                    [5, 0, 0, 0, 7, 7, 7, 7]]
    assert ('skip', 3, 2, 4) in log


# ---- README influence KAT --------------------------------------------------------------

TOP_ROW = [1, 4, 10, 20, 35, 56, 84, 120, 165, 220, 286, 364, 455, 560, 680, 816, 966, 1128,
           1300, 1480, 1666, 1856, 2048, 2240, 2430, 2616, 2796, 2968, 3130, 3280, 3416, 3536,
           3641, 3732, 3810, 3876, 3931, 3976, 4012, 4040, 4061, 4076, 4086, 4092, 4095, 4096]
SECOND_ROW = [2, 8, 20, 40, 70, 112, 168, 240, 328, 432, 552, 688, 840, 1008, 1192, 1392,
              1604, 1824, 2048, 2272, 2492, 2704, 2904, 3088]


def test_readme_influence_kat():
    dil = [1, 2, 4, 8] * 3
    x = np.array([0] * 8 + [4096] * 56, np.float64)
    rows, _ = R.influence_stack(x, dil)
    top, second = rows[-1], rows[-2]
    assert top[:8].tolist() == [0] * 8
    assert top[8:8 + len(TOP_ROW)].tolist() == TOP_ROW
    assert second[8:8 + len(SECOND_ROW)].tolist() == SECOND_ROW
    # staged at the black line (column 32) with the saved D-separation nodes == unstaged
    r1, sv = R.influence_stack(x[:32], dil)
    r2, _ = R.influence_stack(x[32:], dil, save=sv)
    np.testing.assert_array_equal(np.concatenate([r1, r2], axis=1), rows)


# ---- training forward: staged == unstaged, finite differences --------------------------

def _setup(arch, B=2, T=24, seed=0, bias_scale=0.1):
    rng = np.random.default_rng(seed)
    P = R.init_params(arch, rng, bias_scale=bias_scale)
    save = R.init_save(arch, B, rng)
    q = rng.integers(0, arch['n_quant'], size=(B, T))
    ids = rng.integers(1, max(arch['n_gc_category'], 1) + 1, size=(B, T))
    ids[:, :5] = 0
    mel = None
    if arch['n_lc_out']:
        hop = int(np.prod(arch['lc_upsample']))
        mel = rng.normal(size=(B, T // hop, arch['n_lc_in']))
    return P, save, q, ids, mel


@pytest.mark.parametrize('gc,lc', [(0, 0), (3, 0), (0, 1), (3, 1)])
def test_staged_equals_unstaged(gc, lc):
    arch = arch_tiny(gc, lc)
    P, save, q, ids, mel = _setup(arch, T=24)
    lg, _, sv = R.forward(arch, P, q, ids, save, mel)
    hop = int(np.prod(arch['lc_upsample'])) if lc else 1
    a, b = 8, 24
    lg1, _, sv1 = R.forward(arch, P, q[:, :a], ids[:, :a], save, None if mel is None else mel[:, :a // hop])
    lg2, _, sv2 = R.forward(arch, P, q[:, a:], ids[:, a:], sv1, None if mel is None else mel[:, a // hop:])
    np.testing.assert_allclose(np.concatenate([lg1, lg2], 1), lg, rtol=1e-12, atol=1e-12)
    for k in sv:
        np.testing.assert_allclose(sv2[k], sv[k], rtol=0, atol=0)


@pytest.mark.parametrize('gc,lc,ub', [(0, 0, True), (3, 1, True), (0, 0, False)])
def test_backward_finite_difference(gc, lc, ub):
    arch = arch_tiny(gc, lc, ub=ub)
    P, save, q, ids, mel = _setup(arch, T=16)
    l2f = 0.01

    def total(P_):
        lg, _, _ = R.forward(arch, P_, q, ids, save, mel)
        st, _ = R.loss_fcn(arch, P_, lg, q, ids, l2f)
        return st['total']

    lg, cache, _ = R.forward(arch, P, q, ids, save, mel)
    st, dlog = R.loss_fcn(arch, P, lg, q, ids, l2f)
    G = R.backward(arch, P, cache, dlog, l2f)
    rng = np.random.default_rng(1)
    eps = 1e-6
    for name in P:
        flat = P[name].reshape(-1)
        for idx in rng.choice(flat.size, size=min(3, flat.size), replace=False):
            old = flat[idx]
            flat[idx] = old + eps
            fp = total(P)
            flat[idx] = old - eps
            fm = total(P)
            flat[idx] = old
            num = (fp - fm) / (2 * eps)
            ana = G[name].reshape(-1)[idx]
            assert abs(num - ana) <= 1e-6 + 1e-5 * abs(num), (name, idx, num, ana)


def test_generation_teacher_forced_equals_training_forward():
    """tests.py:1 intent: imodel and tmodel are equivalent functions.  Teacher-forced
    generation (PRE bias on) with SAVE built from gen's step-0 state == training logits."""
    arch = arch_tiny(gc=3)
    P, _, q, _, _ = _setup(arch, B=1, T=20)
    teacher = q[0]
    gc_id = 2
    _, _, glog = R.generate(arch, P, 1, len(teacher) + 1, teacher_q=teacher, gc_ids=[gc_id],
                            return_logits=True)
    # gen time 0 (zero input) is the step before training position 0: SAVE_l = [0..0, g_l]
    z0 = np.zeros((1, arch['n_res'])) + P['PRE_BIAS']
    save = {}
    L = R.n_layers(arch)
    emb = P['GC_EMBED'][[gc_id]]
    z = z0
    for l in range(L):
        b, bl, d = R.layer_index(arch, l)
        sfx = '_%d_%d' % (b, bl)
        sv = np.zeros((1, d, arch['n_res']))
        sv[0, -1] = z[0]
        save['SAVE_%d%s' % (d, sfx)] = sv
        v = {nm: z @ P[nm + sfx][1] + P[nm + '_BIAS' + sfx] + emb @ P['GC_' + nm + sfx]
             for nm in ('SIGNAL', 'GATE')}
        zz = np.tanh(v['SIGNAL']) * R._sigmoid(v['GATE'])
        z = z + zz @ P['RESIDUAL' + sfx] + P['RESIDUAL_BIAS' + sfx]
    ids = np.full((1, len(teacher)), gc_id)
    lg, _, _ = R.forward(arch, P, teacher[None, :], ids, save)
    np.testing.assert_allclose(glog[0, 1:], lg[0], rtol=1e-10, atol=1e-10)


def test_generation_forced_trajectory():
    """generate(..., forced_q=) (the GPU full-ring-depth test's checker): forcing a run's own
    draws reproduces it exactly, and forcing another trajectory changes only the inputs -- each
    draw is then the inverse-CDF draw of the logits computed along that trajectory.  The d <= 4
    rings wrap >= 7x in 30 steps."""
    arch = arch_tiny(gc=0)
    P, _, _, _, _ = _setup(arch, B=2, T=8)
    s0, w0, lg0 = R.generate(arch, P, 2, 30, seed=3, return_logits=True)
    s1, w1, lg1 = R.generate(arch, P, 2, 30, seed=3, return_logits=True, forced_q=s0)
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(lg0, lg1)
    other = (s0 + 17) % arch['n_quant']
    s2, _, lg2 = R.generate(arch, P, 2, 30, seed=3, return_logits=True, forced_q=other)
    np.testing.assert_array_equal(lg2[:, 0], lg0[:, 0])            # step 0: zero input either way
    assert not np.allclose(lg2[:, 1:], lg0[:, 1:])
    for b in range(2):
        for i in range(30):
            assert s2[b, i] == R.sample_from_logits(lg2[b, i], R.philox_uniform(3, b, i))


def test_generation_resume_equals_one_run():
    """generate(..., start=, init_rings=, init_q=) (the GPU C3-length test's checker): a run of 30
    steps equals 17 steps then 13 resumed from the first call's rings and last draw -- the ring
    slots and the draws' uniforms follow the global step index."""
    arch = arch_tiny(gc=0)
    P, _, _, _, _ = _setup(arch, B=2, T=8)
    s0, w0, lg0 = R.generate(arch, P, 2, 30, seed=3, return_logits=True)
    s1, _, lg1, rings = R.generate(arch, P, 2, 17, seed=3, return_logits=True, return_state=True)
    s2, _, lg2 = R.generate(arch, P, 2, 13, seed=3, return_logits=True, start=17, init_rings=rings,
                            init_q=s1[:, -1])
    np.testing.assert_array_equal(np.concatenate([s1, s2], 1), s0)
    np.testing.assert_allclose(np.concatenate([lg1, lg2], 1), lg0, rtol=0, atol=1e-12)


def test_adam_tf1():
    opt = R.AdamTF1(0.1)
    P = {'w': np.array([1.0, -2.0])}
    G = {'w': np.array([0.5, -0.25])}
    opt.step(P, G)
    # t=1: lr_t = lr·sqrt(1-b2)/(1-b1); m=(1-b1)g; v=(1-b2)g² -> step = lr_t·m/(sqrt(v)+eps)
    lr_t = 0.1 * np.sqrt(1 - 0.999) / (1 - 0.9)
    exp = np.array([1.0, -2.0]) - lr_t * 0.1 * G['w'] / (np.sqrt(0.001) * np.abs(G['w']) + 1e-8)
    np.testing.assert_allclose(P['w'], exp, rtol=1e-12)
