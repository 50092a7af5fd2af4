"""CPU restatement of hrbigelow/lb-wavenet's hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker / the
timed CPU baseline.  The product path (``lb-wavenet_amd/lbwn``) never imports it and
fails loudly when the HIP library is missing.

Pinning status:
  * mu-law codec (numpy variant) and the invalid-window id dealer/mask are PINNED
    bit-exact against golden vectors produced by importing the reference's own
    ``ops.py`` / ``data.py`` with tensorflow/librosa stubbed (tests/golden/make_golden.py).
  * The D-separation prepend/save mechanism is PINNED by the README influence-diagram
    known-answer test (README.md:62-85, images/wavenet_influence.png).
  * The TensorFlow arithmetic itself (conv / gate / 1x1 / softmax-xent / autodiff / Adam)
    lives in third-party TensorFlow 1.x (unpinned version, inferred 1.12-1.15; not
    vendored, not installable here).  It is restated from TF's published semantics and
    the reference call sites cited per function; no reference test pins it, so that
    part is "parity unpinned" beyond the self-consistency invariants in tests/
    (finite differences, staged == unstaged, teacher-forced generation == training
    forward).

Everything is plain numpy; float64 by default (the checker), float32 for the timed
CPU baseline.  Layout is the reference's channels-last [B][T][C].
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

# ----------------------------------------------------------------------------------
# A1/A2  mu-law codec
# ----------------------------------------------------------------------------------


def mu_encode_np(x, n_quanta):
    """ops.py:23-28 (numpy variant): amp = sign(x)·log1p(mu|x|)/log1p(mu);
    quant = (amp+1)·0.5·mu + 0.5, truncated to int32."""
    mu = n_quanta - 1
    amp = np.sign(x) * np.log1p(mu * np.abs(x)) / np.log1p(mu)
    quant = (amp + 1) * 0.5 * mu + 0.5
    return quant.astype(np.int32)


def mu_decode_np(quant, n_quanta):
    """ops.py:31-39: a = (2q-1)/mu - 1; x = sign(a)·((1+mu)^|a| - 1)/mu."""
    mu = n_quanta - 1
    qf = np.asarray(quant).astype(np.float32)
    inv_mu = 1.0 / mu
    a = (2 * qf - 1) * inv_mu - 1
    return np.sign(a) * ((1 + mu) ** np.fabs(a) - 1) * inv_mu


def mu_encode_tf32(x, n_quanta):
    """ops.py:4-9 (TF variant, every op in float32, tf.to_int32 truncates)."""
    x = np.asarray(x, np.float32)
    mu = np.float32(n_quanta - 1)
    amp = np.sign(x) * np.log1p(mu * np.abs(x)) / np.log1p(mu)
    quant = (amp + np.float32(1)) * np.float32(0.5) * mu + np.float32(0.5)
    return quant.astype(np.float32).astype(np.int32)


def mu_decode_tf32(quant, n_quanta):
    """ops.py:12-20 (TF variant, float32)."""
    mu = np.float32(n_quanta - 1)
    qf = np.asarray(quant).astype(np.float32)
    inv_mu = np.float32(1.0) / mu
    a = (np.float32(2) * qf - np.float32(1)) * inv_mu - np.float32(1)
    return (np.sign(a) * ((np.float32(1) + mu) ** np.abs(a) - np.float32(1)) * inv_mu).astype(np.float32)


# ----------------------------------------------------------------------------------
# A3  receptive field, dealer and the invalid-window mask
# ----------------------------------------------------------------------------------


def recep_field_sz(n_blocks, n_block_layers):
    """tmodel.py:50-51."""
    return n_blocks * sum(2 ** l for l in range(n_block_layers))


def _slot_generator(files, slice_sz, recep_field_sz, mel_hop_sz, mel_spectrum_sz, log):
    """data.py:115-190 (gen_fcn): virtually concatenate files into slice_sz pieces.
    ``files`` is ONE iterator shared by every slot (data.py:211)."""
    need_sz = slice_sz
    spliced_wav = np.empty(0, np.float64)
    spliced_mel = np.empty([0, mel_spectrum_sz], np.float64)
    spliced_ids = np.empty(0, np.int32)
    recep_bound = recep_field_sz - 1

    def mc(v):
        return v // mel_hop_sz

    while True:
        try:
            vid, wav, mel = next(files)
            snip = len(wav) % mel_hop_sz
            wav = wav[:-snip or None]
            if len(wav) != len(mel) * mel_hop_sz:
                log.append(('len_mismatch', len(wav), len(mel) * mel_hop_sz))
        except StopIteration:
            break
        wav_sz = wav.shape[0]
        if wav_sz < recep_field_sz:
            log.append(('skip', wav_sz, vid, recep_field_sz))
            continue
        ids = np.concatenate([np.full(recep_bound, 0, np.int32),
                              np.full(wav_sz - recep_bound, vid, np.int32)])
        cur_pos = 0
        while need_sz <= (wav_sz - cur_pos):
            spliced_wav = np.append(spliced_wav, wav[cur_pos:cur_pos + need_sz], axis=0)
            spliced_mel = np.append(spliced_mel, mel[mc(cur_pos):mc(cur_pos + need_sz)], axis=0)
            spliced_ids = np.append(spliced_ids, ids[cur_pos:cur_pos + need_sz], axis=0)
            cur_pos += need_sz
            yield spliced_wav, spliced_mel, spliced_ids
            spliced_wav = np.empty(0, np.float64)
            spliced_mel = np.empty([0, mel_spectrum_sz], np.float64)
            spliced_ids = np.empty(0, np.int32)
            need_sz = slice_sz
        if cur_pos != wav_sz:
            spliced_wav = np.append(spliced_wav, wav[cur_pos:], axis=0)
            spliced_mel = np.append(spliced_mel, mel[mc(cur_pos):], axis=0)
            spliced_ids = np.append(spliced_ids, ids[cur_pos:], axis=0)
            need_sz -= (wav_sz - cur_pos)


def deal_batches(file_list, batch_sz, slice_sz, recep_field_sz, mel_hop_sz, mel_spectrum_sz):
    """data.py:194-227 (_gen_slice_batch): B slot generators over one shared file
    iterator, advanced in slot order; stops at the first exhausted slot.
    Returns (list of (wav[B,T], mel[B,T/hop,C], ids[B,T]), log)."""
    log = []
    files = iter(file_list)
    gens = [_slot_generator(files, slice_sz, recep_field_sz, mel_hop_sz, mel_spectrum_sz, log)
            for _ in range(batch_sz)]
    out = []
    while True:
        try:
            batch = [next(g) for g in gens]
        except StopIteration:
            break
        out.append((np.stack([b[0] for b in batch]), np.stack([b[1] for b in batch]),
                    np.stack([b[2] for b in batch])))
    return out, log


# ----------------------------------------------------------------------------------
# A15  parameter table (arch.py:85-103, names arch.py:142)
# ----------------------------------------------------------------------------------


def n_layers(arch):
    return arch['n_blocks'] * arch['n_block_layers']


def layer_index(arch, l):
    """(b, bl, dilation) for flat layer l (tmodel.py:313-325)."""
    nbl = arch['n_block_layers']
    return l // nbl, l % nbl, 2 ** (l % nbl)


def param_shapes(arch):
    """Ordered {serial_name: (shape, trainable, is_bias)} in reference layout."""
    Q, Cr, Cd, Cs, Cp = arch['n_quant'], arch['n_res'], arch['n_dil'], arch['n_skip'], arch['n_post']
    Ge, Gc = arch['n_gc_embed'], arch['n_gc_category']
    Li, Lo = arch['n_lc_in'], arch['n_lc_out']
    ub = arch['use_bias']
    p = OrderedDict()
    if Ge > 0:
        p['GC_EMBED'] = ([Gc + 1, Ge], True, False)
    p['PRE'] = ([Q, Cr], True, False)
    if ub:
        p['PRE_BIAS'] = ([Cr], True, True)
    if Lo > 0:
        for i, s in enumerate(arch['lc_upsample']):
            p['LC_UPSAMPLE_%d' % i] = ([s, Lo, Li if i == 0 else Lo], True, False)
    for l in range(n_layers(arch)):
        b, bl, _ = layer_index(arch, l)
        sfx = '_%d_%d' % (b, bl)
        for nm in ('SIGNAL', 'GATE'):
            p[nm + sfx] = ([2, Cr, Cd], True, False)
            if ub:
                p[nm + '_BIAS' + sfx] = ([Cd], True, True)
        if Ge > 0:
            p['GC_SIGNAL' + sfx] = ([Ge, Cd], True, False)
            p['GC_GATE' + sfx] = ([Ge, Cd], True, False)
        if Lo > 0:
            p['LC_SIGNAL' + sfx] = ([Lo, Cd], True, False)
            p['LC_GATE' + sfx] = ([Lo, Cd], True, False)
        p['RESIDUAL' + sfx] = ([Cd, Cr], True, False)
        if ub:
            p['RESIDUAL_BIAS' + sfx] = ([Cr], True, True)
        p['SKIP' + sfx] = ([Cd, Cs], True, False)
        if ub:
            p['SKIP_BIAS' + sfx] = ([Cs], True, True)
    p['POST1'] = ([Cs, Cp], True, False)
    if ub:
        p['POST1_BIAS'] = ([Cp], True, True)
    p['POST2'] = ([Cp, Q], True, False)
    if ub:
        p['POST2_BIAS'] = ([Q], True, True)
    return p


def save_shapes(arch, batch_sz):
    """SAVE_{d}_{b}_{bl} of shape [B, d, n_res] (arch.py:82-83, :100; tmodel.py:123)."""
    out = OrderedDict()
    for l in range(n_layers(arch)):
        b, bl, d = layer_index(arch, l)
        out['SAVE_%d_%d_%d' % (d, b, bl)] = [batch_sz, d, arch['n_res']]
    return out


def xavier_limit(shape):
    """tf.contrib.layers.xavier_initializer(_conv2d) fan computation (arch.py:63)."""
    if len(shape) == 0:
        fi = fo = 1
    elif len(shape) == 1:
        fi = fo = shape[0]
    elif len(shape) == 2:
        fi, fo = shape
    else:
        rf = int(np.prod(shape[:-2]))
        fi, fo = shape[-2] * rf, shape[-1] * rf
    return math.sqrt(6.0 / (fi + fo))


def init_params(arch, rng, bias_scale=0.0, dtype=np.float64):
    """Xavier-uniform weights, biases U(-bias_scale, bias_scale) (0 = reference zeros)."""
    out = OrderedDict()
    for name, (shape, _, is_bias) in param_shapes(arch).items():
        if is_bias:
            v = rng.uniform(-bias_scale, bias_scale, size=shape) if bias_scale else np.zeros(shape)
        else:
            lim = xavier_limit(shape)
            v = rng.uniform(-lim, lim, size=shape)
        out[name] = v.astype(dtype)
    return out


def init_save(arch, batch_sz, rng, dtype=np.float64):
    out = OrderedDict()
    for name, shape in save_shapes(arch, batch_sz).items():
        lim = xavier_limit(shape)
        out[name] = rng.uniform(-lim, lim, size=shape).astype(dtype)
    return out


# ----------------------------------------------------------------------------------
# A4-A13  training forward + loss  (tmodel.py:53-289)
# ----------------------------------------------------------------------------------


def _sigmoid(x):
    return 0.5 * (1.0 + np.tanh(0.5 * x))


def lc_upsample_fwd(arch, P, mel):
    """tmodel.py:68-83: tf.contrib.nn.conv1d_transpose with kernel = stride = s, SAME
    => out[b, s·t + j, o] = Σ_i in[b, t, i] · F[j, o, i]  (non-overlapping)."""
    acts = [mel]
    cur = mel
    for i, s in enumerate(arch['lc_upsample']):
        F = P['LC_UPSAMPLE_%d' % i]                     # [s, O, I]
        B_, T_, _ = cur.shape
        out = np.einsum('bti,joi->btjo', cur, F).reshape(B_, T_ * s, F.shape[1])
        cur = out
        acts.append(cur)
    return cur, acts


def lc_upsample_bwd(arch, P, acts, dout, grads):
    for i in reversed(range(len(arch['lc_upsample']))):
        s = arch['lc_upsample'][i]
        F = P['LC_UPSAMPLE_%d' % i]
        inp = acts[i]
        B_, T_, _ = inp.shape
        d4 = dout.reshape(B_, T_, s, F.shape[1])
        grads['LC_UPSAMPLE_%d' % i] = np.einsum('btjo,bti->joi', d4, inp)
        dout = np.einsum('btjo,joi->bti', d4, F)
    return dout


def forward(arch, P, wav_q, ids, save, mel=None):
    """tmodel.py:292-327.  wav_q int [B,T] (mu_law_quant input), ids int [B,T],
    save {SAVE_*: [B,d,Cr]}.  Returns (logits[B,T,Q], cache, new_save)."""
    dt = P['PRE'].dtype
    B, T = wav_q.shape
    L = n_layers(arch)
    ub = arch['use_bias']
    x = P['PRE'][wav_q]                                   # one-hot · PRE == row gather
    if ub:
        x = x + P['PRE_BIAS']
    lc = None
    lc_acts = None
    if arch['n_lc_out'] > 0:
        lc, lc_acts = lc_upsample_fwd(arch, P, mel.astype(dt))
    emb = P['GC_EMBED'][ids] if arch['n_gc_embed'] > 0 else None
    S = np.zeros((B, T, arch['n_skip']), dt)
    cache = {'x': [], 'prev': [], 'th': [], 'sg': [], 'z': [], 'lc': lc, 'lc_acts': lc_acts,
             'emb': emb, 'wav_q': wav_q, 'ids': ids}
    new_save = OrderedDict()
    for l in range(L):
        b, bl, d = layer_index(arch, l)
        sfx = '_%d_%d' % (b, bl)
        sv = save['SAVE_%d%s' % (d, sfx)].astype(dt)
        full = np.concatenate([sv, x], axis=1)            # tmodel.py:127
        prev = full[:, :T]                                # tap 0 <-> x[t-d]
        v = {}
        for nm in ('SIGNAL', 'GATE'):
            W = P[nm + sfx]
            v[nm] = prev @ W[0] + x @ W[1]                # tmodel.py:143-144 (VALID, dilation d)
            if ub:
                v[nm] = v[nm] + P[nm + '_BIAS' + sfx]
        if emb is not None:                               # tmodel.py:150-154
            v['SIGNAL'] = v['SIGNAL'] + emb @ P['GC_SIGNAL' + sfx]
            v['GATE'] = v['GATE'] + emb @ P['GC_GATE' + sfx]
        if lc is not None:                                # tmodel.py:155-160
            v['SIGNAL'] = v['SIGNAL'] + lc @ P['LC_SIGNAL' + sfx]
            v['GATE'] = v['GATE'] + lc @ P['LC_GATE' + sfx]
        new_save['SAVE_%d%s' % (d, sfx)] = full[:, -d:].copy()   # tmodel.py:165
        th = np.tanh(v['SIGNAL'])
        sg = _sigmoid(v['GATE'])
        z = th * sg                                       # tmodel.py:167
        res = z @ P['RESIDUAL' + sfx]                     # tmodel.py:171-184
        skp = z @ P['SKIP' + sfx]
        if ub:
            res = res + P['RESIDUAL_BIAS' + sfx]
            skp = skp + P['SKIP_BIAS' + sfx]
        cache['x'].append(x)
        cache['prev'].append(prev)
        cache['th'].append(th)
        cache['sg'].append(sg)
        cache['z'].append(z)
        S = S + skp
        x = x + res
    cache['x_out'] = x
    cache['S'] = S
    h1 = np.maximum(S, 0) @ P['POST1']                    # tmodel.py:187-215
    if ub:
        h1 = h1 + P['POST1_BIAS']
    r2 = np.maximum(h1, 0)
    logits = r2 @ P['POST2']
    if ub:
        logits = logits + P['POST2_BIAS']
    cache['h1'] = h1
    cache['r2'] = r2
    return logits, cache, new_save


def l2_loss(P, shapes=None):
    """tmodel.py:250-261: Σ over trainable non-BIAS vars of tf.nn.l2_loss = Σv²/2."""
    tot = 0.0
    for k, v in P.items():
        if 'BIAS' in k:
            continue
        tot += 0.5 * float(np.sum(np.asarray(v, np.float64) ** 2))
    return tot


def loss_fcn(arch, P, logits, wav_q, ids, l2_factor):
    """tmodel.py:218-289.  Returns dict(total, mean_xent, l2, avg_diff, n_valid,
    sum_xent) and dlogits of the mean xent (zeros when n_valid == 0)."""
    B, T, Q = logits.shape
    lg = logits[:, :-1, :]                                # logits[t] predicts input[t+1]
    tgt = wav_q[:, 1:]
    mask = (ids[:, 1:] != 0)
    m = lg.max(axis=2, keepdims=True)
    e = np.exp(lg - m)
    se = e.sum(axis=2, keepdims=True)
    lse = (m + np.log(se))[..., 0]
    picked = np.take_along_axis(lg, tgt[..., None], axis=2)[..., 0]
    xent = lse - picked
    n_valid = int(mask.sum())
    sum_xent = float((xent * mask).sum())
    mean = sum_xent / n_valid if n_valid else 0.0
    diffs = tgt.astype(np.int64) - np.argmax(lg, axis=2).astype(np.int64)
    sum_absdiff = int(np.abs(diffs * mask).sum())
    avg_diff = sum_absdiff // (B * (T - 1))   # int32 reduce_mean
    l2 = l2_loss(P)
    total = mean + l2_factor * l2
    dlog = np.zeros_like(logits)
    if n_valid:
        sm = e / se
        onehot = np.zeros_like(lg)
        np.put_along_axis(onehot, tgt[..., None], 1.0, axis=2)
        dlog[:, :-1, :] = (sm - onehot) * mask[..., None] / n_valid
    stats = dict(total=total, mean_xent=mean, l2=l2, avg_diff=avg_diff, n_valid=n_valid,
                 sum_xent=sum_xent, sum_absdiff=sum_absdiff)
    return stats, dlog


def backward(arch, P, cache, dlogits, l2_factor):
    """Reverse-mode derivative of tmodel's total loss (TF autodiff restated,
    tmodel.py:354-358).  Returns {name: grad} for every trainable parameter,
    including the l2_factor·θ term for non-BIAS vars."""
    ub = arch['use_bias']
    L = n_layers(arch)
    g = OrderedDict((k, np.zeros_like(v)) for k, v in P.items())
    r2, h1, S = cache['r2'], cache['h1'], cache['S']
    g['POST2'] += np.einsum('btp,btq->pq', r2, dlogits)
    if ub:
        g['POST2_BIAS'] += dlogits.sum(axis=(0, 1))
    dh1 = (dlogits @ P['POST2'].T) * (h1 > 0)
    g['POST1'] += np.einsum('bts,btp->sp', np.maximum(S, 0), dh1)
    if ub:
        g['POST1_BIAS'] += dh1.sum(axis=(0, 1))
    dS = (dh1 @ P['POST1'].T) * (S > 0)
    dx = np.zeros_like(cache['x_out'])
    emb, lc = cache['emb'], cache['lc']
    demb = np.zeros_like(emb) if emb is not None else None
    dlc = np.zeros_like(lc) if lc is not None else None
    for l in reversed(range(L)):
        b, bl, d = layer_index(arch, l)
        sfx = '_%d_%d' % (b, bl)
        z, th, sg = cache['z'][l], cache['th'][l], cache['sg'][l]
        x, prev = cache['x'][l], cache['prev'][l]
        g['SKIP' + sfx] += np.einsum('btc,bts->cs', z, dS)
        g['RESIDUAL' + sfx] += np.einsum('btc,btr->cr', z, dx)
        if ub:
            g['SKIP_BIAS' + sfx] += dS.sum(axis=(0, 1))
            g['RESIDUAL_BIAS' + sfx] += dx.sum(axis=(0, 1))
        dz = dS @ P['SKIP' + sfx].T + dx @ P['RESIDUAL' + sfx].T
        dv = {'SIGNAL': dz * sg * (1 - th * th), 'GATE': dz * th * sg * (1 - sg)}
        dprev = np.zeros_like(x)
        dcur = np.zeros_like(x)
        for nm in ('SIGNAL', 'GATE'):
            W = P[nm + sfx]
            g[nm + sfx][0] += np.einsum('btr,btc->rc', prev, dv[nm])
            g[nm + sfx][1] += np.einsum('btr,btc->rc', x, dv[nm])
            if ub:
                g[nm + '_BIAS' + sfx] += dv[nm].sum(axis=(0, 1))
            dprev += dv[nm] @ W[0].T
            dcur += dv[nm] @ W[1].T
        if emb is not None:
            g['GC_SIGNAL' + sfx] += np.einsum('bte,btc->ec', emb, dv['SIGNAL'])
            g['GC_GATE' + sfx] += np.einsum('bte,btc->ec', emb, dv['GATE'])
            demb += dv['SIGNAL'] @ P['GC_SIGNAL' + sfx].T + dv['GATE'] @ P['GC_GATE' + sfx].T
        if lc is not None:
            g['LC_SIGNAL' + sfx] += np.einsum('bti,btc->ic', lc, dv['SIGNAL'])
            g['LC_GATE' + sfx] += np.einsum('bti,btc->ic', lc, dv['GATE'])
            dlc += dv['SIGNAL'] @ P['LC_SIGNAL' + sfx].T + dv['GATE'] @ P['LC_GATE' + sfx].T
        dxn = dx + dcur
        if d < dx.shape[1]:
            dxn[:, :-d] += dprev[:, d:]                    # gradient into SAVE is dropped
        dx = dxn
    np.add.at(g['PRE'], cache['wav_q'], dx)
    if ub:
        g['PRE_BIAS'] += dx.sum(axis=(0, 1))
    if emb is not None:
        np.add.at(g['GC_EMBED'], cache['ids'], demb)
    if lc is not None:
        lc_upsample_bwd(arch, P, cache['lc_acts'], dlc, g)
    for k in g:
        if 'BIAS' not in k:
            g[k] = g[k] + l2_factor * P[k]
    return g


class AdamTF1:
    """tf.train.AdamOptimizer (TF1 defaults β1=.9, β2=.999, ε=1e-8; train.py:178):
    lr_t = lr·√(1-β2^t)/(1-β1^t);  m = β1m+(1-β1)g;  v = β2v+(1-β2)g²;
    θ -= lr_t·m/(√v + ε)."""

    def __init__(self, lr, b1=0.9, b2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps
        self.t = 0
        self.m, self.v = {}, {}

    def step(self, P, G):
        self.t += 1
        lr_t = self.lr * math.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        for k in P:
            m = self.m.get(k, np.zeros_like(P[k]))
            v = self.v.get(k, np.zeros_like(P[k]))
            m = self.b1 * m + (1 - self.b1) * G[k]
            v = self.b2 * v + (1 - self.b2) * G[k] * G[k]
            self.m[k], self.v[k] = m, v
            P[k] = P[k] - lr_t * m / (np.sqrt(v) + self.eps)
        return P


# ----------------------------------------------------------------------------------
# G1-G5  cached single-step generation (imodel.py:61-272)
# ----------------------------------------------------------------------------------

def philox_uniform(seed, stream, step):
    """Counter-based uniform in [0,1): splitmix64 over (seed, stream, step).  The
    reference draws with tf.multinomial (TF RNG, not reproducible); the build's sampler
    takes uniforms from this hash so GPU and oracle draw the same variates."""
    M = (1 << 64) - 1
    z = (seed * 0x9E3779B97F4A7C15 + (stream << 32) + step + 0x632BE59BD9B4E019) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    z = z ^ (z >> 31)
    return (z >> 40) / float(1 << 24)


def sample_from_logits(logits_row, u):
    """Inverse-CDF draw of softmax(logits): smallest k with cumsum(p)[k] > u·Σp.
    Restates tf.multinomial(logits, 1) (imodel.py:179) as a deterministic transform."""
    m = np.max(logits_row)
    e = np.exp(logits_row - m)
    c = np.cumsum(e)
    k = int(np.searchsorted(c, u * c[-1], side='right'))
    return min(k, len(logits_row) - 1)


def generate(arch, P, batch_sz, n_steps, seed=0, teacher_q=None, gc_ids=None,
             pre_bias=True, return_logits=False, forced_q=None, start=0, init_rings=None, init_q=None,
             return_state=False):
    """imodel.py:214-272 restated with ring lookback buffers (semantically the
    reference's shift-by-chunk buffers, imodel.py:88-98, :190-207).
    Step i: input = zero vector (i=0) else onehot(prev draw) or onehot(teacher_q[i-1]).
    ``pre_bias``=True adds PRE_BIAS (tmodel-consistent; imodel.py:75-77 omits it).
    ``forced_q`` [B, >= n-1] (test use): step i's input is forced_q[:, i-1] per stream instead
    of this run's own draw, so the logits and draws are evaluated along another run's
    trajectory (e.g. the GPU's) and compared draw by draw without a single near-tie flip
    making the two streams diverge.
    Resuming (test use): ``start`` = the global index of this call's first step (ring slot
    (start + i) mod d, the draw's uniform of step start + i), ``init_rings`` = every layer's
    [B, d, Cr] ring at that point (layer order, slot = step mod d, as the GPU's "rings"), and
    ``init_q`` [B] = the code the first step takes as input (the previous step's draw);
    ``return_state`` appends the rings after the last step (the next call's init_rings).
    Returns (samples int[B,n], wav float[B,n], [logits[B,n,Q]], [rings])."""
    dt = P['PRE'].dtype
    L = n_layers(arch)
    ub = arch['use_bias']
    Cr = arch['n_res']
    rings = []
    for l in range(L):
        _, _, d = layer_index(arch, l)
        rings.append(np.zeros((batch_sz, d, Cr), dt) if init_rings is None
                     else np.array(init_rings[l], dt).reshape(batch_sz, d, Cr))   # ring of the last d inputs
    gce = None
    if arch['n_gc_embed'] > 0:
        gce = P['GC_EMBED'][np.asarray(gc_ids)]
    samples = np.zeros((batch_sz, n_steps), np.int32)
    all_logits = np.zeros((batch_sz, n_steps, arch['n_quant']), dt) if return_logits else None
    prev_q = None
    for i in range(n_steps):
        t = start + i
        if i == 0 and init_q is not None:
            z = P['PRE'][np.asarray(init_q, np.int64)].copy()
        elif i == 0:
            assert start == 0, 'a resumed run needs init_q'
            z = np.zeros((batch_sz, Cr), dt)
        else:
            if teacher_q is not None and i - 1 < len(teacher_q):
                q = np.full(batch_sz, teacher_q[i - 1], np.int64)
            elif forced_q is not None:
                q = np.asarray(forced_q[:, i - 1], np.int64)
            else:
                q = prev_q
            z = P['PRE'][q].copy()
        if pre_bias and ub:
            z = z + P['PRE_BIAS']
        skip = np.zeros((batch_sz, arch['n_skip']), dt)
        for l in range(L):
            b, bl, d = layer_index(arch, l)
            sfx = '_%d_%d' % (b, bl)
            slot = t % d
            prev = rings[l][:, slot].copy()                # input d steps ago (0 if none)
            rings[l][:, slot] = z
            v = {}
            for nm in ('SIGNAL', 'GATE'):
                W = P[nm + sfx]
                v[nm] = prev @ W[0] + z @ W[1]             # imodel.py:107-108
                if ub:
                    v[nm] = v[nm] + P[nm + '_BIAS' + sfx]
            if gce is not None:
                v['SIGNAL'] = v['SIGNAL'] + gce @ P['GC_SIGNAL' + sfx]
                v['GATE'] = v['GATE'] + gce @ P['GC_GATE' + sfx]
            zz = np.tanh(v['SIGNAL']) * _sigmoid(v['GATE'])
            res = zz @ P['RESIDUAL' + sfx]
            skp = zz @ P['SKIP' + sfx]
            if ub:
                res = res + P['RESIDUAL_BIAS' + sfx]
                skp = skp + P['SKIP_BIAS' + sfx]
            skip = skip + skp
            z = z + res
        h1 = np.maximum(skip, 0) @ P['POST1']
        if ub:
            h1 = h1 + P['POST1_BIAS']
        lg = np.maximum(h1, 0) @ P['POST2']
        if ub:
            lg = lg + P['POST2_BIAS']
        if return_logits:
            all_logits[:, i] = lg
        q = np.array([sample_from_logits(lg[bb], philox_uniform(seed, bb, t))
                      for bb in range(batch_sz)], np.int64)
        samples[:, i] = q
        prev_q = q
    wav = mu_decode_tf32(samples, arch['n_quant'])
    out = (samples, wav) + ((all_logits,) if return_logits else ()) + ((rings,) if return_state else ())
    return out


# ----------------------------------------------------------------------------------
# README influence-diagram known-answer test (README.md:62-85, images/wavenet_influence.png)
# ----------------------------------------------------------------------------------

def influence_stack(x, dilations, save=None):
    """Plain dilated stack, every filter [0.5, 0.5] (tap0·x[t-d] + tap1·x[t]), no gate/
    residual; D-separation prepend/save exactly as tmodel.py:122-127/:165.
    Returns (rows [len(dilations)+1, T] bottom=input, new_save list)."""
    rows = [np.asarray(x, np.float64)]
    cur = rows[0]
    new_save = []
    for li, d in enumerate(dilations):
        sv = np.zeros(d) if save is None else save[li]
        full = np.concatenate([sv, cur])
        out = 0.5 * full[:len(cur)] + 0.5 * cur
        new_save.append(full[-d:].copy())
        cur = out
        rows.append(cur)
    return np.stack(rows), new_save
