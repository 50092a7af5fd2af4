"""Architecture surface: par/arch*.json normalisation, the ArchCat parameter table and the
flat fp32 parameter layout the HIP kernels consume.

Mirrors arch.py of the reference: ``ArchCat`` (arch.py:6-22), the shape table
(arch.py:85-103) and serial names ``NAME[_BIAS]_{indices}`` (arch.py:142).  Every
trainable tensor is a view into ONE flat buffer (so Adam, the L2 term and the
data-parallel all-reduce each run as a single kernel/bucket); per-layer tensors of one
kind are contiguous over layers, so kernels address them by (base, layer stride).
"""
import json
import math
from collections import OrderedDict
from enum import IntEnum


class ArchCat(IntEnum):
    """arch.py:6-22."""
    PRE = 1
    LC_UPSAMPLE = 2
    RESIDUAL = 3
    SKIP = 4
    SIGNAL = 5
    GATE = 6
    GC_SIGNAL = 7
    GC_GATE = 8
    GC_EMBED = 9
    LC_SIGNAL = 10
    LC_GATE = 11
    POST1 = 12
    POST2 = 13
    SAVE = 14
    GLOBAL_STEP = 15
    VALID_SAMPLES = 16


ARCH_KEYS = ('n_blocks', 'n_block_layers', 'n_quant', 'n_res', 'n_dil', 'n_skip', 'n_post',
             'n_gc_embed', 'n_gc_category', 'n_lc_in', 'n_lc_out', 'lc_upsample', 'use_bias',
             'wav_input_type')


class ArchError(ValueError):
    pass


def normalize_arch(arch, num_global_cond=None):
    """Bring any shipped par/arch*.json to the 14 keys WaveNetTrain takes (tmodel.py:10-23).

    Reference quirks handled: arch1/arch3 use the generator key ``n_post1``
    (par/arch1.json:8) and lack the LC keys and ``wav_input_type``; arch1 lacks
    ``use_bias``; arch2 lacks ``n_gc_category`` (needs -gc); arch4 carries ``lc_hop_sz``
    (par/arch4.json:12), which must equal prod(lc_upsample).  ``num_global_cond``
    overrides n_gc_category like train.py:140-146.
    """
    a = dict(arch)
    if 'n_post1' in a:
        a.setdefault('n_post', a.pop('n_post1'))
    a.setdefault('n_gc_embed', 0)
    a.setdefault('n_lc_in', 0)
    a.setdefault('n_lc_out', 0)
    a.setdefault('lc_upsample', [])
    a.setdefault('use_bias', True)
    a.setdefault('wav_input_type', 'mu_law_quant')
    if 'lc_hop_sz' in a:
        hop = a.pop('lc_hop_sz')
        if hop != _prod(a['lc_upsample']):
            raise ArchError('lc_hop_sz %d != prod(lc_upsample) %d' % (hop, _prod(a['lc_upsample'])))
    if num_global_cond is not None:
        a['n_gc_category'] = num_global_cond
    if 'n_gc_category' not in a:
        raise ArchError('Error: must provide n_gc_category in ARCH_FILE, or --num-global-cond')
    if a['n_gc_embed'] == 0:
        a['n_gc_category'] = a.get('n_gc_category', 0)
    missing = [k for k in ARCH_KEYS if k not in a]
    if missing:
        raise ArchError('arch is missing keys %s' % missing)
    extra = [k for k in a if k not in ARCH_KEYS]
    if extra:
        raise ArchError('arch has unknown keys %s' % extra)
    if a['wav_input_type'] not in ('mu_law_quant', 'raw'):
        raise ArchError('wav_input_type must be mu_law_quant or raw')
    a['use_bias'] = bool(a['use_bias'])
    a['lc_upsample'] = list(a['lc_upsample'])
    return a


def load_arch(path, num_global_cond=None):
    with open(path) as fp:
        return normalize_arch(json.load(fp), num_global_cond)


def _prod(xs):
    p = 1
    for x in xs:
        p *= x
    return p


def mel_hop_sz(arch):
    """train.py:130: reduce(mul, lc_upsample)."""
    return _prod(arch['lc_upsample'])


def n_layers(arch):
    return arch['n_blocks'] * arch['n_block_layers']


def recep_field_sz(arch):
    """tmodel.py:50-51."""
    return arch['n_blocks'] * sum(2 ** l for l in range(arch['n_block_layers']))


def layer_iter(arch):
    """(flat l, block b, layer bl, dilation) in tmodel.py:313-325 order."""
    for b in range(arch['n_blocks']):
        for bl in range(arch['n_block_layers']):
            yield b * arch['n_block_layers'] + bl, b, bl, 2 ** bl


def xavier_limit(shape):
    """tf.contrib.layers.xavier_initializer(_conv2d) (arch.py:63) fan computation."""
    if len(shape) == 0:
        fi = fo = 1
    elif len(shape) == 1:
        fi = fo = shape[0]
    elif len(shape) == 2:
        fi, fo = shape
    else:
        rf = _prod(shape[:-2])
        fi, fo = shape[-2] * rf, shape[-1] * rf
    return math.sqrt(6.0 / (fi + fo))


class Entry:
    __slots__ = ('name', 'shape', 'offset', 'numel', 'is_bias', 'cat')

    def __init__(self, name, shape, offset, is_bias, cat):
        self.name, self.shape, self.offset, self.is_bias, self.cat = name, list(shape), offset, is_bias, cat
        self.numel = _prod(shape)


class ParamLayout:
    """Flat fp32 layout.  Region [0, n_weights): non-BIAS trainables (get the L2 term,
    tmodel.py:250-261); [n_weights, n_total): biases.  Every kind (the per-layer arrays the
    engine addresses as base + l·numel, and the single tensors) starts at a multiple of 4
    floats; the layers of a kind are dense (no padding between them, e.g. RESIDUAL_BIAS
    [n_res = 3] of par/arch2.json at stride 3)."""

    def __init__(self, arch):
        self.arch = arch
        Q, Cr, Cd, Cs, Cp = (arch[k] for k in ('n_quant', 'n_res', 'n_dil', 'n_skip', 'n_post'))
        Ge, Gc, Li, Lo = arch['n_gc_embed'], arch['n_gc_category'], arch['n_lc_in'], arch['n_lc_out']
        ub = arch['use_bias']
        layers = list(layer_iter(arch))
        self.entries = OrderedDict()
        self._cur = 0
        self.kind_base = {}
        self._kind_of = {}

        def add(name, shape, is_bias, cat, kind=None):
            if kind is None or kind not in self.kind_base:
                self._cur = (self._cur + 3) // 4 * 4
                if kind is not None:
                    self.kind_base[kind] = self._cur
            e = Entry(name, shape, self._cur, is_bias, cat)
            self.entries[name] = e
            self._kind_of[name] = kind
            self._cur += e.numel

        def sfx(b, bl):
            return '_%d_%d' % (b, bl)

        add('PRE', [Q, Cr], False, ArchCat.PRE, 'pre')
        for kind, cat in (('sig', ArchCat.SIGNAL), ('gate', ArchCat.GATE)):
            for l, b, bl, d in layers:
                add(cat.name + sfx(b, bl), [2, Cr, Cd], False, cat, kind)
        for l, b, bl, d in layers:
            add('RESIDUAL' + sfx(b, bl), [Cd, Cr], False, ArchCat.RESIDUAL, 'res')
        for l, b, bl, d in layers:
            add('SKIP' + sfx(b, bl), [Cd, Cs], False, ArchCat.SKIP, 'skip')
        if Ge > 0:
            add('GC_EMBED', [Gc + 1, Ge], False, ArchCat.GC_EMBED, 'gc_embed')
            for kind, cat in (('gc_sig', ArchCat.GC_SIGNAL), ('gc_gate', ArchCat.GC_GATE)):
                for l, b, bl, d in layers:
                    add(cat.name + sfx(b, bl), [Ge, Cd], False, cat, kind)
        if Lo > 0:
            for i, s in enumerate(arch['lc_upsample']):
                add('LC_UPSAMPLE_%d' % i, [s, Lo, Li if i == 0 else Lo], False, ArchCat.LC_UPSAMPLE,
                    'lc_up%d' % i)
            for kind, cat in (('lc_sig', ArchCat.LC_SIGNAL), ('lc_gate', ArchCat.LC_GATE)):
                for l, b, bl, d in layers:
                    add(cat.name + sfx(b, bl), [Lo, Cd], False, cat, kind)
        add('POST1', [Cs, Cp], False, ArchCat.POST1, 'post1')
        add('POST2', [Cp, Q], False, ArchCat.POST2, 'post2')
        self.n_weights = self._cur = (self._cur + 3) // 4 * 4
        if ub:
            add('PRE_BIAS', [Cr], True, ArchCat.PRE, 'pre_b')
            for kind, cat in (('sig_b', ArchCat.SIGNAL), ('gate_b', ArchCat.GATE)):
                for l, b, bl, d in layers:
                    add(cat.name + '_BIAS' + sfx(b, bl), [Cd], True, cat, kind)
            for l, b, bl, d in layers:
                add('RESIDUAL_BIAS' + sfx(b, bl), [Cr], True, ArchCat.RESIDUAL, 'res_b')
            for l, b, bl, d in layers:
                add('SKIP_BIAS' + sfx(b, bl), [Cs], True, ArchCat.SKIP, 'skip_b')
            add('POST1_BIAS', [Cp], True, ArchCat.POST1, 'post1_b')
            add('POST2_BIAS', [Q], True, ArchCat.POST2, 'post2_b')
        self.n_total = (self._cur + 3) // 4 * 4
        self._check_contiguity()

    def _check_contiguity(self):
        # per-layer kinds must be dense arrays over layers for (base, stride) addressing
        for kind in set(self.kind_base):
            es = [e for e in self.entries.values() if self._kind_of.get(e.name) == kind]
            for i in range(1, len(es)):
                assert es[i].offset == es[i - 1].offset + es[i - 1].numel, (kind, es[i].name)

    def names(self):
        return list(self.entries)

    def views(self, flat):
        """{serial name: view of flat with the reference shape}."""
        out = OrderedDict()
        for n, e in self.entries.items():
            out[n] = flat[e.offset:e.offset + e.numel].view(*e.shape)
        return out


def save_layout(arch, batch_sz):
    """SAVE_{d}_{b}_{bl} [B, d, n_res] (arch.py:82-83, :100), packed in layer order."""
    out = OrderedDict()
    off = 0
    for l, b, bl, d in layer_iter(arch):
        shape = [batch_sz, d, arch['n_res']]
        out['SAVE_%d_%d_%d' % (d, b, bl)] = (off, shape)
        off += _prod(shape)
    return out, off
