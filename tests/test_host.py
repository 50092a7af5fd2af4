"""Host-side (CPU) logic of the product package: arch normalisation, parameter layout,
and the slice dealer against the reference's own golden vectors."""
import os

import numpy as np
import pytest

from lbwn import arch as A
from lbwn.data import SliceDealer, SyntheticSource
from oracle import wavenet_ref as R
from tests.conftest import GOLDEN, ROOT
from tests.golden.make_golden import CASES, make_files


@pytest.mark.parametrize('name', ['small', 'hop4_b3', 'hop256_b4', 'recep5115_b2', 'hop4_b3_resume'])
def test_product_dealer_matches_reference_golden(name):
    """wav/mel/ids and latest_file_read_count (data.py:220) against the reference's own
    dealer; the _resume case starts at ckpt_position = 6 (data.py:79, :250)."""
    g = np.load(os.path.join(GOLDEN, 'dealer_%s.npz' % name))
    if name == 'small':
        files = [(int(g['file_vid_%d' % i]), g['file_wav_%d' % i], g['file_mel_%d' % i])
                 for i in range(int(g['n_files']))]
    else:
        seed, nf, lo, hi, B, T, F, hop, nmel, mv = CASES[name.replace('_resume', '')]
        files = make_files(seed, nf, lo, hi, hop, nmel, mv)
    B, T, F, hop, nmel, start = (int(g[k]) for k in ('B', 'T', 'F', 'hop', 'nmel', 'start'))
    import io
    d = SliceDealer(files[start:], B, T, F, hop, nmel, log=io.StringIO(), start=start)
    out = list(d)
    assert len(out) == int(g['n_batches'])
    for j, (cnt, w, m, ids) in enumerate(out):
        assert cnt == int(g['cnt_%d' % j]), j
        np.testing.assert_array_equal(ids, g['ids_%d' % j])
        np.testing.assert_array_equal(w.astype(np.int64), g['wav_%d' % j])
        np.testing.assert_array_equal(m.astype(np.int64), g['mel_%d' % j])


@pytest.mark.parametrize('f', ['arch1', 'arch2', 'arch3', 'arch4', 'arch5'])
def test_normalize_shipped_arch_files(f):
    gc = 10 if f in ('arch2', 'arch4') else None
    a = A.load_arch(os.path.join(ROOT, 'par', f + '.json'), num_global_cond=gc)
    assert set(a) == set(A.ARCH_KEYS)
    assert A.recep_field_sz(a) == 5115
    lay = A.ParamLayout(a)
    shapes = R.param_shapes(a)
    assert set(lay.entries) == set(shapes)
    for n, e in lay.entries.items():
        assert e.shape == shapes[n][0] and e.is_bias == shapes[n][2], n
        assert (e.offset < lay.n_weights) == (not e.is_bias)
    assert all(o % 4 == 0 for o in lay.kind_base.values())
    # per-layer kinds are dense (the engine addresses layer l at base + l·numel)
    for kind, base in lay.kind_base.items():
        es = sorted((e for n, e in lay.entries.items() if lay._kind_of[n] == kind), key=lambda e: e.offset)
        assert es[0].offset == base
        for a, b in zip(es, es[1:]):
            assert b.offset == a.offset + a.numel, (kind, b.name)


def test_arch_param_counts():
    a3 = A.load_arch(os.path.join(ROOT, 'par', 'arch3.json'))
    assert sum(e.numel for e in A.ParamLayout(a3).entries.values()) == 1507808
    a5 = A.load_arch(os.path.join(ROOT, 'par', 'arch5.json'))
    assert sum(e.numel for e in A.ParamLayout(a5).entries.values()) == 1923440
    a1 = A.load_arch(os.path.join(ROOT, 'par', 'arch1.json'))
    assert sum(e.numel for e in A.ParamLayout(a1).entries.values()) == 1568634


def test_arch_errors():
    with pytest.raises(A.ArchError):
        A.load_arch(os.path.join(ROOT, 'par', 'arch2.json'))       # no n_gc_category, no -gc
    with pytest.raises(A.ArchError):
        A.normalize_arch(dict(A.load_arch(os.path.join(ROOT, 'par', 'arch3.json')), bogus=1))


def test_synthetic_source_shapes():
    s = SyntheticSource(seed=1, n_mel=80, n_voices=5)
    for _ in range(3):
        vid, wav, mel = next(s)
        assert 1 <= vid <= 5 and len(wav) % 256 == 0 and 16000 <= len(wav) + 256 and len(wav) <= 64000
        assert wav.dtype == np.int32 and wav.min() >= 0 and wav.max() <= 255
        assert mel.shape == (len(wav) // 256, 80)
