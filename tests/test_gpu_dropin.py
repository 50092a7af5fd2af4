"""The drop-in entry points end to end on the GPU: train.py on a .npy sample catalog
(train.py:12-244: train, checkpoint at --save-interval, resume from --resume-step) and
generate.py from the resulting checkpoint (generate.py:1-120)."""
import json
import os
import sys

import numpy as np
import pytest
import torch

from lbwn.ckpt import ckpt_file, load_tensors
from lbwn.ops import mu_encode_np
from tests.conftest import ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))


def _dataset(tmp_path, n_files=6, voices=3):
    rng = np.random.default_rng(0)
    lines = []
    for i in range(n_files):
        n = int(rng.integers(600, 1400))
        t = np.arange(n) / 16000.0
        x = 0.8 * np.sin(2 * np.pi * rng.uniform(100, 300) * t) + rng.normal(0, 0.05, n)
        wav = mu_encode_np(np.clip(x, -1, 1), 256).astype(np.int32)
        wp, mp = tmp_path / ('w%d.npy' % i), tmp_path / ('m%d.npy' % i)
        np.save(wp, wav)
        np.save(mp, np.zeros((n, 0), np.float32))
        lines.append('%d\t%s\t%s' % (i % voices + 1, wp, mp))
    cat = tmp_path / 'samples.txt'
    cat.write_text('\n'.join(lines) + '\n')
    return str(cat)


def test_train_resume_generate(tmp_path, capsys):
    import generate
    import train
    arch = dict(n_blocks=1, n_block_layers=4, n_quant=256, n_res=32, n_dil=32, n_skip=64, n_post=32,
                n_gc_embed=8, n_gc_category=3, n_lc_in=0, n_lc_out=0, lc_upsample=[], use_bias=True,
                wav_input_type='mu_law_quant')
    par = dict(batch_sz=2, sample_rate=16000, slice_sz=128, l2_factor=1e-3, learning_rate=1e-3, prefetch_sz=4,
               add_summary=False, n_keep_checkpoints=3, n_valid_total=100000)
    af, pf = tmp_path / 'arch.json', tmp_path / 'par.json'
    af.write_text(json.dumps(arch))
    pf.write_text(json.dumps(par))
    cat = _dataset(tmp_path)
    pfx = str(tmp_path / 'ck' / 'run')
    net = train.main(['--max-steps', '5', '--save-interval', '2', '--progress-interval', '1', '--seed', '1',
                      pfx, str(af), str(pf), cat])
    err = capsys.readouterr().err
    assert 'Starting training...' in err and 'Saved checkpoints to' in err
    lines = [l for l in err.splitlines() if l and l.split('\t')[0].strip().isdigit()]
    assert len(lines) >= 4                             # progress columns, tmodel.py:263-267
    assert all(np.isfinite(float(l.split('\t')[1])) for l in lines)
    assert int(net.counters[0]) == 4                   # steps 1..4 (train.py:213 loop)
    for s in (2, 4):
        assert os.path.exists(ckpt_file(pfx + '.net', s)) and os.path.exists(ckpt_file(pfx + '.dset', s))
    t = load_tensors(pfx + '.net-4')
    assert int(t['GLOBAL_STEP'][0]) == 4
    np.testing.assert_array_equal(t['SIGNAL_0_3'].numpy(), net.vars['SIGNAL_0_3'].cpu().numpy())
    # resume from step 4 and take two more steps
    net2 = train.main(['--max-steps', '7', '--resume-step', '4', '--save-interval', '2', pfx, str(af), str(pf), cat])
    assert int(net2.counters[0]) == 7                  # the reference resumes AT resume_step (train.py:212)
    assert os.path.exists(ckpt_file(pfx + '.net', 6))
    assert 'Restored net and dset from checkpoint' in capsys.readouterr().err
    # generate from the step-6 checkpoint (GC arch: voice ids cycled over the batch)
    wav = generate.main(['--gen-seconds', '0.05', '--batch-size', '3', '--chunk-size', '200', '--gc-ids', '1,3',
                         str(af), pfx + '.net-6', str(tmp_path / 'out')])
    assert wav.shape == (3, 800)
    assert np.all(np.abs(wav) <= 1.03)
    for i in range(3):
        assert os.path.exists(tmp_path / 'out' / ('gen.i%d.wav' % i))
