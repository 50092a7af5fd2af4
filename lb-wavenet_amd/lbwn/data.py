"""Slice dealer and sample sources — drop-in for data.MaskedSliceWav's slicing logic.

``SliceDealer`` restates data.py:110-227: B slot generators over ONE shared file iterator
(data.py:211), advanced in slot order each step (data.py:217); every slot virtually
concatenates files into slice_sz pieces and emits ids = 0 for the first F-1 samples of
each file (the invalid, junction-spanning windows; data.py:133, :156-159) and the voice
id elsewhere.  Files shorter than F are skipped (data.py:150-154); wav is trimmed to a
multiple of the mel hop (data.py:141-142).  Bit-exact with the reference's own
generator (tests/golden/dealer_*.npz).

Sources: ``npy_catalog`` (the reference's tab-separated samples file of
``vid \t wav.npy \t mel.npy`` lines, data.py:43-48) and ``SyntheticSource`` (seeded
16 kHz harmonic tones) for benchmarks.
"""
import sys

import numpy as np

from .ops import mu_encode_np


class SliceDealer:
    def __init__(self, files, batch_sz, slice_sz, recep_field_sz, mel_hop_sz=1, mel_spectrum_sz=0,
                 log=sys.stderr):
        if slice_sz % mel_hop_sz != 0:      # data.py:32-36
            requested = slice_sz
            slice_sz += mel_hop_sz - (slice_sz % mel_hop_sz)
            print('Warning: aligning slice size from {} to {} for mel_hop_sz {}'.format(
                requested, slice_sz, mel_hop_sz), file=log)
        self.slice_sz = slice_sz
        self.batch_sz = batch_sz
        self.recep_field_sz = recep_field_sz
        self.mel_hop_sz = mel_hop_sz
        self.mel_spectrum_sz = mel_spectrum_sz
        self.log = log
        self.files_read = 0
        self._files = iter(files)
        self._gens = [self._slot() for _ in range(batch_sz)]

    def _next_file(self):
        vid, wav, mel = next(self._files)
        self.files_read += 1
        return vid, wav, mel

    def _slot(self):
        hop, F, T = self.mel_hop_sz, self.recep_field_sz, self.slice_sz
        need = T
        parts_w, parts_m, parts_i = [], [], []
        while True:
            try:
                vid, wav, mel = self._next_file()
            except StopIteration:
                return
            snip = len(wav) % hop
            wav = wav[:-snip or None]
            if mel is not None and len(wav) != len(mel) * hop:
                print('Error: len(wav) = {}, len(mel) * mel_hop_sz = {}'.format(len(wav), len(mel) * hop),
                      file=self.log)
            n = wav.shape[0]
            if n < F:
                print(('Warning: skipping length {} wav file (voice id {}).  '
                       'Shorter than receptive field size of {}').format(n, vid, F), file=self.log)
                continue
            ids = np.concatenate([np.zeros(F - 1, np.int32), np.full(n - (F - 1), vid, np.int32)])
            pos = 0
            while need <= n - pos:
                parts_w.append(wav[pos:pos + need])
                parts_i.append(ids[pos:pos + need])
                if mel is not None:
                    parts_m.append(mel[pos // hop:(pos + need) // hop])
                pos += need
                yield (np.concatenate(parts_w), np.concatenate(parts_m) if parts_m else None,
                       np.concatenate(parts_i))
                parts_w, parts_m, parts_i = [], [], []
                need = T
            if pos != n:
                parts_w.append(wav[pos:])
                parts_i.append(ids[pos:])
                if mel is not None:
                    parts_m.append(mel[pos // hop:])
                need -= n - pos

    def __iter__(self):
        return self

    def __next__(self):
        """(files_read, wav[B,T], mel[B,T/hop,C] or None, ids[B,T]); StopIteration when
        the shared file iterator runs dry (data.py:219-227)."""
        batch = [next(g) for g in self._gens]
        wav = np.stack([b[0] for b in batch])
        mel = np.stack([b[1] for b in batch]) if batch[0][1] is not None else None
        ids = np.stack([b[2] for b in batch])
        return self.files_read, wav, mel, ids


def npy_catalog(sam_file, repeat=True, shuffle_seed=None, skip=0):
    """data.py:43-48, :236-256: parse `vid \\t wav.npy \\t mel.npy` lines; repeat,
    shuffle (seeded) and skip `skip` files (resume position)."""
    cat = []
    with open(sam_file) as fh:
        for line in fh:
            line = line.strip()
            if not line:
                continue
            vid, wav_path, mel_path = line.split('\t')
            cat.append((int(vid), wav_path, mel_path))

    def gen():
        rng = np.random.default_rng(shuffle_seed)
        count = 0
        while True:
            order = rng.permutation(len(cat)) if shuffle_seed is not None else range(len(cat))
            for i in order:
                count += 1
                if count <= skip:
                    continue
                vid, wp, mp = cat[i]
                yield vid, np.load(wp), np.load(mp)
            if not repeat:
                return
    return cat, gen()


class SyntheticSource:
    """Seeded 16 kHz 'speech-like' files: length U[1,4] s rounded down to the
    mel hop, 3 harmonics of f0 ~ U[80,400] Hz + N(0, 0.05²) noise, peak 0.9; voice ids
    U{1..n_voices}; mel N(0,1) [len/hop, n_mel] when n_mel > 0.  Values are µ-law codes
    (mu_encode_np, ops.py:23-28) when ``quantize``."""

    def __init__(self, seed=1234, sample_rate=16000, hop=256, n_mel=0, n_voices=1, n_quant=256, quantize=True):
        self.rng = np.random.default_rng(seed)
        self.sr, self.hop, self.n_mel, self.n_voices, self.nq = sample_rate, hop, n_mel, max(1, n_voices), n_quant
        self.quantize = quantize

    def __iter__(self):
        return self

    def __next__(self):
        r = self.rng
        n = int(r.uniform(1.0, 4.0) * self.sr)
        n -= n % self.hop
        t = np.arange(n) / self.sr
        f0 = r.uniform(80, 400)
        x = sum(np.sin(2 * np.pi * f0 * (k + 1) * t + r.uniform(0, 2 * np.pi)) / (k + 1) for k in range(3))
        x = x + r.normal(0, 0.05, n)
        x = 0.9 * x / np.max(np.abs(x))
        wav = mu_encode_np(x, self.nq) if self.quantize else x
        mel = r.normal(size=(n // self.hop, self.n_mel)).astype(np.float32) if self.n_mel else None
        vid = int(r.integers(1, self.n_voices + 1))
        return vid, wav, mel
