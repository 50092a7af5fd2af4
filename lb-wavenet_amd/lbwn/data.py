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
                 log=None, start=0):
        if slice_sz % mel_hop_sz != 0:      # data.py:32-36
            requested = slice_sz
            slice_sz += mel_hop_sz - (slice_sz % mel_hop_sz)
            print('Warning: aligning slice size from {} to {} for mel_hop_sz {}'.format(
                requested, slice_sz, mel_hop_sz), file=log or sys.stderr)
        self.slice_sz = slice_sz
        self.batch_sz = batch_sz
        self.recep_field_sz = recep_field_sz
        self.mel_hop_sz = mel_hop_sz
        self.mel_spectrum_sz = mel_spectrum_sz
        self.log = log or sys.stderr
        # the shared read counter is seeded with the resume position (ckpt_position), as
        # _wav_gen seeds datum_count (data.py:79, :96): counts stay absolute across resumes
        self.files_read = int(start)
        self._files = iter(files)
        self._gens = [self._slot() for _ in range(batch_sz)]

    def _next_file(self):
        vid, wav, mel = next(self._files)
        self.files_read += 1
        return self.files_read, vid, wav, mel

    def _slot(self):
        hop, F, T = self.mel_hop_sz, self.recep_field_sz, self.slice_sz
        need = T
        parts_w, parts_m, parts_i = [], [], []
        while True:
            try:
                cnt, vid, wav, mel = self._next_file()
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
                yield (cnt, np.concatenate(parts_w), np.concatenate(parts_m) if parts_m else None,
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
        """(latest_file_read_count, wav[B,T], mel[B,T/hop,C] or None, ids[B,T]);
        StopIteration when the shared file iterator runs dry (data.py:217-227).  The count is
        that of the file the LAST slot's slice ended in (``batch[-1][0]``, data.py:220), not
        the number of reads so far: later slots may have read ahead."""
        batch = [next(g) for g in self._gens]
        wav = np.stack([b[1] for b in batch])
        mel = np.stack([b[2] for b in batch]) if batch[0][2] is not None else None
        ids = np.stack([b[3] for b in batch])
        return batch[-1][0], wav, mel, ids


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


class MaskedSliceWav:
    """data.MaskedSliceWav (data.py:20-293) on the host: same constructor, catalog methods,
    iterator contract ``(file_read_count, wav[B,T], mel[B,T/hop,C], ids[B,T])`` and
    checkpointed position.  The tf.data graph (repeat → shuffle(seed) → skip(position) →
    slice generator → prefetch, data.py:236-268) becomes: a seeded per-epoch permutation of
    the catalog, a skip of ``ckpt_position`` file reads on resume, the SliceDealer, and a
    prefetch thread of ``prefetch_sz`` batches.  TF's shuffle RNG stream cannot be
    reproduced without TF, so the file ORDER differs from a TF run with the same seed
    (distribution and slicing semantics are identical; SliceDealer is golden-exact)."""

    def __init__(self, sess, sam_file, sample_rate, slice_sz, prefetch_sz, mel_spectrum_sz, mel_hop_sz, batch_sz,
                 n_keep_checkpoints, ckpt_path, resume_step, random_seed=None, rows=None):
        from .ckpt import Checkpoint
        self.sam_file = sam_file
        self.sample_rate = sample_rate
        self.prefetch_sz = max(1, int(prefetch_sz or 1))
        self.mel_spectrum_sz = mel_spectrum_sz or 0
        self.mel_hop_sz = mel_hop_sz
        if slice_sz % mel_hop_sz != 0:      # data.py:32-36 (the dealer repeats the warning)
            slice_sz += mel_hop_sz - (slice_sz % mel_hop_sz)
        self.slice_sz = slice_sz
        self.batch_sz = batch_sz
        self.rows = rows            # DP: this rank's slot range of the global batch
        self.random_seed = np.array([random_seed if random_seed is not None
                                     else np.random.randint(np.iinfo(np.int32).max)], np.int64)
        self.ckpt_position = np.zeros(1, np.int64)
        self.ckpt = Checkpoint(ckpt_path, n_keep_checkpoints, resume_step)
        self.recep_field_sz = None
        self.sample_catalog = None
        self._itr = None

    def init_sample_catalog(self):
        self.sample_catalog = []
        with open(self.sam_file) as fh:
            for s in fh:
                s = s.strip()
                if s:
                    vid, wav_path, mel_path = s.split('\t')
                    self.sample_catalog.append([int(vid), wav_path, mel_path])

    def set_receptive_field_size(self, r_sz):
        self.recep_field_sz = r_sz

    def get_max_id(self):
        return max(self.sample_catalog, key=lambda x: x[0])[0]

    def _files(self):
        cat = self.sample_catalog
        rng = np.random.default_rng(int(self.random_seed[0]))
        skip = int(self.ckpt_position[0])
        count = 0
        want_mel = self.mel_spectrum_sz > 0
        while True:
            for i in rng.permutation(len(cat)):
                count += 1
                if count <= skip:
                    continue
                vid, wp, mp = cat[i]
                wav = np.load(wp)                          # never allow_pickle
                mel = np.load(mp).astype(np.float32) if want_mel else None
                yield vid, wav, mel

    def build(self):
        if self.sample_catalog is None:
            self.init_sample_catalog()
        if self.recep_field_sz is None:
            raise ValueError('set_receptive_field_size first (data.py:55-56, train.py:167)')

    def init_vars(self):
        self._itr = None

    def get_itr(self):
        """Iterator of prefetched batches (starts the producer thread on first use)."""
        if self._itr is None:
            import queue
            import threading
            dealer = SliceDealer(self._files(), self.batch_sz, self.slice_sz, self.recep_field_sz,
                                 self.mel_hop_sz, self.mel_spectrum_sz, start=int(self.ckpt_position[0]))
            q = queue.Queue(maxsize=self.prefetch_sz)
            rows = self.rows

            def produce():
                for cnt, wav, mel, ids in dealer:
                    if rows is not None:
                        wav, ids = wav[rows], ids[rows]
                        mel = mel[rows] if mel is not None else None
                    q.put((cnt, wav, mel, ids))
                q.put(None)

            threading.Thread(target=produce, daemon=True).start()

            def gen():
                while True:
                    item = q.get()
                    if item is None:
                        return
                    yield item
            self._itr = gen()
        return self._itr

    def get_op(self):
        return next(self.get_itr())

    def save(self, step, read_count):
        self.ckpt_position[0] = read_count
        self.ckpt.saveable_objects = {'random_seed': torch_tensor(self.random_seed),
                                      'ckpt_position': torch_tensor(self.ckpt_position)}
        return self.ckpt.save(step)

    def restore(self):
        from .ckpt import load_tensors
        t = load_tensors('{}-{}'.format(self.ckpt.ckpt_path, self.ckpt.resume_step))
        self.random_seed[0] = int(t['random_seed'][0])
        self.ckpt_position[0] = int(t['ckpt_position'][0])
        self._itr = None


class DeviceBatches:
    """Host -> device stage of the training input (the reference's tf.data prefetch feeding
    the session, data.py:267-268): each numpy batch of the prefetch thread is copied into a
    pinned host buffer and sent to the GPU with a non-blocking copy on the current stream, so
    the host never waits for the GPU (a pageable ``torch.as_tensor(..., device=)`` copy
    synchronised every step with the previous step's kernels).  ``depth`` slots rotate; a slot's
    pinned buffers are refilled only after its previous copy completed (its event), and its
    device buffers are reused in stream order after the step that read them.
    Yields (file_read_count, wav int32 [B,T], mel f32 [B,T/hop,C] or None, ids int32 [B,T]),
    the last three on ``device``."""

    def __init__(self, itr, device, depth=3):
        self.itr, self.device, self.depth = itr, device, depth
        self.slots = [None] * depth
        self.k = 0

    def __iter__(self):
        return self

    def _slot(self, wav, mel, ids):
        import torch
        k = self.k
        self.k = (self.k + 1) % self.depth
        s = self.slots[k]
        shapes = (wav.shape, None if mel is None else mel.shape)
        if s is None or s['shapes'] != shapes:
            def pair(shape, dt):
                return (torch.empty(shape, dtype=dt, pin_memory=True), torch.empty(shape, dtype=dt, device=self.device))
            s = {'shapes': shapes, 'wav': pair(wav.shape, torch.int32), 'ids': pair(ids.shape, torch.int32),
                 'mel': None if mel is None else pair(mel.shape, torch.float32), 'ev': None}
            self.slots[k] = s
        elif s['ev'] is not None:
            s['ev'].synchronize()          # this slot's previous copy (depth batches ago) has landed
        return s

    def __next__(self):
        import torch
        cnt, wav, mel, ids = next(self.itr)
        s = self._slot(wav, mel, ids)
        out = []
        for key, a, dt in (('wav', wav, np.int32), ('mel', mel, np.float32), ('ids', ids, np.int32)):
            if a is None:
                out.append(None)
                continue
            host, dev = s[key]
            host.numpy()[...] = np.asarray(a, dtype=dt)
            dev.copy_(host, non_blocking=True)
            out.append(dev)
        ev = torch.cuda.Event()
        ev.record()
        s['ev'] = ev
        return (cnt, out[0], out[1], out[2])


def torch_tensor(a):
    import torch
    return torch.as_tensor(np.asarray(a))
