"""Generate golden vectors from the reference's OWN code (run in the build container,
where /root/reference exists; the GPU box only reads the committed .npz files).

The reference modules import tensorflow/librosa at top level (ops.py:1, data.py:16,
ckpt.py:1); neither is installed, so they are replaced by empty stub modules.  Only
the pure-numpy functions are executed:
  * ops.mu_encode_np / ops.mu_decode_np            (ops.py:23-39)
  * data.MaskedSliceWav._gen_concat_slice_factory  (data.py:110-191)
  * data.MaskedSliceWav._gen_slice_batch's batching loop (data.py:194-227), driven with
    the same shared-iterator semantics (its TF iterator plumbing is replaced by a
    plain Python generator; the loop body is the reference's).
numpy>=1.24 removed ``np.float`` (used at data.py:130-131/:179-180); it is aliased to
``float`` for the duration of the run.  Nothing is written to /root/reference.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import os
import sys
import types

import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.dont_write_bytecode = True
    for name in ('tensorflow', 'librosa'):
        sys.modules.setdefault(name, types.ModuleType(name))
    if not hasattr(np, 'float'):
        np.float = float
    sys.path.insert(0, REF)
    import ops  # noqa: E402
    import data  # noqa: E402
    sys.path.remove(REF)
    return ops, data


def _dealer(data_mod, files, batch_sz, slice_sz, recep, hop, nmel, start=0):
    """Drive the reference's slice factory + batch loop with a plain shared iterator.
    ``start`` plays the dataset's ckpt_position: _wav_gen seeds its counter with it and
    the file stream is skipped by it (data.py:79-88, :250), so the i-th file read after a
    resume carries the count start + i."""
    dset = data_mod.MaskedSliceWav.__new__(data_mod.MaskedSliceWav)
    dset.slice_sz = slice_sz
    dset.batch_sz = batch_sz
    dset.mel_hop_sz = hop
    dset.mel_spectrum_sz = nmel
    dset.recep_field_sz = recep
    shared = iter([(start + i + 1, vid, wav, mel) for i, (vid, wav, mel) in enumerate(files[start:])])
    gens = [dset._gen_concat_slice_factory(shared)() for _ in range(batch_sz)]
    out = []
    while True:
        try:
            batch = [next(g) for g in gens]           # data.py:217 (slot order)
        except StopIteration:
            break
        out.append((np.stack([b[1] for b in batch]), np.stack([b[2] for b in batch]),
                    np.stack([b[3] for b in batch]), batch[-1][0]))     # data.py:220
    return out


def make_files(seed, n_files, min_len, max_len, hop, nmel, max_vid):
    """Deterministic ramp 'files': wav[i] = f·2^20 + i, mel[r, c] = f·2^20 + r·nmel + c
    (exact in float64), so every dealt sample names its source file and position."""
    rng = np.random.default_rng(seed)
    files = []
    for f in range(n_files):
        n = int(rng.integers(min_len, max_len))
        wav = f * 2.0 ** 20 + np.arange(n, dtype=np.float64)
        nm = (n - n % hop) // hop
        mel = f * 2.0 ** 20 + np.arange(nm * nmel, dtype=np.float64).reshape(nm, nmel)
        files.append((int(rng.integers(1, max_vid + 1)), wav, mel))
    return files


CASES = {
    # name: (seed, n_files, min_len, max_len, B, T, F, hop, nmel, max_vid)
    'hop4_b3': (7, 23, 5, 90, 3, 16, 15, 4, 3, 9),
    'hop256_b4': (8, 30, 200, 9000, 4, 512, 1023, 256, 5, 376),
    'recep5115_b2': (9, 12, 3000, 30000, 2, 4096, 5115, 256, 2, 17),
}
RESUME_AT = 6


def main():
    ops, data = _import_reference()
    # ---- A1/A2 mu-law ------------------------------------------------------------------
    rng = np.random.default_rng(1234)
    x = np.concatenate([np.linspace(-1, 1, 9), rng.uniform(-1, 1, 4096),
                        rng.uniform(-1e-3, 1e-3, 512), np.array([0.0, -0.0, 1.0, -1.0])])
    out = {'mu_x': x}
    for q in (256, 64):
        out['mu_enc_%d' % q] = ops.mu_encode_np(x, q)
        qs = np.arange(q, dtype=np.int32)
        out['mu_dec_q_%d' % q] = qs
        out['mu_dec_%d' % q] = ops.mu_decode_np(qs, q)
    x32 = x.astype(np.float32)
    out['mu_x32'] = x32
    out['mu_enc32_256'] = ops.mu_encode_np(x32, 256)
    np.savez_compressed(os.path.join(HERE, 'mulaw.npz'), **out)

    # ---- A3 dealer / ids / mask ----------------------------------------------------------
    cases = {}
    # the SURVEY's worked case: F=4, slice 8, hop 1
    f_small = [(3, np.arange(10, dtype=np.float64), np.zeros((10, 2))),
               (5, np.arange(7, dtype=np.float64) + 100, np.zeros((7, 2))),
               (2, np.arange(3, dtype=np.float64) + 200, np.zeros((3, 2))),
               (7, np.arange(12, dtype=np.float64) + 300, np.zeros((12, 2)))]
    cases['small'] = (f_small, 1, 8, 4, 1, 2, 0)
    for name, (seed, nf, lo, hi, B, T, F, hop, nmel, mv) in CASES.items():
        cases[name] = (make_files(seed, nf, lo, hi, hop, nmel, mv), B, T, F, hop, nmel, 0)
    # a resumed stream: the same files with ckpt_position = RESUME_AT
    seed, nf, lo, hi, B, T, F, hop, nmel, mv = CASES['hop4_b3']
    cases['hop4_b3_resume'] = (make_files(seed, nf, lo, hi, hop, nmel, mv), B, T, F, hop, nmel, RESUME_AT)
    meta = []
    for name, (files, B, T, F, hop, nmel, start) in cases.items():
        batches = _dealer(data, files, B, T, F, hop, nmel, start)
        d = {'n_batches': np.array(len(batches)), 'B': np.array(B), 'T': np.array(T),
             'F': np.array(F), 'hop': np.array(hop), 'nmel': np.array(nmel),
             'n_files': np.array(len(files)), 'start': np.array(start)}
        if name == 'small':
            for i, (vid, wav, mel) in enumerate(files):
                d['file_vid_%d' % i] = np.array(vid)
                d['file_wav_%d' % i] = wav
                d['file_mel_%d' % i] = mel
        for j, (w, m, ids, cnt) in enumerate(batches):
            d['wav_%d' % j] = w.astype(np.int64)          # ramps: exact integers
            d['mel_%d' % j] = m.astype(np.int64)
            d['ids_%d' % j] = ids
            d['cnt_%d' % j] = np.array(int(cnt))           # latest_file_read_count
        np.savez_compressed(os.path.join(HERE, 'dealer_%s.npz' % name), **d)
        meta.append('%s: %d files -> %d batches of [%d,%d]' % (name, len(files), len(batches), B, T))
    print('\n'.join(meta))
    print('mu_encode_np(linspace(-1,1,9),256) =', out['mu_enc_256'][:9].tolist())


if __name__ == '__main__':
    main()
