"""generate.py drop-in (generate.py:1-120 of the reference) on MI355X.

Same flags and positionals (ARCH_FILE CHECKPOINT_PREFIX OUTPUT_WAV_DIR).  The checkpoint is
a '<prefix>.safetensors' written by this build's train.py (reference serial names).  The TF
while_loop becomes WaveNetGen's device-resident generation (hipGraph-replayed chunks);
librosa (absent here) is replaced by scipy.io.wavfile for reading the teacher wav and
writing 'gen.i<k>.wav' (float32).  The reference hard-codes gc_ids = [5, 6]
(generate.py:94); --gc-ids overrides, and the list is cycled over the batch.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def get_args(argv=None):
    p = argparse.ArgumentParser(description='WaveNet')
    p.add_argument('--teacher-wav', '-w', type=str,
                   help='Provide a preliminary teacher-forcing vector to prime the generation')
    p.add_argument('--teacher-start', '-ts', type=float, help='Number of seconds to parse from <teacher_wav>')
    p.add_argument('--teacher-duration', '-td', type=float, help='Number of seconds to parse from <teacher_wav>')
    p.add_argument('--gen-seconds', '-g', type=float, default=5, help='Number of additional seconds to generate')
    p.add_argument('--sample-rate', '-s', type=int, default=16000,
                   help='Number of samples per second for parsed .wav files')
    p.add_argument('--chunk-size', '-c', type=int, default=1000,
                   help='Number of timesteps to generate between internal buffer shifts')
    p.add_argument('--batch-size', '-b', type=int, default=10, help='Number of .wav files to generate simultaneously')
    p.add_argument('--gc-ids', type=str, default='5,6', help='(build extension) voice ids, cycled over the batch')
    p.add_argument('--seed', type=int, default=0, help='(build extension) sampling seed')
    p.add_argument('arch_file', type=str, metavar='ARCH_FILE')
    p.add_argument('ckpt', metavar='CHECKPOINT_PREFIX', type=str)
    p.add_argument('wav_dir', metavar='OUTPUT_WAV_DIR', type=str)
    return p.parse_args(argv)


def load_teacher(path, sample_rate, start=None, duration=None):
    """librosa.load(path, sr, offset, duration, mono=True) restated with scipy: float in
    [-1, 1], mono mix, polyphase resampling to sample_rate."""
    import numpy as np
    from math import gcd
    from scipy.io import wavfile
    from scipy.signal import resample_poly
    sr, x = wavfile.read(path)
    if x.dtype.kind == 'i':
        x = x.astype(np.float32) / float(np.iinfo(x.dtype).max + 1)
    elif x.dtype.kind == 'u':
        x = (x.astype(np.float32) - 128.0) / 128.0
    x = x.astype(np.float32)
    if x.ndim > 1:
        x = x.mean(axis=1)
    if start:
        x = x[int(round(start * sr)):]
    if duration is not None:
        x = x[:int(round(duration * sr))]
    if sr != sample_rate:
        g = gcd(sr, sample_rate)
        x = resample_poly(x, sample_rate // g, sr // g).astype(np.float32)
    return x


def main(argv=None):
    args = get_args(argv)
    from sys import stderr
    import numpy as np
    import torch
    from lbwn.arch import normalize_arch
    from lbwn.ckpt import ckpt_file
    from lbwn.imodel import WaveNetGen

    with open(args.arch_file) as fp:
        arch = normalize_arch(json.load(fp))
    if not os.access(ckpt_file(args.ckpt), os.R_OK):                   # generate.py:43-47
        print("Couldn't find checkpoint file {}".format(ckpt_file(args.ckpt)), file=stderr)
        sys.exit(1)
    if args.teacher_wav is not None:
        teacher_vec = load_teacher(args.teacher_wav, args.sample_rate, args.teacher_start, args.teacher_duration)
        teacher_seconds = teacher_vec.shape[0] / args.sample_rate
    else:
        teacher_vec, teacher_seconds = None, 0

    net = WaveNetGen(arch['n_blocks'], arch['n_block_layers'], arch['n_quant'], arch['n_res'], arch['n_dil'],
                     arch['n_skip'], arch['n_post'], arch['n_gc_embed'], arch['n_gc_category'], arch['use_bias'],
                     args.batch_size, args.chunk_size, teacher_vec, seed=args.seed)
    print('Building graph.')
    print('Restoring from {}'.format(args.ckpt))
    net.restore(args.ckpt)
    print('Initializing buffers.')
    ids = [int(v) for v in args.gc_ids.split(',') if v.strip()]
    gc_ids = [ids[i % len(ids)] for i in range(args.batch_size)] if arch['n_gc_embed'] else None
    gen_sz = int((args.gen_seconds + teacher_seconds) * args.sample_rate)
    print('Starting inference...')
    n, wav_streams, wpos = net.run(gen_sz, gc_ids=gc_ids)
    wav_streams = wav_streams.cpu().numpy()

    from scipy.io import wavfile
    print('Writing wav files.')
    os.makedirs(args.wav_dir, exist_ok=True)
    for i in range(args.batch_size):
        path = os.path.join(args.wav_dir, 'gen.i{}.wav'.format(i))
        wavfile.write(path, args.sample_rate, wav_streams[i].astype(np.float32))
        print('Wrote {}'.format(path))
    print('Finished.')
    return wav_streams


if __name__ == '__main__':
    main()
