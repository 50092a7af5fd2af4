"""Host-side drop-in surface (CPU): checkpoints (ckpt.py), the MaskedSliceWav dataset
(data.py:20-293), train.py argument handling (train.py:12-80), and the data-parallel
gradient reduction over gloo with world_size 2."""
import json
import os
import re
import sys

import numpy as np
import pytest
import torch

from lbwn.arch import load_arch, normalize_arch, ParamLayout
from lbwn.ckpt import ckpt_file, load_tensors
from lbwn.data import MaskedSliceWav, SliceDealer
from lbwn.optim import AdamOptimizer
from lbwn.tmodel import WaveNetTrain
from tests.conftest import ROOT


def small_arch():
    return normalize_arch(dict(n_blocks=1, n_block_layers=3, n_quant=256, n_res=8, n_dil=8, n_skip=16, n_post=8,
                               n_gc_embed=0, n_gc_category=0, use_bias=True))


def test_checkpoint_roundtrip_reference_names(tmp_path):
    arch = load_arch(os.path.join(ROOT, 'par', 'arch5.json'))
    a = WaveNetTrain(**arch, batch_sz=2, l2_factor=1e-3, device='cpu', ckpt_path=str(tmp_path / 'run.net'), seed=3)
    opt = AdamOptimizer()
    m, v = opt.slots(a)
    m.uniform_(-1, 1)
    v.uniform_(0, 1)
    a.counters[:3] = torch.tensor([17, 12345, 16])
    pfx = a.save(17, opt)
    assert pfx == str(tmp_path / 'run.net') + '-17'
    t = load_tensors(pfx)
    # the reference's serial names (arch.py:142) and TF's Adam slot names
    for k in ('PRE', 'SIGNAL_0_0', 'SIGNAL_4_9', 'GC_EMBED', 'LC_UPSAMPLE_3', 'LC_GATE_2_5', 'POST2_BIAS',
              'SAVE_1_0_0', 'SAVE_512_4_9', 'GLOBAL_STEP', 'VALID_SAMPLES', 'SIGNAL_0_0/Adam', 'POST1/Adam_1'):
        assert k in t, k
    assert tuple(t['SAVE_512_4_9'].shape) == (2, 512, 32)
    b = WaveNetTrain(**arch, batch_sz=2, l2_factor=1e-3, device='cpu', ckpt_path=str(tmp_path / 'run.net'),
                     resume_step=17, seed=9)
    opt2 = AdamOptimizer()
    b.restore(opt2)
    assert torch.equal(a.flat, b.flat) and torch.equal(a.save_flat, b.save_flat)
    assert torch.equal(a.counters[:3], b.counters[:3]) and b.global_step_host == 17
    assert all(torch.equal(x, y) for x, y in zip(opt.slots(a), opt2.slots(b)))


def test_checkpoint_rotation_and_missing(tmp_path):
    net = WaveNetTrain(**small_arch(), batch_sz=1, l2_factor=0.0, device='cpu', n_keep_checkpoints=2,
                       ckpt_path=str(tmp_path / 'r.net'))
    for s in (1, 2, 3):
        net.save(s)
    assert not os.path.exists(ckpt_file(str(tmp_path / 'r.net'), 1))
    assert os.path.exists(ckpt_file(str(tmp_path / 'r.net'), 3))
    with pytest.raises(SystemExit):
        load_tensors(str(tmp_path / 'r.net-9'))


def _write_catalog(tmp_path, n_files=5, hop=4, n_mel=3):
    rng = np.random.default_rng(0)
    lines = []
    for i in range(n_files):
        n = int(rng.integers(40, 90)) * hop + int(rng.integers(0, hop))
        wav = rng.integers(0, 256, n).astype(np.int32)
        mel = rng.standard_normal((n // hop, n_mel)).astype(np.float32)
        wp, mp = tmp_path / ('f%d.wav.npy' % i), tmp_path / ('f%d.mel.npy' % i)
        np.save(wp, wav)
        np.save(mp, mel)
        lines.append('%d\t%s\t%s' % (i % 3 + 1, wp, mp))
    cat = tmp_path / 'samples.txt'
    cat.write_text('\n'.join(lines) + '\n')
    return str(cat)


def test_masked_slice_wav_matches_dealer(tmp_path):
    cat = _write_catalog(tmp_path)
    F, T, B, hop = 13, 64, 3, 4
    ds = MaskedSliceWav(None, cat, 16000, T, 2, 3, hop, B, 5, str(tmp_path / 'x.dset'), 0, random_seed=42)
    ds.init_sample_catalog()
    assert ds.get_max_id() == 3
    ds.set_receptive_field_size(F)
    ds.build()
    got = [ds.get_op() for _ in range(6)]
    src = MaskedSliceWav(None, cat, 16000, T, 2, 3, hop, B, 5, None, 0, random_seed=42)
    src.init_sample_catalog()
    ref = SliceDealer(src._files(), B, T, F, hop, 3)
    for g, r in zip(got, ref):
        assert g[0] == r[0]
        np.testing.assert_array_equal(g[1], r[1])
        np.testing.assert_array_equal(g[2], r[2])
        np.testing.assert_array_equal(g[3], r[3])


def test_masked_slice_wav_resume_and_rows(tmp_path):
    cat = _write_catalog(tmp_path)
    ds = MaskedSliceWav(None, cat, 16000, 64, 2, 3, 4, 2, 5, str(tmp_path / 'x.dset'), 0, random_seed=7)
    ds.init_sample_catalog()
    files = ds._files()
    order = [next(files)[1][:5].tolist() for _ in range(8)]
    ds.set_receptive_field_size(13)
    ds.build()
    cnt = ds.get_op()[0]
    ds.save(4, cnt)
    r = MaskedSliceWav(None, cat, 16000, 64, 2, 3, 4, 2, 5, str(tmp_path / 'x.dset'), 4)
    r.init_sample_catalog()
    r.restore()
    assert int(r.random_seed[0]) == 7 and int(r.ckpt_position[0]) == cnt
    resumed = [next(r._files())[1][:5].tolist()]
    assert resumed[0] == order[cnt]          # continues after the files already read
    # DP: a rank's rows of the globally dealt batch
    full = MaskedSliceWav(None, cat, 16000, 64, 2, 3, 4, 4, 5, None, 0, random_seed=1)
    part = MaskedSliceWav(None, cat, 16000, 64, 2, 3, 4, 4, 5, None, 0, random_seed=1, rows=slice(2, 4))
    for d in (full, part):
        d.init_sample_catalog()
        d.set_receptive_field_size(13)
        d.build()
    a, b = full.get_op(), part.get_op()
    np.testing.assert_array_equal(a[1][2:4], b[1])
    np.testing.assert_array_equal(a[3][2:4], b[3])


def test_masked_slice_wav_double_resume_counts_are_absolute(tmp_path):
    """save -> resume -> save -> resume: the read counter is seeded with ckpt_position
    (data.py:79, :96), so the second resume continues after every file read so far."""
    cat = _write_catalog(tmp_path, n_files=7)
    mk = lambda step, **kw: MaskedSliceWav(None, cat, 16000, 64, 2, 3, 4, 2, 5, str(tmp_path / 'x.dset'), step, **kw)
    ref = mk(0, random_seed=11)
    ref.init_sample_catalog()
    files = ref._files()
    order = [next(files)[1][:6].tolist() for _ in range(40)]
    ds = mk(0, random_seed=11)
    ds.init_sample_catalog()
    ds.set_receptive_field_size(13)
    ds.build()
    for _ in range(3):
        cnt1 = ds.get_op()[0]
    ds.save(3, cnt1)
    r1 = mk(3)
    r1.init_sample_catalog()
    r1.set_receptive_field_size(13)
    r1.build()
    r1.restore()
    assert next(r1._files())[1][:6].tolist() == order[cnt1]
    for _ in range(4):
        cnt2 = r1.get_op()[0]
    assert cnt2 > cnt1                       # absolute, not counted from the resume
    r1.save(7, cnt2)
    r2 = mk(7)
    r2.init_sample_catalog()
    r2.restore()
    assert int(r2.ckpt_position[0]) == cnt2
    assert next(r2._files())[1][:6].tolist() == order[cnt2]


def test_train_cli_errors(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
    import train
    arch = tmp_path / 'a.json'
    arch.write_text('{"n_blocks": 1, "n_block_layers": 2, "n_quant": 256, "n_res": 8, "n_dil": 8, '
                    '"n_skip": 8, "n_post": 8, "n_gc_embed": 4, "use_bias": true}')
    par = os.path.join(ROOT, 'par', 'par1.json')
    with pytest.raises(SystemExit) as e:     # n_gc_category missing and no --num-global-cond
        train.main([str(tmp_path / 'ck'), str(arch), par, 'none.txt'])
    assert e.value.code == 1
    with pytest.raises(SystemExit) as e:
        train.main(['--cpu-only', str(tmp_path / 'ck'), os.path.join(ROOT, 'par', 'arch3.json'), par, 'none.txt'])
    assert e.value.code == 1
    # -gc supplies n_gc_category for arch files that lack it (train.py:77-80, :138-146)
    for f in ('arch2', 'arch4'):
        with open(os.path.join(ROOT, 'par', f + '.json')) as fp:
            raw = json.load(fp)
        with pytest.raises(SystemExit) as e:
            train.prepare_arch(raw, None)
        assert e.value.code == 1
        a = train.prepare_arch(raw, 12)
        assert a['n_gc_category'] == 12 and 'lc_hop_sz' not in a
    args = train.get_args(['-bs', '4', '-ss', '1024', '-lr', '0.01', '-rs', '7', 'p', 'a', 'b', 'c'])
    assert (args.batch_size, args.slice_size, args.learning_rate, args.resume_step) == (4, 1024, 0.01, 7)


# ---- data parallel over gloo, world_size 2 -----------------------------------------------------

class _FakeNet:
    def __init__(self, grads, stats, layout, status=0):
        self.grad_flat = grads
        self.stats = stats
        self.layout = layout
        self._status = torch.tensor([status], dtype=torch.int32)

    def status_word(self):
        return self._status


def _dp_worker(rank, world, port, q_np, ids_np, out_path):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
    from oracle import wavenet_ref as R
    from lbwn.dist import DPContext
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    arch = small_arch()
    rng = np.random.default_rng(0)
    P = R.init_params(arch, rng, dtype=np.float64)
    S = R.init_save(arch, 4, rng, dtype=np.float64)
    dp = DPContext(world, rank, rank)
    rows = dp.rows(2)
    Sr = {k: v[rows] for k, v in S.items()}
    lg, cache, _ = R.forward(arch, P, q_np[rows], ids_np[rows], Sr)
    st, dlog = R.loss_fcn(arch, P, lg, q_np[rows], ids_np[rows], 0.0)
    G = R.backward(arch, P, cache, dlog, 0.0)
    lay = ParamLayout(arch)
    flat = np.zeros(lay.n_total)
    for n, e in lay.entries.items():       # raw Σ-xent gradient, as the device buffer holds it
        flat[e.offset:e.offset + e.numel] = (G[n] * st['n_valid']).reshape(-1)
    net = _FakeNet(torch.tensor(flat, dtype=torch.float32),
                   torch.tensor([st['mean_xent'] * st['n_valid'], st['n_valid'], 0.0, 0.0], dtype=torch.float32), lay)
    dp.reduce_grads(net)
    if rank == 0:
        np.savez(out_path, grads=net.grad_flat.numpy(), stats=net.stats.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_dp_gloo_two_ranks_equals_single_process(tmp_path):
    import torch.multiprocessing as mp
    sys.path.insert(0, ROOT)
    from oracle import wavenet_ref as R
    arch = small_arch()
    rng = np.random.default_rng(5)
    B, T = 4, 48
    q = rng.integers(0, 256, (B, T))
    ids = np.ones((B, T), np.int32)
    ids[:, :5] = 0
    ids[3, 20:30] = 0
    out = str(tmp_path / 'dp.npz')
    port = 29500 + os.getpid() % 1000
    mp.spawn(_dp_worker, args=(2, port, q, ids, out), nprocs=2, join=True)
    got = np.load(out)
    # single process over all 4 streams
    rng0 = np.random.default_rng(0)
    P = R.init_params(arch, rng0, dtype=np.float64)
    S = R.init_save(arch, 4, rng0, dtype=np.float64)
    lg, cache, _ = R.forward(arch, P, q, ids, S)
    st, dlog = R.loss_fcn(arch, P, lg, q, ids, 0.0)
    G = R.backward(arch, P, cache, dlog, 0.0)
    assert int(got['stats'][1]) == st['n_valid']
    lay = ParamLayout(arch)
    for n, e in lay.entries.items():   # Adam divides the summed raw grads by the GLOBAL n_valid
        np.testing.assert_allclose(got['grads'][e.offset:e.offset + e.numel] / got['stats'][1], G[n].reshape(-1),
                                   rtol=2e-4, atol=1e-7, err_msg=n)


def _bucket_worker(rank, world, port, out_path):
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
    from lbwn.dist import DPContext
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    dp = DPContext(world, rank, rank)
    lay = ParamLayout(load_arch(os.path.join(ROOT, 'par', 'arch5.json')))
    g = torch.Generator().manual_seed(100 + rank)
    grads = torch.randn(lay.n_total, generator=g) * 10.0 ** torch.randint(-6, 4, (lay.n_total,), generator=g)
    stats = torch.tensor([123.25 + rank, 1000.0 + rank, 7.0 * rank, 0.5])
    a = _FakeNet(grads.clone(), stats.clone(), lay, status=1 + 2 * rank)     # ranks: 0b01, 0b11
    b = _FakeNet(grads.clone(), stats.clone(), lay, status=1 + 2 * rank)
    dp.reduce_grads(a)          # three buckets (head / side / rest)
    dp.reduce_grads_flat(b)     # one message
    if rank == 0:
        np.savez(out_path, ga=a.grad_flat.numpy(), gb=b.grad_flat.numpy(), sa=a.stats.numpy(), sb=b.stats.numpy(),
                 wa=a.status_word().numpy(), wb=b.status_word().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('arch_file', ['arch1', 'arch2', 'arch3', 'arch4', 'arch5'])
def test_dp_buckets_tile_the_gradient(arch_file):
    """The all-reduce buckets cover every flat gradient range exactly once, by the stream that
    finalises it: head = POST1 / POST2 / SKIP_BIAS and the head biases (after the backward
    chain), side = PRE / SIGNAL / GATE / RESIDUAL / GC and their biases (after the side
    stream), rest = SKIP and LC (after the whole backward)."""
    from lbwn.dist import _Buckets
    lay = ParamLayout(load_arch(os.path.join(ROOT, 'par', arch_file + '.json'), num_global_cond=7))
    bk = _Buckets(_FakeNet(torch.zeros(lay.n_total), torch.zeros(4), lay))
    owner = np.full(lay.n_total, -1)
    assert bk.tensors(0, _FakeNet(torch.zeros(lay.n_total), torch.zeros(4), lay))[-1].numel() == 3   # + the stats
    for k, rs in enumerate(bk.ranges):
        for a, b in rs:
            assert (owner[a:b] == -1).all()
            owner[a:b] = k
    assert (owner >= 0).all()
    want = {'POST1': 0, 'POST2': 0, 'SKIP_BIAS': 0, 'POST1_BIAS': 0, 'POST2_BIAS': 0, 'PRE': 1, 'PRE_BIAS': 1,
            'SIGNAL': 1, 'GATE': 1, 'RESIDUAL': 1, 'SIGNAL_BIAS': 1, 'GATE_BIAS': 1, 'RESIDUAL_BIAS': 1,
            'GC_EMBED': 1, 'GC_SIGNAL': 1, 'GC_GATE': 1, 'SKIP': 2, 'LC_UPSAMPLE': 2, 'LC_SIGNAL': 2, 'LC_GATE': 2}
    for n, e in lay.entries.items():
        stem = re.sub(r'(_\d+)+$', '', n)
        assert (owner[e.offset:e.offset + e.numel] == want[stem]).all(), n


def test_dp_bucketed_equals_flat(tmp_path):
    """The three-bucket all-reduce (lbwn.dist: head bucket beside the backward's tail, side
    bucket beside dSKIP, the rest after it; every range reduced in place) gives bitwise the flat
    one-message result, for the gradient, the loss stats and the status word (any rank's timeout
    reaches every rank as the MAX of the words: max(0b01, 0b11) = 0b11, where a SUM would read
    0b100), over 2 gloo ranks at arch5's layout (GC + LC kinds included)."""
    import torch.multiprocessing as mp
    out = str(tmp_path / 'bk.npz')
    port = 29500 + (os.getpid() + 13) % 1000
    mp.spawn(_bucket_worker, args=(2, port, out), nprocs=2, join=True)
    r = np.load(out)
    assert np.array_equal(r['ga'].view(np.uint32), r['gb'].view(np.uint32))
    assert np.array_equal(r['sa'][:3], r['sb'][:3])
    assert int(r['wa'][0]) == int(r['wb'][0]) == 3


def _ckpt_worker(rank, world, port, path):
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
    from lbwn.dist import DPContext
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    dp = DPContext(world, rank, rank)
    net = WaveNetTrain(**small_arch(), batch_sz=2, l2_factor=0.0, device='cpu', ckpt_path=path, seed=0)
    net.dp = dp
    net.save_flat.copy_(torch.arange(net.save_flat.numel(), dtype=torch.float32) + 1000.0 * rank)
    ret = net.save(5)                       # collective
    assert (ret is None) == (rank != 0)
    dist.barrier()
    back = WaveNetTrain(**small_arch(), batch_sz=2, l2_factor=0.0, device='cpu', ckpt_path=path, resume_step=5,
                        seed=1)
    back.dp = dp
    back.restore()
    assert torch.equal(back.save_flat, net.save_flat), rank     # each rank gets its own rows back
    dist.barrier()
    dist.destroy_process_group()


def test_dp_checkpoint_gathers_per_rank_save(tmp_path):
    """SAVE is per stream: under DP the checkpoint holds the global batch's SAVE rows
    (what one process over world·B streams writes) and each rank restores its own."""
    import torch.multiprocessing as mp
    path = str(tmp_path / 'dp.net')
    port = 29500 + (os.getpid() + 7) % 1000
    mp.spawn(_ckpt_worker, args=(2, port, path), nprocs=2, join=True)
    t = load_tensors(path + '-5')
    one = WaveNetTrain(**small_arch(), batch_sz=4, l2_factor=0.0, device='cpu', seed=0)
    for n, v in one.save_vars.items():
        assert tuple(t[n].shape) == tuple(v.shape), n
        per_rank = t[n].shape[0] // 2
        assert torch.all(t[n][per_rank:] - t[n][:per_rank] == 1000.0), n


def test_bench_self_launch_dry_run():
    """`bench.py --gpus 2` outside torch.distributed.run spawns its own ranks (children,
    no exec) and the DP plumbing reduces through lbwn.dist over gloo; --dry-run stops
    before any GPU call."""
    import json as _json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--dry-run'],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout
    d = _json.loads(lines[0])
    assert d['world_size'] == 2 and d['backend'] == 'gloo' and d['reduce_ok']
    assert d['arch'] == 'arch3.json' and d['batch_per_gpu'] == 8
