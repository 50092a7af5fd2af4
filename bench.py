#!/usr/bin/env python
"""Benchmark: WaveNet training step (forward + masked xent + backward + TF1 Adam) on
MI355X, arch3 (par/arch3.json) with B = 8 streams x T = 4096 samples per GPU (BASELINE.json
configs[1]), synthetic 16 kHz µ-law input dealt by the reference's slicing
semantics.  Data-parallel over N GPUs (one process per GPU, RCCL all-reduce of the flat
gradient bucket + loss stats): per-GPU work is fixed, so scaling is weak.

Prints ONE JSON line (rank 0).  `value` = audio samples/s for the whole job (all ranks):
N·B·T / step time.  `roofline` is for the dominant kernel, timed live with HIP events
recorded by the plan around that launch on the plan's stream; `roofline_dilconv` is the
same for the residual-layer forward kernel (the dilated-conv path, HBM-bound).
`cpu_baseline` times the CPU restatement (oracle/, numpy fp32; the reference's TF-CPU path
cannot run here: TensorFlow 1.x is not installable) on a bounded sample on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from lbwn import _lib  # noqa: E402
from lbwn import dist as lbdist  # noqa: E402
from lbwn.arch import load_arch, mel_hop_sz, n_layers, recep_field_sz  # noqa: E402
from lbwn.data import SliceDealer, SyntheticSource  # noqa: E402
from lbwn.imodel import WaveNetGen  # noqa: E402
from lbwn.optim import AdamOptimizer  # noqa: E402
from lbwn.tmodel import WaveNetTrain  # noqa: E402

HBM_PEAK = 8.0e12        # B/s, MI355X_MICROARCH.md chip table
FP32_MFMA_PEAK = 157.3e12  # FLOP/s dense fp32 MFMA


def kernel_work(name, arch, M):
    """Algorithmic work per launch."""
    L, Cr, Cd, Cs, Cp, Q = (n_layers(arch), arch['n_res'], arch['n_dil'], arch['n_skip'], arch['n_post'],
                            arch['n_quant'])
    flops = {
        'dskip': 2.0 * M * L * Cd * Cs,
        'post1_fwd': 2.0 * M * Cs * Cp, 'dpost1': 2.0 * M * Cs * Cp, 'ds': 2.0 * M * Cs * Cp,
        'post2_fwd': 2.0 * M * Cp * Q, 'dpost2': 2.0 * M * Cp * Q, 'dh': 2.0 * M * Cp * Q,
    }
    if name in flops:
        return 'mfma', flops[name]
    if name == 'layer_bwd':
        # the whole residual stack backward (persistent chain): conv bwd 2 x (8 Cr Cd) and
        # residual bwd 2 x (2 Cd Cr) FLOP per layer and position; at
        # AI = 20 Cr Cd / 640 B = 32 FLOP/B it sits right of the fp32 ridge (19.7): MFMA-bound.
        # (The gate recompute and the weight-gradient products the chain also does are not
        # counted: algorithmic work only.)
        return 'mfma', 20.0 * M * Cr * Cd * L
    if name == 'layer_fwd':
        # the whole residual stack (persistent chain launch, or the span of the L per-layer
        # launches): per layer and position x_l in (Cr), x_{l+1} out (Cr), z out (Cd); the
        # dilated tap x[t-d] is re-read from LDS / the neighbour tile and counted once.
        return 'hbm', 4.0 * M * (2 * Cr + Cd) * L
    raise KeyError(name)


def gen_bytes_per_step(arch, B):
    """every weight read once per step (PRE table excluded: one row per stream)
    + per stream 50 lookback reads/writes of n_res floats + PRE row, skip/head vectors."""
    from lbwn.arch import ParamLayout
    lay = ParamLayout(arch)
    w = sum(e.numel for n, e in lay.entries.items() if n != 'PRE') * 4
    L, Cr = n_layers(arch), arch['n_res']
    per_stream = L * 2 * 4 * Cr + 4 * Cr + 4 * (arch['n_skip'] + arch['n_post'] + arch['n_quant']) + 4 * L * arch['n_dil']
    return w + B * per_stream


def bench_gen(net, arch, B=10, seconds=3.0, sr=16000, chunk=1000):
    """imodel.py cached generation, arch3, B=10, 3 s @ 16 kHz (BASELINE configs[2]), graph
    replay of chunk-sized step sequences; weights = the benchmark net's."""
    g = WaveNetGen(arch['n_blocks'], arch['n_block_layers'], arch['n_quant'], arch['n_res'], arch['n_dil'],
                   arch['n_skip'], arch['n_post'], arch['n_gc_embed'], arch['n_gc_category'], arch['use_bias'],
                   B, chunk, None, seed=1, graph=True)
    g.load_params(net)
    n = int(seconds * sr)
    g.build_graph(n)
    gc = list(range(1, B + 1)) if arch['n_gc_embed'] else None
    g.init_buffers(gc)
    g.step(chunk)   # capture + warm
    torch.cuda.synchronize()
    g.init_buffers(gc)
    t0 = time.perf_counter()
    g.step(n)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    bps = gen_bytes_per_step(arch, B)
    return {'metric': 'cached autoregressive gen audio samples/s (B streams x steps / wall)',
            'value': B * n / dt, 'unit': 'audio samples/s', 'steps': n, 'batch': B, 'wall_s': dt,
            'us_per_step': dt / n * 1e6, 'config': 'imodel.py cached gen, par/arch3.json, B=%d, %.0f s @ %d Hz, '
                                                   'chunk %d, hipGraph replay' % (B, seconds, sr, chunk),
            'roofline': {'bound': 'hbm', 'bytes_per_step': bps, 'achieved': bps * n / dt / 1e9, 'peak': HBM_PEAK / 1e9,
                         'unit': 'GB/s', 'frac': bps * n / dt / HBM_PEAK,
                         'note': 'weights are L2/MALL-resident across steps; the step is a 55-stage dependent '
                                 'chain, latency- not bandwidth-bound'}}


def cpu_baseline(arch, seconds):
    """Oracle (numpy fp32) fwd+loss+bwd+Adam at B=1, T=512 for ~`seconds`."""
    sys.path.insert(0, ROOT)
    from oracle import wavenet_ref as R
    try:
        from threadpoolctl import threadpool_info
        cores = max([x.get('num_threads', 1) for x in threadpool_info()] or [1])
    except Exception:
        cores = os.cpu_count() or 1
    rng = np.random.default_rng(0)
    P = R.init_params(arch, rng, dtype=np.float32)
    S = R.init_save(arch, 1, rng, dtype=np.float32)
    B, T = 1, 512
    q = rng.integers(0, arch['n_quant'], (B, T))
    ids = np.ones((B, T), np.int32)
    opt = R.AdamTF1(1e-3)

    def step():
        nonlocal S
        lg, cache, S = R.forward(arch, P, q, ids, S)
        st, dlog = R.loss_fcn(arch, P, lg, q, ids, 1e-3)
        G = R.backward(arch, P, cache, dlog, 1e-3)
        opt.step(P, G)

    step()  # warm-up (BLAS init)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        step()
        n += 1
    dt = time.perf_counter() - t0
    return {'value': B * T * n / dt, 'unit': 'audio samples/s', 'cores': int(cores), 'kind': 'port',
            'sample': 'oracle/wavenet_ref.py numpy fp32 train step (fwd+xent+bwd+TF1 Adam), arch3, B=1, '
                      'T=512, %d steps in %.1f s on the GPU box host (TF-CPU reference not installable)' % (n, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=8)
    ap.add_argument('--arch', default=os.path.join(ROOT, 'par', 'arch3.json'))
    ap.add_argument('--batch', type=int, default=8, help='streams per GPU')
    ap.add_argument('--slice', type=int, default=4096)
    ap.add_argument('--probe', default='auto')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--gc', type=int, default=None, help='--num-global-cond for GC archs')
    ap.add_argument('--no-gen', action='store_true')
    ap.add_argument('--gen-seconds', type=float, default=3.0)
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        raise SystemExit('--gpus %d but WORLD_SIZE=%d (launch N>1 with torch.distributed.run)' % (args.gpus, world))
    dp = lbdist.init()          # one process per GPU; RCCL when WORLD_SIZE > 1
    rank = dp.rank

    arch = load_arch(args.arch, num_global_cond=args.gc)
    B, T = args.batch, args.slice
    net = WaveNetTrain(**arch, batch_sz=B, l2_factor=1e-3, print_interval=0, seed=0)   # par1.json values
    opt = AdamOptimizer(1e-3)
    dev = net.device

    # synthetic data: the GLOBAL dealer over world·B slots; each rank keeps its rows
    hop = mel_hop_sz(arch)
    src = SyntheticSource(seed=1234, hop=hop, n_mel=arch['n_lc_in'] if arch['n_lc_out'] else 0,
                          n_voices=max(1, arch['n_gc_category']), n_quant=arch['n_quant'])
    dealer = SliceDealer(src, world * B, T, recep_field_sz(arch), hop, arch['n_lc_in'])
    ring = []
    for _ in range(8):
        _, wav, mel, ids = next(dealer)
        rows = dp.rows(B)
        ring.append((torch.as_tensor(wav[rows], dtype=torch.int32).to(dev),
                     None if mel is None else torch.as_tensor(mel[rows], dtype=torch.float32).to(dev),
                     torch.as_tensor(ids[rows], dtype=torch.int32).to(dev)))
    torch.cuda.synchronize()
    plan = net._plan(T)

    def step(i):
        q, mel, ids = ring[i % len(ring)]
        net.forward(q, mel, ids, backward=True)
        dp.reduce_grads(net)
        opt.apply(net)

    def probe(name):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        e.record()   # materialise the HIP events
        _lib.check(net.lib.lbwn_plan_probe(plan, name.encode(), s.cuda_event, e.cuda_event))
        return s, e

    M = B * T
    # candidates for the dominant kernel, likeliest first (one probe per warmup step): the
    # backward and forward layer chains, then the single-launch GEMMs
    cands = ['layer_bwd', 'dskip', 'layer_fwd', 'post1_fwd', 'dpost1', 'ds', 'post2_fwd', 'dpost2', 'dh']
    warm_t = {}
    for i in range(args.warmup):
        pr = None
        if args.probe == 'auto' and i >= 1 and i - 1 < len(cands):
            pr = (cands[i - 1], probe(cands[i - 1]))
        step(i)
        if pr:
            torch.cuda.synchronize()
            warm_t[pr[0]] = pr[1][0].elapsed_time(pr[1][1])
    dom = args.probe if args.probe != 'auto' else (max(warm_t, key=warm_t.get) if warm_t else 'layer_bwd')

    # ---- timed region ----
    samples = {dom: [], 'layer_fwd': []}
    pending = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i % 2 == 0:
            pending.append((dom, probe(dom)))
        else:
            pending.append(('layer_fwd', probe('layer_fwd')))
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    for name, (s, e) in pending:
        samples[name].append(s.elapsed_time(e))
    ms = dt * 1000.0 / args.steps
    ms = dp.max_over_ranks(ms, dev)
    value = world * B * T / (ms / 1000.0)

    def roof(name, ms_list):
        bound, work = kernel_work(name, arch, M)
        avg = float(np.mean(ms_list)) / 1000.0
        peak = FP32_MFMA_PEAK if bound == 'mfma' else HBM_PEAK
        ach = work / avg
        return {'kernel': name, 'bound': bound, 'achieved': ach / 1e12 if bound == 'mfma' else ach / 1e9,
                'peak': peak / 1e12 if bound == 'mfma' else peak / 1e9,
                'unit': 'TFLOP/s' if bound == 'mfma' else 'GB/s', 'frac': ach / peak,
                'avg_launch_us': avg * 1e6, 'work_per_launch': work, 'traffic': traffic_from_profiles(name)}

    out = {
        'metric': 'audio samples/sec: train fwd+bwd & cached autoregressive gen, 1/2/4/8 GPU',
        'value': value, 'unit': 'audio samples/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': ms, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
        'gemm_arith': ('f32 operands split exactly into 3 bf16 terms, 6 products on bf16 MFMA, f32 accumulation '
                       '(error vs fp64 <= the f32 MFMA: tests/test_gpu_parity.py::test_gemm_split_accuracy)'
                       if net.lib.lbwn_gemm_get_mode() == 1 else 'f32 MFMA (v_mfma_f32_32x32x2_f32)'),
        'data': 'synthetic 16 kHz harmonic tones, mu-law 256, dealt with the reference slicing/mask semantics',
        'config': {'workload': 'train step fwd+xent+bwd+TF1-Adam, par/arch3.json (5x10 layers, res/dil 32, '
                               'skip/post 512, Q 256), B=%d streams x T=%d per GPU' % (B, T),
                   'arch': os.path.basename(args.arch), 'batch_per_gpu': B, 'global_batch': world * B,
                   'slice_sz': T, 'parallelism': 'dp%d' % world},
        'roofline': roof(dom, samples[dom]),
        'roofline_dilconv': roof('layer_fwd', samples['layer_fwd']),
        'warmup_probe_ms': warm_t,
    }
    if world == 1 and not args.no_gen and arch['n_lc_out'] == 0:
        out['gen'] = bench_gen(net, arch, B=10, seconds=args.gen_seconds)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(arch, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def traffic_from_profiles(kernel):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_traffic.json,
    written by tools/pmc_traffic.py from separate rocprofv3 --pmc passes, FETCH_SIZE x2
    gfx950 correction), or None when not collected."""
    p = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        with open(p) as f:
            d = json.load(f)
        v = d.get(kernel)
        return None if v is None else v.get('hbm_bytes_per_launch')
    except Exception:
        return None


if __name__ == '__main__':
    main()
