#!/usr/bin/env python
"""Benchmark: WaveNet training step (forward + masked xent + backward + TF1 Adam) on
MI355X with synthetic 16 kHz µ-law input dealt by the reference's slicing semantics.

* N = 1: arch3 (par/arch3.json), B = 8 streams x T = 4096 (BASELINE.json configs[1], SURVEY
  §8 C2) is the headline line; the same run adds C4 (arch5, B = 32), the per-GPU share of C5
  (arch5, B = 8, one GPU), C1 (arch1, B = 2, T = 512, forward + loss) and C3 (cached
  generation, arch3, B = 10) as sub-objects, each with its CPU baseline where one applies.
* N > 1: data-parallel (one process per GPU, RCCL all-reduce of the flat gradient bucket +
  loss stats), per-GPU work fixed, so scaling is weak.  The headline line keeps the N = 1
  configuration per GPU (arch3, B = 8 per GPU) so that value(N) / value(1) is a true
  weak-scaling ratio; the same run then measures C5 -- arch5 at 8 streams per GPU, B = 8N
  in total (BASELINE configs[4] at N = 8) -- as the ``c5`` sub-object, whose one-GPU
  reference is the N = 1 line's ``c5_per_gpu``.  ``python bench.py --gpus N`` without
  torch.distributed.run spawns the N ranks itself (before anything touches the GPU; no
  exec); under torch.distributed.run it reads RANK / LOCAL_RANK / WORLD_SIZE like any worker.

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
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))

import numpy as np  # noqa: E402

HBM_PEAK = 8.0e12        # B/s, MI355X_MICROARCH.md chip table
FP32_MFMA_PEAK = 157.3e12  # FLOP/s dense fp32 MFMA
PROBE_EVERY = 4          # timed steps per probed step (bench run())
X3_PEAK = 2.5e15 / 6       # f32-equivalent FLOP/s of the exact 3-term bf16 split (6 dense bf16 products)


def chain_forms():
    """(forward, backward) chain forms of the plans this process creates (LBWN_CHAIN_TILE =
    <fwd>[:<bwd>], engine.cpp; unset = DEFAULT_TILE for both)."""
    v = os.environ.get('LBWN_CHAIN_TILE') or DEFAULT_TILE
    f, _, b = v.partition(':')
    return f, (b or f)


def chain_ceiling(name, arch, x3):
    """Peak of the arithmetic the chain kernel actually runs (f32-equivalent FLOP/s), per
    algorithmic FLOP: in the bf16-split build the backward chain (chain_bwd16_kernel, the default
    form) does dx, dSIG/dGATE and, since round 5, dz (18·Cr·Cd per position and layer) as split
    products and dRES (2·Cr·Cd) on the f32 MFMA (358 TF; 313 TF while dz was on the f32 MFMA too);
    the forward chain does its conv and residual (10·Cr·Cd) as split products."""
    if not x3:
        return FP32_MFMA_PEAK
    if name == 'layer_bwd':
        return 20.0 / (18.0 / X3_PEAK + 2.0 / FP32_MFMA_PEAK)
    return X3_PEAK


def chain_fwd_latency_floor(arch, B, T, clock_ghz=2.4, ncu=256):
    """Latency floor of the persistent forward chain (chain_fwd_kernel): per layer the
    cross-tile dependency runs producer's x_{l+1} stores -> drain -> flag -> consumer poll -> halo
    loads -> dilated tap -> gate -> residual -> stores, at MI355X_MICROARCH.md's constants:
      * sc1 store drain 332 cyc ('L2-warm vmcnt(N) drain 156 -> 332 cyc'), one-way flag 0.3 us
        (price table 'handoff-flag': 0.3-0.6 idle), halo payload read ~500 cyc (4 b128 loads per
        lane from L2: 'global_load L2-hit latency ~180-225 cyc' + the in-order drain), two
        workgroup barriers (20 cyc each, taken) and the halo LDS write/read (2 x 50);
      * the dilated tap: 2 k-steps x 2 (sig, gate) x 6 split products = 24 v_mfma_f32_32x32x16_bf16
        at 32 cyc; the residual 12 of them; the gate 16 x (exp, rcp, exp, rcp) at 8 cyc issue
        + 6 VALU at 4 = 16 x 56 (one reciprocal since round 3: exp, exp, rcp + 6 VALU = 16 x 48);
        splitting z into bf16 terms 16 x 22 cyc (5.5 VALU each).
    Rounds: tiles beyond one per CU run as further rounds of the whole chain."""
    from lbwn.arch import n_layers
    L = n_layers(arch)
    handoff = 332 + 0.3 * clock_ghz * 1e3 + 500 + 2 * 20 + 2 * 50
    compute = 24 * 32 + 12 * 32 + 16 * 48 + 16 * 22
    layer = handoff + compute
    tiles = B * ((T + 127) // 128)
    rounds = (tiles + ncu - 1) // ncu
    return {'layer_cycles': round(layer), 'handoff_cycles': round(handoff), 'compute_cycles': compute,
            'layers': L, 'rounds': rounds, 'launch_us': rounds * L * layer / (clock_ghz * 1e3),
            'clock_ghz': clock_ghz}


def kernel_work(name, arch, M):
    """Algorithmic work per launch."""
    from lbwn.arch import n_layers
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
    if name == 'layer_wgrad':
        # the residual stack's weight gradients over the backward chain's exports (LBWN_BWD_WGRAD=1):
        # per layer and position x_l (Cr; the dilated tap re-read from cache), z (Cd), dv (2 Cd)
        # and G (Cr) read once
        return 'hbm', 4.0 * M * (2 * Cr + 3 * Cd) * L
    if name == 'layer_fwd':
        # the whole residual stack (persistent chain launch, or the span of the L per-layer
        # launches): per layer and position x_l in (Cr), x_{l+1} out (Cr), z out (Cd); the
        # dilated tap x[t-d] is re-read from LDS / the neighbour tile and counted once.
        return 'hbm', 4.0 * M * (2 * Cr + Cd) * L
    raise KeyError(name)


def gen_bytes_per_step(arch, B):
    """every weight read once per step (PRE table excluded: one row per stream)
    + per stream 50 lookback reads/writes of n_res floats + PRE row, skip/head vectors."""
    from lbwn.arch import ParamLayout, n_layers
    lay = ParamLayout(arch)
    w = sum(e.numel for n, e in lay.entries.items() if n != 'PRE') * 4
    L, Cr = n_layers(arch), arch['n_res']
    per_stream = L * 2 * 4 * Cr + 4 * Cr + 4 * (arch['n_skip'] + arch['n_post'] + arch['n_quant']) + 4 * L * arch['n_dil']
    return w + B * per_stream


def _gen(net, arch, B, chunk, max_steps, env=None):
    """A generator with the benchmark net's weights and its plan built (the plan reads
    LBWN_GEN_* at creation, so `env` applies there)."""
    from lbwn.imodel import WaveNetGen
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        g = WaveNetGen(arch['n_blocks'], arch['n_block_layers'], arch['n_quant'], arch['n_res'], arch['n_dil'],
                       arch['n_skip'], arch['n_post'], arch['n_gc_embed'], arch['n_gc_category'], arch['use_bias'],
                       B, chunk, None, seed=1, graph=True)
        g.load_params(net)
        g.build_graph(max_steps)
        return g
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _gen_form(g, B):
    if g.persistent:
        groups = (B + 15) // 16
        return 'persistent (one launch per chunk%s)' % (', %d stream groups' % groups if groups > 1 else '')
    return 'per-step, head as MFMA GEMMs' if B > 16 else 'per-step, head as vector GEMVs'


def _gen_rate(g, arch, B, n, chunk):
    """wall time of n steps (graph replay of chunk-step runs), after a warm chunk."""
    import torch
    gc = [1 + b % max(1, arch['n_gc_category']) for b in range(B)] if arch['n_gc_embed'] else None
    g.init_buffers(gc)
    g.step(chunk)   # capture + warm
    torch.cuda.synchronize()
    g.init_buffers(gc)
    t0 = time.perf_counter()
    g.step(n)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    g.check_status()
    return dt


def gen_layer_latency(net, arch, B):
    """Median wall time of one layer of the dependent per-stream chain (conv -> gate ->
    residual), from the persistent kernel's in-kernel stamps (LBWN_GEN_TRACE plan)."""
    import torch
    from lbwn.arch import n_layers
    g = _gen(net, arch, B, 50, 400, env={'LBWN_GEN_TRACE': '1'})
    if not g.persistent:
        return None
    g.init_buffers([1 + b % max(1, arch['n_gc_category']) for b in range(B)] if arch['n_gc_embed'] else None)
    g.step(300)
    torch.cuda.synchronize()
    tr = g.tensor('trace', torch.int64).cpu().numpy().astype(np.int64)
    L = n_layers(arch)
    lay = np.diff(np.concatenate([[tr[0]], tr[8:8 + L]])) / 100.0   # wall_clock64: 100 MHz
    return float(np.median(lay))


def gen_latency_floor(arch, clock_ghz=2.4):
    """Latency floor of one cached-generation step (imodel.py:214-272) for this design (one CU
    per stream, the layer chain's dependent instructions on the critical path, three hand-offs to
    and from the head), from MI355X_MICROARCH.md's constants:
      * ds_read issue -> use 50 cyc (cycle table, 'ds_read_b32 latency'); a write made visible to
        the other waves = its lgkmcnt drain (taken as 50) + s_barrier (taken as 20: one 4-wave
        workgroup; the guide prices only grid barriers);
      * dependent v_fma_f32 4 cyc ('Dependent-chain latency'); v_exp_f32 / v_rcp_f32 8 cyc
        ('vector-instruction ISSUE cost'); a DPP / permlane step 8 cyc (one VALU + its nop);
      * a granule hand-off 0.8 us (price table 'handoff-1to1', idle, 8 B).
    Per layer: x and z LDS reads (2 x 50), two write->barrier hops (2 x 70), the conv dot chain (two
    4-wide dot4 per lane: 8 dependent FMA + 1 add = 36), two DPP reduction steps + bias + the
    gate pairing (2 x 12 + 4 + 8 = 36), tanh/sigmoid (mul, exp, add, rcp, fma, then z = t*s: 32),
    the residual dot chain (8 FMA + add: 36) and its permlane32 half-swap + adds (24).
    Per step: + three hand-offs (chain -> head skip columns, skip all-gather, partial logits ->
    draw) and the draw's wave scans (~30 dependent DPP steps: 240 cyc)."""
    from lbwn.arch import n_layers
    L = n_layers(arch)
    layer_cyc = 2 * 50 + 2 * (50 + 20) + 36 + 36 + 32 + 36 + 24
    step_us = L * layer_cyc / (clock_ghz * 1e3) + 3 * 0.8 + 240 / (clock_ghz * 1e3)
    return {'layer_cycles': layer_cyc, 'layer_us': layer_cyc / (clock_ghz * 1e3), 'layers': L,
            'handoffs': 3, 'handoff_us': 0.8, 'step_us': step_us, 'clock_ghz': clock_ghz}


def bench_gen(net, arch, B=10, seconds=3.0, sr=16000, chunk=1000, sweep=(16, 64, 80, 256)):
    """imodel.py cached generation, arch3, B=10, 3 s @ 16 kHz (BASELINE configs[2]), graph
    replay of chunk-sized step sequences; weights = the benchmark net's.  Also a B sweep and
    the step time against the latency floor of its dependent chain."""
    from lbwn.arch import n_layers
    n = int(seconds * sr)
    g = _gen(net, arch, B, chunk, n + chunk)
    dt = _gen_rate(g, arch, B, n, chunk)
    us = dt / n * 1e6
    bps = gen_bytes_per_step(arch, B)
    out = {'metric': 'cached autoregressive gen audio samples/s (B streams x steps / wall)',
           'value': B * n / dt, 'unit': 'audio samples/s', 'steps': n, 'batch': B, 'wall_s': dt,
           'us_per_step': us, 'form': _gen_form(g, B),
           'config': 'imodel.py cached gen, par/arch3.json, B=%d, %.0f s @ %d Hz, chunk %d, hipGraph replay'
                     % (B, seconds, sr, chunk)}
    # latency roofline: a step is L dependent layers (conv -> gate -> residual on one CU per
    # stream) plus the head's hand-offs; the floor is derived from instruction latencies
    # (gen_latency_floor), not from this kernel's own timings
    fl = gen_latency_floor(arch)
    t_layer = gen_layer_latency(net, arch, B)
    out['roofline'] = {'bound': 'latency', 'unit': 'us/step', 'achieved': us, 'peak': fl['step_us'],
                       'frac': fl['step_us'] / us, 'floor': fl,
                       'measured_per_layer_us': t_layer,
                       'mfma_busy': mfma_from_profiles('gen_persist_kernel', 'gen'),
                       'note': 'peak = the dependent chain of one step at MI355X_MICROARCH.md latencies '
                               '(gen_latency_floor); frac = floor / measured step'}
    out['roofline_hbm'] = {'bound': 'hbm', 'bytes_per_step': bps, 'achieved': bps * n / dt / 1e9, 'peak': HBM_PEAK / 1e9,
                           'unit': 'GB/s', 'frac': bps * n / dt / HBM_PEAK,
                           'note': 'weights are L2/MALL- and LDS/register-resident across steps: not bandwidth-bound'}
    rows = []
    for Bs in sweep:
        ns = 2000
        gs = _gen(net, arch, Bs, 500, ns + 500)
        dts = _gen_rate(gs, arch, Bs, ns, 500)
        bs = gen_bytes_per_step(arch, Bs)
        rows.append({'batch': Bs, 'us_per_step': dts / ns * 1e6, 'samples_per_s': Bs * ns / dts,
                     'weight_and_state_GB_per_s': bs * ns / dts / 1e9,
                     'form': _gen_form(gs, Bs)})
    out['sweep'] = rows
    return out


def _cores():
    try:
        from threadpoolctl import threadpool_info
        return int(max([x.get('num_threads', 1) for x in threadpool_info()] or [1]))
    except Exception:
        return os.cpu_count() or 1


def _oracle():
    sys.path.insert(0, ROOT)
    from oracle import wavenet_ref as R
    return R


def _timed(fn, seconds):
    fn()    # warm-up (BLAS init)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        n += 1
    return n, time.perf_counter() - t0


def cpu_baseline(arch, seconds, B=1, T=512, backward=True, label='arch3'):
    """Oracle (numpy fp32) train step (fwd+xent+bwd+TF1 Adam), or fwd+loss only, for
    ~`seconds` on the host cores (the TF-CPU reference cannot run: TF is not installable)."""
    R = _oracle()
    rng = np.random.default_rng(0)
    P = R.init_params(arch, rng, dtype=np.float32)
    S = R.init_save(arch, B, rng, dtype=np.float32)
    q = rng.integers(0, arch['n_quant'], (B, T))
    ids = rng.integers(1, max(1, arch['n_gc_category']) + 1, (B, T)).astype(np.int32)
    hop = 1
    for u in arch['lc_upsample'] if arch['n_lc_out'] else []:
        hop *= u
    mel = rng.standard_normal((B, T // hop, arch['n_lc_in'])).astype(np.float32) if arch['n_lc_out'] else None
    opt = R.AdamTF1(1e-3)

    def step():
        nonlocal S
        lg, cache, S = R.forward(arch, P, q, ids, S, mel)
        st, dlog = R.loss_fcn(arch, P, lg, q, ids, 1e-3)
        if backward:
            G = R.backward(arch, P, cache, dlog, 1e-3)
            opt.step(P, G)

    n, dt = _timed(step, seconds)
    what = 'train step (fwd+xent+bwd+TF1 Adam)' if backward else 'forward + loss'
    return {'value': B * T * n / dt, 'unit': 'audio samples/s', 'cores': _cores(), 'kind': 'port',
            'sample': 'oracle/wavenet_ref.py numpy fp32 %s, %s, B=%d, T=%d, %d steps in %.1f s on the GPU box '
                      'host (TF-CPU reference not installable)' % (what, label, B, T, n, dt)}


def cpu_baseline_gen(arch, seconds, B=10):
    """Oracle cached generation (imodel.py:214-272 restated) at C3's B for ~`seconds`."""
    R = _oracle()
    P = R.init_params(arch, np.random.default_rng(0), dtype=np.float32)
    n0 = 20
    t0 = time.perf_counter()
    R.generate(arch, P, B, n0, seed=1)
    per = (time.perf_counter() - t0) / n0
    n = max(n0, int(seconds / max(per, 1e-6)))
    t0 = time.perf_counter()
    R.generate(arch, P, B, n, seed=1)
    dt = time.perf_counter() - t0
    return {'value': B * n / dt, 'unit': 'audio samples/s', 'cores': _cores(), 'kind': 'port',
            'sample': 'oracle/wavenet_ref.py numpy fp32 cached generation, arch3, B=%d, %d steps in %.1f s '
                      '(C3 runs 48,000 steps; rate is per step, so the sample is scaled down)' % (B, n, dt)}


class TrainBench:
    """One (arch, B, T) training configuration on this rank: synthetic data from the GLOBAL
    dealer over world·B slots (each rank keeps its rows, data.py:210-224), the plan, and a
    step = forward + loss + backward + DP gradient all-reduce + TF1 Adam."""

    def __init__(self, arch, B, T, dp, backward=True):
        import torch
        from lbwn.arch import mel_hop_sz, recep_field_sz
        from lbwn.data import SliceDealer, SyntheticSource
        from lbwn.optim import AdamOptimizer
        from lbwn.tmodel import WaveNetTrain
        self.arch, self.B, self.T, self.dp, self.backward = arch, B, T, dp, backward
        self.net = WaveNetTrain(**arch, batch_sz=B, l2_factor=1e-3, print_interval=0, seed=0)   # par1.json values
        self.opt = AdamOptimizer(1e-3)
        dev = self.net.device
        hop = mel_hop_sz(arch)
        src = SyntheticSource(seed=1234, hop=hop, n_mel=arch['n_lc_in'] if arch['n_lc_out'] else 0,
                              n_voices=max(1, arch['n_gc_category']), n_quant=arch['n_quant'])
        dealer = SliceDealer(src, dp.world * B, T, recep_field_sz(arch), hop, arch['n_lc_in'])
        self.ring = []
        rows = dp.rows(B)
        for _ in range(8):
            _, wav, mel, ids = next(dealer)
            self.ring.append((torch.as_tensor(wav[rows], dtype=torch.int32).to(dev),
                              None if mel is None else torch.as_tensor(mel[rows], dtype=torch.float32).to(dev),
                              torch.as_tensor(ids[rows], dtype=torch.int32).to(dev)))
        torch.cuda.synchronize()
        self.plan = self.net._plan(T)

    def step(self, i):
        q, mel, ids = self.ring[i % len(self.ring)]
        self.net.forward(q, mel, ids, backward=self.backward)
        if self.backward:
            self.dp.reduce_grads(self.net)
            self.opt.apply(self.net)

    def probe(self, name):
        import torch
        from lbwn import _lib
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        e.record()   # materialise the HIP events
        _lib.check(self.net.lib.lbwn_plan_probe(self.plan, name.encode(), s.cuda_event, e.cuda_event))
        return s, e

    def run(self, steps, warmup, probes=None, probe_mode='auto'):
        """Warm up (one probe per warmup step to find the dominant kernel), then time
        exactly `steps` steps between barrier + synchronize pairs; max over ranks."""
        import torch
        import torch.distributed as dist
        from lbwn import _lib
        world = self.dp.world
        cands = probes or []
        warm_t = {}
        for i in range(warmup):
            pr = None
            if probe_mode == 'auto' and i >= 1 and i - 1 < len(cands):
                pr = (cands[i - 1], self.probe(cands[i - 1]))
            self.step(i)
            if pr:
                torch.cuda.synchronize()
                warm_t[pr[0]] = pr[1][0].elapsed_time(pr[1][1])
        dom = None
        if cands:
            dom = probe_mode if probe_mode != 'auto' else (max(warm_t, key=warm_t.get) if warm_t else cands[0])
        samples = {dom: [], 'layer_fwd': []} if dom else {}
        # probe pairs (a HIP event on each side of one launch) on every PROBE_EVERY-th timed step,
        # alternating the dominant kernel and the forward chain; the events are materialised
        # (first record) before the timed region, so a probed step adds only its two records
        # (~8 us each on this stack, profiles/r04_v1_step_timeline.txt) and unprobed steps none
        every = max(1, min(PROBE_EVERY, steps // 2))
        pairs = {}
        if dom:
            for k, i in enumerate(range(0, steps, every)):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                e.record()
                pairs[i] = (dom if k % 2 == 0 else 'layer_fwd', s, e)
        pending = []
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            if i in pairs:
                name, s, e = pairs[i]
                _lib.check(self.net.lib.lbwn_plan_probe(self.plan, name.encode(), s.cuda_event, e.cuda_event))
                pending.append((name, (s, e)))
            self.step(warmup + i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        # a chain hand-off that timed out in ANY step leaves its code in the cumulative status
        # (counters[3], ORed in by the optimizer kernel every step): such a run's numbers are
        # computed on garbage and must not be reported
        self.net.check_status(self.T)
        for name, (s, e) in pending:
            samples[name].append(s.elapsed_time(e))
        ms = self.dp.max_over_ranks(dt * 1000.0 / steps, self.net.device)
        return ms, dom, samples, warm_t

    def roof(self, name, ms_list, traffic=True):
        """`traffic`: PMC bytes from profiles/pmc_traffic.json, which holds the headline (C2)
        configuration only -- sub-benchmarks pass False.  MFMA-bound kernels are quoted against
        the peak of the arithmetic they run (chain_ceiling); the forward chain (HBM-quoted, as
        north_star asks) also carries its fraction of that MFMA floor: it is bound by neither,
        but by the per-layer hand-off latency."""
        bound, work = kernel_work(name, self.arch, self.B * self.T)
        avg = float(np.mean(ms_list)) / 1000.0
        x3 = self.net.lib.lbwn_gemm_get_mode() == 1
        peak = chain_ceiling(name, self.arch, x3) if bound == 'mfma' else HBM_PEAK
        ach = work / avg
        out = {'kernel': name, 'bound': bound, 'achieved': ach / 1e12 if bound == 'mfma' else ach / 1e9,
               'peak': peak / 1e12 if bound == 'mfma' else peak / 1e9,
               'unit': 'TFLOP/s' if bound == 'mfma' else 'GB/s', 'frac': ach / peak,
               'avg_launch_us': avg * 1e6, 'work_per_launch': work,
               'traffic': traffic_from_profiles(name, traffic if isinstance(traffic, str) else None) if traffic else None,
               'mfma_busy': mfma_from_profiles(name, traffic if isinstance(traffic, str) else None) if traffic else None}
        if bound == 'mfma':
            out['arith'] = ('bf16-split (6 products) for dx, dz and dSIG/dGATE, f32 MFMA for dRES'
                            if x3 and name == 'layer_bwd' else ('bf16-split' if x3 else 'f32 MFMA'))
            out['frac_of_f32_peak'] = ach / FP32_MFMA_PEAK
        if name == 'layer_fwd':
            L, Cr, Cd = self.arch['n_blocks'] * self.arch['n_block_layers'], self.arch['n_res'], self.arch['n_dil']
            # conv + residual, + the in-chain LC term (2 Lo 2Cd per position) when the chain computes it
            lo = self.arch['n_lc_out'] if 64 < self.arch['n_lc_out'] <= 80 and x3 else 0
            fl = (10.0 * Cr * Cd + 4.0 * lo * Cd) * self.B * self.T * L
            cp = chain_ceiling(name, self.arch, x3)
            out['mfma'] = {'flop_per_launch': fl, 'achieved_tflops': fl / avg / 1e12, 'peak_tflops': cp / 1e12,
                           'frac': fl / avg / cp, 'floor_us': fl / cp * 1e6}
            # the chain is bound by neither HBM nor MFMA but by its per-layer dependent path:
            # quoted HBM (north_star) with the latency floor beside it
            out['bound'] = 'latency'
            out['hbm_frac'] = out['frac']
            lf = chain_fwd_latency_floor(self.arch, self.B, self.T)
            out['latency_floor'] = lf
            out['latency_frac'] = lf['launch_us'] / (avg * 1e6)
        return out

    def close(self):
        import torch
        del self.net, self.ring
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


FWD_TILES = {'128': dict(positions=128, waves=8, waves_per_simd=2, kernel='chain_fwd16_kernel<8> / chain_bwd16_kernel<8>'),
             '64': dict(positions=64, waves=4, waves_per_simd=1, kernel='chain_fwd16_kernel<4> / chain_bwd16_kernel<4>'),
             'w32': dict(positions=128, waves=4, waves_per_simd=1,
                         kernel='chain_fwd_kernel / chain_bwd_x3_kernel (32-position waves)')}


def chain_dilation_sweep(arch_file, B, T, dp, steps=4, gc=None, tile=None):
    """C4's LDS-tile x dilation sweep (BASELINE configs[3], SURVEY §8d "Shapes"): for one forward
    chain tile (LBWN_CHAIN_TILE, read at plan creation: '128' / '64' = 16-position waves on 128- /
    64-position tiles, 'w32' = 32-position waves on 128), the timed step and the in-kernel clock
    stamps of one chain block's tile (LBWN_CHAIN_TRACE), which give each layer's start-to-start
    time in the forward and the backward chain; layers grouped by dilation d = 2^bl
    (tmodel.py:313-325), median over the n_blocks layers of each d and over steps.  The tile
    applies to both chains (chain_fwd16_kernel / chain_bwd16_kernel, or the w32 pair)."""
    import torch
    from lbwn.arch import load_arch, n_layers
    arch = load_arch(arch_file, num_global_cond=gc)
    saved = {k: os.environ.get(k) for k in ('LBWN_CHAIN_TRACE', 'LBWN_CHAIN_TILE')}

    def restore():
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    if tile is not None:
        os.environ['LBWN_CHAIN_TILE'] = tile
    try:
        tb = TrainBench(arch, B, T, dp)          # untraced: the tile's step time
        ms, _, _, _ = tb.run(10, 3)
        tb.close()
        os.environ['LBWN_CHAIN_TRACE'] = '1'
        tb = TrainBench(arch, B, T, dp)
    finally:
        restore()
    L, nbl = n_layers(arch), arch['n_block_layers']
    runs = []
    for i in range(steps + 1):
        tb.step(i)
        torch.cuda.synchronize()
        if i >= 1:
            runs.append(tb.net.plan_tensor(T, 'ctrace').view(torch.int64).cpu().numpy().reshape(2, L, 16).copy())
    tb.net.check_status(T)
    tb.close()
    r = np.array(runs)                          # [steps][fwd, bwd][L][16]
    fwd = r[:, 0, 1:, 0] - r[:, 0, :-1, 0]      # layer l = 0..L-2: start(l+1) - start(l)
    bwd = r[:, 1, :-1, 0] - r[:, 1, 1:, 0]      # layer l = 1..L-1 (runs L-1 .. 0): start(l-1) - start(l)
    rows = []
    for bl in range(nbl):
        fl = [l for l in range(L - 1) if l % nbl == bl]
        bls = [l - 1 for l in range(1, L) if l % nbl == bl]
        fc, bc = float(np.median(fwd[:, fl])), float(np.median(bwd[:, bls]))
        rows.append({'d': 1 << bl, 'fwd_cycles': round(fc), 'bwd_cycles': round(bc),
                     'fwd_us': round(fc / 2400.0, 3), 'bwd_us': round(bc / 2400.0, 3)})
    t = tile or os.environ.get('LBWN_CHAIN_TILE') or DEFAULT_TILE
    info = FWD_TILES.get(t, {})
    return {'tile': t, 'fwd_tile_positions': info.get('positions'), 'fwd_waves_per_block': info.get('waves'),
            'fwd_waves_per_simd': info.get('waves_per_simd'), 'fwd_kernel': info.get('kernel'),
            'bwd_tile_positions': info.get('positions'), 'tile_channels': 32, 'blocks_per_cu': 1,
            'ms_per_step': ms,
            'clock': 'clock64 cycles, us at 2.4 GHz', 'traced_block': 1, 'per_dilation': rows,
            'note': 'per-layer start-to-start time of one chain block (its first tile), median over the '
                    'n_blocks layers of each dilation and %d steps; ms_per_step: 10 timed steps after 3 '
                    'warmup' % steps}


DEFAULT_TILE = '128'    # the library's default chain form (engine.cpp, LBWN_CHAIN_TILE unset)


def wgrad_out():
    """The plans of this process take the residual stack's weight gradients out of the backward
    chain (LBWN_BWD_WGRAD, read at plan creation, engine.cpp; default: in the chain)."""
    return os.environ.get('LBWN_BWD_WGRAD', '0') == '1'


def cands():
    """Launches probed during warmup (one per warmup step) to find the dominant kernel."""
    wg = ['layer_wgrad'] if wgrad_out() else []
    return ['layer_bwd'] + wg + ['dskip', 'layer_fwd', 'post1_fwd', 'dpost1', 'ds', 'post2_fwd', 'dpost2', 'dh']


def sub_bench(arch_file, B, T, dp, steps, warmup, gc=None, backward=True, label='', traffic_tag=None):
    """A secondary configuration (C1 / C4 / C5-per-GPU) in the same run."""
    from lbwn.arch import load_arch
    arch = load_arch(arch_file, num_global_cond=gc)
    tb = TrainBench(arch, B, T, dp, backward=backward)
    ms, dom, samples, warm_t = tb.run(steps, warmup, probes=cands() if backward else None)
    out = {'workload': label, 'arch': os.path.basename(arch_file), 'batch_per_gpu': B, 'slice_sz': T,
           'value': dp.world * B * T / (ms / 1000.0), 'unit': 'audio samples/s', 'ms_per_step': ms,
           'steps': steps, 'warmup': warmup}
    if dom:
        out['roofline'] = tb.roof(dom, samples[dom], traffic=traffic_tag or False)
        out['roofline_dilconv'] = tb.roof('layer_fwd', samples['layer_fwd'], traffic=traffic_tag or False)
    tb.close()
    return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=8)
    ap.add_argument('--arch', default=None, help='default: par/arch3.json (C2 per GPU); C5 (arch5) rides along')
    ap.add_argument('--batch', type=int, default=8, help='streams per GPU')
    ap.add_argument('--slice', type=int, default=4096)
    ap.add_argument('--probe', default='auto')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--gc', type=int, default=None, help='--num-global-cond for GC archs')
    ap.add_argument('--no-gen', action='store_true')
    ap.add_argument('--no-extras', action='store_true', help='skip the C1 / C4 / C5 sub-benchmarks')
    ap.add_argument('--gen-seconds', type=float, default=3.0)
    ap.add_argument('--dry-run', action='store_true',
                    help='launcher + DP plumbing only, on the CPU over gloo (no GPU call): tests')
    return ap.parse_args(argv)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch(args, argv):
    """`bench.py --gpus N` outside torch.distributed.run: start N rank processes of this
    script (children, never an exec) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, and
    exit with the worst child status.  This parent never touches the GPU."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')    # dmabuf IPC only on this pool (RCCL)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in procs:          # one rank failed: the collective would hang
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc if rc >= 0 else 128 - rc


def dry_run(args):
    """Rank processes join a gloo group, reduce a gradient-sized buffer through
    lbwn.dist exactly as a training step does, and rank 0 prints one JSON line."""
    import torch
    from lbwn import dist as lbdist
    from lbwn.arch import ParamLayout, load_arch
    dp = lbdist.init(device_type='cpu')
    arch = load_arch(args.arch or os.path.join(ROOT, 'par', 'arch3.json'), num_global_cond=args.gc)
    n = ParamLayout(arch).n_total

    class _Net:
        grad_flat = torch.full((n,), float(dp.rank + 1))
        stats = torch.tensor([1.0, 10.0 * (dp.rank + 1), 2.0, 0.0])
        layout = ParamLayout(arch)
        _status = torch.zeros(1, dtype=torch.int32)

        def status_word(self):
            return self._status
    net = _Net()
    t0 = time.perf_counter()
    dp.reduce_grads(net)
    ms = dp.max_over_ranks((time.perf_counter() - t0) * 1e3, 'cpu')
    want = dp.world * (dp.world + 1) / 2
    ok = bool(torch.all(net.grad_flat == want)) and float(net.stats[1]) == 10.0 * want
    if dp.rank == 0:
        print(json.dumps({'dry_run': True, 'world_size': dp.world, 'backend': torch.distributed.get_backend()
                          if dp.enabled else None, 'grad_floats': n, 'reduce_ok': ok, 'reduce_ms': ms,
                          'arch': os.path.basename(args.arch or 'arch3.json'),
                          'batch_per_gpu': args.batch}), flush=True)
    if dp.enabled:
        torch.distributed.destroy_process_group()
    return 0 if ok else 1


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        return launch(args, argv)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        raise SystemExit('--gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
    if args.dry_run:
        return dry_run(args)

    import torch
    import torch.distributed as dist
    from lbwn import dist as lbdist
    from lbwn.arch import load_arch
    dp = lbdist.init()          # one process per GPU; RCCL when WORLD_SIZE > 1
    rank = dp.rank
    arch_file = args.arch or os.path.join(ROOT, 'par', 'arch3.json')
    arch = load_arch(arch_file, num_global_cond=args.gc)
    B, T = args.batch, args.slice
    tb = TrainBench(arch, B, T, dp)
    net = tb.net
    ms, dom, samples, warm_t = tb.run(args.steps, args.warmup, probes=cands(), probe_mode=args.probe)
    value = world * B * T / (ms / 1000.0)
    cid = {'arch3.json': 'C2' + (' per GPU' if world > 1 else ''),
           'arch5.json': 'C5' if B == 8 and world > 1 else 'arch5'}.get(os.path.basename(arch_file), 'custom')
    name = os.path.basename(arch_file)
    out = {
        'metric': 'audio samples/sec: train fwd+bwd & cached autoregressive gen, 1/2/4/8 GPU',
        'value': value, 'unit': 'audio samples/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': ms, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
        'gemm_arith': ('f32 operands split exactly into 3 bf16 terms, 6 products on bf16 MFMA, f32 accumulation '
                       '(error vs fp64 <= the f32 MFMA: tests/test_gpu_parity.py::test_gemm_split_accuracy)'
                       if net.lib.lbwn_gemm_get_mode() == 1 else 'f32 MFMA (v_mfma_f32_32x32x2_f32)'),
        'data': 'synthetic 16 kHz harmonic tones, mu-law 256, dealt with the reference slicing/mask semantics',
        'config': {'workload': '%s: train step fwd+xent+bwd+TF1-Adam, par/%s (5x10 layers, res/dil %d, skip/post %d, '
                               'Q %d%s), B=%d streams x T=%d per GPU' % (
                                   cid, name, arch['n_res'], arch['n_skip'], arch['n_quant'],
                                   (', GC %d/%d' % (arch['n_gc_embed'], arch['n_gc_category']) if arch['n_gc_embed']
                                    else '') + (', LC %d->%d x%s' % (arch['n_lc_in'], arch['n_lc_out'],
                                                                     arch['lc_upsample']) if arch['n_lc_out'] else ''),
                                   B, T),
                   'arch': name, 'batch_per_gpu': B, 'global_batch': world * B,
                   'slice_sz': T, 'parallelism': 'dp%d' % world, 'world_size_seen': dist.get_world_size()
                   if dist.is_initialized() else 1},
        'roofline': tb.roof(dom, samples[dom]),
        'roofline_dilconv': tb.roof('layer_fwd', samples['layer_fwd']),
        'warmup_probe_ms': warm_t,
    }
    if world == 1 and not args.no_gen and arch['n_lc_out'] == 0:
        out['gen'] = bench_gen(net, arch, B=10, seconds=args.gen_seconds)
        if not args.no_cpu_baseline:
            out['gen']['cpu_baseline'] = cpu_baseline_gen(arch, args.cpu_seconds * 0.5)
    tb.close()
    if world == 1 and not args.no_extras and args.arch is None:
        par = lambda f: os.path.join(ROOT, 'par', f)   # noqa: E731
        out['c4'] = sub_bench(par('arch5.json'), 32, 4096, dp, 10, 3, label='C4: arch5 deep stack, B=32 x T=4096, '
                              'train fwd+bwd+Adam, 1 GPU', traffic_tag='c4')
        out['c4']['sweep'] = {'default_tile': os.environ.get('LBWN_CHAIN_TILE') or DEFAULT_TILE,
                              'tiles': [chain_dilation_sweep(par('arch5.json'), 32, 4096, dp, tile=t)
                                        for t in ('128', '64', 'w32')]}
        out['c5_per_gpu'] = sub_bench(par('arch5.json'), 8, 4096, dp, 10, 3,
                                      label='C5 per-GPU share on one GPU: arch5, B=8 x T=4096 (the N>1 runs '
                                            'default to this per rank: scaling reference)', traffic_tag='c5')
        out['c1'] = sub_bench(par('arch1.json'), 2, 512, dp, 20, 5, backward=False,
                              label='C1: arch1 (GC 17/377), B=2 x T=512, forward + masked xent loss')
        if not args.no_cpu_baseline:
            out['c1']['cpu_baseline'] = cpu_baseline(load_arch(par('arch1.json')), args.cpu_seconds * 0.5, B=2,
                                                     T=512, backward=False, label='arch1')
    if world > 1 and not args.no_extras and args.arch is None:
        out['c5'] = sub_bench(os.path.join(ROOT, 'par', 'arch5.json'), 8, 4096, dp, 10, 3,
                              label='C5: arch5, B=8 per GPU x %d GPUs = global B=%d, T=4096, DP over RCCL '
                                    '(one-GPU reference: the N=1 line\'s c5_per_gpu)' % (world, 8 * world))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(arch, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def traffic_from_profiles(kernel, tag=None):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_traffic.json for the
    headline C2 configuration, profiles/pmc_traffic_<tag>.json for another one, written by
    tools/pmc_traffic.py from separate rocprofv3 --pmc passes, FETCH_SIZE x2 gfx950
    correction), or None when not collected."""
    p = os.path.join(ROOT, 'profiles', 'pmc_traffic%s.json' % ('_' + tag if tag else ''))
    try:
        with open(p) as f:
            d = json.load(f)
        v = d.get(kernel)
        return None if v is None else v.get('hbm_bytes_per_launch')
    except Exception:
        return None


def mfma_from_profiles(kernel, tag=None):
    """Matrix-pipe utilisation of a launch from the committed PMC summary (profiles/pmc_mfma.json
    for C2, profiles/pmc_mfma_<tag>.json for c4 / gen; tools/pmc_mfma.py over one counter-only
    rocprofv3 pass): {'mfma_busy': SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs),
    'kernel', 'source'}, or None when not collected."""
    p = os.path.join(ROOT, 'profiles', 'pmc_mfma%s.json' % ('_' + tag if tag else ''))
    try:
        with open(p) as f:
            d = json.load(f)
        v = d.get(kernel)
        if v is None or v.get('mfma_busy') is None:
            return None
        return {'frac': v['mfma_busy'], 'kernel': v['kernel'], 'source': 'profiles/' + os.path.basename(p)}
    except Exception:
        return None


if __name__ == '__main__':
    sys.exit(main())
