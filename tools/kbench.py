#!/usr/bin/env python
"""Per-kernel timing of the training plan via the plan's HIP-event probes (arch3 B=8 T=4096
by default).  Variant builds: python tools/with_lib.py VARIANT.so tools/kbench.py ..."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lbwn import _lib  # noqa: E402
from lbwn.arch import load_arch  # noqa: E402
from lbwn.tmodel import WaveNetTrain  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--arch', default=os.path.join(ROOT, 'par', 'arch3.json'))
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--slice', type=int, default=4096)
    ap.add_argument('--iters', type=int, default=4)
    ap.add_argument('--probes', default='layer_fwd@25,layer_bwd@25,layer_fwd@9,layer_bwd@9,layer_bwd@0')
    ap.add_argument('--tag', default='default')
    args = ap.parse_args()
    arch = load_arch(args.arch)
    net = WaveNetTrain(**arch, batch_sz=args.batch, l2_factor=1e-3, print_interval=0)
    rng = np.random.default_rng(0)
    q = torch.as_tensor(rng.integers(0, 256, (args.batch, args.slice)), dtype=torch.int32).cuda()
    ids = torch.ones_like(q)
    plan = net._plan(args.slice)
    net.forward(q, None, ids)
    torch.cuda.synchronize()
    res = {}
    for name in args.probes.split(','):
        ts = []
        for _ in range(args.iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            e.record()
            _lib.check(net.lib.lbwn_plan_probe(plan, name.encode(), s.cuda_event, e.cuda_event))
            net.forward(q, None, ids)
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) * 1000)
        res[name] = round(float(np.median(ts)), 2)
    print(json.dumps({'tag': os.path.basename(args.tag), 'us': res}))


if __name__ == '__main__':
    main()
