"""Cached generation timing: arch3 (or --arch), B streams, N steps after a warm chunk,
graph replay; prints us/step.  Run under rocprofv3 --kernel-trace --stats for the split."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import torch  # noqa: E402
from lbwn.arch import load_arch  # noqa: E402
from lbwn.imodel import WaveNetGen  # noqa: E402
from lbwn.tmodel import WaveNetTrain  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--arch', default=os.path.join(ROOT, 'par', 'arch3.json'))
ap.add_argument('--batch', type=int, default=10)
ap.add_argument('--steps', type=int, default=4000)
ap.add_argument('--chunk', type=int, default=1000)
ap.add_argument('--no-graph', action='store_true')
a = ap.parse_args()
arch = load_arch(a.arch)
net = WaveNetTrain(**arch, batch_sz=1, l2_factor=0.0, print_interval=0, seed=0)
g = WaveNetGen(arch['n_blocks'], arch['n_block_layers'], arch['n_quant'], arch['n_res'], arch['n_dil'],
               arch['n_skip'], arch['n_post'], arch['n_gc_embed'], arch['n_gc_category'], arch['use_bias'],
               a.batch, a.chunk, None, seed=1, graph=not a.no_graph)
g.load_params(net)
g.build_graph(a.steps + a.chunk)
gc = list(range(1, a.batch + 1)) if arch['n_gc_embed'] else None
g.init_buffers(gc)
g.step(a.chunk)
torch.cuda.synchronize()
t0 = time.perf_counter()
g.step(a.steps)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print('B=%d steps=%d  %.2f us/step  %.0f samples/s' % (a.batch, a.steps, dt / a.steps * 1e6, a.batch * a.steps / dt))
