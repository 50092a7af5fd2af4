"""Cycle-stamp trace of one cached-generation step (stream 0): prologue (weights + taps),
step input, then per layer conv+gate and residual.  Needs LBWN_GEN_TRACE=1 (set here)."""
import os
import sys

os.environ['LBWN_GEN_TRACE'] = '1'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from lbwn.arch import load_arch  # noqa: E402
from lbwn.imodel import WaveNetGen  # noqa: E402
from lbwn.tmodel import WaveNetTrain  # noqa: E402

arch = load_arch(os.path.join(ROOT, 'par', 'arch3.json'))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 10
net = WaveNetTrain(**arch, batch_sz=1, l2_factor=0.0, print_interval=0, seed=0)
g = WaveNetGen(arch['n_blocks'], arch['n_block_layers'], arch['n_quant'], arch['n_res'], arch['n_dil'],
               arch['n_skip'], arch['n_post'], arch['n_gc_embed'], arch['n_gc_category'], arch['use_bias'],
               B, 200, None, seed=1, graph=False)
g.load_params(net)
g.build_graph(2000)
g.init_buffers(list(range(1, B + 1)) if arch['n_gc_embed'] else None)
g.step(1000)
torch.cuda.synchronize()
L = arch['n_blocks'] * arch['n_block_layers']
rows, gv, ps = [], [], []
for _ in range(5):
    g.step(2)   # the second launch draws the first step itself (the fused path)
    torch.cuda.synchronize()
    full = g.tensor('trace', torch.int64).cpu().numpy()
    tr = full[:4 + 2 * L]
    rows.append(np.diff(np.concatenate([tr[:3], tr[4:4 + 2 * L]])))
    gv.append(full[2 * L + 8:2 * L + 8 + 24].reshape(3, 8).astype(np.int64))
    ps.append(full[2 * L + 40:2 * L + 40 + 3 * B].reshape(B, 3).astype(np.int64))
d = np.median(np.array(rows), axis=0)
print('cycles: input %d  wait for taps+layer 0 %d  first-conv %d' % (d[0], d[1], d[2]))
conv, res = d[4::2], d[3::2][:L]
print('per layer (median over layers): conv+gate %.0f  residual %.0f   total %.0f cycles' %
      (np.median(conv), np.median(res), np.median(conv) + np.median(res)))
print('layers:', ' '.join('%d/%d' % (c, r) for c, r in zip(d[2::2][:L], d[3::2][:L])))
print('total kernel cycles (stamps): %d' % (np.sum(d)))
gm = np.median(np.array(gv), axis=0)
w = gm[0]
print('wall (us from chain block 0 start): chain end %.2f; last skip helper start %.2f, end %.2f'
      % ((w[1] - w[0]) / 100.0, (w[2] - w[0]) / 100.0, (w[3] - w[0]) / 100.0))
print('  last helper: layer-a poll done %.2f, layer-b poll done %.2f, accumulated %.2f'
      % ((w[4] - w[0]) / 100.0, (w[6] - w[0]) / 100.0, (w[5] - w[0]) / 100.0))
for name, s in zip(['post1', 'post2'], gm[1:]):
    print('gemv %-5s block0 %5.2f us (staged %d cyc, compute+store %d cyc); last block starts +%.2f us, ends +%.2f us'
          % (name, (s[1] - s[0]) / 100.0, s[3] - s[2], s[4] - s[3], (s[6] - s[0]) / 100.0, (s[7] - s[0]) / 100.0))
print('gap: post1->post2 start %.2f us' % ((gm[2][0] - gm[1][0]) / 100.0))
pm = np.median(np.array(ps) - np.array(gv)[:, :1, :1], axis=0) / 100.0
print('per stream (us from chain block 0 start): start / input ready / chain end')
for b in range(B):
    print('  stream %2d  %6.2f %6.2f %6.2f' % (b, pm[b, 0], pm[b, 1], pm[b, 2]))
