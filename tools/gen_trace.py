"""Wall-clock trace of one cached-generation step (LBWN_GEN_TRACE=1, set here), arch3, B
streams.  Persistent form (default for B <= 80, groups of <= 16): the run's last step as seen by chain block 0
and the last head block; per-step form (LBWN_GEN_PERSIST=0): per-layer cycles of stream 0's
gen_wave and the GEMV stamps.  Usage: python tools/gen_trace.py [B]"""
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
g.build_graph(4000)
g.init_buffers(list(range(1, B + 1)) if arch['n_gc_embed'] else None)
g.step(1000)
torch.cuda.synchronize()
L = arch['n_blocks'] * arch['n_block_layers']
runs = []
for _ in range(5):
    g.step(20)
    torch.cuda.synchronize()
    runs.append(g.tensor('trace', torch.int64).cpu().numpy().astype(np.int64).copy())
tr = np.median(np.array(runs), axis=0)
if g.persistent:
    us = lambda x: (x - tr[0]) / 100.0   # noqa: E731  (wall_clock64: 100 MHz)
    print('persistent, B=%d; us from chain block 0 starting step n-1 (after its draw):' % B)
    lay = np.diff(np.concatenate([[tr[0]], tr[8:8 + L]])) / 100.0
    print('  chain 0: layers end %.2f  (per layer median %.3f us, first %.3f)' % (us(tr[1]), np.median(lay), lay[0]))
    nr = 1 + (L - 1 + 7) // 8
    hl = us(tr[8 + L:8 + L + nr])
    print('  chain 0 layer ends: ' + ' '.join('%.2f' % x for x in us(tr[8:8 + L])[7::8]) + ' (every 8th)')
    print('  last head, thread 0 (stream 0) sweep done:  ' + ' '.join('%.2f' % x for x in us(tr[8 + L + 40:8 + L + 40 + nr])))
    print('  last head, round barrier passed:            ' + ' '.join('%.2f' % x for x in us(tr[8 + L + 80:8 + L + 80 + nr])))
    print('  last head: 8-layer rounds accumulated at    ' + ' '.join('%.2f' % x for x in hl))
    print('  last head: phase A done %.2f, skip gathered %.2f, partial logits published %.2f'
          % (us(tr[2]), us(tr[3]), us(tr[4])))
    print('  last head C: post1 partials %.2f, barrier %.2f, h %.2f' % tuple(us(tr[8 + L + 120:8 + L + 123])))
    print('  chain 0: logits gathered %.2f (heads 0-15, compute waves), barrier D passed %.2f (heads 16-31, '
          'loader waves), draw done %.2f' % (us(tr[5]), us(tr[7]), us(tr[6])))
    print('  step period ~ %.2f us (draw done - start of the step it drew)' % us(tr[6]))
    hs = tr[2 * L + 136:2 * L + 136 + 64].reshape(32, 2)
    if np.all(hs > 0):
        pub, got = us(hs[:, 0]), us(hs[:, 1])
        print('  every head: skip columns published %.2f .. %.2f (median %.2f; latest head %d), whole vector gathered '
              '%.2f .. %.2f' % (pub.min(), pub.max(), np.median(pub), int(np.argmax(pub)), got.min(), got.max()))
        print('  published by head: ' + ' '.join('%.2f' % x for x in pub))
    sub = tr[8 + L + 128:8 + L + 128 + 48].reshape(8, 6)
    if np.all(sub > 0):
        seg = np.diff(np.concatenate([sub, sub[1:, :1].tolist() + [[sub[-1, 5]]]], axis=1), axis=1)
        med = np.median(seg[:7], axis=0)
        print('  chain 0, layers 16-22, shader cycles: reads+conv dot+DPP %d, gate %d, z write+barrier %d, '
              'residual %d, x write+sync %d, to next layer start %d' % tuple(med[:6]))
else:
    rows = np.diff(np.concatenate([tr[:3], tr[4:4 + 2 * L]]))
    conv, res = rows[4::2], rows[3::2][:L]
    print('per-step form, B=%d: input %d cyc, taps+layer 0 wait %d cyc; per layer conv+gate %.0f, residual %.0f cycles'
          % (B, rows[0], rows[1], np.median(conv), np.median(res)))
    gm = tr[2 * L + 8:2 * L + 8 + 24].reshape(3, 8)
    for name, s in zip(['skip', 'post1', 'post2'], gm):
        print('gemv %-5s block0 %5.2f us (staged %d cyc, compute+store %d cyc); last block ends +%.2f us'
              % (name, (s[1] - s[0]) / 100.0, s[3] - s[2], s[4] - s[3], (s[7] - s[0]) / 100.0))
