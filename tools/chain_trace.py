"""Cycle-stamp trace of the backward layer chain for one block's tile (arch3, B=8, T=4096):
per layer, the segments between the stamps in chain_bwd_kernel.  LBWN_CHAIN_TRACE=<block>
(set here; block k runs tile ntiles-1-k).  Usage: python tools/chain_trace.py [block]"""
import os
import sys

BLK = sys.argv[1] if len(sys.argv) > 1 else '1'
os.environ['LBWN_CHAIN_TRACE'] = BLK
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from lbwn.arch import load_arch, n_layers  # noqa: E402
from lbwn.tmodel import WaveNetTrain  # noqa: E402

arch = load_arch(os.path.join(ROOT, 'par', 'arch3.json'))
B, T = 8, 4096
L = n_layers(arch)
net = WaveNetTrain(**arch, batch_sz=B, l2_factor=0.0, print_interval=0, seed=0)
g = torch.Generator().manual_seed(0)
q = torch.randint(0, 256, (B, T), generator=g, dtype=torch.int32).cuda()
ids = torch.ones(B, T, dtype=torch.int32).cuda()
runs = []
for i in range(6):
    net.forward(q, None, ids, backward=True)
    torch.cuda.synchronize()
    if i >= 2:
        runs.append(net.plan_tensor(T, 'ctrace').view(torch.int64).cpu().numpy().reshape(2, L, 16).copy())
allr = np.median(np.array(runs), axis=0).astype(np.int64)
fw = allr[0]
fnames = ['image prefetch issue', 'producer wait', 'halo loads + bar', 'dilated conv + gate',
          'residual + next own tap', 'drain + bar + publish + image', 'z / sigma store issue']
fseg = np.diff(fw[:, :8], axis=1)
fmed = np.median(fseg[1:-1], axis=0)
ftot = np.median(fw[:, 7] - fw[:, 0])
print('chain_fwd block %s, per layer (median cycles over layers):' % BLK)
for n, m in zip(fnames, fmed):
    print('  %-26s %6d  (%4.1f %%)' % (n, m, 100.0 * m / ftot))
print('  layer total                %6d  = %.2f us at 2.4 GHz' % (ftot, ftot / 2400.0))
print('    of which residual + stores %6d, next own tap %6d' % (np.median(fw[1:-2, 8] - fw[1:-2, 4]), np.median(fw[1:-2, 5] - fw[1:-2, 8])))
print('    drain (vmcnt 0) %6d, barrier %6d, publish + image %6d' % (np.median(fw[1:-2, 9] - fw[1:-2, 5]),
      np.median(fw[1:-2, 10] - fw[1:-2, 9]), np.median(fw[1:-2, 6] - fw[1:-2, 10])))
tr = allr[1]   # backward
if net.lib.lbwn_gemm_get_mode() == 1:      # chain_bwd_x3_kernel: XSTAMP(0..6)
    names = ['G wait+build, DMA issue', 'dz,dv,DV', 'dx MFMA + OC', 'publish+img DMA+prefetch', 'dSIG MFMA',
             'dRES+bias+slab+bar']
    if os.environ.get('LBWN_BWD_WGRAD') == '1':   # export form: no weight gradients in the chain
        names = ['G build (G rows landed)', 'dz,dv, DV+G export', 'dx MFMA + OC', 'drain+bar+publish',
                 'image DMA + flag poll', 'G row loads issue']
    order = list(range(L - 1, -1, -1))
    seg = np.diff(tr[:, :7], axis=1)[order]
    med = np.median(seg[1:-1], axis=0)
    per = np.median(np.diff(tr[order, 0]))          # layer start to next layer start
    print('chain_bwd_x3 block %s, per layer (median cycles over layers):' % BLK)
    for n, m in zip(names, med):
        print('  %-26s %6d  (%4.1f %%)' % (n, m, 100.0 * m / per))
    print('  layer period               %6d  = %.2f us at 2.4 GHz;  whole tile %d cycles' %
          (per, per / 2400.0, tr[0, 6] - tr[L - 1, 0]))
    sub = tr[order][1:-1]
    if np.all(sub[:, 13] > 0):   # sub-stamps of dSIG (8 reads, 9 DMA issue, 10 k-step 0) and the tail
        for n, i, j in [('dSIG: operand reads', 4, 8), ('dSIG: DMA + row issue', 8, 9), ('dSIG: k-step 0', 9, 10),
                        ('dSIG: k-step 1', 10, 5), ('dRES', 5, 11), ('bias + dRES slab + bar', 11, 12),
                        ('dSIG partials + bar', 12, 13), ('dSIG sum + slab', 13, 6)]:
            print('    %-26s %6d' % (n, np.median(sub[:, j] - sub[:, i])))
    if os.environ.get('TRACE_TAIL') == '1' and np.all(sub[:, 15] > 0):
        # a timing variant with stamps 7 / 14 / 15 moved into the weight-gradient tail (after the
        # bias sums, after the flag wait, after the barrier): where the tail's cycles go
        for n, i, j in [('tail: bias sums (waves 0-2)', 11, 7), ('tail: flag wait (tid 0)', 7, 14),
                        ('tail: barrier', 14, 15), ('tail: G-row loads + bias sum + store', 15, 12),
                        ('tail: partials park + barrier', 12, 13), ('tail: partial sums + slab', 13, 6)]:
            print('    %-36s %6d' % (n, np.median(sub[:, j] - sub[:, i])))
    elif np.all(sub[:, 15] > 0):   # sub-stamps of the G build (7 flag barrier, 14 G written, 15 vmcnt drained)
        for n, i, j in [('G: flag wait + barrier', 0, 7), ('G: loads + LDS writes', 7, 14), ('G: vmcnt(0)', 14, 15),
                        ('G: barrier', 15, 1)]:
            print('    %-26s %6d' % (n, np.median(sub[:, j] - sub[:, i])))
    sys.exit(0)
names = ['stage x/dz + bar', 'gate recompute', 'G wait+build', 'dz,dv,DV', 'dx MFMA+OC', 'publish bar',
         'dSIG MFMA', 'bar+dRES', 'bias+slab+bar', 'image+bar']
seg = np.diff(tr[:, :11], axis=1)          # [L][10]
order = list(range(L - 1, -1, -1))         # execution order: top layer first
seg = seg[order]
med = np.median(seg[1:-1], axis=0)
tot = np.median(tr[:, 10] - tr[:, 0])
print('chain_bwd block %s, per layer (median cycles over layers):' % BLK)
for n, m in zip(names, med):
    print('  %-18s %6d  (%4.1f %%)' % (n, m, 100.0 * m / tot))
print('  layer total        %6d  = %.2f us at 2.4 GHz;  whole tile %d cycles = %.0f us' %
      (tot, tot / 2400.0, tr[0, 10] - tr[L - 1, 0], (tr[0, 10] - tr[L - 1, 0]) / 2400.0))
