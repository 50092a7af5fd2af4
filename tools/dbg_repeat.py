"""Debug: run-to-run determinism of the training step in a given mode."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import torch
from tests.test_gpu_parity import small_arch, make_net, rand_batch
B, T, nbl, mode = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
os.environ['LBWN_NO_CHAIN'] = '1' if mode == 'layers' else '0'
arch = small_arch(nb=1, nbl=nbl)
q, ids = rand_batch(arch, B, T)
ref = None
for rep in range(4):
    net = make_net(arch, B, l2=0.0)
    net.forward(q, None, ids, backward=True)
    torch.cuda.synchronize()
    g = {n: x.clone() for n, x in net.grads.items()}
    if ref is None:
        ref = g
    else:
        worst = max(((g[n] - ref[n]).abs().max().item(), n) for n in g)
        print(mode, 'rep', rep, 'max diff vs rep0', worst)
