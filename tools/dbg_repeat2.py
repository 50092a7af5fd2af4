"""Debug: determinism and chain-vs-layers for the conditioning arch."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import numpy as np
import torch
from tests.test_gpu_parity import cond_arch, make_net, rand_batch
gc, lc, C = (int(x) for x in sys.argv[1:4])
arch = cond_arch(gc, lc, C)
B, T = 2, 256
q, ids = rand_batch(arch, B, T)
rng = np.random.default_rng(3)
if gc:
    for b in range(B):
        cuts = np.sort(rng.choice(np.arange(40, T), 3, replace=False))
        v = rng.integers(1, arch['n_gc_category'] + 1, 4)
        ids[b] = np.repeat(v, np.diff(np.r_[0, cuts, T]))
        ids[b, cuts[1]:cuts[1] + 20] = 0
mel = rng.standard_normal((B, T // 8, arch['n_lc_in'])).astype(np.float32) if lc else None
res = []
for mode in ('0', '0', '1', '1'):
    os.environ['LBWN_NO_CHAIN'] = mode
    net = make_net(arch, B)
    net.forward(q, mel, ids, backward=True)
    torch.cuda.synchronize()
    res.append(({n: g.clone() for n, g in net.grads.items()}, net.plan_tensor(T, 'dvall').clone() if lc else None))
for i, j in ((0, 1), (2, 3), (0, 2)):
    worst = max(((res[i][0][n] - res[j][0][n]).abs().max().item(), n) for n in res[i][0])
    dv = (res[i][1] - res[j][1]).abs().max().item() if lc else 0
    print('run', i, 'vs', j, 'worst grad diff', worst, 'dvall diff', dv)
