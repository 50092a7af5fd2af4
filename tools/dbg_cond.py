"""Debug: per-gradient errors of the conditioning parity case."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import numpy as np
import torch
from tests.test_gpu_parity import cond_arch, make_net, rand_batch, oracle_params
from oracle import wavenet_ref as R
gc, lc, C = (int(x) for x in sys.argv[1:4])
arch = cond_arch(gc, lc, C)
B, T = 2, 256
net = make_net(arch, B)
q, ids = rand_batch(arch, B, T)
rng = np.random.default_rng(3)
if gc:
    for b in range(B):
        cuts = np.sort(rng.choice(np.arange(40, T), 3, replace=False))
        v = rng.integers(1, arch['n_gc_category'] + 1, 4)
        ids[b] = np.repeat(v, np.diff(np.r_[0, cuts, T]))
        ids[b, cuts[1]:cuts[1] + 20] = 0
mel = rng.standard_normal((B, T // 8, arch['n_lc_in'])).astype(np.float32) if lc else None
P, S = oracle_params(net)
lg, cache, new_save = R.forward(arch, P, q, ids, S, mel=mel)
st, dlog = R.loss_fcn(arch, P, lg, q, ids, 0.0)
net.forward(q, mel, ids, backward=True)
torch.cuda.synchronize()
G = R.backward(arch, P, cache, dlog, 0.0)
for nm in ('x', 'z', 's', 'dz', 'ds', 'cond', 'dvall', 'gctab', 'gcd'):
    try:
        v = net.plan_tensor(T, nm)
    except Exception as ex:
        continue
    print('tensor', nm, 'nan', int(torch.isnan(v).sum()), 'inf', int(torch.isinf(v).sum()), 'absmax', float(v.abs().max()))
M = B * T
h1 = cache['h1'].reshape(M, -1); Sx = cache['S'].reshape(M, -1)
print('min |h1|', np.abs(h1).min(), 'min |S|', np.abs(Sx).min())
s_gpu = net.plan_tensor(T, 's').view(M, -1).cpu().double().numpy()
print('S flips', int(((s_gpu > 0) != (Sx > 0)).sum()))
for n in net.layout.names():
    o = G[n]; g = net.grads[n].cpu().double().numpy() / st['n_valid']
    print('%-22s %.3g  gpu_nan %d oracle_nan %d gpu_max %.3g oracle_max %.3g' % (n, np.abs(g - o).max() / max(1, np.abs(o).max()),
          np.isnan(g).sum(), np.isnan(o).sum(), np.abs(g).max(), np.abs(o).max()))
