"""Debug: check backward GEMM outputs against torch on the GPU's own inputs."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import torch
from tests.test_gpu_parity import small_arch, make_net, rand_batch
B, T, nbl, mode = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
os.environ['LBWN_NO_CHAIN'] = '1' if mode == 'layers' else '0'
arch = small_arch(nb=1, nbl=nbl)
q, ids = rand_batch(arch, B, T)
net = make_net(arch, B, l2=0.0)
net.forward(q, None, ids, backward=True)
torch.cuda.synchronize()
M = B * T
t = lambda n: net.plan_tensor(T, n).double()
LOG, R2, S = t('logits').view(M, -1), t('r2').view(M, -1), t('s').view(M, -1)
DH, DS, DZ = t('dh').view(M, -1), t('ds').view(M, -1), t('dz').view(M, -1)
v = {k: x.double() for k, x in net.vars.items()}
dh = (LOG @ v['POST2'].T) * (R2 > 0)
ds = (DH @ v['POST1'].T) * (S > 0)
L = 10 if nbl == 10 else nbl
skip = torch.cat([v['SKIP_0_%d' % l] for l in range(nbl)], 0)
dz = DS @ skip.T
for nm, a, b in (('dh', DH, dh), ('ds', DS, ds), ('dz', DZ, dz)):
    err = (a - b).abs()
    bad = (err > 1e-4 * b.abs().max()).nonzero()
    print(nm, 'max err %.3g (scale %.3g)' % (err.max(), b.abs().max()), 'bad', bad.shape[0],
          'first rows', sorted(set(bad[:, 0].tolist()))[:10], 'cols', sorted(set(bad[:, 1].tolist()))[:10])
gp1 = torch.relu(S).T @ DH
print('dPOST1 err %.3g scale %.3g' % ((net.grads['POST1'].double() - gp1).abs().max(), gp1.abs().max()))
