"""Debug: chain vs per-layer vs oracle grads when tiles exceed one round."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'lb-wavenet_amd'))
import numpy as np
import torch
from tests.test_gpu_parity import small_arch, make_net, rand_batch, oracle_params
from oracle import wavenet_ref as R

B, T = int(sys.argv[1]), int(sys.argv[2])
nbl = int(sys.argv[3]) if len(sys.argv) > 3 else 3
arch = small_arch(nb=1, nbl=nbl)
q, ids = rand_batch(arch, B, T)
res = {}
modes = sys.argv[4].split(',') if len(sys.argv) > 4 else ['chain', 'layers']
for mode in modes:
    os.environ['LBWN_NO_CHAIN'] = '1' if mode == 'layers' else '0'
    net = make_net(arch, B, l2=0.0)
    if mode == modes[0]:
        P, S = oracle_params(net)
    net.forward(q, None, ids, backward=True)
    torch.cuda.synchronize()
    print(mode, 'status', int(net.plan_tensor(T, 'status').view(torch.int32)[0]))
    res[mode] = {n: g.cpu().double().numpy() for n, g in net.grads.items()}
    res[mode]['_z'] = net.plan_tensor(T, 'z').view(B * T, -1).cpu().double().numpy()
    res[mode]['_s'] = net.plan_tensor(T, 's').view(B * T, -1).cpu().double().numpy()
    res[mode]['_r2'] = net.plan_tensor(T, 'r2').view(B * T, -1).cpu().double().numpy()
    res[mode]['_dlog'] = net.plan_tensor(T, 'logits').view(B * T, -1).cpu().double().numpy()
    res[mode]['_stats'] = net.stats.cpu().double().numpy()
lg, cache, _ = R.forward(arch, P, q, ids, S)
st, dlog = R.loss_fcn(arch, P, lg, q, ids, 0.0)
G = R.backward(arch, P, cache, dlog, 0.0)
L = R.n_layers(arch)
zc = np.concatenate([cache['z'][l].reshape(B * T, -1) for l in range(L)], 1)
print('oracle n_valid', st['n_valid'], 'mean_xent', st['mean_xent'], {m: res[m]['_stats'] for m in res})
for nm, ref in (('_z', zc), ('_s', cache['S'].reshape(B * T, -1)), ('_r2', cache['r2'].reshape(B * T, -1)),
                ('_dlog', dlog.reshape(B * T, -1) * st['n_valid'])):
    for mode in res:
        err = np.abs(res[mode][nm] - ref)
        i = np.unravel_index(err.argmax(), err.shape)
        print(nm, mode, 'max abs err %.3g at (t=%d, col=%d)' % (err.max(), i[0] % T, i[1]), 'rows>1e-6:',
              sorted(set((np.nonzero(err.max(1) > 1e-5)[0] % T).tolist()))[:20])
for m in res:
    P2 = P['POST2']; P1 = P['POST1']
    dh = (res[m]['_dlog'] @ P2.T) * (res[m]['_r2'] > 0)
    gp1 = np.maximum(res[m]['_s'], 0).T @ dh
    o = G['POST1'] * st['n_valid']
    print(m, 'POST1 gpu-vs-recomputed %.3g  recomputed-vs-oracle %.3g  gpu-vs-oracle %.3g  (scale %.3g)' % (
        np.abs(res[m]['POST1'] - gp1).max(), np.abs(gp1 - o).max(), np.abs(res[m]['POST1'] - o).max(), np.abs(o).max()))
    print(m, 'oracle S vs cache', np.abs(cache['S'].reshape(B*T,-1) - res[m]['_s']).max(), 'dh oracle', np.abs(dh - cache.get('dh', dh)).max() if 'dh' in cache else '-')
for n in res[modes[0]]:
    if n.startswith('_'):
        continue
    o = G[n] * st['n_valid']
    sc = max(1.0, np.abs(o).max())
    print('%-20s' % n, '  '.join('%s %.3g' % (md, np.abs(res[md][n] - o).max() / sc) for md in modes))
