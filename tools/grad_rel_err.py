import sys, os
sys.path.insert(0, 'lb-wavenet_amd'); sys.path.insert(0, '.')
import numpy as np, torch
from tests.test_gpu_parity import make_net, rand_batch, _run_oracle, arch3, small_arch, R
for which, B, T in [('arch3', 8, 4096), ('arch3', 2, 512)]:
    arch = arch3()
    net = make_net(arch, B)
    q, ids = rand_batch(arch, B, T)
    P, S, lg, cache, new_save, st, dlog = _run_oracle(arch, net, q, ids)
    net.forward(q, None, ids, backward=True)
    torch.cuda.synchronize()
    G = R.backward(arch, P, cache, dlog, 0.0)
    inv = 1.0 / st['n_valid']
    worst = []
    for name in net.layout.names():
        ours = net.grads[name].cpu().double().numpy() * inv
        ref = G[name]
        mx = float(np.max(np.abs(ref)))
        err = float(np.max(np.abs(ours - ref)))
        worst.append((err / max(mx, 1e-30), name, err, mx))
    worst.sort(reverse=True)
    print(which, B, T, 'worst rel-to-max:', ['%s %.2e (err %.2e max %.2e)' % (n, r, e, m) for r, n, e, m in worst[:8]], flush=True)
    print('median rel', np.median([w[0] for w in worst]), 'n', len(worst), flush=True)
