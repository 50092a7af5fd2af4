"""Time lbwn_split_planes (the per-step pre-split of a GEMM weight into three bf16 planes) for the
arch3 head / skip weights, both orientations: us per call over 200 calls (one GPU).
Usage: python tools/split_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import torch  # noqa: E402
from lbwn import _lib  # noqa: E402

lib = _lib.load()
# (name, W rows x cols as stored, rows of the product N, K, trans): w3_shape in engine.cpp
jobs = [('SKIP_F', 1600, 512, 512, 1600, 1), ('SKIP_B', 1600, 512, 1600, 512, 0),
        ('POST1_F', 512, 512, 512, 512, 1), ('POST1_B', 512, 512, 512, 512, 0),
        ('POST2_F', 512, 256, 256, 512, 1), ('POST2_B', 512, 256, 512, 256, 0)]
for name, wr, wc, rows, K, trans in jobs:
    W = torch.randn(wr, wc, device='cuda')
    out = torch.empty(int(lib.lbwn_split_planes_elems_abi(rows, K)), dtype=torch.int16, device='cuda')
    for _ in range(10):
        _lib.check(lib.lbwn_split_planes(W.data_ptr(), wc, rows, K, trans, out.data_ptr(), None))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(200):
        _lib.check(lib.lbwn_split_planes(W.data_ptr(), wc, rows, K, trans, out.data_ptr(), None))
    e.record()
    torch.cuda.synchronize()
    print('%-8s %5d x %4d trans=%d  %.2f us per call' % (name, rows, K, trans, s.elapsed_time(e) * 1e3 / 200))
