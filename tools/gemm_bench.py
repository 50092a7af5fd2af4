"""Time lbwn_gemm_f32 on the training step's GEMM shapes (arch3, M = 32768) next to
torch.matmul fp32 (the vendor BLAS) on the same operands.  Usage: python tools/gemm_bench.py (a variant build: python tools/with_lib.py VARIANT.so tools/gemm_bench.py)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import torch  # noqa: E402
from lbwn import _lib  # noqa: E402

lib = _lib.load()
M = 32768
# name, M, N, K, a_kcontig, b_kcontig, split
SHAPES = [('skip_fwd', M, 512, 1600, 1, 0, 1), ('dz', M, 1600, 512, 1, 1, 1), ('dskip', 1600, 512, M, 0, 0, 19),
          ('post1_fwd', M, 512, 512, 1, 0, 1), ('ds', M, 512, 512, 1, 1, 1), ('dpost1', 512, 512, M, 0, 0, 4),
          ('post2_fwd', M, 256, 512, 1, 0, 1), ('dh', M, 512, 256, 1, 1, 1), ('dpost2', 512, 256, M, 0, 0, 8),
          # arch5 local conditioning (M = B·T = 32768 at B = 8): COND = lc·LCcat, dlc = DV·LCcatᵀ,
          # dLCCAT = lcᵀ·DV (K = 80 channels, or padded to 96)
          ('lc_cond', M, 3200, 80, 1, 0, 1), ('lc_cond96', M, 3200, 96, 1, 0, 1),
          ('lc_dlc', M, 80, 3200, 1, 1, 1), ('lc_dlc96', M, 96, 3200, 1, 1, 1),
          ('lc_dcat', 80, 3200, M, 0, 0, 8), ('lc_dcat96', 96, 3200, M, 0, 0, 8),
          # C4 (arch5 B = 32): dlc over M = 131072
          ('lc_dlc_c4', 4 * M, 80, 3200, 1, 1, 1), ('lc_dlc_c4_128', 4 * M, 128, 3200, 1, 1, 1)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


# GEMM_KSCAN=1: the post1 shape (N = 512, pre-split B) at K = 128 .. 2048 -- time against K separates
# the per-tile fixed cost (prologue fill, epilogue) from the k-loop
SHAPES += [('kscan%d' % k, M, 512, k, 1, 0, 1) for k in (128, 256, 512, 1024, 1600, 2048)]
only = os.environ.get('GEMM_ONLY') or ('kscan' if os.environ.get('GEMM_KSCAN') else None)
splits = os.environ.get('GEMM_SPLITS')   # e.g. "4,9,16": every listed split-K for the selected shapes
runs = [(s[0], s[1], s[2], s[3], s[4], s[5], int(x)) for s in SHAPES for x in splits.split(',')] if splits else SHAPES
for name, m, n, k, akc, bkc, split in runs:
    if only and name not in only.split(',') and not (only == 'kscan' and name.startswith('kscan')):
        continue
    if not only and name.startswith('kscan'):
        continue
    A = torch.randn(m, k, device='cuda') if akc else torch.randn(k, m, device='cuda')
    B = torch.randn(n, k, device='cuda') if bkc else torch.randn(k, n, device='cuda')
    C = torch.empty(m, n, device='cuda')
    slab = torch.empty(max(1, split) * m * n, device='cuda')
    st = _lib.stream_ptr()

    def ours():
        _lib.check(lib.lbwn_gemm_f32(A.data_ptr(), A.shape[1], akc, B.data_ptr(), B.shape[1], bkc, C.data_ptr(), n,
                                     m, n, k, None, 0, 0, None, 0, 0, split, slab.data_ptr(), st))
    b3 = None
    if akc and split == 1 and k % 32 == 0:   # the step's form: B pre-split once per step
        b3 = torch.empty(int(lib.lbwn_split_planes_elems_abi(n, k)), dtype=torch.int16, device='cuda')
        _lib.check(lib.lbwn_split_planes(B.data_ptr(), B.shape[1], n, k, 0 if bkc else 1, b3.data_ptr(), st))

    def ours_pre():
        _lib.check(lib.lbwn_gemm_f32_presplit(A.data_ptr(), A.shape[1], akc, b3.data_ptr(), n, B.data_ptr(),
                                              B.shape[1], bkc, C.data_ptr(), n, m, k, None, 0, 0, None, 0, 0, st))
    Am = A if akc else A.t()
    Bm = B.t() if bkc else B

    def ref():
        torch.matmul(Am, Bm, out=C)
    fl = 2.0 * m * n * k
    res = []
    for mode in (0, 1):
        _lib.check(lib.lbwn_gemm_set_mode(mode))
        t = timeit(ours)
        res.append('%s %7.1f us %6.1f TF' % (('f32 ', 'x3  ')[mode], t * 1e6, fl / t / 1e12))
    if b3 is not None:
        t = timeit(ours_pre)
        res.append('x3pre %7.1f us %6.1f TF' % (t * 1e6, fl / t / 1e12))
    t1 = timeit(ref)
    print('%-10s M%6d N%5d K%6d split %2d | %s | torch %7.1f us %6.1f TF' % (
        name, m, n, k, split, ' | '.join(res), t1 * 1e6, fl / t1 / 1e12), flush=True)
