"""Step time of the C2 bench loop with and without the live kernel probes (HIP events around the
probed launch, every step), interleaved: the events' cost inside the timed region."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'lb-wavenet_amd'))
import bench  # noqa: E402
from lbwn import dist as lbdist  # noqa: E402
from lbwn.arch import load_arch  # noqa: E402

tb = bench.TrainBench(load_arch(os.path.join(ROOT, 'par', 'arch3.json')), 8, 4096, lbdist.DPContext())
for r in range(3):
    a, _, _, _ = tb.run(40, 4, probes=None)
    b, dom, _, _ = tb.run(40, 4, probes=bench.CANDS)
    print('round %d: no probes %.4f ms, probed (%s) %.4f ms' % (r, a, dom, b), flush=True)
