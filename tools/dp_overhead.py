"""Cost of the data-parallel gradient reduction on one GPU with the real RCCL collective: the C2
training step timed with lbwn.dist's bucketed reduce_grads through a one-rank "nccl" process
group (SUM over one rank = identity, so the same numbers; pack, RCCL all_reduce kernel and unpack
on the comm stream, the head_grads / side_grads wait points) against the plain step, interleaved.
What it measures is the device path's own cost and how much of it hides under the backward's
tail -- not the xGMI transfer, which needs a second GPU.

Usage: python tools/dp_overhead.py [--arch par/arch3.json] [--batch 8] [--steps 20] [--rounds 3]
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'lb-wavenet_amd')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--arch', default=os.path.join(ROOT, 'par', 'arch3.json'))
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--slice', type=int, default=4096)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--mode', choices=('both', 'dp', 'plain'), default='both')
    ap.add_argument('--last-on-comm', dest='last_on_main', action='store_false',
                    help='issue the last bucket from the comm stream (the round-5 order)')
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import bench
    from lbwn import dist as lbdist
    from lbwn.arch import load_arch
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))

    class ForcedDP(lbdist.DPContext):
        on = False

        @property
        def enabled(self):
            return self.on

    dp = ForcedDP(world=1, rank=0, local_rank=0, last_on_main=a.last_on_main)
    tb = bench.TrainBench(load_arch(a.arch), a.batch, a.slice, dp)
    for i in range(6):
        dp.on = bool(i & 1)
        tb.step(i)
    torch.cuda.synchronize()
    res = {'plain': [], 'rccl_buckets': []}
    host = {'plain': [], 'rccl_buckets': []}   # host time to enqueue the steps (before the sync)
    for _ in range(a.rounds):
        for on, key in ((False, 'plain'), (True, 'rccl_buckets')):
            if a.mode != 'both' and (a.mode == 'dp') != on:
                continue
            dp.on = on
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                tb.step(i)
            host[key].append((time.perf_counter() - t0) * 1e3 / a.steps)
            torch.cuda.synchronize()
            res[key].append((time.perf_counter() - t0) * 1e3 / a.steps)
    tb.net.check_status()
    out = {k: round(min(v), 4) for k, v in res.items() if v}
    out['all_ms'] = {k: [round(x, 4) for x in v] for k, v in res.items() if v}
    out['host_enqueue_ms'] = {k: round(min(v), 4) for k, v in host.items() if v}
    if a.mode == 'both':
        out['overhead_us'] = round((out['rccl_buckets'] - out['plain']) * 1e3, 1)
    out['config'] = {'arch': os.path.basename(a.arch), 'batch': a.batch, 'slice': a.slice, 'steps': a.steps,
                     'last_bucket_on_main': a.last_on_main}
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
