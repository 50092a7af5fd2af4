"""Per-launch HBM bytes from two rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE, kB per
dispatch).  gfx950: FETCH_SIZE counts ½ of the bytes of wide coalesced reads, so
hbm_bytes = (2·FETCH_SIZE + WRITE_SIZE)·1024 (MI355X_MICROARCH.md § HBM).  Dispatches are
split into training steps at the step-prologue (or weight-pack) kernel and named in launch order: the chain
kernels by name, the GEMMs by their position in engine.cpp's fixed enqueue sequence (skip_fwd,
post1_fwd, post2_fwd, then dh, ds, dz, dpost2, dpost1 before the backward chain and dskip after
it; an LC arch's dLCcat, dlc and upsample GEMMs in between, gemm_key; dispatch ids follow
enqueue order)."""
import csv
import glob
import json
import sys

GEMM_ORDER = ['skip_fwd', 'post1_fwd', 'post2_fwd', 'dh', 'ds', 'dz', 'dpost2', 'dpost1', 'dskip']
NAMED = {'chain_fwd_kernel': 'layer_fwd', 'chain_bwd_kernel': 'layer_bwd', 'chain_bwd_x3_kernel': 'layer_bwd',
         'chain_fwd16_kernel': 'layer_fwd', 'chain_bwd16_kernel': 'layer_bwd',
         'head_kernel': 'head', 'head_reg_kernel': 'head',
         'layer_reduce_all_kernel': 'layer_reduce', 'pre_grad_part_kernel': 'dpre'}


def dispatches(d, counter):
    rows = []
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter:
                rows.append((int(r['Dispatch_Id']), r['Kernel_Name'], float(r['Counter_Value'])))
    rows.sort()
    return rows


def per_name(rows, skip_steps=8):
    steps, cur = [], None
    for did, name, v in rows:
        if 'pack_layers' in name or 'step_prologue' in name:   # the kernel that opens each step
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((name, v))
    out = {}
    for st in steps[skip_steps:-1] or steps[-2:-1]:
        gi = 0
        for name, v in st:
            key = None
            for k, n in NAMED.items():
                if k in name:
                    key = n
            if is_gemm(name):
                key = gemm_key(gi, name)
                gi += 1
            if key:
                out.setdefault(key, []).append(v)
    return {k: sum(v) / len(v) for k, v in out.items()}


def is_gemm(name):
    return any(g in name for g in ('gemm_f32_kernel', 'gemm_x3_kernel', 'gemm_x3r_kernel', 'gemm_x3q_kernel'))


def gemm_key(gi, name):
    """The gi-th GEMM dispatch of a step.  The first eight are the fixed head sequence; after the
    backward chain an LC arch enqueues dLCcat (side stream), dlc (96-column tiles) and the
    upsample's per-stage GEMMs before dSKIP (engine.cpp lbwn_train_backward), so those are named
    by their kernel form."""
    if gi < 8:
        return GEMM_ORDER[gi]
    if 'gemm_x3q_kernel<8, true>' in name:
        return 'dskip'
    if gi == 8:
        return 'lc_wgrad'
    if 'gemm_x3q_kernel<6' in name or 'gemm_x3r_kernel<3' in name:
        return 'lc_dlc'
    return 'lc_up_bwd_gemm'



def main(fdir, wdir, out_path):
    fetch = per_name(dispatches(fdir, 'FETCH_SIZE'))
    write = per_name(dispatches(wdir, 'WRITE_SIZE'))
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k), write.get(k)
        res[k] = {'fetch_size_kb': f, 'write_size_kb': w,
                  'hbm_bytes_per_launch': None if f is None or w is None else (2 * f + w) * 1024.0}
    json.dump(res, open(out_path, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(*sys.argv[1:4])
