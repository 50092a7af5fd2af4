"""MFMA utilisation per launch from one rocprofv3 counter pass (SQ_VALU_MFMA_BUSY_CYCLES,
SQ_INSTS_MFMA, SQ_BUSY_CYCLES, SQ_WAVES, SQ_WAVE_CYCLES, SQ_INSTS_VALU, GRBM_GUI_ACTIVE,
GRBM_COUNT).  SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-pipe cycles summed over the SIMDs
(= 32 x SQ_INSTS_MFMA for 32-cycle MFMAs, MI355X_MICROARCH.md § Per-instruction cycle
constants); GRBM_GUI_ACTIVE is the dispatch's GPU-busy cycles summed over the 8 XCDs, so

    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)

is the fraction of all SIMD cycles of the launch that the matrix pipe was busy.  Training
dispatches are named like tools/pmc_traffic.py (probe names); any other kernel (generation)
by its kernel name.  Usage: python tools/pmc_mfma.py DIR OUT.json [label]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import NAMED, gemm_key, is_gemm   # noqa: E402

SIMDS = 1024
COUNTERS = ('SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_INSTS_MFMA', 'SQ_BUSY_CYCLES', 'SQ_WAVES', 'SQ_WAVE_CYCLES',
            'SQ_INSTS_VALU', 'GRBM_GUI_ACTIVE', 'GRBM_COUNT')


def load(d):
    disp = defaultdict(dict)
    names = {}
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            i = int(r['Dispatch_Id'])
            disp[i][r['Counter_Name']] = disp[i].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
            names[i] = r['Kernel_Name']
    return [(i, names[i], disp[i]) for i in sorted(disp)]


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0]


def name_dispatches(rows, skip_steps=4):
    """Training runs: per step (opened by the prologue kernel), probe names for the chains, the
    head and the GEMMs in engine.cpp's enqueue order; other dispatches by kernel name."""
    out = defaultdict(list)
    kname = {}
    steps, cur = [], None
    for did, name, c in rows:
        if 'pack_layers' in name or 'step_prologue' in name:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((name, c))
        elif not steps:
            out[short(name)].append(c)
            kname[short(name)] = short(name)
    for st in steps[skip_steps:-1] or steps[-2:-1]:
        gi = 0
        for name, c in st:
            key = None
            for k, n in NAMED.items():
                if k in name:
                    key = n
            if is_gemm(name):
                key = gemm_key(gi, name)
                gi += 1
            if key:
                out[key].append(c)
                kname[key] = short(name)
    return out, kname


def main(d, out_path, label=''):
    rows = load(d)
    groups, kname = name_dispatches(rows)
    res = {'_about': {'label': label, 'formula': 'mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * %d)' % SIMDS,
                      'counters': list(COUNTERS), 'source': d}}
    for k, lst in sorted(groups.items()):
        mean = {c: sum(x.get(c, 0.0) for x in lst) / len(lst) for c in COUNTERS}
        cyc = mean['GRBM_GUI_ACTIVE'] / 8.0
        res[k] = {'kernel': kname.get(k, k), 'dispatches': len(lst), 'counters_per_dispatch': mean,
                  'gpu_cycles': cyc,
                  'mfma_busy': mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * SIMDS) if cyc else None,
                  'mfma_cycles_per_inst': (mean['SQ_VALU_MFMA_BUSY_CYCLES'] / mean['SQ_INSTS_MFMA']
                                           if mean['SQ_INSTS_MFMA'] else None)}
    json.dump(res, open(out_path, 'w'), indent=1)
    for k, v in res.items():
        if k.startswith('_'):
            continue
        print('%-14s %-44s mfma_busy %s  cycles %.0f  n=%d' % (
            k, v['kernel'][:44], '%.3f' % v['mfma_busy'] if v['mfma_busy'] is not None else '-', v['gpu_cycles'],
            v['dispatches']))


if __name__ == '__main__':
    main(*sys.argv[1:4])
