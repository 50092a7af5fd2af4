"""Sum rocprofv3 counter-collection CSVs per kernel (kernel-name substring filter): value per dispatch
(mean over dispatches).  Usage: python tools/pmc_summary.py DIR [kernel-name-substring]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
pref = sys.argv[2] if len(sys.argv) > 2 else ''
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if pref and pref not in k:
            continue
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k in sorted(acc):
    print(k[:90])
    for c in sorted(acc[k]):
        v = acc[k][c]
        print('   %-26s %16.0f  (per dispatch, n=%d)' % (c, sum(v) / len(v), len(v)))
