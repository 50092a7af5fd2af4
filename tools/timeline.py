"""Print one training step's kernel timeline from a rocprofv3 kernel_trace CSV:
start offset, duration, queue, name.  Usage: timeline.py trace.csv [step_index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
step = int(sys.argv[2]) if len(sys.argv) > 2 else -3
starts = [i for i, r in enumerate(rows) if 'pack_layers' in r['Kernel_Name'] or 'step_prologue' in r['Kernel_Name']]
i0 = starts[step]
i1 = starts[step + 1] if step + 1 < len(starts) and step != -1 else len(rows)
seg = sorted(rows[i0:i1], key=lambda r: int(r['Start_Timestamp']))
t0 = int(seg[0]['Start_Timestamp'])
for r in seg:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    name = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '')
    name = name.split('(')[0][:60]
    print('%9.1f %8.1f q%-3s %s' % ((s - t0) / 1e3, (e - s) / 1e3, r['Queue_Id'], name))
