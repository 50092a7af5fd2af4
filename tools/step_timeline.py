"""Print one training step's kernels (start offset, duration) from a rocprofv3 kernel trace:
the step between the 11th and 12th adam_kernel.  Usage: python tools/step_timeline.py TRACE.csv [k]"""
import csv
import sys


def main(path, k=10):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
    a, b = idx[k], idx[k + 1]
    t0 = int(rows[a]['End_Timestamp'])
    for r in rows[a + 1:b + 1]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '')
        print('%8.1f %7.1f  %s' % ((s - t0) / 1e3, (e - s) / 1e3, name[:70]))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
