#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel calls, total and average
duration, share; written as markdown next to the raw stats CSV copied into profiles/."""
import csv
import sys


def main(stats_csv, out_md, steps=None, title=''):
    rows = list(csv.DictReader(open(stats_csv)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    lines = ['# %s' % (title or stats_csv), '',
             '| kernel | calls | total us | avg us | % |', '|---|---:|---:|---:|---:|']
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
        lines.append('| `%s` | %s | %.1f | %.2f | %.1f |' % (
            r['Name'].replace('(anonymous namespace)::', '')[:90], r['Calls'], float(r['TotalDurationNs']) / 1e3,
            float(r['AverageNs']) / 1e3, 100 * float(r['TotalDurationNs']) / tot))
    lines.append('')
    lines.append('Total kernel time %.1f us%s' % (tot / 1e3, (' = %.1f us per step over %d steps' % (
        tot / 1e3 / steps, steps)) if steps else ''))
    open(out_md, 'w').write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None,
         sys.argv[4] if len(sys.argv) > 4 else '')
