"""Report, per kernel of a hipcc --save-temps .s file, the vmcnt waits that fall between the first
and last MFMA (a wait there usually means a load was consumed right after it was issued).
Usage: python tools/isa_waits.py FILE.s [NAME_SUBSTRING]"""
import re
import sys


def main(path, sub=''):
    s = open(path).read()
    for name in re.findall(r'^(_Z\w+):', s, re.M):
        if sub not in name:
            continue
        a = s.index(name + ':')
        b = s.index('.Lfunc_end', a)
        lines = [ln.strip() for ln in s[a:b].split('\n')]
        idx = [i for i, ln in enumerate(lines) if ln.startswith('v_mfma')]
        if not idx:
            continue
        region = lines[idx[0]:idx[-1]]
        waits = [ln for ln in region if 'vmcnt' in ln]
        print('%-70s mfma %4d  vmcnt waits in MFMA region %3d %s' % (name[:70], len(idx), len(waits), waits[:4]))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else '')
