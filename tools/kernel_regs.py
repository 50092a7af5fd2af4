"""Register budget of every kernel in the built library, read from its gfx950 code objects (no GPU).

The side stream's gradient kernels run beside dSKIP's weight-gradient GEMM only while they fit in
the VGPRs its two waves per SIMD leave free: a kernel that grows past that
waits for dSKIP's blocks instead, silently (round 6: the AMN GEMM at 238 -> 242 VGPRs pushed
pre_grad_part from 74 to 306 us at C2).  This reads `.vgpr_count` / `.agpr_count` /
`.sgpr_count` / `.group_segment_fixed_size` per kernel from the AMDGPU metadata notes of each
offload bundle in liblbwn.so's .hip_fatbin section.

Usage: python tools/kernel_regs.py [lib.so] [name-substring ...]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'lb-wavenet_amd', 'lbwn', 'liblbwn.so')
READELF = '/opt/rocm/lib/llvm/bin/llvm-readelf'
MAGIC = b'__CLANG_OFFLOAD_BUNDLE__'


def code_objects(path=LIB, arch='gfx950'):
    """The device ELF images for `arch` of every offload bundle in the library."""
    data = open(path, 'rb').read()
    out, pos = [], data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from('<Q', data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from('<QQQ', data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith(arch) or (arch + ':') in triple or triple.endswith(arch + '-'):
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 32)
    return out


def kernel_resources(path=LIB, arch='gfx950'):
    """{symbol name: {'vgpr': n, 'agpr': n, 'sgpr': n, 'lds': bytes}} over all bundles."""
    res = {}
    for img in code_objects(path, arch):
        with tempfile.NamedTemporaryFile(suffix='.co') as f:
            f.write(img)
            f.flush()
            txt = subprocess.run([READELF, '--notes', f.name], capture_output=True, text=True, check=True).stdout
        # one metadata map per kernel: '- .agpr_count: ...' starts it, keys indented below
        for blk in re.split(r'\n\s*- \.', txt)[1:]:
            blk = '.' + blk
            name = re.search(r'\.name:\s+(\S+)', blk)
            if not name:
                continue
            def num(key):
                m = re.search(r'\.%s:\s+(\d+)' % key, blk)
                return int(m.group(1)) if m else 0
            res[name.group(1)] = {'vgpr': num('vgpr_count'), 'agpr': num('agpr_count'),
                                  'sgpr': num('sgpr_count'), 'lds': num('group_segment_fixed_size')}
    return res


def demangled(names):
    try:
        out = subprocess.run(['c++filt'], input='\n'.join(names), capture_output=True, text=True,
                             check=True).stdout.splitlines()
        return dict(zip(names, out))
    except (OSError, subprocess.CalledProcessError):
        return {n: n for n in names}


if __name__ == '__main__':
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith('.so') else LIB
    pats = [a for a in sys.argv[1:] if not a.endswith('.so')]
    r = kernel_resources(lib)
    dm = demangled(sorted(r))
    for k in sorted(r, key=lambda k: dm[k]):
        if pats and not any(p in dm[k] for p in pats):
            continue
        v = r[k]
        print('%4d vgpr %4d agpr %4d sgpr %6d lds  %s' % (v['vgpr'], v['agpr'], v['sgpr'], v['lds'], dm[k][:110]))
