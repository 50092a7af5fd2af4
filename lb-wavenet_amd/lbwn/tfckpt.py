"""TF V2 checkpoint bundles (``<prefix>.index`` + ``<prefix>.data-00000-of-00001``), weights only.

The reference saves its serial-named variables (arch.py:142: ``SIGNAL_2_7``, ``SAVE_128_2_7``,
``GLOBAL_STEP`` ...) with tf.train.Saver (ckpt.py:54-61, tmodel.py:330).  This module reads such a
bundle into numpy arrays, so a model trained by the reference resumes or generates here, and writes
one, so weights trained here load back into the reference's Saver.  Nothing in a file is executed:
the index is parsed as data (table blocks, varints and the two small protobuf messages below).

Format restated from TensorFlow's published sources (TensorFlow is not importable here, and the
reference ships no checkpoint, so byte-level parity with a TF-written file is UNPINNED; the
tests pin the CRC-32C known answer and the write -> read round trip):

* ``.index`` is a TF table (tensorflow/core/lib/io/table_format.txt, the LevelDB layout):
  data blocks of prefix-compressed entries [varint shared, varint non_shared, varint value_len,
  key delta, value] + uint32 restart offsets + uint32 restart count, each block followed by a
  5-byte trailer (compression type 0, masked CRC-32C of block + type byte); an index block whose
  values are BlockHandles (varint offset, varint size) of the data blocks; an empty metaindex
  block; a 48-byte footer (metaindex handle, index handle, zero padding to 40 bytes, magic
  0xdb4775248b80fb57 as two little-endian uint32).
* Entries (tensorflow/core/protobuf/tensor_bundle.proto): key "" holds BundleHeaderProto
  {1: num_shards, 2: endianness (0 = little), 3: VersionDef {1: producer}}; every other key is a
  variable name holding BundleEntryProto {1: dtype, 2: TensorShapeProto {2: Dim {1: size}},
  3: shard_id, 4: offset, 5: size, 6: fixed32 masked CRC-32C of the tensor bytes}.
* ``.data-00000-of-00001`` is the tensors' raw little-endian bytes at their offsets.
"""
import os
import struct

import numpy as np

MAGIC = 0xdb4775248b80fb57
DATA_SUFFIX = '.data-00000-of-00001'
INDEX_SUFFIX = '.index'

# tensorflow/core/framework/types.proto DataType values for the dtypes a WaveNet checkpoint holds
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64, 19: np.float16, 10: np.bool_}
_DT_OF = {np.dtype(v): k for k, v in _DT.items()}


# ---- CRC-32C (Castagnoli, reflected 0x82F63B78) ------------------------------------------------
def _table():
    t = np.zeros(256, dtype=np.uint32)
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t[i] = c
    return t


_T = _table()
_TL = [int(x) for x in _T]
_CHUNK = 4096
_SHIFT = None   # 32 columns: the register after _CHUNK zero bytes, from each basis bit


def _raw(reg, data):
    for byte in data:
        reg = _TL[(reg ^ byte) & 0xFF] ^ (reg >> 8)
    return reg


def _shift_cols():
    global _SHIFT
    if _SHIFT is None:
        r = np.array([1 << i for i in range(32)], dtype=np.uint32)
        for _ in range(_CHUNK):
            r = _T[r & 0xFF] ^ (r >> 8)
        _SHIFT = [int(x) for x in r]
    return _SHIFT


def crc32c(data, crc=0):
    """CRC-32C of ``data`` (bytes-like), continuing ``crc``.  Long inputs run as _CHUNK-byte
    chunks stepped side by side in numpy (each from register 0), folded in order by the linear
    map of _CHUNK zero bytes: reg(A‖B) = shift(reg(A)) ^ reg0(B)."""
    mv = memoryview(data).cast('B')
    reg = crc ^ 0xFFFFFFFF
    n = len(mv)
    nfull = n // _CHUNK if n >= 8 * _CHUNK else 0
    if nfull:
        blk = np.frombuffer(mv[:nfull * _CHUNK], dtype=np.uint8).reshape(nfull, _CHUNK)
        r = np.zeros(nfull, dtype=np.uint32)
        for j in range(_CHUNK):
            r = _T[(r ^ blk[:, j]) & 0xFF] ^ (r >> 8)
        cols = _shift_cols()
        for c in r.tolist():
            s = 0
            i = 0
            while reg:
                if reg & 1:
                    s ^= cols[i]
                reg >>= 1
                i += 1
            reg = s ^ c
    reg = _raw(reg, mv[nfull * _CHUNK:])
    return reg ^ 0xFFFFFFFF


def mask(crc):
    """LevelDB / TF masked CRC (crc32c::Mask)."""
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def unmask(m):
    rot = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---- varints and protobuf fields ----------------------------------------------------------------
def _put_varint(out, v):
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return


def _get_varint(buf, pos):
    shift = result = 0
    while True:
        if pos >= len(buf):
            raise ValueError('truncated varint')
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError('varint too long')


def _fields(buf):
    """Yield (field number, wire type, value) of a protobuf message; length-delimited values
    are bytes, fixed32/64 ints."""
    pos = 0
    while pos < len(buf):
        key, pos = _get_varint(buf, pos)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _get_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from('<Q', buf, pos)[0]
            pos += 8
        elif wt == 2:
            ln, pos = _get_varint(buf, pos)
            v = bytes(buf[pos:pos + ln])
            pos += ln
        elif wt == 5:
            v = struct.unpack_from('<I', buf, pos)[0]
            pos += 4
        else:
            raise ValueError('unsupported protobuf wire type %d' % wt)
        yield f, wt, v


def _pb_varint(out, field, v):
    _put_varint(out, field << 3)
    _put_varint(out, v & 0xFFFFFFFFFFFFFFFF)


def _pb_bytes(out, field, payload):
    _put_varint(out, (field << 3) | 2)
    _put_varint(out, len(payload))
    out += payload


def _entry_proto(dtype, shape, offset, size, crc):
    shp = bytearray()
    for d in shape:
        dim = bytearray()
        _pb_varint(dim, 1, int(d))
        _pb_bytes(shp, 2, dim)
    out = bytearray()
    _pb_varint(out, 1, dtype)
    _pb_bytes(out, 2, shp)
    if offset:
        _pb_varint(out, 4, offset)
    _pb_varint(out, 5, size)
    _put_varint(out, (6 << 3) | 5)
    out += struct.pack('<I', mask(crc))
    return bytes(out)


def _parse_entry(buf):
    e = {'dtype': 0, 'shape': [], 'shard_id': 0, 'offset': 0, 'size': 0, 'crc32c': None, 'slices': False}
    for f, _, v in _fields(buf):
        if f == 1:
            e['dtype'] = v
        elif f == 2:
            for sf, _, sv in _fields(v):
                if sf == 2:
                    size = 0
                    for df, _, dv in _fields(sv):
                        if df == 1:
                            size = dv - (1 << 64) if dv >= 1 << 63 else dv
                    e['shape'].append(size)
                elif sf == 3 and sv:
                    raise ValueError('unknown-rank shape in checkpoint entry')
        elif f == 3:
            e['shard_id'] = v
        elif f == 4:
            e['offset'] = v
        elif f == 5:
            e['size'] = v
        elif f == 6:
            e['crc32c'] = v
        elif f == 7:
            e['slices'] = True
    return e


# ---- table blocks -------------------------------------------------------------------------------
def _block(entries):
    """A block of (key, value) byte pairs, every entry a restart point (no prefix sharing)."""
    out = bytearray()
    restarts = []
    for k, v in entries:
        restarts.append(len(out))
        _put_varint(out, 0)
        _put_varint(out, len(k))
        _put_varint(out, len(v))
        out += k
        out += v
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack('<I', r)
    out += struct.pack('<I', len(restarts))
    return bytes(out)


def _put_block(f, contents):
    off = f.tell()
    f.write(contents)
    f.write(b'\x00' + struct.pack('<I', mask(crc32c(contents + b'\x00'))))
    return off, len(contents)


def _handle(off, size):
    out = bytearray()
    _put_varint(out, off)
    _put_varint(out, size)
    return bytes(out)


def _read_block(buf, handle, verify):
    off, pos = _get_varint(handle, 0)
    size, _ = _get_varint(handle, pos)
    if off + size + 5 > len(buf):
        raise ValueError('block handle past the end of the index file')
    contents = buf[off:off + size]
    if buf[off + size] != 0:
        raise ValueError('compressed table blocks are not supported (type %d)' % buf[off + size])
    if verify:
        want = unmask(struct.unpack_from('<I', buf, off + size + 1)[0])
        if crc32c(bytes(contents) + b'\x00') != want:
            raise ValueError('index block checksum mismatch at offset %d' % off)
    return contents


def _block_entries(block):
    n_restarts = struct.unpack_from('<I', block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * n_restarts
    pos, key = 0, b''
    while pos < end:
        shared, pos = _get_varint(block, pos)
        non_shared, pos = _get_varint(block, pos)
        vlen, pos = _get_varint(block, pos)
        key = key[:shared] + bytes(block[pos:pos + non_shared])
        pos += non_shared
        yield key, bytes(block[pos:pos + vlen])
        pos += vlen


# ---- bundles ------------------------------------------------------------------------------------
def exists(prefix):
    return os.access(prefix + INDEX_SUFFIX, os.R_OK)


def read_bundle(prefix, verify=True):
    """{variable name: numpy array} of a TF V2 bundle.  ``verify`` checks the index blocks' and
    every tensor's CRC-32C.  Raises ValueError on anything it does not understand (several data
    shards, partitioned variables, string tensors, big-endian bundles)."""
    with open(prefix + INDEX_SUFFIX, 'rb') as f:
        idx = f.read()
    if len(idx) < 48:
        raise ValueError('%s: too short for a table footer' % (prefix + INDEX_SUFFIX))
    lo, hi = struct.unpack_from('<II', idx, len(idx) - 8)
    if (hi << 32) | lo != MAGIC:
        raise ValueError('%s: not a TF table (bad magic)' % (prefix + INDEX_SUFFIX))
    footer = idx[len(idx) - 48:len(idx) - 8]
    _, pos = _get_varint(footer, 0)
    _, pos = _get_varint(footer, pos)       # metaindex handle (unused)
    index_handle = footer[pos:]
    index_block = _read_block(idx, index_handle, verify)
    out = {}
    data = None
    try:
        for _, handle in _block_entries(index_block):
            for key, val in _block_entries(_read_block(idx, handle, verify)):
                if key == b'':
                    for fnum, _, v in _fields(val):
                        if fnum == 1 and v != 1:
                            raise ValueError('bundles of %d data shards are not supported' % v)
                        if fnum == 2 and v != 0:
                            raise ValueError('big-endian bundles are not supported')
                    continue
                e = _parse_entry(val)
                if e['slices']:
                    raise ValueError('%s: partitioned variables are not supported' % key.decode())
                if e['dtype'] not in _DT:
                    raise ValueError('%s: unsupported dtype %d' % (key.decode(), e['dtype']))
                if e['shard_id'] != 0:
                    raise ValueError('%s: shard %d of a one-shard reader' % (key.decode(), e['shard_id']))
                if data is None:
                    data = np.memmap(prefix + DATA_SUFFIX, dtype=np.uint8, mode='r')
                raw = data[e['offset']:e['offset'] + e['size']]
                if len(raw) != e['size']:
                    raise ValueError('%s: tensor bytes past the end of the data file' % key.decode())
                if verify and e['crc32c'] is not None and crc32c(raw) != unmask(e['crc32c']):
                    raise ValueError('%s: tensor checksum mismatch' % key.decode())
                dt = np.dtype(_DT[e['dtype']]).newbyteorder('<')
                n = int(np.prod(e['shape'], dtype=np.int64)) if e['shape'] else 1
                if n * dt.itemsize != e['size']:
                    raise ValueError('%s: %d bytes for shape %s' % (key.decode(), e['size'], e['shape']))
                out[key.decode()] = np.frombuffer(bytes(raw), dtype=dt).astype(dt.newbyteorder('='))\
                    .reshape(e['shape'])
    finally:
        del data
    return out


def write_bundle(prefix, tensors):
    """Write {name: array-like} as a one-shard TF V2 bundle (keys sorted, as TF's BundleWriter
    requires); returns the prefix.  No ``.meta`` graph is written: tf.train.Saver.restore reads
    the bundle alone, while the reference's restore() (ckpt.py:71-75) also wants the ``.meta``
    file its own save() wrote beside it."""
    d = os.path.dirname(os.path.abspath(prefix))
    os.makedirs(d, exist_ok=True)
    entries = []
    with open(prefix + DATA_SUFFIX + '.tmp', 'wb') as df:
        for name in sorted(tensors, key=lambda s: s.encode()):
            a = tensors[name]
            if hasattr(a, 'detach'):
                a = a.detach().cpu().numpy()
            a = np.asarray(a)
            shape = a.shape            # (np.ascontiguousarray would make a 0-d array 1-d)
            if a.dtype not in _DT_OF:
                raise ValueError('%s: dtype %s has no TF DataType here' % (name, a.dtype))
            raw = a.astype(a.dtype.newbyteorder('<'), copy=False).tobytes()
            off = df.tell()
            df.write(raw)
            entries.append((name.encode(), _entry_proto(_DT_OF[a.dtype], shape, off, len(raw), crc32c(raw))))
    header = bytearray()
    _pb_varint(header, 1, 1)                       # num_shards
    ver = bytearray()
    _pb_varint(ver, 1, 1)                          # producer = kTensorBundleVersion
    _pb_bytes(header, 3, ver)
    entries.insert(0, (b'', bytes(header)))
    with open(prefix + INDEX_SUFFIX + '.tmp', 'wb') as f:
        # data blocks of ~4 KiB, as TF's table builder cuts them; the index keys are each block's
        # last key (a valid separator: >= every key of its block, < every key after it)
        index, cur, cur_sz = [], [], 0
        for k, v in entries:
            cur.append((k, v))
            cur_sz += len(k) + len(v) + 8
            if cur_sz >= 4096:
                index.append((cur[-1][0], _handle(*_put_block(f, _block(cur)))))
                cur, cur_sz = [], 0
        if cur:
            index.append((cur[-1][0], _handle(*_put_block(f, _block(cur)))))
        meta = _handle(*_put_block(f, _block([])))
        ih = _handle(*_put_block(f, _block(index)))
        footer = meta + ih
        f.write(footer + b'\x00' * (40 - len(footer)) + struct.pack('<II', MAGIC & 0xFFFFFFFF, MAGIC >> 32))
    os.replace(prefix + DATA_SUFFIX + '.tmp', prefix + DATA_SUFFIX)
    os.replace(prefix + INDEX_SUFFIX + '.tmp', prefix + INDEX_SUFFIX)
    return prefix


def main(argv=None):
    """python -m lbwn.tfckpt {import|export} SRC DST: TF bundle prefix <-> .safetensors file."""
    import argparse
    from . import ckpt
    p = argparse.ArgumentParser(description=main.__doc__)
    p.add_argument('direction', choices=['import', 'export'])
    p.add_argument('src')
    p.add_argument('dst')
    a = p.parse_args(argv)
    if a.direction == 'import':
        arrs = read_bundle(a.src)
        ckpt.save_tensors(ckpt.ckpt_file(a.dst), arrs)
        print('Wrote {} tensors to {}'.format(len(arrs), ckpt.ckpt_file(a.dst)))
    else:
        t = ckpt.load_tensors(a.src)
        ckpt.export_tf_bundle(t, a.dst)
        print('Wrote {} tensors to {}{{{},{}}}'.format(len(t), a.dst, INDEX_SUFFIX, DATA_SUFFIX))


if __name__ == '__main__':
    main()
