"""Checkpoints: this framework's torch files and the reference's TF-1.x tensor bundles.

The reference saves and restores with tf.train.Saver (train.py:176, 237-243, 282; partial
restore of `backbone.+|refine.+` at train.py:155-158, 191-193; evaluate.py:221-224 takes the
latest checkpoint of a directory).  Saver writes a *tensor bundle*:

  <prefix>.index                  an SSTable (LevelDB table format) mapping each variable name
                                  to a BundleEntryProto (dtype, shape, shard, offset, size,
                                  masked CRC32C); key "" holds the BundleHeaderProto
  <prefix>.data-00000-of-00001    the raw little-endian tensor bytes
  checkpoint                      text proto naming the latest prefix (model_checkpoint_path)

`load_variables` reads either format into a ParamStore: names are the slim variable names
(mobilenet.py:275 scopes, catch_net.py:53/289/298/324), so the map is 1:1; TF's HWIO conv
weights [kh, kw, Cin, Cout] become [Cout, kh, kw, Cin], depthwise [3, 3, C, 1] becomes
[3, 3, C]; conv2d_transpose weights [2, 2, F, Cin] are stored as TF stores them.
`save_tf_bundle` writes the inverse, so the reference's Saver can restore what this
framework trained.  Parity unpinned: no TF checkpoint of the reference exists here (the
format follows tensorflow/core/util/tensor_bundle and tensorflow/core/lib/io/table as
published; the round trip is tested against the reader).
"""
from __future__ import annotations

import os
import re
import struct

import numpy as np
import torch

from . import io_native, pbwire

TABLE_MAGIC = 0xdb4775248b80fb57
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64, 10: np.bool_,
       19: np.float16}
_DT_INV = {np.dtype(v): k for k, v in _DT.items()}
DT_BFLOAT16 = 14


# ---------------------------------------------------------------- SSTable

def _crc_ok(block, typ, stored):
    return io_native.masked_crc32c(bytes(block) + bytes([typ])) == stored


def _snappy_decompress(src):
    """Raw snappy block (leveldb kSnappyCompression)."""
    src = bytes(src)
    n, pos = pbwire.read_varint(src, 0)
    out = bytearray()
    while pos < len(src):
        tag = src[pos]
        pos += 1
        t = tag & 3
        if t == 0:                                   # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(src[pos:pos + nb], 'little')
                pos += nb
            ln += 1
            out += src[pos:pos + ln]
            pos += ln
            continue
        if t == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | src[pos]
            pos += 1
        elif t == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 2], 'little')
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(src[pos:pos + 4], 'little')
            pos += 4
        if off == 0 or off > len(out):
            raise ValueError('corrupt snappy block')
        for _ in range(ln):                          # overlapping copies are legal
            out.append(out[-off])
    if len(out) != n:
        raise ValueError('snappy length mismatch')
    return bytes(out)


def _read_block(data, handle, verify=True):
    off, size = handle
    contents = data[off:off + size]
    typ = data[off + size]
    stored = struct.unpack_from('<I', data, off + size + 1)[0]
    if verify and not _crc_ok(contents, typ, stored):
        raise IOError('SSTable block at %d: checksum mismatch' % off)
    if typ == 1:
        contents = _snappy_decompress(contents)
    elif typ != 0:
        raise IOError('SSTable block at %d: unknown compression %d' % (off, typ))
    return bytes(contents)


def _block_entries(block):
    nrest = struct.unpack_from('<I', block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    pos, key = 0, b''
    while pos < end:
        shared, pos = pbwire.read_varint(block, pos)
        nonshared, pos = pbwire.read_varint(block, pos)
        vlen, pos = pbwire.read_varint(block, pos)
        key = key[:shared] + block[pos:pos + nonshared]
        pos += nonshared
        yield key, block[pos:pos + vlen]
        pos += vlen


def _handle(buf, pos=0):
    off, pos = pbwire.read_varint(buf, pos)
    size, pos = pbwire.read_varint(buf, pos)
    return (off, size), pos


def read_sstable(path, verify=True):
    """[(key bytes, value bytes)] of a LevelDB-format table (TF's tensor-bundle index)."""
    data = open(path, 'rb').read()
    if len(data) < 48 or struct.unpack_from('<Q', data, len(data) - 8)[0] != TABLE_MAGIC:
        raise IOError('%s is not an SSTable (bad magic)' % path)
    foot = data[len(data) - 48:]
    _meta, pos = _handle(foot)
    index_h, _ = _handle(foot, pos)
    out = []
    for _, v in _block_entries(_read_block(data, index_h, verify)):
        h, _ = _handle(v)
        out.extend(_block_entries(_read_block(data, h, verify)))
    return out


def _block_bytes(entries, restart_interval=16):
    buf, restarts, last = bytearray(), [], b''
    for i, (k, v) in enumerate(entries):
        shared = 0
        if i % restart_interval == 0:
            restarts.append(len(buf))
        else:
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        buf += pbwire.varint(shared) + pbwire.varint(len(k) - shared) + pbwire.varint(len(v))
        buf += k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack('<I', r)
    buf += struct.pack('<I', len(restarts))
    return bytes(buf)


def write_sstable(path, entries):
    """Uncompressed LevelDB-format table of sorted (key, value) byte pairs."""
    entries = sorted(entries)
    out = bytearray()

    def put(block):
        off = len(out)
        out.extend(block + b'\x00' + struct.pack('<I', io_native.masked_crc32c(block + b'\x00')))
        return pbwire.varint(off) + pbwire.varint(len(block))
    data_h = put(_block_bytes(entries))
    meta_h = put(_block_bytes([]))
    last = entries[-1][0] if entries else b''
    index_h = put(_block_bytes([(last, data_h)]))
    foot = meta_h + index_h
    out.extend(foot + b'\x00' * (40 - len(foot)) + struct.pack('<Q', TABLE_MAGIC))
    with open(path, 'wb') as f:
        f.write(out)


# ---------------------------------------------------------------- tensor bundle

def _parse_entry(v):
    e = {'dtype': 0, 'shape': [], 'shard_id': 0, 'offset': 0, 'size': 0, 'crc32c': None, 'slices': False}
    for fno, _, val in pbwire.iter_fields(v):
        if fno == 1:
            e['dtype'] = val
        elif fno == 2:
            for f2, _, dim in pbwire.iter_fields(val):
                if f2 == 2:
                    size = 0
                    for f3, _, x in pbwire.iter_fields(dim):
                        if f3 == 1:
                            size = pbwire.signed64(x)
                    e['shape'].append(size)
        elif fno == 3:
            e['shard_id'] = val
        elif fno == 4:
            e['offset'] = pbwire.signed64(val)
        elif fno == 5:
            e['size'] = pbwire.signed64(val)
        elif fno == 6:
            e['crc32c'] = val
        elif fno == 7:
            e['slices'] = True
    return e


def read_tf_bundle(prefix, verify=True):
    """{variable name: numpy array} of a TF-1.x checkpoint prefix."""
    rows = read_sstable(prefix + '.index', verify)
    nshards = 1
    out = {}
    entries = []
    for k, v in rows:
        if k == b'':
            for fno, _, val in pbwire.iter_fields(v):
                if fno == 1:
                    nshards = val
                elif fno == 2 and val != 0:
                    raise IOError('big-endian tensor bundles are not supported')
            continue
        entries.append((k.decode(), _parse_entry(v)))
    shards = {}
    for name, e in entries:
        if e['slices']:
            raise IOError('%s: partitioned (sliced) variables are not supported' % name)
        sid = e['shard_id']
        if sid not in shards:
            shards[sid] = open('%s.data-%05d-of-%05d' % (prefix, sid, nshards), 'rb').read()
        raw = shards[sid][e['offset']:e['offset'] + e['size']]
        if len(raw) != e['size']:
            raise IOError('%s: data shard truncated' % name)
        if verify and e['crc32c'] is not None:
            c = io_native.crc32c(raw)
            if e['crc32c'] not in (io_native.mask(c), c):
                raise IOError('%s: checksum mismatch' % name)
        if e['dtype'] == DT_BFLOAT16:
            a = (np.frombuffer(raw, '<u2').astype(np.uint32) << 16).view(np.float32)
        elif e['dtype'] in _DT:
            a = np.frombuffer(raw, np.dtype(_DT[e['dtype']]).newbyteorder('<'))
        else:
            raise IOError('%s: unsupported dtype %d' % (name, e['dtype']))
        out[name] = a.reshape(e['shape']).copy()
    return out


def write_tf_bundle(prefix, tensors):
    """Write {name: numpy array} as a single-shard TF-1.x tensor bundle (+ `checkpoint` file)."""
    os.makedirs(os.path.dirname(prefix) or '.', exist_ok=True)
    data = bytearray()
    rows = [(b'', pbwire.f_varint(1, 1) + pbwire.f_varint(2, 0) + pbwire.f_bytes(3, pbwire.f_varint(1, 1)))]
    for name in sorted(tensors):
        a = np.array(tensors[name], order="C")   # (ascontiguousarray would make a 0-d value 1-d)
        if a.dtype not in _DT_INV:
            raise TypeError('%s: dtype %s' % (name, a.dtype))
        raw = a.astype(a.dtype.newbyteorder('<')).tobytes()
        shape = b''.join(pbwire.f_bytes(2, pbwire.f_varint(1, int(d))) for d in a.shape)
        ent = (pbwire.f_varint(1, _DT_INV[a.dtype]) + pbwire.f_bytes(2, shape) + pbwire.f_varint(4, len(data)) +
               pbwire.f_varint(5, len(raw)) + pbwire.f_fixed32(6, io_native.mask(io_native.crc32c(raw))))
        rows.append((name.encode(), ent))
        data += raw
    with open(prefix + '.data-00000-of-00001', 'wb') as f:
        f.write(data)
    write_sstable(prefix + '.index', rows)
    with open(os.path.join(os.path.dirname(prefix) or '.', 'checkpoint'), 'w') as f:
        base = os.path.basename(prefix)
        f.write('model_checkpoint_path: "%s"\nall_model_checkpoint_paths: "%s"\n' % (base, base))


def tf_latest_checkpoint(directory):
    """tf.train.latest_checkpoint: the prefix named by <directory>/checkpoint, if it exists."""
    p = os.path.join(directory, 'checkpoint')
    if not os.path.exists(p):
        return None
    m = re.search(r'^model_checkpoint_path:\s*"(.*)"\s*$', open(p).read(), re.M)
    if not m:
        return None
    prefix = m.group(1) if os.path.isabs(m.group(1)) else os.path.join(directory, m.group(1))
    return prefix if os.path.exists(prefix + '.index') else None


def is_tf_bundle(path):
    return os.path.exists(path + '.index') and not os.path.isfile(path)


def exists(path):
    return os.path.isfile(path) or is_tf_bundle(path)


# ---------------------------------------------------------------- ParamStore <-> formats

def tf_to_store_layout(name, a, shape):
    """A TF variable value in this framework's layout for parameter `name` of `shape`."""
    a = np.asarray(a)
    if a.ndim == 4 and name.endswith('depthwise_weights') and len(shape) == 3:
        a = a.reshape(a.shape[:3])                   # [3, 3, C, 1] -> [3, 3, C]
    elif a.ndim == 4 and name.endswith('/weights'):
        a = a.transpose(3, 0, 1, 2)                  # HWIO -> [Cout, kh, kw, Cin]
    if tuple(a.shape) != tuple(shape):
        raise ValueError('%s: checkpoint shape %s does not match %s' % (name, a.shape, tuple(shape)))
    return np.ascontiguousarray(a, np.float32)


def store_to_tf_layout(name, a):
    a = np.asarray(a)
    if a.ndim == 3 and name.endswith('depthwise_weights'):
        return a[..., None]
    if a.ndim == 4 and name.endswith('/weights'):
        return a.transpose(1, 2, 3, 0)
    return a


def load_variables(store, path, names_regex=None):
    """Restore a ParamStore from a torch checkpoint or a TF tensor bundle; returns global_step.
    names_regex: restore only matching names (the reference's restore_saver filter)."""
    if is_tf_bundle(path):
        tf = read_tf_bundle(path)
        step = int(np.asarray(tf.get('global_step', 0)).reshape(-1)[0]) if 'global_step' in tf else 0
        sd = {}
        for n, t in list(store.params.items()) + list(store.buffers.items()):
            if n in tf:
                sd[n] = torch.from_numpy(tf_to_store_layout(n, tf[n], t.shape))
        store.load_state_dict(sd, strict=names_regex is None, names_regex=names_regex)
        return step
    if not os.path.isfile(path):
        raise FileNotFoundError('checkpoint %r not found' % path)
    sd = torch.load(path, map_location='cpu', weights_only=True)
    store.load_state_dict(sd['variables'], strict=names_regex is None, names_regex=names_regex)
    return int(sd.get('global_step', 0))


def save_variables(store, path, step, fmt='torch'):
    """fmt 'torch' (default, what train.py writes) or 'tf' (a tensor bundle at prefix `path`)."""
    os.makedirs(os.path.dirname(path) or '.', exist_ok=True)
    if fmt == 'tf':
        t = {n: store_to_tf_layout(n, v.numpy()) for n, v in store.state_dict().items()}
        t['global_step'] = np.array(step, np.int64)
        write_tf_bundle(path, t)
        return
    torch.save({'variables': store.state_dict(), 'global_step': step}, path)
