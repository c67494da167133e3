"""Protocol-buffer wire format, just what the readers need (no generated code, no TF).

Used for tf.train.Example records (rod.tfrecord; schema of the reference's
dataset/pascalvoc_common.py:75-88) and for the BundleHeaderProto / BundleEntryProto values
of TF tensor bundles (rod.checkpoint).  Wire types: 0 varint, 1 fixed64, 2 length-delimited,
5 fixed32.
"""
from __future__ import annotations

import struct

VARINT, FIXED64, LEN, FIXED32 = 0, 1, 2, 5


def read_varint(buf, pos):
    result = shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError('varint too long')


def signed64(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def iter_fields(buf):
    """Yield (field number, wire type, value): int for varint / fixed, memoryview for LEN."""
    mv = memoryview(buf)
    pos, end = 0, len(mv)
    while pos < end:
        key, pos = read_varint(mv, pos)
        fno, wt = key >> 3, key & 7
        if wt == VARINT:
            v, pos = read_varint(mv, pos)
        elif wt == FIXED64:
            v = struct.unpack_from('<Q', mv, pos)[0]
            pos += 8
        elif wt == FIXED32:
            v = struct.unpack_from('<I', mv, pos)[0]
            pos += 4
        elif wt == LEN:
            n, pos = read_varint(mv, pos)
            if pos + n > end:
                raise ValueError('truncated length-delimited field')
            v = mv[pos:pos + n]
            pos += n
        else:
            raise ValueError('unsupported wire type %d' % wt)
        yield fno, wt, v


def varint(v):
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def key(fno, wt):
    return varint((fno << 3) | wt)


def f_varint(fno, v):
    return key(fno, VARINT) + varint(v)


def f_bytes(fno, b):
    b = bytes(b)
    return key(fno, LEN) + varint(len(b)) + b


def f_fixed32(fno, v):
    return key(fno, FIXED32) + struct.pack('<I', v)
