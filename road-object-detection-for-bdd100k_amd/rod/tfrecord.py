"""TFRecord files of tf.train.Example protos — the reference's on-disk dataset format.

The reference writes BDD100K / VOC as TFRecords (dataset/pascalvoc_to_tfrecords.py:131-160,
files `bdd100k_train_*.tfrecord`, dataset/bdd100k.py:9) and reads them with slim's
TFExampleDecoder over the schema of dataset/pascalvoc_common.py:75-88:

  image/encoded (bytes, JPEG)   image/format (bytes)   image/height|width|channels (int64)
  image/shape (int64 [3])       image/object/bbox/{xmin,ymin,xmax,ymax} (float, per box)
  image/object/bbox/label|difficult|truncated (int64, per box)   [+ label_text (bytes)]

Framing (tensorflow/core/lib/io/record_writer.cc): uint64 length, masked CRC32C of the
length, payload, masked CRC32C of the payload.  The scan and the checksums are native
(librodio, rod.io_native); the Example protos are decoded here from the wire format.
"""
from __future__ import annotations

import mmap
import os
import struct

import numpy as np

from . import io_native, pbwire

# ---------------------------------------------------------------- framing


class TFRecordFile:
    """Random access to the records of one file (memory-mapped; offsets from the native scan,
    every checksum verified once when opened unless verify=False)."""

    def __init__(self, path, verify=True):
        self.path = path
        self.offsets, self.lengths = io_native.tfrecord_scan(path, verify_data=verify)
        self._f = open(path, 'rb')
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ) if os.path.getsize(path) else b''

    def __len__(self):
        return len(self.offsets)

    def __getitem__(self, i):
        o, n = int(self.offsets[i]), int(self.lengths[i])
        return memoryview(self._mm)[o:o + n]

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]

    def close(self):
        if isinstance(self._mm, mmap.mmap):
            self._mm.close()
        self._f.close()


class TFRecordWriter:
    """tf.python_io.TFRecordWriter (uncompressed)."""

    def __init__(self, path):
        self._f = open(path, 'wb')

    def write(self, payload):
        payload = bytes(payload)
        head = struct.pack('<Q', len(payload))
        self._f.write(head + struct.pack('<I', io_native.masked_crc32c(head)))
        self._f.write(payload + struct.pack('<I', io_native.masked_crc32c(payload)))

    def close(self):
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ---------------------------------------------------------------- tf.train.Example

def _decode_list(kind, mv):
    """Values of a BytesList (1) / FloatList (2) / Int64List (3), packed or not."""
    out = []
    for fno, wt, v in pbwire.iter_fields(mv):
        if fno != 1:
            continue
        if kind == 1:
            out.append(bytes(v))
        elif kind == 2:
            if wt == pbwire.LEN:
                out.extend(np.frombuffer(v, '<f4').tolist())
            else:
                out.append(struct.unpack('<f', struct.pack('<I', v))[0])
        else:
            if wt == pbwire.LEN:
                pos, n = 0, len(v)
                while pos < n:
                    x, pos = pbwire.read_varint(v, pos)
                    out.append(pbwire.signed64(x))
            else:
                out.append(pbwire.signed64(v))
    return out


def decode_example(payload):
    """{feature name: ('bytes'|'float'|'int64', [values])} of a serialized tf.train.Example."""
    feats = {}
    for fno, _, ex in pbwire.iter_fields(payload):
        if fno != 1:                      # Example.features
            continue
        for f2, _, entry in pbwire.iter_fields(ex):
            if f2 != 1:                   # Features.feature (map entry)
                continue
            name, feature = None, None
            for f3, _, v in pbwire.iter_fields(entry):
                if f3 == 1:
                    name = bytes(v).decode()
                elif f3 == 2:
                    feature = v
            kind, vals = None, []
            if feature is not None:
                for f4, _, lst in pbwire.iter_fields(feature):
                    kind = f4
                    vals = _decode_list(f4, lst)
            feats[name] = ({1: 'bytes', 2: 'float', 3: 'int64'}.get(kind, 'bytes'), vals)
    return feats


def encode_example(features):
    """Serialize {name: ('bytes'|'float'|'int64', values)} as a tf.train.Example
    (packed float / int64 lists, as TF's Python API writes them)."""
    body = b''
    for name, (kind, vals) in features.items():
        if kind == 'bytes':
            lst = b''.join(pbwire.f_bytes(1, v) for v in vals)
            feat = pbwire.f_bytes(1, lst)
        elif kind == 'float':
            lst = pbwire.f_bytes(1, np.asarray(vals, '<f4').tobytes()) if len(vals) else b''
            feat = pbwire.f_bytes(2, lst)
        elif kind == 'int64':
            lst = pbwire.f_bytes(1, b''.join(pbwire.varint(int(v)) for v in vals)) if len(vals) else b''
            feat = pbwire.f_bytes(3, lst)
        else:
            raise ValueError(kind)
        body += pbwire.f_bytes(1, pbwire.f_bytes(1, name.encode()) + pbwire.f_bytes(2, feat))
    return pbwire.f_bytes(1, body)


# ---------------------------------------------------------------- the detection schema

def _first(feats, name, default=None):
    kind, vals = feats.get(name, (None, []))
    return vals[0] if vals else default


def decode_detection_example(payload):
    """slim TFExampleDecoder with the items of pascalvoc_common.py:89-98: (encoded image bytes,
    format, shape [3], boxes [G, 4] (ymin, xmin, ymax, xmax) float32, labels [G] int64,
    difficult [G], truncated [G])."""
    f = decode_example(payload)
    enc = _first(f, 'image/encoded', b'')
    fmt = _first(f, 'image/format', b'jpeg')
    shape = np.asarray(f.get('image/shape', ('int64', []))[1], np.int64)
    coords = [np.asarray(f.get('image/object/bbox/' + k, ('float', []))[1], np.float32)
              for k in ('ymin', 'xmin', 'ymax', 'xmax')]
    G = min(len(c) for c in coords)
    boxes = np.stack([c[:G] for c in coords], -1) if G else np.zeros((0, 4), np.float32)
    lab = np.asarray(f.get('image/object/bbox/label', ('int64', []))[1], np.int64)
    dif = np.asarray(f.get('image/object/bbox/difficult', ('int64', []))[1], np.int64)
    tru = np.asarray(f.get('image/object/bbox/truncated', ('int64', []))[1], np.int64)
    return enc, fmt, shape, boxes, lab, dif, tru


def encode_detection_example(image_bytes, shape, boxes, labels, labels_text=None, difficult=None, truncated=None,
                             fmt=b'JPEG'):
    """_convert_to_example of dataset/pascalvoc_to_tfrecords.py:131-171 (boxes [G, 4] as
    (ymin, xmin, ymax, xmax) normalised)."""
    boxes = np.asarray(boxes, np.float32).reshape(-1, 4)
    G = boxes.shape[0]
    labels = [int(v) for v in labels]
    feats = {
        'image/height': ('int64', [int(shape[0])]),
        'image/width': ('int64', [int(shape[1])]),
        'image/channels': ('int64', [int(shape[2])]),
        'image/shape': ('int64', [int(s) for s in shape]),
        'image/object/bbox/xmin': ('float', boxes[:, 1].tolist()),
        'image/object/bbox/xmax': ('float', boxes[:, 3].tolist()),
        'image/object/bbox/ymin': ('float', boxes[:, 0].tolist()),
        'image/object/bbox/ymax': ('float', boxes[:, 2].tolist()),
        'image/object/bbox/label': ('int64', labels),
        'image/object/bbox/label_text': ('bytes', list(labels_text) if labels_text is not None else
                                         [b''] * G),
        'image/object/bbox/difficult': ('int64', list(difficult) if difficult is not None else [0] * G),
        'image/object/bbox/truncated': ('int64', list(truncated) if truncated is not None else [0] * G),
        'image/format': ('bytes', [fmt]),
        'image/encoded': ('bytes', [bytes(image_bytes)]),
    }
    return encode_example(feats)


def decode_image(data, fmt=b'jpeg'):
    """tf.image.decode_jpeg / decode_png (slim tfexample_decoder.Image, 3 channels) -> uint8
    [H, W, 3].  PIL (libjpeg, ISLOW DCT, fancy upsampling — TF's defaults)."""
    import io
    from PIL import Image
    with Image.open(io.BytesIO(bytes(data))) as im:
        return np.asarray(im.convert('RGB'), dtype=np.uint8)
