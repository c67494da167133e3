"""Host I/O (CPU): CRC32C, TFRecord framing, tf.train.Example wire format, the committed
BDD100K-schema fixture, and TF-1.x tensor bundles (rod.checkpoint).

Pinning: CRC32C against the RFC 3720 (iSCSI) test vectors; the Example encoder / decoder
against google.protobuf's own serializer on a descriptor of tensorflow/core/example/
{example,feature}.proto built at run time; the fixture against the annotations and the
pixels recorded when it was written (tests/golden/make_tfrecord.py)."""
import os
import struct

import numpy as np
import pytest
import torch

from rod import io_native, tfrecord

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'tfrecord')


def test_crc32c_rfc3720_vectors():
    assert io_native.crc32c(b'123456789') == 0xE3069283
    assert io_native.crc32c(bytes(32)) == 0x8A9136AA
    assert io_native.crc32c(b'\xff' * 32) == 0x62A8AB43
    assert io_native.crc32c(bytes(range(32))) == 0x46DD794E
    assert io_native.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    data = os.urandom(1000)
    assert io_native.crc32c(data[600:], io_native.crc32c(data[:600])) == io_native.crc32c(data)
    c = io_native.crc32c(b'abc')
    assert io_native.unmask(io_native.mask(c)) == c
    assert io_native.masked_crc32c(b'abc') == io_native.mask(c)


def test_librodio_exports_header():
    L = io_native.lib()
    for name in io_native.exported_symbols():
        assert hasattr(L, name), name
    assert L.rodio_abi_version() == 1


def test_tfrecord_roundtrip_and_corruption(tmp_path):
    p = str(tmp_path / 'x.tfrecord')
    payloads = [b'', b'a', os.urandom(5000), b'xyz' * 77]
    with tfrecord.TFRecordWriter(p) as w:
        for pl in payloads:
            w.write(pl)
    f = tfrecord.TFRecordFile(p)
    assert [bytes(r) for r in f] == payloads
    f.close()
    raw = bytearray(open(p, 'rb').read())
    # framing of record 0: uint64 length 0, masked crc of the 8 length bytes, masked crc of b''
    assert raw[:8] == bytes(8)
    assert struct.unpack('<I', raw[8:12])[0] == io_native.masked_crc32c(bytes(8))
    assert struct.unpack('<I', raw[12:16])[0] == io_native.masked_crc32c(b'')
    bad = bytearray(raw)
    bad[100] ^= 1                               # inside record 2's payload (starts at 45)
    q = str(tmp_path / 'bad.tfrecord')
    open(q, 'wb').write(bad)
    with pytest.raises(IOError, match='corrupted record data'):
        tfrecord.TFRecordFile(q)
    assert len(tfrecord.TFRecordFile(q, verify=False)) == 4    # lengths still intact
    open(q, 'wb').write(raw[:-3])
    with pytest.raises(IOError, match='truncated'):
        tfrecord.TFRecordFile(q)


def _example_classes():
    """tf.train.Example & co. built from a runtime FileDescriptorProto (field numbers of
    tensorflow/core/example/feature.proto and example.proto)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name='rod_test_example.proto', package='tfx', syntax='proto3')
    F = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
        return m
    rep, opt = F.LABEL_REPEATED, F.LABEL_OPTIONAL
    msg('BytesList', [('value', 1, F.TYPE_BYTES, rep, None)])
    msg('FloatList', [('value', 1, F.TYPE_FLOAT, rep, None)])
    msg('Int64List', [('value', 1, F.TYPE_INT64, rep, None)])
    feat = msg('Feature', [('bytes_list', 1, F.TYPE_MESSAGE, opt, '.tfx.BytesList'),
                           ('float_list', 2, F.TYPE_MESSAGE, opt, '.tfx.FloatList'),
                           ('int64_list', 3, F.TYPE_MESSAGE, opt, '.tfx.Int64List')])
    feat.oneof_decl.add(name='kind')
    for f in feat.field:
        f.oneof_index = 0
    feats = msg('Features', [('feature', 1, F.TYPE_MESSAGE, rep, '.tfx.Features.FeatureEntry')])
    ent = feats.nested_type.add(name='FeatureEntry')
    ent.field.add(name='key', number=1, type=F.TYPE_STRING, label=opt)
    ent.field.add(name='value', number=2, type=F.TYPE_MESSAGE, label=opt, type_name='.tfx.Feature')
    ent.options.map_entry = True
    msg('Example', [('features', 1, F.TYPE_MESSAGE, opt, '.tfx.Features')])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName('tfx.Example'))


def test_example_wire_format_against_protobuf():
    Example = _example_classes()
    feats = {'image/encoded': ('bytes', [b'\xff\xd8jpegbytes', b'']), 'f': ('float', [0.5, -1.25, 3e-8]),
             'i': ('int64', [0, 1, -7, 2 ** 40]), 'empty': ('float', [])}
    mine = tfrecord.encode_example(feats)
    ex = Example()
    ex.ParseFromString(mine)                      # protobuf accepts our bytes ...
    fm = ex.features.feature
    assert list(fm['image/encoded'].bytes_list.value) == feats['image/encoded'][1]
    assert list(fm['f'].float_list.value) == list(np.float32(feats['f'][1]))
    assert list(fm['i'].int64_list.value) == feats['i'][1]
    # ... and we decode protobuf's own serialization (packed lists, any map order)
    got = tfrecord.decode_example(ex.SerializeToString())
    assert got['image/encoded'] == feats['image/encoded']
    assert got['f'] == ('float', list(np.float32(feats['f'][1])))
    assert got['i'] == feats['i']
    # unpacked repeated scalars (legacy writers) decode too
    from rod import pbwire
    lst = b''.join(pbwire.f_varint(1, v) for v in (3, 4))
    raw = pbwire.f_bytes(1, pbwire.f_bytes(1, pbwire.f_bytes(1, b'k') + pbwire.f_bytes(2, pbwire.f_bytes(3, lst))))
    assert tfrecord.decode_example(raw)['k'] == ('int64', [3, 4])


def test_bdd_fixture_decodes():
    exp = np.load(os.path.join(GOLD, 'expected.npz'))
    f = tfrecord.TFRecordFile(os.path.join(GOLD, 'bdd100k_train_000.tfrecord'))
    assert len(f) == int(exp['n'])
    for i, rec in enumerate(f):
        enc, fmt, shape, boxes, labels, dif, tru = tfrecord.decode_detection_example(rec)
        assert fmt == b'JPEG' and list(shape) == [*exp['image_%d' % i].shape]
        np.testing.assert_array_equal(boxes, exp['boxes_%d' % i])
        np.testing.assert_array_equal(labels, exp['labels_%d' % i])
        assert (dif == 0).all() and (tru == 0).all() and len(dif) == len(labels)
        np.testing.assert_array_equal(tfrecord.decode_image(enc, fmt), exp['image_%d' % i])


def test_make_source_requires_data_or_synthetic(tmp_path):
    from rod.dataio import make_source
    with pytest.raises(FileNotFoundError, match='--synthetic'):
        make_source(str(tmp_path), 2, (64, 64), 'cpu')


# ---------------------------------------------------------------- tensor bundles

def test_sstable_roundtrip_and_snappy(tmp_path):
    from rod import checkpoint as ck
    rows = [(b'', b'hdr'), (b'a/b', b'1' * 10)] + [(b'k%03d' % i, os.urandom(i)) for i in range(40)]
    p = str(tmp_path / 't.index')
    ck.write_sstable(p, rows)
    assert ck.read_sstable(p) == sorted(rows)
    raw = bytearray(open(p, 'rb').read())
    raw[20] ^= 0x40
    open(p, 'wb').write(raw)
    with pytest.raises(IOError, match='checksum'):
        ck.read_sstable(p)
    # snappy: literal "abcd" + copy(offset 4, len 8) -> "abcdabcdabcd"
    comp = bytes([12, (4 - 1) << 2]) + b'abcd' + bytes([((8 - 4) << 2) | 1, 4])
    assert ck._snappy_decompress(comp) == b'abcdabcdabcd'


def test_tf_bundle_roundtrip_into_store(tmp_path):
    import config
    from nets.catch_net import CatchNet
    from rod import checkpoint as ck
    cfg = {'train_range': config.train_range.REFINE, 'process_backbone_method': config.process_backbone_method.NONE,
           'deconv_method': config.deconv_method.LEARN_HALF, 'merge_method': config.merge_method.ADD}
    a = CatchNet('mobilenet_v2', cfg, 'cpu', seed=1)
    b = CatchNet('mobilenet_v2', cfg, 'cpu', seed=2)
    prefix = str(tmp_path / 'refine' / 'mobilenet_v2.model')
    ck.save_variables(a.store, prefix, 123, fmt='tf')
    tf = ck.read_tf_bundle(prefix)
    w = tf['backbone/MobilenetV2/expanded_conv_1/expand/weights']
    assert w.shape == (1, 1, 16, 96)                                         # TF HWIO
    assert tf['backbone/MobilenetV2/expanded_conv/depthwise/depthwise_weights'].shape == (3, 3, 32, 1)
    assert int(tf['global_step']) == 123
    assert ck.exists(prefix) and ck.tf_latest_checkpoint(str(tmp_path / 'refine')) == prefix
    step = ck.load_variables(b.store, prefix)
    assert step == 123
    for n, p in a.store.params.items():
        assert torch.equal(p.detach(), b.store.params[n].detach()), n
    # partial restore (restore_saver of backbone.+|refine.+, train.py:155-158): others untouched
    c = CatchNet('mobilenet_v2', cfg, 'cpu', seed=3)
    before = c.store.params['refine/block_1/Conv/weights'].detach().clone()
    ck.load_variables(c.store, prefix, names_regex=r'backbone.+')
    assert torch.equal(c.store.params['backbone/MobilenetV2/Conv/weights'], a.store.params['backbone/MobilenetV2/Conv/weights'])
    assert torch.equal(c.store.params['refine/block_1/Conv/weights'].detach(), before)
    # a corrupted data shard is detected by the entry checksum
    d = prefix + '.data-00000-of-00001'
    raw = bytearray(open(d, 'rb').read())
    raw[100] ^= 1
    open(d, 'wb').write(raw)
    with pytest.raises(IOError, match='checksum'):
        ck.read_tf_bundle(prefix)


# ---------------------------------------------------------------- F2: tensor-bundle layout vs TF's protos

def _crc32c_py(data, crc=0):
    """Bitwise CRC32C (Castagnoli, reflected 0x82F63B78): independent of librodio."""
    crc ^= 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 & -(crc & 1))
    return crc ^ 0xFFFFFFFF


def _mask_py(c):   # tensorflow/core/lib/hash/crc32c.h Mask()
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xa282ead8) & 0xFFFFFFFF


def _leveldb_rows(raw):
    """Minimal reader of the LevelDB table format as published (table_format.md, which TF's
    tensorflow/core/lib/io/table follows): 48-byte footer (metaindex + index BlockHandles,
    zero padding, magic 0xdb4775248b80fb57 LE), blocks of prefix-compressed entries with a
    restart array, each block followed by a type byte and the masked CRC32C of block + type."""
    def varint(b, p):
        v = s = 0
        while True:
            x = b[p]
            p += 1
            v |= (x & 0x7F) << s
            s += 7
            if x < 0x80:
                return v, p

    def block(off, size):
        blk, typ = raw[off:off + size], raw[off + size]
        assert typ == 0, 'compressed block'
        assert struct.unpack_from('<I', raw, off + size + 1)[0] == _mask_py(_crc32c_py(raw[off:off + size + 1]))
        n = struct.unpack_from('<I', blk, len(blk) - 4)[0]
        end, p, key, rows = len(blk) - 4 - 4 * n, 0, b'', []
        while p < end:
            sh, p = varint(blk, p)
            ns, p = varint(blk, p)
            vl, p = varint(blk, p)
            key = key[:sh] + blk[p:p + ns]
            p += ns
            rows.append((key, blk[p:p + vl]))
            p += vl
        return rows
    foot = raw[-48:]
    assert struct.unpack_from('<Q', foot, 40)[0] == 0xdb4775248b80fb57
    _, p = varint(foot, 0)
    _, p = varint(foot, p)
    io_, p = varint(foot, p)
    isz, p = varint(foot, p)
    rows = []
    for _, h in block(io_, isz):
        o, q = varint(h, 0)
        sz, _ = varint(h, q)
        rows += block(o, sz)
    return rows


def _bundle_classes():
    """BundleHeaderProto / BundleEntryProto (tensorflow/core/protobuf/tensor_bundle.proto) with
    VersionDef (framework/versions.proto), TensorShapeProto (tensor_shape.proto),
    TensorSliceProto (tensor_slice.proto) and DataType (types.proto), from field numbers."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    fd = descriptor_pb2.FileDescriptorProto(name='rod_test_bundle.proto', package='tfb', syntax='proto3')
    F = descriptor_pb2.FieldDescriptorProto
    rep, opt = F.LABEL_REPEATED, F.LABEL_OPTIONAL
    dt = fd.enum_type.add(name='DataType')
    for n, v in [('DT_INVALID', 0), ('DT_FLOAT', 1), ('DT_DOUBLE', 2), ('DT_INT32', 3), ('DT_UINT8', 4),
                 ('DT_INT16', 5), ('DT_INT8', 6), ('DT_STRING', 7), ('DT_INT64', 9), ('DT_BOOL', 10),
                 ('DT_BFLOAT16', 14), ('DT_HALF', 19)]:
        dt.value.add(name=n, number=v)

    def msg(parent, name, fields):
        m = parent.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
        return m
    msg(fd.message_type, 'VersionDef', [('producer', 1, F.TYPE_INT32, opt, None),
                                        ('min_consumer', 2, F.TYPE_INT32, opt, None),
                                        ('bad_consumers', 3, F.TYPE_INT32, rep, None)])
    shp = msg(fd.message_type, 'TensorShapeProto', [('dim', 2, F.TYPE_MESSAGE, rep, '.tfb.TensorShapeProto.Dim'),
                                                    ('unknown_rank', 3, F.TYPE_BOOL, opt, None)])
    msg(shp.nested_type, 'Dim', [('size', 1, F.TYPE_INT64, opt, None), ('name', 2, F.TYPE_STRING, opt, None)])
    msg(fd.message_type, 'TensorSliceProto', [])
    hdr = msg(fd.message_type, 'BundleHeaderProto', [('num_shards', 1, F.TYPE_INT32, opt, None),
                                                     ('endianness', 2, F.TYPE_ENUM, opt,
                                                      '.tfb.BundleHeaderProto.Endianness'),
                                                     ('version', 3, F.TYPE_MESSAGE, opt, '.tfb.VersionDef')])
    en = hdr.enum_type.add(name='Endianness')
    en.value.add(name='LITTLE', number=0)
    en.value.add(name='BIG', number=1)
    msg(fd.message_type, 'BundleEntryProto', [('dtype', 1, F.TYPE_ENUM, opt, '.tfb.DataType'),
                                              ('shape', 2, F.TYPE_MESSAGE, opt, '.tfb.TensorShapeProto'),
                                              ('shard_id', 3, F.TYPE_INT32, opt, None),
                                              ('offset', 4, F.TYPE_INT64, opt, None),
                                              ('size', 5, F.TYPE_INT64, opt, None),
                                              ('crc32c', 6, F.TYPE_FIXED32, opt, None),
                                              ('slices', 7, F.TYPE_MESSAGE, rep, '.tfb.TensorSliceProto')])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName('tfb.' + n))
    return get('BundleHeaderProto'), get('BundleEntryProto')


_BUNDLE = {'global_step': np.array(77, np.int64),
           'backbone/MobilenetV2/Conv/weights': np.arange(3 * 3 * 3 * 4, dtype=np.float32).reshape(3, 3, 3, 4) / 7,
           'refine/block_1/Conv/biases': np.array([-1.5, 0.25, 3e-8], np.float32),
           'deconv/block_2/weight_1': np.linspace(-1, 1, 2 * 2 * 5 * 6).astype(np.float32).reshape(2, 2, 5, 6),
           'counts': np.array([[1, -2], [3, 2 ** 40]], np.int64), 'flags': np.array([True, False, True])}


def test_tf_bundle_layout_against_tf_protos(tmp_path):
    """F2 (ref train.py:155-158, 191-193, 278-283 — tf.train.Saver bundles).  What
    rod.checkpoint writes is read back with an independent LevelDB-table reader and TF's own
    message layouts (protobuf from descriptors): header (1 shard, little endian, version
    producer 1), one BundleEntryProto per variable in key order (dtype enum, shape dims,
    shard 0, back-to-back offsets / sizes into .data-00000-of-00001, masked CRC32C of the
    bytes); and a bundle whose index values protobuf itself serialised reads back through
    rod.checkpoint.read_tf_bundle."""
    from rod import checkpoint as ck
    Header, Entry = _bundle_classes()
    prefix = str(tmp_path / 'a' / 'model')
    ck.write_tf_bundle(prefix, _BUNDLE)
    rows = _leveldb_rows(open(prefix + '.index', 'rb').read())
    assert [k for k, _ in rows] == [b''] + sorted(k.encode() for k in _BUNDLE)
    h = Header()
    h.ParseFromString(rows[0][1])
    assert h.num_shards == 1 and h.endianness == 0 and h.version.producer == 1
    data = open(prefix + '.data-00000-of-00001', 'rb').read()
    dtnum = {np.dtype(np.float32): 1, np.dtype(np.int64): 9, np.dtype(np.bool_): 10}
    pos = 0
    for k, v in rows[1:]:
        e = Entry()
        e.ParseFromString(v)
        a = _BUNDLE[k.decode()]
        assert e.dtype == dtnum[a.dtype] and [d.size for d in e.shape.dim] == list(a.shape)
        assert e.shard_id == 0 and e.offset == pos and e.size == a.nbytes and not e.slices
        raw = data[e.offset:e.offset + e.size]
        assert raw == a.astype(a.dtype.newbyteorder('<')).tobytes()
        assert e.crc32c == _mask_py(_crc32c_py(raw))
        pos += e.size
    assert pos == len(data)
    # the other direction: index values serialised by protobuf (field order, defaults and
    # encodings of its choosing) in a table, read by rod.checkpoint
    q = str(tmp_path / 'b' / 'model')
    os.makedirs(os.path.dirname(q))
    h2 = Header(num_shards=1)
    h2.version.producer = 1
    rows2, blob = [(b'', h2.SerializeToString())], bytearray()
    for name in sorted(_BUNDLE):
        a = _BUNDLE[name]
        raw = a.astype(a.dtype.newbyteorder('<')).tobytes()
        e = Entry(dtype=dtnum[a.dtype], offset=len(blob), size=len(raw), crc32c=_mask_py(_crc32c_py(raw)))
        for d in a.shape:
            e.shape.dim.add(size=d)
        rows2.append((name.encode(), e.SerializeToString()))
        blob += raw
    open(q + '.data-00000-of-00001', 'wb').write(bytes(blob))
    ck.write_sstable(q + '.index', rows2)
    got = ck.read_tf_bundle(q)
    assert set(got) == set(_BUNDLE)
    for k, a in _BUNDLE.items():
        np.testing.assert_array_equal(got[k], a)
        assert got[k].shape == a.shape
