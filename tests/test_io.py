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
