"""CPU: host-side guards of the data and parameter plumbing.

  * rodio_tfrecord_scan rejects a record whose (checksum-valid) length runs past the end of
    the file, with an error instead of an allocation abort;
  * TFRecordSource under data parallel: every rank reads a disjoint slice of one shared
    shuffle, so one global batch never holds the same record twice (the reference reads the
    data set on one device, dataset/pascalvoc_common.py:40-107);
  * the dropout seed differs per rank (ops.dropout);
  * ParamStore.eval_views serves a BatchNorm's eval slices only for buffers that really are
    views of the flat moving-statistics buffer.
"""
import struct

import numpy as np
import pytest
import torch

from rod import io_native, ops
from rod.params import ParamStore


def _record(payload):
    ln = struct.pack('<Q', len(payload))
    return ln + struct.pack('<I', io_native.masked_crc32c(ln)) + payload + \
        struct.pack('<I', io_native.masked_crc32c(payload))


def test_tfrecord_scan_rejects_length_past_eof(tmp_path):
    good = _record(b'abc') + _record(b'hello world')
    p = tmp_path / 'ok.tfrecord'
    p.write_bytes(good)
    off, ln = io_native.tfrecord_scan(str(p))
    assert list(ln) == [3, 11] and list(off) == [12, 12 + 3 + 4 + 12]
    # a header whose length CRC is valid but whose length (2^62) exceeds the file
    huge = struct.pack('<Q', 1 << 62)
    bad = good + huge + struct.pack('<I', io_native.masked_crc32c(huge)) + b'xy'
    q = tmp_path / 'bad.tfrecord'
    q.write_bytes(bad)
    for verify in (True, False):
        with pytest.raises(Exception, match='past the end'):
            io_native.tfrecord_scan(str(q), verify_data=verify)
    # a length that fits the payload but leaves no room for the footer CRC
    short = _record(b'abcdef')[:-2]
    r = tmp_path / 'short.tfrecord'
    r.write_bytes(short)
    with pytest.raises(Exception):
        io_native.tfrecord_scan(str(r))


def test_tfrecord_source_ranks_read_disjoint_slices(golden_dir):
    import os
    from rod.dataio import TFRecordSource, tfrecord_files
    files = tfrecord_files(os.path.join(golden_dir, 'tfrecord'))
    world = 2
    srcs = [TFRecordSource(files, 1, (32, 32), torch.device('cpu'), torch.float32, train=True, seed=9, rank=r,
                           world=world, prefetch=False) for r in range(world)]
    n = len(srcs[0].index)
    assert len(srcs[0]) == n // world   # records this rank reads per epoch
    for epoch in range(3):
        orders = [s.order.tolist() for s in srcs]
        assert all(len(o) == n // world for o in orders)
        assert not set(orders[0]) & set(orders[1])
        assert sorted(orders[0] + orders[1]) == sorted(set(orders[0] + orders[1]))
        for s in srcs:                       # next epoch: same shared reshuffle on every rank
            s.pos = len(s.order)
            s._take()
    one = TFRecordSource(files, 1, (32, 32), torch.device('cpu'), torch.float32, train=True, seed=9)
    assert len(one.order) == n and sorted(one.order.tolist()) == list(range(n))


def test_dropout_seed_differs_per_rank(monkeypatch):
    seeds = []

    class _Rec(object):
        @staticmethod
        def apply(x, keep, seed):
            seeds.append(seed)
            return x, None
    monkeypatch.setattr(ops, '_Dropout', _Rec)
    x = torch.zeros(4)
    old = list(ops.DROPOUT_RANK)
    try:
        for rank in range(2):
            ops.DROPOUT_RANK[:] = [rank, 2]
            ops._DROPOUT_CALLS[0] = 0
            ops.dropout(x, 0.5, True)
            ops.dropout(x, 0.5, True)
    finally:
        ops.DROPOUT_RANK[:] = old
    assert len(set(seeds)) == 4, seeds


def test_eval_views_checks_buffer_bounds():
    st = ParamStore()
    st.add_buffer('a/moving_mean', np.zeros(3, np.float32))
    st.add_buffer('a/moving_variance', np.ones(3, np.float32))
    st.add_buffer('b/moving_mean', np.zeros(5, np.float32))
    st.add_buffer('b/moving_variance', np.ones(5, np.float32))
    st.finalize('cpu')
    st._eval_eps = 1e-3          # as after eval_refresh (no kernel launch needed for the views)
    st._eval_out = torch.arange(2 * 16, dtype=torch.float32).view(2, 16)
    m, v = st.eval_views(st.buffers['b/moving_mean'], st.buffers['b/moving_variance'], 1e-3)
    assert m.tolist() == list(range(6, 11)) and v.tolist() == list(range(16 + 11, 16 + 16))
    # a rebound buffer (not a view of flat_buf) falls back to the per-BatchNorm path
    st.buffers['b/moving_mean'] = torch.zeros(5)
    assert st.eval_views(st.buffers['b/moving_mean'], st.buffers['b/moving_variance'], 1e-3) is None
    # a view that runs past the end of flat_buf, or another eps, also falls back
    assert st.eval_views(st.flat_buf[14:16], st.flat_buf[14:16], 1e-3) is not None
    assert st.eval_views(st.flat_buf[10:16], st.flat_buf[14:16], 1e-3) is None
    assert st.eval_views(st.buffers['a/moving_mean'], st.buffers['a/moving_variance'], 1e-5) is None
    # load_state_dict updates in place: the views stay valid
    sd = st.state_dict()
    sd['b/moving_mean'] = torch.ones(5)
    st.buffers['b/moving_mean'] = st.flat_buf[6:11]
    st.load_state_dict(sd)
    assert st.eval_views(st.buffers['b/moving_mean'], st.buffers['b/moving_variance'], 1e-3) is not None
    assert st.flat_buf[6:11].tolist() == [1.0] * 5


def test_bn_parts_handoff_rejects_summed_gradient():
    """The BatchNorm-sum hand-off from the fused depthwise backward to its producer (ops._BN_PARTS)
    is taken only for the very gradient it was formed from: not after an in-place sum into it
    (a second consumer of the depthwise input), not for another tensor of the same shape."""
    dx = torch.zeros(4, 8)
    parts = torch.ones(2, 2, 8)
    ops._put_bn_parts(dx, parts)
    assert ops._take_bn_parts(dx) is parts
    ops._put_bn_parts(dx, parts)
    dx.add_(torch.ones(4, 8))            # autograd accumulating a second branch in place
    assert ops._take_bn_parts(dx) is None
    ops._put_bn_parts(dx, parts)
    other = torch.zeros(4, 8)            # same shape, different storage (an out-of-place sum)
    assert ops._take_bn_parts(other) is None
    ops._put_bn_parts(dx, parts)
    assert ops._take_bn_parts(dx.view(4, 8)) is parts   # a view of the same, unchanged storage
    ops.clear_bn_parts()
