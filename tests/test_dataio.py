"""Host half of the TFRecord training source (CPU): fixed box padding for graph replay, the
prefetching thread's batch sequence, and the evaluation order (no sharding, no drops)."""
import os

import numpy as np
import torch

from rod import tfrecord
from rod.dataio import GMAX, TFRecordSource, tfrecord_files

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'tfrecord')
CPU = torch.device('cpu')


def _host_batches(src, k):
    if src._ahead is None:
        return [src._host() for _ in range(k)]
    out = []
    for _ in range(k):   # what __next__ does, minus the device half
        fut = src._next_host if src._next_host is not None else src._ahead.submit(src._host)
        out.append(fut.result())
        src._next_host = src._ahead.submit(src._host)
    return out


def test_training_batches_padded_to_fixed_count():
    files = tfrecord_files(GOLD)
    src = TFRecordSource(files, 3, (96, 160), CPU, torch.float32, train=True, seed=5, prefetch=False)
    counts = set()
    for flat, boxes, labels, n, hw, offs, draws, _ in _host_batches(src, 6):
        assert boxes.shape == (3, GMAX, 4) and labels.shape == (3, GMAX)
        counts.add(tuple(n.tolist()))
        for b in range(3):   # zero past the real count
            assert not boxes[b, n[b]:].any() and not labels[b, n[b]:].any()
    assert len(counts) > 1   # real counts differ between batches, the shape does not
    src.close()


def test_prefetch_yields_the_same_sequence():
    files = tfrecord_files(GOLD)
    a = TFRecordSource(files, 3, (96, 160), CPU, torch.float32, train=True, seed=9, prefetch=False)
    b = TFRecordSource(files, 3, (96, 160), CPU, torch.float32, train=True, seed=9, prefetch=True)
    for ha, hb in zip(_host_batches(a, 5), _host_batches(b, 5)):
        assert torch.equal(ha[0], hb[0])
        for x, y in zip(ha[1:6], hb[1:6]):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(ha[6], hb[6]):   # crop / ref / mode / colour draws
            np.testing.assert_array_equal(x, y)
    a.close()
    b.close()


def test_batch_with_more_boxes_pads_to_next_multiple(tmp_path):
    import io
    from PIL import Image
    path = str(tmp_path / 'bdd100k_train_000.tfrecord')
    rng = np.random.default_rng(0)
    buf = io.BytesIO()
    Image.fromarray(rng.integers(0, 256, (40, 64, 3), dtype=np.uint8)).save(buf, format='JPEG')
    with tfrecord.TFRecordWriter(path) as w:
        for g in (3, 70):
            c = np.sort(rng.uniform(0.05, 0.95, (g, 2, 2)), axis=1).reshape(g, 4)[:, [0, 2, 1, 3]].astype(np.float32)
            w.write(tfrecord.encode_detection_example(buf.getvalue(), (40, 64, 3), c, np.ones(g, np.int64)))
    src = TFRecordSource([path], 2, (32, 48), CPU, torch.float32, train=True, seed=1, prefetch=False)
    _, boxes, labels, n, _, _, _, _ = src._host()
    assert sorted(n.tolist()) == [3, 70] and boxes.shape == (2, 2 * GMAX, 4)
    src.close()


def test_eval_order_not_sharded():
    files = tfrecord_files(GOLD)
    full = TFRecordSource(files, 2, (96, 160), CPU, torch.float32, train=False)
    r1 = TFRecordSource(files, 2, (96, 160), CPU, torch.float32, train=False, rank=1, world=3)
    assert len(full) == len(r1) == 8 and (r1.order == np.arange(8)).all()
    assert full._ahead is None   # evaluation reads in the caller's thread
    tr = TFRecordSource(files, 2, (96, 160), CPU, torch.float32, train=True, rank=1, world=3, prefetch=False)
    assert len(tr) == 8 // 3   # training: this rank's disjoint slice of the shared shuffle
    for s in (full, r1, tr):
        s.close()
