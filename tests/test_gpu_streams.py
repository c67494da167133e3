"""The detector heads run one pyramid level per HIP stream (rod.ops.LEVELS, nets/catch_net.py
head_out): the same kernels in the same per-level order, so a training step — eager or replayed
as a HIP graph, REFINE and ALL — and the predict path are bit-identical to the heads run one
after another on the calling stream (ROD_HEAD_STREAMS=0)."""
import pytest
import torch

import config
from rod import ops

pytestmark = pytest.mark.gpu


def _steps(train_range, n_streams, graphed, dev, steps=3):
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    ops.LEVELS.n = n_streams
    try:
        tr = Trainer((160, 288), 2, dtype=torch.bfloat16, train_range=train_range, device=dev, seed=5)
        batches = [synthetic_batch(2, 160, 288, dev, seed=30 + i) for i in range(2)]
        step = tr.step_graphed if graphed else tr.step
        losses = [step(*batches[i % 2])[0].detach().clone() for i in range(steps)]
        torch.cuda.synchronize()
        return tr.net.store.flat.detach().clone(), torch.stack([l.reshape(()) for l in losses]), \
            {k: v.clone() for k, v in tr.net.store.buffers.items()}
    finally:
        ops.LEVELS.n = 3


@pytest.mark.parametrize('train_range', ['REFINE', 'ALL'])
@pytest.mark.parametrize('graphed', [False, True])
def test_level_streams_bit_identical(train_range, graphed, dev):
    tr_range = getattr(config.train_range, train_range)
    f0, l0, b0 = _steps(tr_range, 0, graphed, dev)
    f3, l3, b3 = _steps(tr_range, 3, graphed, dev)
    assert torch.equal(l0, l3), (l0, l3)
    assert torch.equal(f0, f3)
    assert all(torch.equal(v, b3[k]) for k, v in b0.items())


def test_level_streams_predict_bit_identical(dev):
    import predict
    from rod.data import synthetic_batch
    img = synthetic_batch(4, 160, 288, dev, seed=12)[0]
    outs = []
    for n in (0, 3):
        ops.LEVELS.n = n
        try:
            pr = predict.Predictor((160, 288), dev, torch.bfloat16)
            scores, boxes = pr(img)
            scores, boxes = pr(img)   # graph replay
            torch.cuda.synchronize()
            outs.append(({k: v.clone() for k, v in scores.items()}, {k: v.clone() for k, v in boxes.items()}))
        finally:
            ops.LEVELS.n = 3
    for a, b in zip(outs[0], outs[1]):
        assert a.keys() == b.keys()
        assert all(torch.equal(a[k], b[k]) for k in a)
