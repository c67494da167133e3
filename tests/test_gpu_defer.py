"""Deferred weight-gradient sums (rod_slab_defer / rod_slab_flush, ABI 11) keep every slab they
will read alive: each entry that queues a sum is in rod._abi.DEFERRING (its tensors stay
referenced until the flush), checked here against the library's own queue length on REFINE and
ALL steps at a size where every backward path of the network runs (320x576: the ABI-20
recompute pair on block 2, the ABI-22 backward-data on the deep expands).  A gap showed as
run-to-run different weight updates: a freed slab reused before the flush read it."""
import os

import pytest
import torch

import config
from rod import _abi

pytestmark = pytest.mark.gpu


def _run(train_range, dev, steps=2):
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    tr = Trainer((320, 576), 2, dtype=torch.bfloat16, train_range=train_range, device=dev, seed=9)
    batches = [synthetic_batch(2, 320, 576, dev, seed=60 + i) for i in range(steps)]
    losses = [tr.step(*b)[0].detach().clone() for b in batches]
    torch.cuda.synchronize()
    return tr.net.store.flat.detach().clone(), torch.stack([l.reshape(()) for l in losses])


@pytest.mark.parametrize('train_range', ['REFINE', 'ALL'])
def test_deferring_entries_listed_and_step_deterministic(train_range, dev):
    tr_range = getattr(config.train_range, train_range)
    _abi.DEFER_UNLISTED.clear()
    _abi.WATCH_DEFER = True     # the registry check (on by default; ROD_DEFER_WATCH=0 turns it off)
    try:
        f0, l0 = _run(tr_range, dev)
    finally:
        _abi.WATCH_DEFER = os.environ.get("ROD_DEFER_WATCH", "1") != "0"
    assert not _abi.DEFER_UNLISTED, sorted(_abi.DEFER_UNLISTED)
    f1, l1 = _run(tr_range, dev)
    assert torch.equal(l0, l1), (l0, l1)
    assert torch.equal(f0, f1)
