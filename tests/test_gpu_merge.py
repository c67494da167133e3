"""BatchNorm statistic merges: the two-level merge in one launch (the last block of each channel
group merges the slice parts the others wrote, csrc/batchnorm.hip bn_parts_merge_kernel) keeps
the grouping and order of two launches, so a training step is bit-identical with it on and off
(ROD_MERGE_TWO_LAUNCH=1), eager and graphed.  The kernel-level check over 1 to 70,000 parts is
tests/test_gpu_kernels.py::test_bn_finalize_many_parts."""
import pytest
import torch

from rod import _abi

pytestmark = pytest.mark.gpu
bf16 = torch.bfloat16


@pytest.fixture(scope='module')
def dev():
    return torch.device('cuda:0')


@pytest.mark.parametrize('graphed', [False, True])
def test_step_single_launch_merge_bit_identical(dev, graphed, monkeypatch):
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    runs = []
    for two in (True, False):
        if two:
            monkeypatch.setenv('ROD_MERGE_TWO_LAUNCH', '1')
        else:
            monkeypatch.delenv('ROD_MERGE_TWO_LAUNCH', raising=False)
        tr = Trainer((320, 576), 2, dtype=bf16, device=dev, seed=7)
        batches = [synthetic_batch(2, 320, 576, dev, seed=50 + i) for i in range(2)]
        step = tr.step_graphed if graphed else tr.step
        losses = [step(*batches[i % 2])[0].detach().clone() for i in range(3)]
        torch.cuda.synchronize()
        runs.append((tr.net.store.flat.detach().clone(), torch.stack([l.reshape(()) for l in losses])))
    (f0, l0), (f1, l1) = runs
    assert torch.equal(l0, l1), (l0, l1)
    assert torch.equal(f0, f1)
