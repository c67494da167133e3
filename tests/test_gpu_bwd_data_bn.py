"""Backward-data of a 1x1 conv through its BatchNorm in one launch (ABI 22,
rod_conv_bwd_data_bn): dy (the BatchNorm-backward apply of (dz, y)) formed in the GEMM's loader
and written once, dx = dy . W — bit-identical to rod_bn_bwd_apply followed by rod_conv_fwd with
the mode-1 weights (FusedBatchNormGrad + Conv2DBackpropInput of the expand convs,
conv_blocks.py:263-294) on every GEMM path (one N tile, several N tiles, split-K), and a REFINE
training step with the entry on / off (ROD_DISABLE=bnbwd) bit-identical, eager and graphed."""
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu
bf16 = torch.bfloat16

# (M, Cout = the GEMM's K, Cin = its N, act): the 720p step's deep expands (blocks 6-16) and
# ragged / multi-tile / split-K cases
CASES = [(115200, 384, 64, ops.ROD_ACT_RELU6), (28800, 576, 96, ops.ROD_ACT_RELU6),
         (7360, 960, 160, ops.ROD_ACT_RELU6), (1920, 960, 160, ops.ROD_ACT_RELU6), (5003, 256, 24, ops.ROD_ACT_LEAKY),
         (3001, 128, 264, ops.ROD_ACT_NONE), (640, 1280, 128, ops.ROD_ACT_LEAKY),
         # the upper limit of rod_conv_bwd_data_bn_supported: the table's 4096 x 8 floats of
         # dynamic LDS beside the static tiles fill gfx950's 160 KB per workgroup
         (515, 4096, 64, ops.ROD_ACT_RELU6)]


def test_bwd_data_bn_supported_bound(dev):
    lib = _abi.lib()
    code = ops.dtcode(torch.empty(1, dtype=bf16))
    assert lib.rod_conv_bwd_data_bn_supported(4096, 64, code) == 1
    assert lib.rod_conv_bwd_data_bn_supported(4104, 64, code) == 0


@pytest.mark.parametrize('M,Cout,Cin,act', CASES)
def test_bwd_data_bn_bit_identical(dev, M, Cout, Cin, act):
    assert _abi.lib().rod_conv_bwd_data_bn_supported(Cout, Cin, ops.dtcode(torch.empty(1, dtype=bf16)))
    g = torch.Generator().manual_seed(M + Cout + Cin)
    y = (torch.randn(1, 1, M, Cout, generator=g) * 1.5 + 0.4).to(dev, bf16)
    dz = torch.randn(1, 1, M, Cout, generator=g).to(dev, bf16)
    mean = y.float().mean((0, 1, 2)) + (torch.randn(Cout, generator=g) * 0.05).to(dev)
    rstd = (torch.rand(Cout, generator=g) + 0.5).to(dev)
    gamma = (torch.rand(Cout, generator=g) + 0.5).to(dev)
    beta = (torch.randn(Cout, generator=g) * 0.2).to(dev)
    coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)
    w = (torch.randn(Cout, 1, 1, Cin, generator=g) * 0.1).to(dev)
    wt1 = ops._prep(w, 1, bf16, Cout, Cin, 1)
    dy_ref = torch.empty_like(y)
    _abi.call('rod_bn_bwd_apply', dz, y, mean, rstd, gamma, beta, coef, dy_ref, M, Cout, act, ops.dtcode(y),
              ops.stream())
    dx_ref = torch.empty(1, 1, M, Cin, dtype=bf16, device=dev)
    ops.conv_fwd_raw(dy_ref, wt1, None, dx_ref, 1, 1, M, Cout, Cin, 1)
    dy, dx = ops.conv_bwd_data_bn(dz, y, mean, rstd, gamma, beta, act, coef, w)
    torch.cuda.synchronize()
    assert torch.equal(dy, dy_ref), float((dy.float() - dy_ref.float()).abs().max())
    assert torch.equal(dx, dx_ref), float((dx.float() - dx_ref.float()).abs().max())


@pytest.mark.parametrize('graphed', [False, True])
def test_step_bwd_data_bn_bit_identical(dev, graphed):
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    runs = []
    for off in (True, False):
        if off:
            ops._DISABLE.add('bnbwd')
        try:
            tr = Trainer((320, 576), 2, dtype=bf16, device=dev, seed=7)
            batches = [synthetic_batch(2, 320, 576, dev, seed=50 + i) for i in range(2)]
            step = tr.step_graphed if graphed else tr.step
            _abi.PROBE.arm(['rod_conv_bwd_data_bn', 'rod_bn_bwd_apply'])
            losses = [step(*batches[i % 2])[0].detach().clone() for i in range(3)]
            torch.cuda.synchronize()
            calls = _abi.PROBE.table()
            _abi.PROBE.disarm()
            runs.append((tr.net.store.flat.detach().clone(), torch.stack([l.reshape(()) for l in losses]), calls))
        finally:
            ops._DISABLE.discard('bnbwd')
    (f0, l0, c0), (f1, l1, c1) = runs
    assert 'rod_conv_bwd_data_bn' not in c0
    assert c1.get('rod_conv_bwd_data_bn', (0,))[0] >= 1, c1
    assert torch.equal(l0, l1), (l0, l1)
    assert torch.equal(f0, f1)
