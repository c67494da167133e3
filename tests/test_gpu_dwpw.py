"""The inverted-residual block's depthwise backward without a materialised dz (ABI 20):
rod_pw_bwd_gred_dyp hands over the project BatchNorm's backward output dy_p instead of writing
dx = dy_p . W_p, and rod_dw3x3_bwd_fused_pw recomputes that dx per tile with the same MFMA.
Against the materialising chain rod_pw_bwd_gred -> rod_dw3x3_bwd_fused on the same inputs:
the project's dW and the depthwise BatchNorm's sums, then the depthwise's dx, dW and the
expand BatchNorm's sums, all bit-identical (ref conv_blocks.py:238-247, 287-294 backward)."""
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu
bf16 = torch.bfloat16
R6 = ops.ROD_ACT_RELU6


def _vec(g, C, lo, dev, scale=1.0):
    return ((torch.rand(C, generator=g) * scale) + lo).to(dev)


# (N, H, W, C, cout): the 720p step's shapes scaled down (block 0: 32 -> 16, block 2: 144 -> 24,
# blocks 4 / 5: 192 -> 32) plus ragged maps and strip / tile edges
CASES = [(2, 37, 45, 144, 24), (1, 64, 70, 32, 16), (2, 23, 40, 192, 32), (3, 19, 33, 144, 24),
         (1, 90, 160, 32, 16), (2, 45, 80, 192, 32)]


@pytest.mark.parametrize('N,H,W,C,cout', CASES)
def test_dw_fused_pw_bit_identical(dev, N, H, W, C, cout):
    assert _abi.lib().rod_dw3x3_bwd_fused_pw_supported(N, H, W, C, cout, R6, R6, ops.dtcode(torch.empty(1, dtype=bf16)))
    g = torch.Generator().manual_seed(N * 1000 + H * 10 + C + cout)
    M = N * H * W
    # the project conv: input x_p = ReLU6(BN_d(yd)), output y_p (linear BatchNorm)
    yd = (torch.randn(N, H, W, C, generator=g) * 1.5 + 0.3).to(dev, bf16)
    yp = (torch.randn(M, cout, generator=g) * 2 + 0.5).to(dev, bf16)
    dzp = torch.randn(M, cout, generator=g).to(dev, bf16)
    wp = (torch.randn(cout, 1, 1, C, generator=g) * 0.2).to(dev)
    pm, pr = yp.float().mean(0), torch.rsqrt(yp.float().var(0, unbiased=False) + 1e-3)
    pg, pb = _vec(g, cout, 0.5, dev), (torch.randn(cout, generator=g) * 0.3).to(dev)
    dm = yd.float().mean((0, 1, 2)) + (torch.randn(C, generator=g) * 0.05).to(dev)
    dr = _vec(g, C, 0.5, dev)
    dg, db = _vec(g, C, 0.5, dev), (torch.randn(C, generator=g) * 0.2).to(dev)
    dpro = (dm, dr, dg, db, R6)
    coef_p = ops.bn_bwd_reduce(dzp, yp, pm, pr, pg, pb, ops.ROD_ACT_NONE, False, False)
    wt1 = ops._prep(wp, 1, bf16, cout, C, 1)
    dwp_a = torch.full((cout, C), float('nan'), device=dev)
    dwp_b = torch.full((cout, C), float('nan'), device=dev)
    dzd, parts_a = ops.pw_bwd_gred(dzp, yp, pm, pr, pg, pb, ops.ROD_ACT_NONE, coef_p, yd.view(M, C), dpro, wt1, dwp_a)
    dyp, parts_b = ops.pw_bwd_gred(dzp, yp, pm, pr, pg, pb, ops.ROD_ACT_NONE, coef_p, yd.view(M, C), dpro, wt1, dwp_b,
                                   dyp=True)
    assert torch.equal(dwp_a, dwp_b) and torch.equal(parts_a, parts_b)
    dyp_ref = torch.empty_like(yp)   # dyp is the BatchNorm-backward output rod_bn_bwd_apply writes
    _abi.call('rod_bn_bwd_apply', dzp, yp, pm, pr, pg, pb, coef_p, dyp_ref, M, cout, ops.ROD_ACT_NONE, ops.dtcode(yp),
              ops.stream())
    assert torch.equal(dyp, dyp_ref)
    # the depthwise: input x = ReLU6(BN_e(ye)), BN_d's coefficients from the project's sums
    ye = (torch.randn(N, H, W, C, generator=g) * 1.3 + 0.2).to(dev, bf16)
    em, er = (torch.randn(C, generator=g) * 0.1).to(dev), _vec(g, C, 0.5, dev)
    eg, eb = _vec(g, C, 0.5, dev), (torch.randn(C, generator=g) * 0.1).to(dev)
    w = (torch.randn(3, 3, C, generator=g) * 0.4).to(dev)
    coef_d = ops.bn_bwd_coef_from_parts(parts_a, M, C, dr, dg, db, False, False)
    nparts = _abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, 1, 1, 1)
    ws_n = _abi.query('rod_dw3x3_bwd_fused_workspace', N, H, W, C, 1, 1, 1)
    outs = []
    for pw in (False, True):
        dx = torch.full_like(ye, float('nan'))
        dw = torch.full((3, 3, C), float('nan'), device=dev)
        gp = torch.full((nparts, 2, C), float('nan'), device=dev)
        ws = ops.workspace(ws_n, dev)
        if pw:
            _abi.call('rod_dw3x3_bwd_fused_pw', ye, em, er, eg, eb, R6, dyp, wt1, cout, yd, dm, dr, dg, db, R6, coef_d,
                      w, dx, dw, gp, ws, N, H, W, C, ops.dtcode(ye), ops.stream())
        else:
            _abi.call('rod_dw3x3_bwd_fused', ye, em, er, eg, eb, R6, dzd.view(N, H, W, C), yd, dm, dr, dg, db, R6,
                      coef_d, w, dx, dw, gp, ws, N, H, W, C, 1, 1, 1, H, W, ops.dtcode(ye), ops.stream())
        outs.append((dx, dw, gp))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert not torch.isnan(a).any()
        assert torch.equal(a, b), float((a.float() - b.float()).abs().max())



@pytest.mark.parametrize('graphed', [False, True])
def test_step_with_recompute_bit_identical(dev, graphed):
    """A bf16 REFINE training step with the depthwise backward recomputing dz (the default) is
    bit-identical to the step that materialises it (ROD_DISABLE=dwpw), eager and HIP-graph replayed,
    and the recompute path actually runs (its entry is called in the eager step)."""
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    runs = []
    for off in (True, False):
        if off:
            ops._DISABLE.add('dwpw')
        try:
            tr = Trainer((160, 288), 2, dtype=bf16, device=dev, seed=6)
            batches = [synthetic_batch(2, 160, 288, dev, seed=40 + i) for i in range(2)]
            step = tr.step_graphed if graphed else tr.step
            _abi.PROBE.arm(['rod_dw3x3_bwd_fused_pw', 'rod_pw_bwd_gred_dyp'])
            losses = [step(*batches[i % 2])[0].detach().clone() for i in range(3)]
            torch.cuda.synchronize()
            calls = _abi.PROBE.table()
            _abi.PROBE.disarm()
            runs.append((tr.net.store.flat.detach().clone(), torch.stack([l.reshape(()) for l in losses]), calls))
        finally:
            ops._DISABLE.discard('dwpw')
    (f0, l0, c0), (f1, l1, c1) = runs
    assert 'rod_dw3x3_bwd_fused_pw' not in c0
    # at 160x288 block 0 (32 -> 16) takes it; the graphed run probes its one eager step
    assert c1.get('rod_dw3x3_bwd_fused_pw', (0,))[0] >= 1 and c1.get('rod_pw_bwd_gred_dyp', (0,))[0] >= 1, c1
    assert torch.equal(l0, l1), (l0, l1)
    assert torch.equal(f0, f1)
