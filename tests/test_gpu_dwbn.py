"""rod_dw3x3_bwd_filter_bn (the depthwise's BatchNorm-backward apply fused into its filter
gradient, ABI 10) against the unfused librod chain it replaces: rod_bn_bwd_reduce (coef) ->
rod_bn_bwd_apply (dy written) -> rod_dw3x3_bwd_filter.  The fused kernel forms dy with
rod_bn_bwd_apply's arithmetic, rounds it the same way and contracts the rounded value in the
same order, so dy and dw are bit-identical; the fp32 path and the non-16-byte fallback too."""
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu

CASES = [  # (N, H, W, C, stride, prologue on x, dtype)
    (2, 37, 45, 96, 1, True, torch.bfloat16),
    (2, 38, 41, 96, 2, True, torch.bfloat16),
    (1, 64, 70, 144, 1, False, torch.bfloat16),
    (3, 23, 40, 192, 2, False, torch.bfloat16),
    (2, 20, 33, 32, 1, True, torch.float32),
    (2, 21, 30, 64, 2, True, torch.float32),
    (2, 19, 25, 12, 1, True, torch.bfloat16),   # C % 8 != 0: apply + plain filter fallback
]


@pytest.mark.parametrize('N,H,W,C,s,pro,dt', CASES)
def test_filter_bn_matches_unfused(dev, N, H, W, C, s, pro, dt):
    g = torch.Generator().manual_seed(N * 1000 + H * 10 + C + s)
    Ho, pt = ops.same_pad(H, s)
    Wo, pl = ops.same_pad(W, s)
    x = (torch.randn(N, H, W, C, generator=g) * 1.3 + 0.2).to(dev, dt)
    y = (torch.randn(N, Ho, Wo, C, generator=g) * 2 + 0.4).to(dev, dt)
    dz = torch.randn(N, Ho, Wo, C, generator=g).to(dev, dt)
    f = lambda *sh, lo=0.5: (torch.rand(*sh, generator=g) + lo).to(dev)
    mean, rstd, gamma, beta = torch.randn(C, generator=g).to(dev) * 0.3, f(C), f(C), torch.randn(C, generator=g).to(dev)
    act = ops.ROD_ACT_RELU6
    pargs = (torch.randn(C, generator=g).to(dev) * 0.1, f(C), f(C), torch.randn(C, generator=g).to(dev) * 0.1,
             ops.ROD_ACT_RELU6) if pro else (None, None, None, None, 0)
    M, st, code = N * Ho * Wo, ops.stream(), ops.dtcode(x)
    coef = torch.empty(3 * C, device=dev)
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    rws = ops.workspace(_abi.query('rod_bn_bwd_workspace', M, C), dev)
    _abi.call('rod_bn_bwd_reduce', dz, y, mean, rstd, gamma, beta, dg, db, coef, rws, M, C, act, code, st)
    fws = ops.workspace(_abi.query('rod_dw3x3_bwd_filter_workspace', N, Ho, Wo, C), dev)
    # unfused reference chain
    dy_ref = torch.empty_like(y)
    _abi.call('rod_bn_bwd_apply', dz, y, mean, rstd, gamma, beta, coef, dy_ref, M, C, act, code, st)
    dw_ref = torch.empty(3, 3, C, device=dev)
    _abi.call('rod_dw3x3_bwd_filter', x, *pargs, dy_ref, dw_ref, fws, N, H, W, C, s, pt, pl, Ho, Wo, code, st)
    # fused
    dy = torch.full_like(y, float('nan'))
    dw = torch.empty(3, 3, C, device=dev)
    _abi.call('rod_dw3x3_bwd_filter_bn', x, *pargs, dz, y, mean, rstd, gamma, beta, act, coef, dy, dw, fws,
              N, H, W, C, s, pt, pl, Ho, Wo, code, st)
    torch.cuda.synchronize()
    assert torch.equal(dy.view(torch.int16 if dt == torch.bfloat16 else torch.int32),
                       dy_ref.view(torch.int16 if dt == torch.bfloat16 else torch.int32))
    assert torch.equal(dw, dw_ref)
