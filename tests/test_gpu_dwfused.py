"""rod_dw3x3_bwd_fused (ABI 12/13: the stride-1 / stride-2 depthwise backward with the BatchNorm-backward
apply of its output and the BatchNorm-backward sums of its input's BatchNorm in one pass)
against the unfused librod chain it replaces (ref conv_blocks.py:238-247 backward,
FusedBatchNormGrad under mobilenet.py:417-420):

  rod_bn_bwd_reduce(dz, yd) -> coef_d            (both paths)
  rod_bn_bwd_apply(dz, yd, coef_d) -> dy          -- fused: in registers
  rod_dw3x3_bwd_data(dy, w) -> dx                 -- bit-identical (C % 8 == 0 bf16, fp32)
  rod_dw3x3_bwd_filter(act_e(BN_e(ye)), dy) -> dw -- reassociated: 1e-6 (fp32) / 1e-5 (bf16) normwise
  rod_bn_bwd_reduce(dx, ye; BN_e) -> coef_e, dgamma_e, dbeta_e
      -- fused: partial sums -> rod_bn_bwd_finalize, reassociated: same bounds
"""
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu

CASES = [  # (N, H, W, C, dtype, BN_e prologue / sums, stride)
    (2, 37, 45, 96, torch.bfloat16, True, 1),
    (1, 64, 70, 144, torch.bfloat16, True, 1),
    (3, 23, 40, 192, torch.bfloat16, True, 1),
    (2, 20, 33, 32, torch.float32, True, 1),
    (2, 19, 25, 12, torch.bfloat16, True, 1),     # C % 8 != 0 (4-channel packs)
    (2, 9, 7, 960, torch.bfloat16, True, 1),      # one strip, narrow map
    (1, 90, 160, 24, torch.float32, False, 1),    # no input BatchNorm (plain x)
    (2, 45, 80, 576, torch.bfloat16, True, 1),
    # stride 2, TF SAME: even sides pad (0, 1), odd sides (1, 1)
    (2, 36, 44, 96, torch.bfloat16, True, 2),
    (2, 37, 45, 144, torch.bfloat16, True, 2),    # odd: pad_t = pad_l = 1
    (1, 90, 160, 32, torch.float32, True, 2),
    (2, 23, 64, 192, torch.bfloat16, True, 2),
    (2, 19, 26, 12, torch.bfloat16, True, 2),
    (1, 45, 80, 96, torch.float32, False, 2),
    (1, 181, 320, 144, torch.bfloat16, True, 2),
]


def _same(n, s):
    o = -(-n // s)
    return o, max((o - 1) * s + 3 - n, 0) // 2


def _nerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


R6, NONE, LEAKY, RELU = ops.ROD_ACT_RELU6, ops.ROD_ACT_NONE, ops.ROD_ACT_LEAKY, 3
# the run-time activation forms (DW_ACT_RT) of both BatchNorms, stride 1 and 2
ACT_CASES = [  # (N, H, W, C, dtype, stride, act of the output BatchNorm, act of the input BatchNorm)
    (2, 37, 45, 96, torch.bfloat16, 1, NONE, LEAKY),
    (2, 37, 45, 96, torch.bfloat16, 1, LEAKY, NONE),
    (2, 20, 33, 32, torch.float32, 1, LEAKY, LEAKY),
    (1, 23, 40, 64, torch.bfloat16, 1, RELU, R6),
    (2, 36, 44, 96, torch.bfloat16, 2, NONE, LEAKY),
    (2, 37, 45, 144, torch.bfloat16, 2, LEAKY, NONE),
    (1, 45, 80, 32, torch.float32, 2, LEAKY, RELU),
]


@pytest.mark.parametrize('N,H,W,C,dt,pro,S', CASES)
def test_fused_matches_unfused_chain(dev, N, H, W, C, dt, pro, S):
    _check(dev, N, H, W, C, dt, pro, S, R6, R6)


@pytest.mark.parametrize('N,H,W,C,dt,S,act_d,act_e', ACT_CASES)
def test_fused_runtime_activations(dev, N, H, W, C, dt, S, act_d, act_e):
    _check(dev, N, H, W, C, dt, True, S, act_d, act_e)


def _check(dev, N, H, W, C, dt, pro, S, act, act_e):
    g = torch.Generator().manual_seed(N * 1000 + H * 10 + C + 7 * act + act_e)
    (Ho, pt), (Wo, pl) = _same(H, S), _same(W, S)
    ye = (torch.randn(N, H, W, C, generator=g) * 1.3 + 0.2).to(dev, dt)
    yd = (torch.randn(N, Ho, Wo, C, generator=g) * 2 + 0.4).to(dev, dt)
    dz = torch.randn(N, Ho, Wo, C, generator=g).to(dev, dt)
    w = (torch.randn(3, 3, C, generator=g) * 0.4).to(dev)
    f = lambda lo=0.5: (torch.rand(C, generator=g) + lo).to(dev)
    dmean, drstd, dgam, dbet = torch.randn(C, generator=g).to(dev) * 0.3, f(), f(), torch.randn(C, generator=g).to(dev)
    emean, erstd, egam, ebet = (torch.randn(C, generator=g).to(dev) * 0.1, f(), f(),
                                torch.randn(C, generator=g).to(dev) * 0.1)
    pargs = (emean, erstd, egam, ebet, act_e) if pro else (None, None, None, None, 0)
    M, Mo, st, code = N * H * W, N * Ho * Wo, ops.stream(), ops.dtcode(ye)
    coef = torch.empty(3 * C, device=dev)
    rws = ops.workspace(_abi.query('rod_bn_bwd_workspace', max(M, Mo), C), dev)
    _abi.call('rod_bn_bwd_reduce', dz, yd, dmean, drstd, dgam, dbet, None, None, coef, rws, Mo, C, act, code, st)
    # unfused reference chain
    dy = torch.empty_like(yd)
    _abi.call('rod_bn_bwd_apply', dz, yd, dmean, drstd, dgam, dbet, coef, dy, Mo, C, act, code, st)
    dx_ref = torch.empty_like(ye)
    _abi.call('rod_dw3x3_bwd_data', dy, w, dx_ref, None, None, None, None, None, 0, None, N, H, W, C, S, pt, pl, Ho,
              Wo, code, st)
    fws = ops.workspace(_abi.query('rod_dw3x3_bwd_filter_workspace', N, Ho, Wo, C), dev)
    dw_ref = torch.empty(3, 3, C, device=dev)
    _abi.call('rod_dw3x3_bwd_filter', ye, *pargs, dy, dw_ref, fws, N, H, W, C, S, pt, pl, Ho, Wo, code, st)
    # fused
    nparts = _abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, S, pt, pl)
    assert nparts > 0
    gparts = torch.full((nparts, 2, C), float('nan'), device=dev) if pro else None
    dx = torch.full_like(ye, float('nan'))
    dw = torch.empty(3, 3, C, device=dev)
    ws = ops.workspace(_abi.query('rod_dw3x3_bwd_fused_workspace', N, H, W, C, S, pt, pl), dev)
    _abi.call('rod_dw3x3_bwd_fused', ye, *pargs, dz, yd, dmean, drstd, dgam, dbet, act, coef, w, dx, dw, gparts, ws,
              N, H, W, C, S, pt, pl, Ho, Wo, code, st)
    torch.cuda.synchronize()
    iv = torch.int16 if dt == torch.bfloat16 else torch.int32
    if C % 8 == 0 or dt == torch.float32 or S == 2:
        # same accumulation order as the backward-data kernel (stride 2: any pack width)
        assert torch.equal(dx.view(iv), dx_ref.view(iv)), float((dx.float() - dx_ref.float()).abs().max())
    else:   # the reference takes the narrow-pack kernel, which sums the taps in another order
        assert (dx.float() - dx_ref.float()).abs().max() <= 2 ** -7 * dx_ref.float().abs().max()
    tol = 1e-5 if dt == torch.bfloat16 else 1e-6
    assert _nerr(dw, dw_ref) < tol, _nerr(dw, dw_ref)
    if pro:
        # BN_e backward from the fused sums against rod_bn_bwd_reduce over (dx, ye)
        ce_ref, dg_ref, db_ref = torch.empty(3 * C, device=dev), torch.empty(C, device=dev), torch.empty(C, device=dev)
        rws2 = ops.workspace(_abi.query('rod_bn_bwd_workspace', M, C), dev)
        _abi.call('rod_bn_bwd_reduce', dx_ref, ye, emean, erstd, egam, ebet, dg_ref, db_ref, ce_ref, rws2, M, C, act_e,
                  code, st)
        ce, dg, db = torch.empty(3 * C, device=dev), torch.empty(C, device=dev), torch.empty(C, device=dev)
        _abi.call('rod_bn_bwd_finalize', gparts, nparts, M, C, erstd, egam, dg, db, ce, st)
        torch.cuda.synchronize()
        for a, b in ((ce, ce_ref), (dg, dg_ref), (db, db_ref)):
            assert _nerr(a, b) < tol, (_nerr(a, b), a[:4], b[:4])
