"""rod_bn_bwd_reduce on tensors of >= 64M elements (the software-pipelined reduction the step's
large BatchNorm backwards take, batchnorm.hip bn_bwd_reduce_kernel PIPE) against a float64
restatement of FusedBatchNormGrad's sums (tf.nn.fused_batch_norm backward, as the oracle's
batchnorm backward): dbeta = sum g, dgamma = sum g * (y - mean) * rstd with g = dz * act'(BN(y)),
and the apply coefficients (rstd * gamma, dbeta / M, dgamma / M).  Ragged row counts exercise
the pipelined loop's batch tail and the per-row remainder."""
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu

CASES = [  # (M, C, act)
    (2_200_003, 32, ops.ROD_ACT_RELU6),
    (1_100_001, 64, ops.ROD_ACT_NONE),
    (460_807, 192, ops.ROD_ACT_RELU6),
]


@pytest.mark.parametrize('M,C,act', CASES)
def test_bn_bwd_reduce_large(dev, M, C, act):
    assert M * C >= 64 << 20
    g = torch.Generator(device=dev).manual_seed(M % 1000 + C)
    y = (torch.randn(M, C, device=dev, generator=g) * 2 + 0.5).to(torch.bfloat16)
    dz = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    mean = torch.randn(C, device=dev, generator=g) * 0.3 + 0.5
    rstd = torch.rand(C, device=dev, generator=g) + 0.5
    gamma = torch.rand(C, device=dev, generator=g) + 0.5
    beta = torch.randn(C, device=dev, generator=g) * 0.2
    coef = torch.empty(3 * C, device=dev)
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    rws = ops.workspace(_abi.query('rod_bn_bwd_workspace', M, C), dev)
    _abi.call('rod_bn_bwd_reduce', dz, y, mean, rstd, gamma, beta, dg, db, coef, rws, M, C, act, ops.dtcode(y),
              ops.stream())
    torch.cuda.synchronize()
    # float64 restatement
    yf, gf = y.double(), dz.double()
    sc = (gamma * rstd).double()
    z = yf * sc + (beta.double() - mean.double() * sc)
    if act == ops.ROD_ACT_RELU6:
        gf = gf * ((z > 0) & (z < 6)).double()
    xhat = (yf - mean.double()) * rstd.double()
    db_ref = gf.sum(0)
    dg_ref = (gf * xhat).sum(0)
    del yf, z, xhat, gf

    def nerr(a, b):
        return float((a.double() - b).norm() / b.norm().clamp_min(1e-30))

    assert nerr(db, db_ref) < 1e-5, nerr(db, db_ref)
    assert nerr(dg, dg_ref) < 1e-5, nerr(dg, dg_ref)
    assert nerr(coef[:C], (rstd * gamma).double()) < 1e-7
    assert nerr(coef[C:2 * C], db_ref / M) < 1e-5
    assert nerr(coef[2 * C:], dg_ref / M) < 1e-5


@pytest.mark.parametrize('M,C', [(65_536, 64), (4096, 256)])
def test_bn_bwd_fp32_large_mean_vs_float64(dev, M, C):
    """fp32 BatchNorm backward on a channel whose |mean| is 5000x its std (mean 50, rstd 100):
    the apply centres y before scaling (rod_common.h bn_bwd_k<float>), as FusedBatchNormGrad does,
    so dx keeps fp32 precision; folding the mean into the constant (the bf16 form) would lose
    ~log2(5000) bits here (~3e-4 relative).  dz is correlated with yhat so that the
    mean(g * yhat) term — the one the fold degrades — carries weight.  (4096, 256) takes the
    one-launch small-tensor kernel, (65536, 64) reduce -> finalize -> apply."""
    g = torch.Generator(device=dev).manual_seed(M + C)
    mean = 50.0 + torch.rand(C, device=dev, generator=g)
    rstd = 100.0 * (torch.rand(C, device=dev, generator=g) + 0.5)
    xh = torch.randn(M, C, device=dev, generator=g)
    y = (mean + xh / rstd).float()
    dz = (0.5 * xh + torch.randn(M, C, device=dev, generator=g)).float()
    gamma = torch.rand(C, device=dev, generator=g) + 0.5
    beta = torch.randn(C, device=dev, generator=g) * 0.2
    act = ops.ROD_ACT_NONE
    dx, dg, db = torch.empty_like(y), torch.empty(C, device=dev), torch.empty(C, device=dev)
    ws = ops.workspace(_abi.query('rod_bn_bwd_workspace', M, C), dev)
    _abi.call('rod_bn_bwd', dz, y, mean, rstd, gamma, beta, dx, dg, db, ws, M, C, C, C, C, act, ops.dtcode(y),
              ops.stream())
    coef = torch.empty(3 * C, device=dev)
    _abi.call('rod_bn_bwd_reduce', dz, y, mean, rstd, gamma, beta, None, None, coef, ws, M, C, act, ops.dtcode(y),
              ops.stream())
    dx2 = torch.empty_like(y)
    _abi.call('rod_bn_bwd_apply', dz, y, mean, rstd, gamma, beta, coef, dx2, M, C, act, ops.dtcode(y), ops.stream())
    torch.cuda.synchronize()
    yf, gf, mu, rs = y.double(), dz.double(), mean.double(), rstd.double()
    xhat = (yf - mu) * rs
    mg, mgx = gf.mean(0), (gf * xhat).mean(0)
    ref = (rs * gamma.double()) * (gf - mg - xhat * mgx)
    for out in (dx, dx2):
        err = float((out.double() - ref).norm() / ref.norm())
        assert err < 2e-6, err
