"""The projects on the streaming 1x1 kernel (csrc/gemm.hip pw_proj_launch: pw_stream_kernel with
the BatchNorm-apply prologue past K = 32: K = 40 .. 192 input channels, Cout = 16 .. 32 outputs,
M >= 65536 rows, ReLU6) against the tiled GEMM it replaces (ROD_PW_PROJ=0, read per call): y
bit-identical (the same MFMA k order and prologue rounding), the BatchNorm statistics parts (one
per 128-row tile in both) equal to fp32 summation-order level, incl. ragged M and a padded last
N tile (Cout = 24).  The step-level check is every training test: the shapes are the backbone's
projects (conv_blocks.py:287-294, project conv + BatchNorm after the depthwise BatchNorm + ReLU6)."""
import numpy as np
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu
bf16 = torch.bfloat16


@pytest.fixture(scope='module')
def dev():
    return torch.device('cuda:0')


@pytest.mark.parametrize('K,Cout,M,act,stats', [
    (96, 24, 65536, ops.ROD_ACT_RELU6, True),      # L3 project 96 -> 24
    (144, 24, 65536 + 77, ops.ROD_ACT_RELU6, True),  # L4 project, ragged last tile
    (144, 32, 70000, ops.ROD_ACT_RELU6, True),
    (192, 32, 65536, ops.ROD_ACT_RELU6, True),     # L6/L7 projects
    (192, 32, 65536, ops.ROD_ACT_RELU6, False),
    (40, 8, 65536, ops.ROD_ACT_RELU6, False),
    (32, 16, 65536, ops.ROD_ACT_RELU6, True),      # K <= 32 (the 720p block-1 project): the tiled kernel
    (96, 24, 65536, ops.ROD_ACT_NONE, True)])      # another activation: the tiled kernel
def test_pw_proj_matches_tiled(dev, K, Cout, M, act, stats, monkeypatch):
    g = torch.Generator().manual_seed(K * 7 + Cout)
    x = (torch.randn(M, K, generator=g) * 2 + 0.5).to(bf16).to(dev)
    w = (torch.randn(Cout, K, generator=g) / np.sqrt(K)).to(dev)
    mean = (torch.randn(K, generator=g) * 0.3).to(dev)
    rstd = (torch.rand(K, generator=g) + 0.5).to(dev)
    gamma = (torch.rand(K, generator=g) + 0.5).to(dev)
    beta = (torch.randn(K, generator=g) * 0.2).to(dev)
    pro = (mean, rstd, gamma, beta, act)
    wt = torch.empty((Cout, K), dtype=bf16, device=dev)
    _abi.call('rod_conv_weight_prep', w.reshape(Cout, 1, 1, K).contiguous(), wt, Cout, K, 1, 0, 1, ops.stream())
    nt = -(-M // 128)

    def run():
        y = torch.full((1, 1, M, Cout), float('nan'), dtype=bf16, device=dev)
        parts = torch.full((nt, 3, Cout), float('nan'), device=dev) if stats else None
        ops.conv_fwd_raw(x.reshape(1, 1, M, K), wt, None, y, 1, 1, M, K, Cout, 1, parts, pro)
        torch.cuda.synchronize()
        return y, parts

    y1, p1 = run()
    monkeypatch.setenv('ROD_PW_PROJ', '0')
    y0, p0 = run()
    assert not torch.isnan(y1.float()).any()
    assert torch.equal(y1, y0)
    if stats:
        assert not torch.isnan(p1).any()
        assert torch.equal(p1[:, 0], p0[:, 0])                     # counts
        torch.testing.assert_close(p1[:, 1], p0[:, 1], rtol=1e-5, atol=1e-5)   # tile means
        torch.testing.assert_close(p1[:, 2], p0[:, 2], rtol=1e-4, atol=1e-3)   # tile M2
