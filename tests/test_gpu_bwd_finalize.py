"""rod_bn_bwd_finalize in one launch (round 5): the column sums of the part-major [nparts][2][C]
backward sums and the coefficients formed from them, bit-exact against a numpy replica of the
fixed summation order (f64 chains over part rows ty, ty + L, ..., lanes added in order, rounded
to float; slab_sum_kernel's order) — the BatchNorm backward of slim.batch_norm
(mobilenet.py:417-420) finished from a producer's epilogue sums."""
import numpy as np
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu


def _slab_cb(nslab, n):
    if n >= 256 * 32 or nslab <= 64:
        return 32
    if n >= 256 * 8:
        return 8
    return 4


def _ordered_colsum(parts):
    """[nparts][n] float32 -> float32 [n], summed in the kernel's order."""
    nparts, n = parts.shape
    L = 256 // _slab_cb(nparts, n)
    x = parts.astype(np.float64)
    red = np.zeros((L, n))
    for ty in range(L):
        s = np.zeros((4, n))
        b = ty
        while b + 3 * L < nparts:
            for q in range(4):
                s[q] += x[b + q * L]
            b += 4 * L
        while b < nparts:
            s[0] += x[b]
            b += L
        red[ty] = (s[0] + s[1]) + (s[2] + s[3])
    t = np.zeros(n)
    for ty in range(L):
        t += red[ty]
    return t.astype(np.float32)


@pytest.mark.parametrize('nparts,C', [(1, 16), (50, 24), (300, 32), (1000, 144), (257, 1280), (4001, 576), (90, 66)])
def test_bwd_finalize_bit_exact(dev, nparts, C):
    g = torch.Generator().manual_seed(nparts * 7 + C)
    parts = (torch.randn(nparts, 2, C, generator=g) * 3).float()
    M = nparts * 97 + 5
    rstd = torch.rand(C, generator=g) + 0.5
    gamma = torch.rand(C, generator=g) + 0.5
    sums = _ordered_colsum(parts.reshape(nparts, 2 * C).numpy())
    sg, sgx = sums[:C], sums[C:]
    for with_gamma in (True, False):
        coef = torch.full((3 * C,), float('nan'), device=dev)
        dg = torch.full((C,), float('nan'), device=dev) if with_gamma else None
        db = torch.full((C,), float('nan'), device=dev)
        _abi.call('rod_bn_bwd_finalize', parts.to(dev), nparts, M, C, rstd.to(dev),
                  gamma.to(dev) if with_gamma else None, dg, db, coef, ops.stream())
        torch.cuda.synchronize()
        c = coef.cpu().numpy()
        k1 = (rstd * gamma).numpy() if with_gamma else rstd.numpy()
        assert np.array_equal(c[:C], k1)
        assert np.array_equal(c[C:2 * C], (sg.astype(np.float64) / M).astype(np.float32))
        assert np.array_equal(c[2 * C:], (sgx.astype(np.float64) / M).astype(np.float32))
        assert np.array_equal(db.cpu().numpy(), sg)
        if with_gamma:
            assert np.array_equal(dg.cpu().numpy(), sgx)
