"""Kernel parity: librod (HIP, cuda:0) against the CPU oracle on seeded inputs.

Tolerances: fp32 storage 1e-4 relative (north_star) with a small absolute floor for
values that cancel; bf16 storage is compared against the fp32 oracle at bf16 resolution.
Integer outputs (positive masks, labels, argmax-selected boxes) are compared bit-exactly.
"""
import numpy as np
import pytest
import torch

import config
from oracle import anchors as oa
from oracle import net as onet
from oracle import targets as ot
from rod import ops

pytestmark = pytest.mark.gpu

TOL = {torch.float32: dict(rtol=1e-4, atol=1e-5), torch.bfloat16: dict(rtol=2e-2, atol=2e-2)}


def _close(a, b, dtype, scale=1.0, **kw):
    tol = dict(TOL[dtype])
    tol['atol'] = tol['atol'] * scale
    tol.update(kw)
    torch.testing.assert_close(a.detach().float().cpu(), b.detach().float().cpu(), **tol)


def _param(t, dev):
    p = t.detach().clone().to(dev).requires_grad_(True)
    p._rod_grad = torch.zeros_like(p)
    return p


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('C,stride,H,W', [(c, s, h, w) for c in (24, 6)
                                          for (s, h, w) in [(1, 13, 17), (2, 13, 17), (2, 12, 16), (1, 4, 5)]] +
                         [(144, 2, 45, 80), (144, 1, 45, 80), (96, 2, 90, 161), (960, 1, 23, 40), (32, 1, 90, 160)])
def test_depthwise(dev, dtype, C, stride, H, W):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, H, W, C, generator=g)
    w = torch.randn(3, 3, C, generator=g) * 0.3
    if dtype == torch.bfloat16:  # the oracle sees the bf16-rounded activations (dw weights stay fp32)
        x = x.to(torch.bfloat16).float()
    xo = x.clone().requires_grad_(True)
    wo = w.clone().requires_grad_(True)
    yo = onet.dwconv(xo.permute(0, 3, 1, 2), wo, stride).permute(0, 2, 3, 1)
    gy = torch.randn(yo.shape, generator=g)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).float()
    (yo * gy).sum().backward()

    xd = x.to(dev, dtype).requires_grad_(True)
    wd = _param(w, dev)
    yd = ops.dw3x3(xd, wd, stride)
    assert yd.shape == yo.shape
    yd.backward(gy.to(dev, dtype))
    _close(yd, yo, dtype, scale=3)
    _close(xd.grad, xo.grad, dtype, scale=3)
    npix = x.shape[0] * yo.shape[1] * yo.shape[2]   # filter gradient = sum over npix products
    _close(wd._rod_grad, wo.grad, dtype, scale=max(10 if dtype == torch.bfloat16 else 3, np.sqrt(npix) / 8))


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('ks,Cin,Cout,NHW', [(1, 16, 96, None), (1, 96, 24, None), (1, 64, 128, None), (1, 40, 66, None),
                                             (3, 3, 32, None), (3, 3, 32, (1, 5, 128)), (3, 128, 128, None), (3, 24, 24, None), (3, 99, 99, None),
                                             (1, 320, 1920, None), (1, 24, 144, (2, 45, 80)), (1, 32, 192, (2, 23, 40)),
                                             (1, 96, 160, (2, 23, 40)), (1, 64, 256, (1, 30, 41)),
                                             (3, 36, 36, (2, 3, 5)), (1, 1920, 320, (2, 3, 5)),
                                             (3, 128, 128, (2, 3, 5)), (3, 128, 128, (2, 5, 9)),
                                             (1, 256, 128, (2, 3, 5)), (1, 128, 36, (2, 3, 5)),
                                             (3, 36, 36, (2, 2, 3)), (3, 128, 128, (2, 2, 3)), (1, 256, 128, (2, 2, 3)),
                                             (1, 128, 36, (2, 2, 3)), (3, 36, 36, (2, 1, 2))])
def test_conv(dev, dtype, ks, Cin, Cout, NHW):
    g = torch.Generator().manual_seed(2)
    N, H, W = NHW or (2, 7, 11)
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(Cout, ks, ks, Cin, generator=g) / np.sqrt(ks * ks * Cin)
    b = torch.randn(Cout, generator=g) * 0.1
    if dtype == torch.bfloat16:  # compare against the oracle on the bf16-rounded operands
        x = x.to(torch.bfloat16).float()
        w = w.to(torch.bfloat16).float()
    xo = x.clone().requires_grad_(True)
    wo = w.clone().requires_grad_(True)
    bo = b.clone().requires_grad_(True)
    yo = onet.conv(xo.permute(0, 3, 1, 2), wo, bo).permute(0, 2, 3, 1)
    gy = torch.randn(yo.shape, generator=g)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).float()
    (yo * gy).sum().backward()

    xd = x.to(dev, dtype).requires_grad_(True)
    wd, bd = _param(w, dev), _param(b, dev)
    yd = ops.conv2d(xd, wd, bd, ks)
    yd.backward(gy.to(dev, dtype))
    _close(yd, yo, dtype, scale=5)
    _close(xd.grad, xo.grad, dtype, scale=5)
    _close(wd._rod_grad, wo.grad, dtype, scale=20, rtol=1e-4 if dtype == torch.float32 else 2e-2)
    _close(bd._rod_grad, bo.grad, dtype, scale=20)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('act', [ops.ROD_ACT_NONE, ops.ROD_ACT_RELU6, ops.ROD_ACT_LEAKY])
@pytest.mark.parametrize('C,gamma,res', [(32, True, False), (24, True, True), (20, False, False), (66, False, False)])
def test_batchnorm(dev, dtype, act, C, gamma, res):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(3, 9, 10, C, generator=g) * 2 + 3  # non-zero mean exercises the pivot
    if dtype == torch.bfloat16:
        x = x.to(torch.bfloat16).float()
    ga = torch.rand(C, generator=g) + 0.5 if gamma else None
    be = torch.randn(C, generator=g) * 0.2
    r = torch.randn(x.shape, generator=g) if res else None
    if r is not None and dtype == torch.bfloat16:
        r = r.to(torch.bfloat16).float()
    mm = torch.randn(C, generator=g) * 0.1
    mv = torch.rand(C, generator=g) + 0.5
    decay = 0.997

    xo = x.clone().requires_grad_(True)
    gao = ga.clone().requires_grad_(True) if gamma else None
    beo = be.clone().requires_grad_(True)
    mov = {}
    yo = onet.batch_norm(xo.permute(0, 3, 1, 2), gao, beo, mm, mv, True, decay, 1e-3, mov, 'bn')
    yo = {ops.ROD_ACT_NONE: lambda t: t, ops.ROD_ACT_RELU6: onet.relu6, ops.ROD_ACT_LEAKY: onet.leaky}[act](yo)
    yo = yo.permute(0, 2, 3, 1)
    if res:
        yo = yo + r
    gy = torch.randn(yo.shape, generator=g)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).float()
    (yo * gy).sum().backward()

    xd = x.to(dev, dtype).requires_grad_(True)
    gad = _param(ga, dev) if gamma else None
    bed = _param(be, dev)
    mmd, mvd = mm.clone().to(dev), mv.clone().to(dev)
    rd = r.to(dev, dtype).requires_grad_(True) if res else None
    yd = ops.bn_act(xd, gad, bed, mmd, mvd, act, True, decay, 1e-3, rd)
    yd.backward(gy.to(dev, dtype))
    _close(yd, yo, dtype, scale=5)
    _close(mmd, mov['bn/moving_mean'], torch.float32)
    _close(mvd, mov['bn/moving_variance'], torch.float32)
    _close(xd.grad, xo.grad, dtype, scale=5)
    _close(bed._rod_grad, beo.grad, dtype, scale=50, rtol=1e-4 if dtype == torch.float32 else 3e-2)
    if gamma:
        _close(gad._rod_grad, gao.grad, dtype, scale=50, rtol=1e-4 if dtype == torch.float32 else 3e-2)
    if res:
        _close(rd.grad, gy, dtype)

    # inference: moving statistics
    with torch.no_grad():
        ye = ops.bn_act(x.to(dev, dtype), gad, bed, mmd, mvd, act, False, decay)
        yeo = onet.batch_norm(x.permute(0, 3, 1, 2), ga, be, mmd.cpu(), mvd.cpu(), False, decay)
        yeo = {ops.ROD_ACT_NONE: lambda t: t, ops.ROD_ACT_RELU6: onet.relu6, ops.ROD_ACT_LEAKY: onet.leaky}[act](
            yeo).permute(0, 2, 3, 1)
    _close(ye, yeo, dtype, scale=5)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('ks,Cin,Cout,NHW', [(1, 16, 96, (2, 45, 80)), (3, 128, 128, (2, 3, 5)), (3, 36, 36, (2, 10, 18)),
                                             (1, 64, 256, (1, 30, 41)), (3, 3, 32, (1, 20, 30)), (3, 3, 32, (2, 9, 256)),
                                             (1, 320, 1920, (2, 3, 5)), (1, 24, 144, (2, 23, 40))])
def test_conv_epilogue_bn_stats(dev, dtype, ks, Cin, Cout, NHW):
    """BatchNorm statistics reduced in the conv epilogue (rod_conv_fwd stat_parts ->
    rod_bn_finalize) against the separate statistics pass (rod_bn_stats) on the same conv
    output: normalised outputs and moving statistics agree to fp32 rounding."""
    g = torch.Generator().manual_seed(4)
    N, H, W = NHW
    x = (torch.randn(N, H, W, Cin, generator=g) + 0.5).to(dev, dtype)
    w = (torch.randn(Cout, ks, ks, Cin, generator=g) / np.sqrt(ks * ks * Cin)).to(dev)
    b = (torch.randn(Cout, generator=g) * 0.3).to(dev)
    be = torch.zeros(Cout, device=dev)
    y1, parts = ops.conv2d(x, w, b, ks, want_stats=True)
    y2 = ops.conv2d(x, w, b, ks)
    assert torch.equal(y1, y2)
    mm1, mv1 = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
    mm2, mv2 = mm1.clone(), mv1.clone()
    z1 = ops.bn_act(y1, None, be, mm1, mv1, ops.ROD_ACT_NONE, True, 0.9, 1e-3, parts=parts)
    z2 = ops.bn_act(y2, None, be, mm2, mv2, ops.ROD_ACT_NONE, True, 0.9, 1e-3)
    torch.testing.assert_close(mm1, mm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mv1, mv2, rtol=1e-5, atol=1e-6)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(z1.float(), z2.float(), **tol)


@pytest.mark.parametrize('Cin,Cout,NHW', [(24, 144, (2, 181, 321)), (16, 96, (1, 257, 259)), (32, 192, (2, 181, 183)),
                                           (64, 96, (3, 97, 227)), (40, 144, (1, 256, 263)), (8, 192, (1, 259, 255)),
                                           (64, 384, (1, 257, 257)), (96, 576, (1, 256, 257))])
def test_pw_stream_expand(dev, Cin, Cout, NHW):
    """The streaming 1x1 forward (pw_stream_kernel: bf16, no bias, K <= 64, Cout % 16 == 0,
    M >= 65536; M here not a multiple of the 128-row part tile) against the oracle conv, and its
    statistics parts against the separate statistics pass (ref conv_blocks.py:264-271 expand +
    BatchNorm).  ROD_PW_STREAM=0 would route these shapes to the tiled kernel."""
    g = torch.Generator().manual_seed(14)
    N, H, W = NHW
    x = (torch.randn(N, H, W, Cin, generator=g) + 0.5).to(torch.bfloat16).float()
    w = (torch.randn(Cout, 1, 1, Cin, generator=g) / np.sqrt(Cin)).to(torch.bfloat16).float()
    yo = onet.conv(x.permute(0, 3, 1, 2).double(), w.double(), None).permute(0, 2, 3, 1)
    xd = x.to(dev, torch.bfloat16)
    y1, parts = ops.conv2d(xd, w.to(dev), None, 1, want_stats=True)
    y2 = ops.conv2d(xd, w.to(dev), None, 1)
    assert torch.equal(y1, y2)
    # fp32 accumulation of exact bf16 products, rounded once to bf16
    err = (y1.double().cpu() - yo).abs().max() / yo.abs().max()
    assert err <= 2 ** -8, float(err)
    be = torch.zeros(Cout, device=dev)
    mm1, mv1 = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
    mm2, mv2 = mm1.clone(), mv1.clone()
    z1 = ops.bn_act(y1, None, be, mm1, mv1, ops.ROD_ACT_NONE, True, 0.9, 1e-3, parts=parts)
    z2 = ops.bn_act(y2, None, be, mm2, mv2, ops.ROD_ACT_NONE, True, 0.9, 1e-3)
    torch.testing.assert_close(mm1, mm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mv1, mv2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(z1.float(), z2.float(), rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('C,stride,H,W', [(144, 1, 45, 80), (96, 2, 90, 161), (6, 1, 13, 17), (960, 1, 3, 5),
                                          (32, 1, 33, 70)])
def test_dw_epilogue_bn_stats(dev, dtype, C, stride, H, W):
    """Depthwise forward with the BatchNorm statistics reduced in its epilogue agrees with
    the separate statistics pass on the same output."""
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(2, H, W, C, generator=g) + 0.3).to(dev, dtype)
    w = (torch.randn(3, 3, C, generator=g) * 0.3).to(dev)
    y1, parts = ops.dw3x3(x, w, stride, want_stats=True)
    y2 = ops.dw3x3(x, w, stride)
    assert torch.equal(y1, y2)
    be = torch.zeros(C, device=dev)
    mm1, mv1 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    mm2, mv2 = mm1.clone(), mv1.clone()
    z1 = ops.bn_act(y1, None, be, mm1, mv1, ops.ROD_ACT_NONE, True, 0.9, 1e-3, parts=parts)
    z2 = ops.bn_act(y2, None, be, mm2, mv2, ops.ROD_ACT_NONE, True, 0.9, 1e-3)
    torch.testing.assert_close(mm1, mm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mv1, mv2, rtol=1e-5, atol=1e-6)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(z1.float(), z2.float(), **tol)


def test_head_chain_small_level(dev):
    """One refine head (catch_net.py:276-342) on a 2x3 map, B=2 (M = 12 rows): conv1x1 ->
    BN -> leaky -> conv3x3 -> BN -> leaky -> conv1x1 -> BN -> leaky -> conv3x3 -> BN -> leaky,
    with the epilogue statistics, against the oracle chain in fp32 (forward and every grad)."""
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 2, 3, 256, generator=g)
    chans = [(256, 128, 1), (128, 128, 3), (128, 36, 1), (36, 36, 3)]
    Ws = [torch.randn(co, k, k, ci, generator=g) / np.sqrt(k * k * ci) for ci, co, k in chans]
    Bs = [torch.randn(co, generator=g) * 0.1 for _, co, _ in chans]
    Be = [torch.randn(co, generator=g) * 0.1 for _, co, _ in chans]
    # oracle
    Wo = [w.clone().requires_grad_(True) for w in Ws]
    Bo = [b.clone().requires_grad_(True) for b in Bs]
    Beo = [b.clone().requires_grad_(True) for b in Be]
    h = x.permute(0, 3, 1, 2)
    for i in range(4):
        h = onet.conv(h, Wo[i], Bo[i])
        h = onet.leaky(onet.batch_norm(h, None, Beo[i], torch.zeros(h.shape[1]), torch.ones(h.shape[1]), True,
                                       0.999, 1e-3, {}, 'b%d' % i))
    gy = torch.randn(h.shape, generator=g)
    (h * gy).sum().backward()
    # librod
    Wd = [_param(w, dev) for w in Ws]
    Bd = [_param(b, dev) for b in Bs]
    Bed = [_param(b, dev) for b in Be]
    hd = x.to(dev).requires_grad_(True)
    t = hd
    for i, (ci, co, k) in enumerate(chans):
        t, st = ops.conv2d(t, Wd[i], Bd[i], k, want_stats=True)
        t = ops.bn_act(t, None, Bed[i], torch.zeros(co, device=dev), torch.ones(co, device=dev), ops.ROD_ACT_LEAKY,
                       True, 0.999, 1e-3, parts=st)
    t.backward(gy.permute(0, 2, 3, 1).contiguous().to(dev))
    _close(t, h.permute(0, 2, 3, 1), torch.float32, scale=10)
    for i in range(4):
        _close(Bed[i]._rod_grad, Beo[i].grad, torch.float32, scale=10, rtol=1e-4)
        _close(Wd[i]._rod_grad, Wo[i].grad, torch.float32, scale=10, rtol=1e-4)
        _close(Bd[i]._rod_grad, Bo[i].grad, torch.float32, scale=10, rtol=1e-4)


def _anchors(H, W):
    init = oa.init_anchor(6, (H, W))
    chain = oa.feat_sizes((H, W), [s for (_, s, _, _, _) in onet.SPEC])
    return [oa.anchors_one_layer((H, W), chain[t - 1], init[i]) for i, t in enumerate(onet.TAPS)]


def _random_gt(rng, B, G, degenerate=False):
    n = rng.integers(1, G + 1, size=B)
    n[0] = G
    cy = rng.uniform(0.05, 0.95, (B, G))
    cx = rng.uniform(0.05, 0.95, (B, G))
    h = np.exp(rng.uniform(np.log(0.01), np.log(0.6), (B, G)))
    w = np.exp(rng.uniform(np.log(0.01), np.log(0.6), (B, G)))
    corner = np.stack([cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2], -1).clip(0, 1).astype(np.float32)
    if degenerate:
        corner[1, 0, 2] = corner[1, 0, 0]  # zero-height box in image 1
    labels = rng.choice([1, 2, 3, 4, 6, 8, 10], size=(B, G)).astype(np.int32)
    return corner, labels, n.astype(np.int32)


@pytest.mark.parametrize('H,W,degenerate', [(300, 300, False), (418, 418, False), (300, 300, True)])
def test_match_anchors_bit_exact(dev, H, W, degenerate):
    from utils import net_tools as nt
    import utils.common_tools as ct
    rng = np.random.default_rng(7)
    B, G = 3, 24
    corner, labels, n = _random_gt(rng, B, G, degenerate)
    anchors = _anchors(H, W)
    center_d = ct.cornerBboxes_2_centerBboxes(torch.from_numpy(corner).to(dev))
    center_o = ot.corner_to_center(corner)
    np.testing.assert_array_equal(center_d.cpu().numpy(), center_o)  # box conversion is bit-exact
    res = nt.refine_groundtruth(anchors, center_d, torch.from_numpy(labels).to(dev), config.refine_method.JACCARD_BIGGER,
                                n_boxes=torch.from_numpy(n).to(dev))
    gt_l, cb_l, lb_l, pm_l = res
    total_pos = 0
    for b in range(B):
        og, oc, ol, op = ot.refine_groundtruth(anchors, center_o[b, :n[b]], labels[b, :n[b]],
                                               config.refine_pos_jac_val_all_layers)
        for l in range(6):
            np.testing.assert_array_equal(pm_l[l][b].cpu().numpy(), op[l])
            np.testing.assert_array_equal(lb_l[l][b].cpu().numpy(), ol[l])
            np.testing.assert_array_equal(cb_l[l][b].cpu().numpy(), oc[l])
            np.testing.assert_array_equal(gt_l[l][b].cpu().numpy(), og[l])  # incl. NaN positions
            total_pos += int(op[l].sum())
    assert total_pos > 50


@pytest.mark.parametrize('H,W', [(300, 300), (418, 418)])
@pytest.mark.parametrize('degenerate', [False, True])
def test_match_anchors_nearest_neighbor_bit_exact(dev, H, W, degenerate):
    """refine_method.NEAREST_NEIGHBOR (net_tools.py:354-380): every anchor positive, matched to
    the box of least squared encoded distance; offsets / boxes / labels bit-exact vs the oracle
    (incl. the NaN poisoning of a zero-size box, as in JACCARD_BIGGER)."""
    from utils import net_tools as nt
    rng = np.random.default_rng(17)
    B, G = 2, 16
    corner, labels, n = _random_gt(rng, B, G, degenerate)
    anchors = _anchors(H, W)
    center_o = ot.corner_to_center(corner)
    res = nt.refine_groundtruth(anchors, torch.from_numpy(center_o).to(dev), torch.from_numpy(labels).to(dev),
                                config.refine_method.NEAREST_NEIGHBOR, n_boxes=torch.from_numpy(n).to(dev))
    gt_l, cb_l, lb_l, pm_l = res
    for b in range(B):
        og, oc, ol, op = ot.refine_groundtruth_nn(anchors, center_o[b, :n[b]], labels[b, :n[b]])
        for l in range(6):
            np.testing.assert_array_equal(pm_l[l][b].cpu().numpy(), op[l])
            np.testing.assert_array_equal(lb_l[l][b].cpu().numpy(), ol[l])
            np.testing.assert_array_equal(cb_l[l][b].cpu().numpy(), oc[l])
            np.testing.assert_array_equal(gt_l[l][b].cpu().numpy(), og[l])


def test_refine_loss(dev):
    from utils import net_tools as nt
    rng = np.random.default_rng(11)
    H = W = 300
    B, G = 2, 16
    corner, labels, n = _random_gt(rng, B, G)
    anchors = _anchors(H, W)
    center = torch.from_numpy(ot.corner_to_center(corner)).to(dev)
    tg = nt.refine_groundtruth(anchors, center, torch.from_numpy(labels).to(dev), config.refine_method.JACCARD_BIGGER,
                               n_boxes=torch.from_numpy(n).to(dev))
    g = torch.Generator().manual_seed(5)
    outs = [torch.randn(B, *a[0].shape[:2], a[2].shape[0], 4, generator=g) for a in anchors]
    outs_d = [o.to(dev).requires_grad_(True) for o in outs]
    loss = nt.refine_loss(outs_d, tg[0], tg[3], targets=tg)
    loss.backward()
    gts = [t.cpu().numpy() for t in tg[0]]
    pms = [t.cpu().numpy() for t in tg[3]]
    per, tot = ot.refine_loss([o.numpy() for o in outs], gts, pms, B)
    np.testing.assert_allclose(nt.refine_loss.last_per_layer[:6].detach().cpu().numpy(), per, rtol=1e-5)
    np.testing.assert_allclose(loss.item(), tot, rtol=1e-5)
    grads = ot.refine_loss_grad([o.numpy() for o in outs], gts, pms, B)
    for gd, go in zip(outs_d, grads):
        np.testing.assert_allclose(gd.grad.cpu().numpy(), go, rtol=1e-6, atol=1e-7)
    # the per-layer list path gives the same loss
    loss2 = nt.refine_loss([o.detach() for o in outs_d], tg[0], tg[3])
    assert loss2.item() == loss.item()


def test_sgd_clip_and_normalize(dev):
    g = torch.Generator().manual_seed(9)
    p = torch.randn(1003, generator=g)
    gr = torch.randn(1003, generator=g) * 10
    pd, gd = p.to(dev), gr.to(dev)
    ops.sgd_clip_(pd, gd, 1e-2, 5.0)
    ref = (p.numpy() - np.float32(1e-2) * np.clip(gr.numpy(), -5, 5)).astype(np.float32)
    np.testing.assert_array_equal(pd.cpu().numpy(), ref)
    # tf.clip_by_value keeps a NaN gradient NaN (Eigen max/min), so the variable turns NaN;
    # +-inf clip to +-5 (vector body and the scalar tail both)
    for n in (8, 7):
        p2 = torch.ones(n)
        g2 = torch.tensor([float('nan'), float('inf'), -float('inf'), 1.0, 0.5, -7.0, float('nan'), 2.0][:n])
        pd2 = p2.to(dev)
        ops.sgd_clip_(pd2, g2.to(dev), 0.5, 5.0)
        got = pd2.cpu().numpy()
        assert np.isnan(got[0]) and (n < 7 or np.isnan(got[6]))
        np.testing.assert_array_equal(got[1:6], np.float32([1 - 2.5, 1 + 2.5, 0.5, 0.75, 1 + 2.5]))
    img = torch.randint(0, 256, (2, 5, 7, 3), dtype=torch.uint8, generator=g)
    out = ops.normalize_image(img.to(dev))
    k = np.float32(2.0 / 255.0)
    np.testing.assert_array_equal(out.cpu().numpy(), k * img.numpy().astype(np.float32) - np.float32(1.0))


def _pending_pair(dev, dtype, shape, act, gamma, seed):
    """Two identical leaf pre-BatchNorm tensors y (for the fused and the materialised path) and
    the BatchNorm parameters; statistics from rod_bn_stats (no moving-average update)."""
    g = torch.Generator().manual_seed(seed)
    C = shape[-1]
    y0 = (torch.randn(*shape, generator=g) * 2 + 0.7).to(dev, dtype)
    ga = _param(torch.rand(C, generator=g) + 0.5, dev) if gamma else None
    be = _param(torch.randn(C, generator=g) * 0.3, dev)
    return y0, ga, be


def _fused_vs_materialised(dev, dtype, shape, act, gamma, consumer, seed):
    """consumer(x) on ops.Pending (BatchNorm-apply in the load prologue, BatchNorm backward in
    the consumer's backward) against consumer(materialize(Pending)) (rod_bn_apply + the plain
    kernel): forward and the consumer's weight gradient bit-exact; the gradients of y / gamma /
    beta agree to fp32 summation order (the fused path reduces the BatchNorm-backward sums in
    the backward-data epilogue, per 128-row tile or per block, rod_bn_bwd_finalize) — for bf16
    dy that is at most one bf16 rounding step."""
    y0, ga, be = _pending_pair(dev, dtype, shape, act, gamma, seed)
    outs = []
    for fused in (True, False):
        y = y0.clone().requires_grad_(True)
        for p in (ga, be):
            if p is not None:
                p._rod_grad.zero_()
        p = ops.bn_pending(y, ga, be, None, None, act, True, 0.9, 1e-3)
        out, wgrad = consumer(p if fused else ops.materialize(p))
        gy = torch.randn(out.shape, generator=torch.Generator().manual_seed(seed + 1)).to(dev, dtype)
        out.backward(gy)
        outs.append((out.detach().clone(), y.grad.clone(), None if ga is None else ga._rod_grad.clone(),
                     be._rod_grad.clone(), wgrad().clone()))
    for i, (a, b) in enumerate(zip(*outs)):
        if a is None:
            continue
        if i in (0, 4):
            assert torch.equal(a, b), (a.float() - b.float()).abs().max()
        else:
            af, bf = a.float().cpu(), b.float().cpu()
            scale = float(bf.abs().max()) + 1e-30
            tol = 1e-5 if (i > 1 or dtype == torch.float32) else 8e-3
            torch.testing.assert_close(af, bf, rtol=tol, atol=tol * scale)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('ks,Cin,Cout,NHW,act,gamma', [
    (1, 144, 24, (2, 23, 40), ops.ROD_ACT_RELU6, True),      # project conv (dw BN prologue)
    (1, 960, 160, (2, 3, 5), ops.ROD_ACT_RELU6, True),       # deep project: split-K path
    (3, 128, 128, (2, 10, 18), ops.ROD_ACT_LEAKY, False),    # head 3x3 after 1x1 (beta only)
    (1, 128, 36, (2, 10, 18), ops.ROD_ACT_LEAKY, False),     # head 1x1 -> k*A
    (3, 36, 36, (2, 10, 18), ops.ROD_ACT_LEAKY, False),      # head 3x3 over k*A (scalar A path)
    (3, 24, 24, (1, 3, 5), ops.ROD_ACT_LEAKY, False)])
def test_conv_bn_prologue(dev, dtype, ks, Cin, Cout, NHW, act, gamma):
    g = torch.Generator().manual_seed(11)
    w = _param(torch.randn(Cout, ks, ks, Cin, generator=g) / np.sqrt(ks * ks * Cin), dev)
    b = _param(torch.randn(Cout, generator=g) * 0.1, dev)

    def consumer(x):
        w._rod_grad.zero_()
        return ops.conv2d(x, w, b, ks), (lambda: w._rod_grad)
    _fused_vs_materialised(dev, dtype, NHW + (Cin,), act, gamma, consumer, 12)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('C,stride,H,W', [(96, 2, 45, 81), (144, 1, 23, 40), (32, 1, 30, 44), (36, 1, 9, 11),
                                          (6, 2, 13, 17), (960, 1, 3, 5)])
def test_dw_bn_prologue(dev, dtype, C, stride, H, W):
    g = torch.Generator().manual_seed(13)
    w = _param(torch.randn(3, 3, C, generator=g) * 0.3, dev)

    def consumer(x):
        w._rod_grad.zero_()
        return ops.dw3x3(x, w, stride), (lambda: w._rod_grad)
    _fused_vs_materialised(dev, dtype, (2, H, W, C), ops.ROD_ACT_RELU6, True, consumer, 14)


@pytest.mark.parametrize('hw,cin', [((2, 3), 256), ((20, 36), 96), ((40, 72), 192), ((40, 72), 64)])
def test_head_chain_nodes_match_float64(dev, hw, cin):
    """The refine head exactly as the product runs it (CatchNet._conv_bn: ops.conv2d_bn nodes,
    BatchNorm + leaky applied in the next conv's load prologue, one materialise at the end)
    on maps of the step's level sizes, fp32, against float64 — forward and every gradient."""
    g = torch.Generator().manual_seed(7)
    H, W = hw
    x = torch.randn(2, H, W, cin, generator=g)
    chans = [(cin, 128, 1), (128, 128, 3), (128, 24, 1), (24, 24, 3)]
    Ws = [torch.randn(co, k, k, ci, generator=g) / np.sqrt(k * k * ci) for ci, co, k in chans]
    Bs = [torch.randn(co, generator=g) * 0.1 for _, co, _ in chans]
    Be = [torch.randn(co, generator=g) * 0.1 for _, co, _ in chans]

    def oracle(dt):
        Wo = [w.to(dt).requires_grad_(True) for w in Ws]
        Beo = [b.to(dt).requires_grad_(True) for b in Be]
        h = x.to(dt).permute(0, 3, 1, 2)
        for i in range(4):
            h = onet.conv(h, Wo[i], Bs[i].to(dt))
            h = onet.leaky(onet.batch_norm(h, None, Beo[i], torch.zeros(h.shape[1], dtype=dt),
                                           torch.ones(h.shape[1], dtype=dt), True, 0.999, 1e-3, {}, 'b%d' % i))
        return h, Wo, Beo
    h64, W64, Be64 = oracle(torch.float64)
    h32, W32, Be32 = oracle(torch.float32)
    gy = torch.randn(h64.shape, generator=g) * (torch.rand(h64.shape, generator=g) < 0.02)
    (h64 * gy.double()).sum().backward()
    (h32 * gy).sum().backward()
    Wd = [_param(w, dev) for w in Ws]
    Bd = [_param(b, dev) for b in Bs]
    Bed = [_param(b, dev) for b in Be]
    t = x.to(dev)
    for i, (ci, co, k) in enumerate(chans):
        t = ops.conv2d_bn(t, Wd[i], Bd[i], k, None, Bed[i], torch.zeros(co, device=dev), torch.ones(co, device=dev),
                          ops.ROD_ACT_LEAKY, True, 0.999)
    t = ops.materialize(t)
    t.backward(gy.permute(0, 2, 3, 1).contiguous().to(dev))

    def ne(a, b):
        return float((a.detach().double().cpu() - b.detach().double()).abs().max() / b.detach().double().abs().max())
    rep = []
    assert ne(t, h64.permute(0, 2, 3, 1)) <= max(1e-5, 4 * ne(h32.permute(0, 2, 3, 1), h64.permute(0, 2, 3, 1)))
    for i in range(4):
        for got, r64, r32 in ((Wd[i]._rod_grad, W64[i].grad, W32[i].grad), (Bed[i]._rod_grad, Be64[i].grad,
                                                                            Be32[i].grad)):
            rep.append((i, ne(got, r64), ne(r32, r64)))
    print('head chain', hw, cin, ['%d %.2e/%.2e' % r for r in rep])
    for i, e, e32 in rep:
        assert e <= max(1e-4, 4 * e32), rep


@pytest.mark.parametrize('act', [ops.ROD_ACT_NONE, ops.ROD_ACT_RELU6])
def test_pw_stream_prologue(dev, act):
    """The streaming 1x1 forward with the BatchNorm-apply prologue (pw_stream_kernel PRO: the
    720p expand 16 -> 96 whose input is block 1's project BatchNorm left pending, no bias,
    M >= 65536) against writing the BatchNorm out first: forward bit-identical, gradients as the
    materialised path."""
    g = torch.Generator().manual_seed(21)
    w = _param(torch.randn(96, 1, 1, 16, generator=g) / 4.0, dev)

    def consumer(x):
        w._rod_grad.zero_()
        return ops.conv2d(x, w, None, 1), (lambda: w._rod_grad)
    _fused_vs_materialised(dev, torch.bfloat16, (1, 257, 259, 16), act, True, consumer, 22)


@pytest.mark.parametrize('nparts,C', [(1, 16), (700, 16), (5000, 16), (57600, 16), (3000, 96), (900, 200), (40000, 1280),
                                     (70000, 64)])
def test_bn_finalize_many_parts(dev, nparts, C, monkeypatch):
    """rod_bn_finalize over a producer's partial statistics (count, mean, M2 per part; one to
    70,000 parts, so one to three merge levels) against a float64 Chan merge, incl. empty parts;
    repeated calls on the same parts are bit-identical, and so are calls inside a replayed
    graph, calls on three streams at once, and the two-level merge in one launch (last-block
    hand-off) against the same two levels in two launches (ROD_MERGE_TWO_LAUNCH=1)."""
    from rod import _abi
    from rod.ops import workspace, stream
    g = torch.Generator().manual_seed(nparts + C)
    cnt = torch.randint(1, 129, (nparts, 1, C), generator=g).double()
    cnt[3::7] = 0.
    mu = torch.randn(nparts, 1, C, generator=g).double() * 0.5 + 3.0
    m2 = torch.rand(nparts, 1, C, generator=g).double() * cnt
    mu[cnt == 0] = 0.
    parts = torch.cat([cnt, mu, m2], 1).float()
    cd, md, qd = (t.double() for t in parts.unbind(1))
    N = cd.sum(0)
    mean = (cd * md).sum(0) / N
    M2 = (qd + cd * (md - mean) ** 2).sum(0)
    M = int(N.max())   # the call's M only scales the variance; use one M for every channel
    var = M2 / M
    pd = parts.to(dev)
    nb = _abi.query("rod_bn_finalize_workspace", nparts, C)
    ws = workspace(nb, dev) if nb else None

    def run():
        mo, ro = torch.empty(C, device=dev), torch.empty(C, device=dev)
        mm, mv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        _abi.call("rod_bn_finalize", pd, nparts, M, C, 1e-3, 0.9, mo, ro, mm, mv, ws, stream())
        return mo, ro, mm, mv

    a = run()
    torch.testing.assert_close(a[0].double().cpu(), mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a[1].double().cpu(), 1.0 / torch.sqrt(var.float().double() + 1e-3), rtol=1e-5, atol=1e-6)
    for _ in range(20):
        b = run()
        for u, v in zip(a, b):
            assert torch.equal(u, v)
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.cuda.graph(gr, stream=s):
        c = run()
    for _ in range(3):
        gr.replay()
        torch.cuda.synchronize()
        for u, v in zip(a, c):
            assert torch.equal(u, v)
    # three streams at once, each with its own workspace (distinct arrival counters)
    wss = [workspace(nb, dev) if nb else None for _ in range(3)]
    outs = []
    sts = [torch.cuda.Stream() for _ in range(3)]
    for st, w in zip(sts, wss):
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            for _ in range(4):
                mo, ro = torch.empty(C, device=dev), torch.empty(C, device=dev)
                mm, mv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
                _abi.call("rod_bn_finalize", pd, nparts, M, C, 1e-3, 0.9, mo, ro, mm, mv, w, stream())
                outs.append((mo, ro, mm, mv))
    torch.cuda.synchronize()
    for o in outs:
        for u, v in zip(a, o):
            assert torch.equal(u, v)
    monkeypatch.setenv('ROD_MERGE_TWO_LAUNCH', '1')
    d = run()
    torch.cuda.synchronize()
    for u, v in zip(a, d):
        assert torch.equal(u, v)
