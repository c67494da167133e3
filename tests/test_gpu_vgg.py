"""VGG-16 backbone (reference nets/backbone/vgg.py:67-137; `--backbone_name=vgg_16`) on the GPU:
the new kernels against PyTorch-CPU restatements, then one REFINE training step against the
float64 oracle (oracle/vgg.py) with the dropout masks the product drew.

Tolerances as in test_gpu_train.py: max pool, dropout and im2col / col2im are bit-exact
(pure data movement / one rounding); convs through the column matrix within fp32 GEMM
rounding; the step's outputs / loss / gradients within max(1e-4 / 2e-3, 4x the spread of the
fp32 oracle) of the float64 truth."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import config
from oracle import anchors as oa
from oracle import net as onet
from oracle import targets as ot
from oracle import vgg as ovgg
from rod import _abi, ops
from rod.data import synthetic_batch
from rod.trainer import Trainer

pytestmark = pytest.mark.gpu


def _nerr(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('hw', [(8, 12), (9, 13)])
def test_maxpool_matches_torch(dev, dtype, hw):
    g = torch.Generator().manual_seed(1)
    x = torch.randn((2, hw[0], hw[1], 16), generator=g)
    x = torch.where(x < 0, torch.zeros_like(x), x).to(dtype)   # relu-like input: tied zero windows
    xd = x.to(dev).requires_grad_(True)
    y = ops.max_pool2x2(xd)
    ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 2, 2)
    assert torch.equal(y.float().cpu(), ref.permute(0, 2, 3, 1))
    gy = torch.randn(y.shape, generator=g).to(dtype)
    y.backward(gy.to(dev))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.max_pool2d(xr, 2, 2).backward(gy.float().permute(0, 3, 1, 2))
    assert torch.equal(xd.grad.float().cpu(), xr.grad.permute(0, 2, 3, 1))   # first max wins, as TF / torch


def test_dropout_mask_and_gradient(dev):
    x = torch.randn((4, 13, 13, 64), device=dev)
    y, m = ops.dropout(x.requires_grad_(True), 0.5, True, seed=1234)
    frac = float(m.float().mean())
    assert 0.48 < frac < 0.52
    assert torch.equal(y, torch.where(m.bool(), x * 2, torch.zeros_like(x)))   # x / 0.5 * binary
    y2, m2 = ops.dropout(x, 0.5, True, seed=1234)
    assert torch.equal(m, m2)
    g = torch.randn_like(x)
    y.backward(g)
    assert torch.equal(x.grad, torch.where(m.bool(), g * 2, torch.zeros_like(g)))
    yi, mi = ops.dropout(x, 0.5, False)
    assert mi is None and yi is x


@pytest.mark.parametrize('geo', [(2, 'VALID', 1, 13, 9), (1, 'VALID', 0, 6, 7), (2, 'VALID', 1, 4, 4)])
def test_strided_conv_matches_torch(dev, geo):
    """pad2d + VALID stride-2 (blocks 8, 9) and VALID stride-1 (block 10) 3x3 convs through
    rod_im2col3x3 / rod_col2im3x3 and the ksize-1 GEMMs, relu after, fp32."""
    s, padding, pad, H, W = geo
    g = torch.Generator().manual_seed(2)
    Cin, Cout = 32, 48
    x = torch.randn((2, H, W, Cin), generator=g)
    w = torch.randn((Cout, 3, 3, Cin), generator=g) * 0.1
    b = torch.randn(Cout, generator=g) * 0.1
    xd, wd, bd = x.to(dev).requires_grad_(True), w.to(dev).requires_grad_(True), b.to(dev).requires_grad_(True)
    gw = torch.zeros_like(wd)
    gb = torch.zeros_like(bd)
    wd._rod_grad, bd._rod_grad = gw, gb
    p = ops.conv2d_act(xd, wd, bd, 3, ops.ROD_ACT_RELU, s, padding, pad)
    y = ops.materialize(p)
    xr, wr, br = x.double().requires_grad_(True), w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = torch.relu(F.conv2d(F.pad(xr.permute(0, 3, 1, 2), (pad,) * 4), wr.permute(0, 3, 1, 2), br, s))
    ref = ref.permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert _nerr(y, ref) < 1e-5
    gy = torch.randn(y.shape, generator=g)
    y.backward(gy.to(dev))
    ref.backward(gy.double())
    assert _nerr(xd.grad, xr.grad) < 1e-5
    assert _nerr(gw, wr.grad) < 1e-5 and _nerr(gb, br.grad) < 1e-5


def _oracle_refine(tr, img, corner, labels, n, H, W, B, dt, masks, buffers):
    P = {k: v.detach().cpu().clone().to(dt).requires_grad_(v.requires_grad) for k, v in tr.net.store.params.items()}
    Bf = {k: v.clone().to(dt) for k, v in buffers.items()}
    x = torch.from_numpy(np.float32(2.0 / 255.0) * img.cpu().numpy().astype(np.float32) - np.float32(1.0)).to(dt)
    mov = {}
    refine = ovgg.forward(x, P, Bf, True, masks=masks, moving=mov)
    init = oa.init_anchor(6, (H, W))
    sizes = config.feat_sizes((H, W), 'vgg_16')
    anchors = [oa.anchors_one_layer((H, W), sizes['layer_%d' % (i + 1)], init[i]) for i in range(6)]
    center = ot.corner_to_center(corner.cpu().numpy())
    loss = 0.
    for b in range(B):
        nb = int(n[b])
        gts, _, _, pms = ot.refine_groundtruth(anchors, center[b, :nb], labels.cpu().numpy()[b, :nb],
                                               config.refine_pos_jac_val_all_layers)
        for l in range(6):
            d = (torch.from_numpy(gts[l]).to(dt) - refine[l][b]) * torch.from_numpy(pms[l]).to(dt)
            ad = d.abs()
            loss = loss + (0.5 * ((ad - 1) * torch.clamp(ad, max=1.0) + ad)).sum() / B
    loss.backward()
    return P, mov, refine, loss


def test_vgg_refine_step_matches_oracle(dev):
    """One REFINE step (train.py:250-327) with --backbone_name=vgg_16 at 288x512 (the smallest
    size whose block-10 VALID conv has an output: 1x2), fp32."""
    H, W, B = 288, 512, 1
    tr = Trainer((H, W), B, dtype=torch.float32, device=dev, learning_rate=1e-2, seed=3, backbone_name='vgg_16')
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=9)
    from nets.catch_net import factory
    import utils.net_tools as nt
    from utils.common_tools import cornerBboxes_2_centerBboxes
    buffers0 = {k: v.detach().cpu().clone() for k, v in tr.net.store.buffers.items()}   # before the update
    x = ops.normalize_image(img, torch.float32)
    tg = nt.refine_groundtruth(tr.anchors, cornerBboxes_2_centerBboxes(corner), labels,
                               config.refine_method.JACCARD_BIGGER, n_boxes=n)
    out = factory(x, 'vgg_16', True, tr.config_dict, torch.float32, net=tr.net).get_output()
    masks = [m.cpu() for m in tr.net.backbone.last_dropout_masks]
    assert len(masks) == 2 and all(0.4 < float(m.float().mean()) < 0.6 for m in masks)
    loss = nt.refine_loss(out, tg[0], tg[3], targets=tg)
    loss.backward()
    P32, mov32, ref32, loss32 = _oracle_refine(tr, img, corner, labels, n, H, W, B, torch.float32, masks, buffers0)
    P64, mov64, ref64, loss64 = _oracle_refine(tr, img, corner, labels, n, H, W, B, torch.float64, masks, buffers0)
    for l, (a, o32, o64) in enumerate(zip(out, ref32, ref64)):
        assert tuple(a.shape) == tuple(o64.shape), (l, a.shape, o64.shape)
        assert _nerr(a, o64) <= max(1e-4, 4 * _nerr(o32, o64)), (l, _nerr(a, o64), _nerr(o32, o64))
    assert abs(loss.item() - loss64.item()) <= max(1e-4, 4 * abs(loss32.item() - loss64.item()) /
                                                   abs(loss64.item())) * abs(loss64.item())
    for k, v in mov64.items():   # the heads' BatchNorm moving statistics
        assert _nerr(tr.net.store.buffers[k], v) <= max(1e-4, 4 * _nerr(mov32[k], v)), k
    bad = []
    for name, p in tr.net.store.params.items():
        g64, g32 = P64[name].grad, P32[name].grad
        if g64 is None or g64.abs().max() == 0:
            continue
        if name.endswith('/biases') and name.startswith('refine') and \
                float(g64.abs().max()) <= 1e-6 * float(P64[name.replace('/biases', '/weights')].grad.abs().max()):
            continue   # head conv bias before a training-mode BatchNorm: exactly zero gradient
        e, e32 = _nerr(p._rod_grad, g64), _nerr(g32, g64)
        if e > max(2e-3, 4 * e32):
            bad.append((name, e, e32))
    assert not bad, bad[:10]


def test_vgg_step_graphed_draws_fresh_dropout_masks(dev):
    """Trainer.step_graphed with the vgg_16 backbone (dropout in training, vgg.py:106, 111) runs
    eager: a replayed graph would reuse one dropout seed forever.  Over three calls it matches
    three eager steps bit for bit (same seed sequence), draws a new mask every step, and
    advances opt.global_step once per call."""
    H, W, B = 288, 512, 1
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=9)
    ta = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=3, backbone_name='vgg_16')
    tb = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=3, backbone_name='vgg_16')
    ops._DROPOUT_CALLS[0] = 0
    masks_a = []
    for _ in range(3):
        la = ta.step(img, corner, labels, n)
        masks_a.append(ta.net.backbone.last_dropout_masks[0].clone())
    ops._DROPOUT_CALLS[0] = 0
    for _ in range(3):
        lb = tb.step_graphed(img, corner, labels, n)
    torch.cuda.synchronize()
    assert getattr(tb, '_graph', None) is None and tb._dropout_seen
    assert not torch.equal(masks_a[0], masks_a[1]) and not torch.equal(masks_a[1], masks_a[2])
    assert torch.equal(tb.net.backbone.last_dropout_masks[0], masks_a[2])
    assert torch.equal(ta.net.store.flat, tb.net.store.flat) and torch.equal(la[0], lb[0])
    assert ta.opt.global_step == tb.opt.global_step == 3
