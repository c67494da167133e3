"""process_backbone_method.PREORDER_MSF (reference nets/catch_net.py:115-152) + se_block
(nets/attention_module.py:3-33) on the GPU: pad / space_to_depth bit-exact against PyTorch,
the SE block forward / backward against a float64 PyTorch restatement, and one REFINE step
against the float64 oracle (oracle.net.feats_aug)."""
import numpy as np
import pytest
import torch

import config
from oracle import net as onet
from rod import ops
from rod.data import synthetic_batch
from rod.trainer import Trainer
from test_gpu_train import _nerr, _oracle_step

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_pad_and_space_to_depth_bit_exact(dev, dtype):
    g = torch.Generator().manual_seed(3)
    x = torch.randn((2, 9, 13, 16), generator=g).to(dtype)
    xd = x.to(dev).requires_grad_(True)
    y = ops.space_to_depth(ops.pad_top_left(xd, 3, 3), 4)
    ref = onet.space_to_depth(torch.nn.functional.pad(x.float().permute(0, 3, 1, 2), (3, 0, 3, 0)), 4)
    assert torch.equal(y.float().cpu(), ref.permute(0, 2, 3, 1))
    gy = torch.randn(y.shape, generator=g).to(dtype)
    y.backward(gy.to(dev))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    onet.space_to_depth(torch.nn.functional.pad(xr, (3, 0, 3, 0)), 4).backward(gy.float().permute(0, 3, 1, 2))
    assert torch.equal(xd.grad.float().cpu(), xr.grad.permute(0, 2, 3, 1))


@pytest.mark.parametrize('shape,sparse', [((3, 12, 20, 192), False), ((2, 40, 72, 192), True)])
def test_se_block_matches_float64(dev, shape, sparse):
    g = torch.Generator().manual_seed(4)
    N, H, W, C = shape
    x = torch.randn((N, H, W, C), generator=g)
    if sparse:   # non-negative activations and a gradient on a few rows, as in the REFINE step
        x = x.clamp(0, 6)
    w1, b1 = torch.randn((C, C // 8), generator=g) * 0.1, torch.randn(C // 8, generator=g) * 0.1
    w2, b2 = torch.randn((C // 8, C), generator=g) * 0.3, torch.randn(C, generator=g) * 0.1
    ps = [t.to(dev).requires_grad_(True) for t in (w1, b1, w2, b2)]
    slots = [torch.zeros_like(p) for p in ps]
    for p, s in zip(ps, slots):
        p._rod_grad = s
    xd = x.to(dev).requires_grad_(True)
    y = ops.se_block(xd, *ps)
    x64 = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    P64 = {'s/bottleneck_fc/kernel': w1.double().requires_grad_(True), 's/bottleneck_fc/bias': b1.double().requires_grad_(True),
           's/recover_fc/kernel': w2.double().requires_grad_(True), 's/recover_fc/bias': b2.double().requires_grad_(True)}
    ref = onet.se_block(x64, P64, 's').permute(0, 2, 3, 1)
    assert _nerr(y, ref) < 1e-5
    gy = torch.randn(y.shape, generator=g)
    if sparse:
        gy = gy * (torch.rand(y.shape[:3], generator=g) < 0.01)[..., None]
    y.backward(gy.to(dev))
    ref.backward(gy.double())
    print('dx', _nerr(xd.grad, x64.grad.permute(0, 2, 3, 1)), [(_nerr(s_, P64[k].grad)) for s_, k in zip(slots, P64)])
    assert _nerr(xd.grad, x64.grad.permute(0, 2, 3, 1)) < 1e-5
    for s, k in zip(slots, ('s/bottleneck_fc/kernel', 's/bottleneck_fc/bias', 's/recover_fc/kernel',
                            's/recover_fc/bias')):
        assert _nerr(s, P64[k].grad) < 1e-5, k


# Gradient floor of this step test: 5e-3 normwise (2e-3 in test_gpu_train.py).  Measured: the
# level-1 refine head here carries 3e-3 relative error in its weight gradient from activation
# kinks (the same head alone, fed a dense gradient, is within 1e-6 of float64:
# test_gpu_kernels.py::test_head_chain_nodes_match_float64), and every tensor upstream of it —
# the SE, the augmentation convs, layers 8-11 through the residual stream — inherits that
# 2-3.5e-3.  The SE block by itself is exact to 1e-7 (test_se_block_matches_float64); forward
# outputs and loss keep 1e-4.
GRAD_FLOOR = 5e-3


def test_preorder_msf_refine_step_matches_oracle(dev):
    """REFINE step with process_backbone_method=PREORDER_MSF at 320x576, fp32: outputs, loss and
    every gradient (backbone, the augmentation convs / BatchNorms / SE, refine heads) within
    max(1e-4 / 2e-3, 4x the fp32 oracle's spread) of the float64 oracle."""
    H, W, B = 320, 576, 2
    tr = Trainer((H, W), B, dtype=torch.float32, device=dev, learning_rate=1e-2, seed=6,
                 process_backbone_method=config.process_backbone_method.PREORDER_MSF)
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=12)
    P32, _, ref32, loss32 = _oracle_step(tr, img, corner, labels, n, H, W, B, torch.float32, msf=True)
    P64, _, ref64, loss64 = _oracle_step(tr, img, corner, labels, n, H, W, B, torch.float64, msf=True)
    # a second fp32 oracle with another convolution algorithm (oneDNN off) and the float64
    # truth under 1e-6 input noise: what any fp32 evaluation order can move (test_gpu_train.py)
    torch.backends.mkldnn.enabled = False
    try:
        P32b = _oracle_step(tr, img, corner, labels, n, H, W, B, torch.float32, msf=True)[0]
    finally:
        torch.backends.mkldnn.enabled = True
    # ReLU6 / leaky kinks: elements within fp32 rounding of zero flip their branch under ANY
    # evaluation order; where the REFINE gradient is concentrated on few rows (level 1: BN_1 /
    # Conv_1 of the refine head) one flip moves a tensor by percents — measured with noise
    Pp = [_oracle_step(tr, img, corner, labels, n, H, W, B, torch.float64, perturb=a, seed=s_, msf=True)[0]
          for s_ in (11, 12) for a in (1e-6, 1e-5)]
    from nets.catch_net import factory
    import utils.net_tools as nt
    from utils.common_tools import cornerBboxes_2_centerBboxes
    x = ops.normalize_image(img, torch.float32)
    tg = nt.refine_groundtruth(tr.anchors, cornerBboxes_2_centerBboxes(corner), labels,
                               config.refine_method.JACCARD_BIGGER, n_boxes=n)
    out = factory(x, 'mobilenet_v2', True, tr.config_dict, torch.float32, net=tr.net).get_output()
    loss = nt.refine_loss(out, tg[0], tg[3], targets=tg)
    loss.backward()
    for l, (a, o32, o64) in enumerate(zip(out, ref32, ref64)):
        assert _nerr(a, o64) <= max(1e-4, 4 * _nerr(o32, o64)), (l, _nerr(a, o64), _nerr(o32, o64))
    assert abs(loss.item() - loss64.item()) <= max(1e-4, 4 * abs(loss32.item() - loss64.item()) /
                                                   abs(loss64.item())) * abs(loss64.item())
    bad, checked = [], 0
    for name, p in tr.net.store.params.items():
        g64, g32 = P64[name].grad, P32[name].grad
        if g64 is None or g64.abs().max() == 0:
            continue
        w = name.replace('/biases', '/weights')
        if name.endswith('/biases') and w in P64 and \
                float(g64.abs().max()) <= 1e-6 * float(P64[w].grad.abs().max()):
            continue   # conv bias before a training-mode BatchNorm: exactly zero gradient
        checked += 1
        e = _nerr(p._rod_grad, g64)
        e32 = max([_nerr(g32, g64), _nerr(P32b[name].grad, g64)] + [_nerr(pp[name].grad, g64) for pp in Pp])
        if e > max(GRAD_FLOOR, 4 * e32):
            bad.append((name, e, e32))
    assert checked > 100 and not bad, bad[:10]
    assert any(k.startswith('backbone/se_aug') for k in tr.net.store.params)
