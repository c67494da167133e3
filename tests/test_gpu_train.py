"""End-to-end parity of one REFINE training step (train.py:250-327) against the oracle:
network outputs, moving statistics, loss, every parameter gradient and the SGD update.

Tolerances (normwise, max|a-b| / max|b|): fp32 forward outputs 1e-4 (north_star),
gradients 2e-3 (24 batch-normalised layers of fp32 reductions in a different order);
bf16 storage: loss within 3 %, gradients cosine similarity > 0.98 per tensor.
"""
import numpy as np
import pytest
import torch

import config
from oracle import anchors as oa
from oracle import net as onet
from oracle import targets as ot
from rod import ops
from rod.data import synthetic_batch
from rod.trainer import Trainer

pytestmark = pytest.mark.gpu


def _nerr(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _oracle_step(tr, img, corner, labels, n, H, W, B):
    P = {k: v.detach().cpu().clone().requires_grad_(v.requires_grad) for k, v in tr.net.store.params.items()}
    Bf = {k: v.detach().cpu().clone() for k, v in tr.net.store.buffers.items()}
    x = torch.from_numpy(np.float32(2.0 / 255.0) * img.cpu().numpy().astype(np.float32) - np.float32(1.0))
    mov = {}
    refine = onet.forward(x, P, Bf, True, moving=mov)
    init = oa.init_anchor(6, (H, W))
    chain = oa.feat_sizes((H, W), [s for (_, s, _, _, _) in onet.SPEC])
    anchors = [oa.anchors_one_layer((H, W), chain[t - 1], init[i]) for i, t in enumerate(onet.TAPS)]
    center = ot.corner_to_center(corner.cpu().numpy())
    gts = [[] for _ in range(6)]
    pms = [[] for _ in range(6)]
    for b in range(B):
        nb = int(n[b])
        g, _, _, p = ot.refine_groundtruth(anchors, center[b, :nb], labels.cpu().numpy()[b, :nb],
                                           config.refine_pos_jac_val_all_layers)
        for l in range(6):
            gts[l].append(g[l])
            pms[l].append(p[l])
    loss = 0.
    for l in range(6):
        y = torch.from_numpy(np.stack(gts[l]))
        m = torch.from_numpy(np.stack(pms[l])).float()
        d = (y - refine[l]) * m
        ad = d.abs()
        loss = loss + (0.5 * ((ad - 1) * torch.clamp(ad, max=1.0) + ad)).sum() / B
    loss.backward()
    return P, mov, refine, loss


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_refine_step_matches_oracle(dev, dtype):
    H, W, B = 64, 96, 2
    tr = Trainer((H, W), B, dtype=dtype, device=dev, learning_rate=1e-2, seed=1)
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=4)
    p0 = tr.net.store.flat.detach().clone()
    P, mov, refine_o, loss_o = _oracle_step(tr, img, corner, labels, n, H, W, B)

    # forward outputs through the drop-in factory API
    from nets.catch_net import factory
    with torch.no_grad():
        pass
    x = ops.normalize_image(img, dtype)
    import utils.net_tools as nt
    from utils.common_tools import cornerBboxes_2_centerBboxes
    tg = nt.refine_groundtruth(tr.anchors, cornerBboxes_2_centerBboxes(corner), labels,
                               config.refine_method.JACCARD_BIGGER, n_boxes=n)
    out = factory(x, 'mobilenet_v2', True, tr.config_dict, dtype, net=tr.net).get_output()
    loss = nt.refine_loss(out, tg[0], tg[3], targets=tg)
    loss.backward()
    if dtype == torch.float32:
        for a, b in zip(out, refine_o):
            assert _nerr(a, b) < 1e-4
        assert abs(loss.item() - loss_o.item()) <= 1e-4 * abs(loss_o.item())
    else:
        assert abs(loss.item() - loss_o.item()) <= 3e-2 * abs(loss_o.item())
    # moving statistics updated once (this forward)
    for k, v in mov.items():
        got = tr.net.store.buffers[k]
        tol = 1e-4 if dtype == torch.float32 else 3e-2
        assert _nerr(got, v) < tol, k
    # every parameter gradient
    bad = []
    for name, p in tr.net.store.params.items():
        go = P[name].grad
        gd = p._rod_grad
        if dtype == torch.float32:
            e = _nerr(gd, go)
            if e > 2e-3:
                bad.append((name, e))
        else:
            cs = torch.nn.functional.cosine_similarity(gd.float().cpu().reshape(-1), go.reshape(-1), dim=0).item()
            if go.abs().max() > 0 and cs < 0.98:
                bad.append((name, cs))
    assert not bad, bad[:10]
    # SGD with clip (net_tools.py:645-651)
    flat_g = tr.net.store.flat_grad.detach().clone()
    tr.opt.step()
    ref = (p0.cpu().numpy() - np.float32(1e-2) * np.clip(flat_g.cpu().numpy(), -5, 5)).astype(np.float32)
    np.testing.assert_array_equal(tr.net.store.flat.detach().cpu().numpy(), ref)


def test_trainer_steps_reduce_loss(dev):
    H, W, B = 96, 160, 2
    tr = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, learning_rate=5e-2, seed=2)
    batch = synthetic_batch(B, H, W, dev, seed=5)
    losses = [tr.step(*batch)[0].item() for _ in range(8)]
    assert np.isfinite(losses).all()
    assert losses[-1] < losses[0], losses
