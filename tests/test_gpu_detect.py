"""Parity of the ALL-mode / inference kernels with the oracle.

Bit-exact: decode, ODM targets (iou, det_pos, det_lbl, det_gt), the hard-negative mask
(k, max_hard_pred, number selected) and the NMS keep lists / output boxes & scores.
fp32 tolerances: losses 1e-5 relative, gradients 1e-5 relative (+1e-8 absolute).
"""
import numpy as np
import pytest
import torch

import config
from oracle import anchors as oa
from oracle import net as onet
from oracle import post as op
from oracle import targets as ot
from rod import ops

pytestmark = pytest.mark.gpu
f32 = np.float32


def _param(t, dev):
    p = t.detach().clone().to(dev).requires_grad_(True)
    p._rod_grad = torch.zeros_like(p)
    return p


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('H,W,Ho,Wo', [(3, 5, 6, 10), (12, 20, 23, 40), (45, 80, 90, 160), (7, 7, 14, 14)])
def test_resize_bilinear_legacy(dev, dtype, H, W, Ho, Wo):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, H, W, 8, generator=g)
    if dtype == torch.bfloat16:
        x = x.to(torch.bfloat16).float()
    xo = x.clone().requires_grad_(True)
    yo = onet.resize_bilinear_legacy(xo.permute(0, 3, 1, 2), (Ho, Wo)).permute(0, 2, 3, 1)
    gy = torch.randn(yo.shape, generator=g)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).float()
    (yo * gy).sum().backward()
    xd = x.to(dev, dtype).requires_grad_(True)
    yd = ops.resize_bilinear(xd, (Ho, Wo))
    yd.backward(gy.to(dev, dtype))
    tol = dict(rtol=1e-5, atol=1e-6) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(yd.float().cpu(), yo.detach(), **tol)
    torch.testing.assert_close(xd.grad.float().cpu(), xo.grad, **tol)


@pytest.mark.parametrize('h,w,Ho,Wo,Cin,F', [(3, 5, 6, 10, 256, 128), (12, 20, 23, 40, 320, 80), (45, 80, 90, 160, 96, 32)])
def test_deconv2x2(dev, h, w, Ho, Wo, Cin, F):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, h, w, Cin, generator=g)
    wt = torch.randn(2, 2, F, Cin, generator=g) * 0.05
    xo, wo = x.clone().requires_grad_(True), wt.clone().requires_grad_(True)
    yo = onet.conv_transpose_2x2(xo.permute(0, 3, 1, 2), wo, (Ho, Wo)).permute(0, 2, 3, 1)
    gy = torch.randn(yo.shape, generator=g)
    (yo * gy).sum().backward()
    xd = x.to(dev).requires_grad_(True)
    wd = _param(wt, dev)
    yd = ops.deconv2x2(xd, wd, (Ho, Wo))
    yd.backward(gy.to(dev))
    torch.testing.assert_close(yd.cpu(), yo.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(xd.grad.cpu(), xo.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(wd._rod_grad.cpu(), wo.grad, rtol=1e-4, atol=1e-4)


def test_concat_and_add(dev):
    g = torch.Generator().manual_seed(3)
    a = torch.randn(2, 5, 7, 24, generator=g).to(dev).requires_grad_(True)
    b = torch.randn(2, 5, 7, 40, generator=g).to(dev).requires_grad_(True)
    c = ops.channel_concat([a, b])
    torch.testing.assert_close(c.cpu(), torch.cat([a.detach().cpu(), b.detach().cpu()], -1), rtol=0, atol=0)
    gc = torch.randn(c.shape, generator=g).to(dev)
    c.backward(gc)
    assert torch.equal(a.grad, gc[..., :24]) and torch.equal(b.grad, gc[..., 24:])
    x = torch.randn(3, 4, 5, 16, generator=g).to(dev)
    y = torch.randn(3, 4, 5, 16, generator=g).to(dev)
    assert torch.equal(ops.add(x, y).cpu(), torch.from_numpy(x.cpu().numpy() + y.cpu().numpy()))


def test_fork_sums_branch_gradients(dev):
    """graph.fork: n aliases whose gradients are summed (fp32 add, bit-exact vs numpy);
    branches that receive no gradient contribute nothing."""
    from rod import graph
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 3, 4, 8, generator=g).to(dev).requires_grad_(True)
    a, b, c = graph.fork(x, 3)
    ga, gb = (torch.randn(x.shape, generator=g) for _ in range(2))
    torch.autograd.backward([ops.add(a, a.detach()), b], [ga.to(dev), gb.to(dev)])
    assert torch.equal(x.grad.cpu(), torch.from_numpy(ga.numpy() + gb.numpy()))
    l1 = torch.tensor(1.5, device=dev, requires_grad=True)
    l2 = torch.tensor(2.25, device=dev, requires_grad=True)
    s = graph.scalar_sum(l1, l2)
    graph.backward(s)
    assert s.item() == 3.75 and l1.grad.item() == 1.0 and l2.grad.item() == 1.0


def _setup(H, W, B, seed):
    from utils import net_tools as nt
    rng = np.random.default_rng(seed)
    config.img_size = (H, W)
    anchors = nt.anchors_all_layer((H, W), config.feat_sizes((H, W)), nt.init_anchor(6))
    tab = nt.AnchorTable(anchors, 'cpu')
    A = tab.A
    return rng, anchors, tab, A


def test_decode_bit_exact(dev):
    from utils import net_tools as nt
    rng, anchors, tab, A = _setup(300, 300, 3, 0)
    a = rng.normal(0, 0.5, (3, A, 4)).astype(f32)
    b = rng.normal(0, 0.1, (3, A, 4)).astype(f32)
    tabd = nt.AnchorTable(anchors, dev)
    got = ops.decode(tabd.center, torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), to_corner=True)
    ref = op.decode_corner(tab.center_np, a + b)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_det_targets_and_hnm_loss(dev):
    from utils import net_tools as nt
    from utils.common_tools import cornerBboxes_2_centerBboxes
    from rod.data import synthetic_boxes
    H, W, B = 300, 300, 4
    rng, anchors, tab, A = _setup(H, W, B, 1)
    corner, labels, n = synthetic_boxes(B, seed=11)
    tg = nt.refine_groundtruth(anchors, cornerBboxes_2_centerBboxes(torch.from_numpy(corner).to(dev)),
                               torch.from_numpy(labels).to(dev), config.refine_method.JACCARD_BIGGER,
                               n_boxes=torch.from_numpy(n).to(dev))
    rgt, cbox, lbl, pos = (t.cpu().numpy() for t in tg.flat)
    # refine_out near the targets so that many ODM positives exist
    ro = (rgt + rng.normal(0, 0.15, rgt.shape)).astype(f32)
    ro_d = torch.from_numpy(ro).to(dev)
    thr = config.det_pos_jac_val_all_layers
    dgt, dpos, dlbl, iou = ops.det_targets(tg.table.center, ro_d, tg.flat[0], tg.flat[1], tg.flat[2], tg.flat[3],
                                           tab.lvl_off, thr)
    r_gt, r_pos, r_lbl, r_iou = op.det_groundtruth(tab.center_np, tab.lvl_off, thr, ro, rgt, cbox, lbl, pos)
    np.testing.assert_array_equal(iou.cpu().numpy(), r_iou)
    np.testing.assert_array_equal(dpos.cpu().numpy(), r_pos)
    np.testing.assert_array_equal(dlbl.cpu().numpy(), r_lbl)
    np.testing.assert_array_equal(dgt.cpu().numpy(), r_gt)
    assert r_pos.sum() > 20

    logits = rng.normal(0, 2.0, (B, A, 11)).astype(f32)
    det_out = rng.normal(0, 0.3, (B, A, 4)).astype(f32)
    ref = op.det_clf_loss(det_out, r_gt, r_pos, logits, r_lbl, r_iou, tab.lvl_off, B)
    ld = torch.from_numpy(logits).to(dev).requires_grad_(True)
    out, clf = ops.softmax_ce_hnm(ld, dlbl, dpos, iou, tab.lvl_off, float(B))
    clf.backward()
    o = out.detach().cpu().numpy()
    assert clf.item() == o[2]
    assert int(o[5]) == ref['k'] and int(o[4]) == ref['n_pos']
    assert o[3] == f32(ref['max_hard_pred'])                 # k-th smallest nvalue, bit-exact
    assert int(o[6]) == ref['n_neg_selected']                # hard-negative mask size
    np.testing.assert_allclose(o[0], ref['pos_loss'], rtol=1e-5)
    np.testing.assert_allclose(o[1], ref['neg_loss'], rtol=1e-5)
    np.testing.assert_allclose(o[2], ref['clf_loss'], rtol=1e-5)
    np.testing.assert_allclose(ld.grad.cpu().numpy(), ref['g_logits'], rtol=1e-5, atol=1e-8)
    # det loss through the shared smooth-L1 kernel
    dd = torch.from_numpy(det_out).to(dev).requires_grad_(True)
    vec, tot = ops.smooth_l1_masked(dd, dgt, dpos, tab.lvl_off, float(B))
    tot.backward()
    np.testing.assert_allclose(vec[6].item(), ref['det_loss'], rtol=1e-5)
    assert tot.item() == vec[6].item()
    np.testing.assert_allclose(dd.grad.cpu().numpy(), ref['g_det'], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize('ranks', [1, 2, 4])
def test_hnm_data_parallel_exchange(dev, ranks):
    """the batch split over `ranks` shards (emulated in one process; the exchange
    sums the int32 counts / histograms over the shards as RCCL all-reduce does across GPUs).
    k, the k-th smallest nvalue and the negative mask equal the single-process ones bit for bit;
    the per-shard gradients are the rows of the full-batch gradient; the loss sums match."""
    from utils import net_tools as nt
    from utils.common_tools import cornerBboxes_2_centerBboxes
    from rod.data import synthetic_boxes
    H, W, B = 300, 300, 4
    rng, anchors, tab, A = _setup(H, W, B, 3)
    corner, labels, n = synthetic_boxes(B, seed=12)
    tg = nt.refine_groundtruth(anchors, cornerBboxes_2_centerBboxes(torch.from_numpy(corner).to(dev)),
                               torch.from_numpy(labels).to(dev), config.refine_method.JACCARD_BIGGER,
                               n_boxes=torch.from_numpy(n).to(dev))
    rgt = tg.flat[0].cpu().numpy()
    ro_d = torch.from_numpy((rgt + rng.normal(0, 0.15, rgt.shape)).astype(f32)).to(dev)
    dgt, dpos, dlbl, iou = ops.det_targets(tg.table.center, ro_d, tg.flat[0], tg.flat[1], tg.flat[2], tg.flat[3],
                                           tab.lvl_off, config.det_pos_jac_val_all_layers)
    logits = torch.from_numpy(rng.normal(0, 2.0, (B, A, 11)).astype(f32)).to(dev)
    ld = logits.clone().requires_grad_(True)
    full, clf = ops.softmax_ce_hnm(ld, dlbl, dpos, iou, tab.lvl_off, float(B))
    clf.backward()
    full = full.cpu().numpy()

    def exchange(ts):       # in-place SUM over the shards (what dist.all_reduce does over ranks)
        tot = ts[0].clone()
        for t in ts[1:]:
            tot += t
        for t in ts:
            t.copy_(tot)
    per = B // ranks
    sl = [slice(r * per, (r + 1) * per) for r in range(ranks)]
    shards = [(logits[s].contiguous(), dlbl[s].contiguous(), dpos[s].contiguous(), iou[s].contiguous()) for s in sl]
    res = ops.hnm_lockstep(shards, tab.lvl_off, float(B), B, exchange)
    outs = np.stack([o.cpu().numpy() for o, _ in res])
    assert (outs[:, 3] == full[3]).all() and (outs[:, 5] == full[5]).all() and (outs[:, 4] == full[4]).all()
    assert int(outs[:, 6].sum()) == int(full[6])
    np.testing.assert_allclose(outs[:, 0].sum(), full[0], rtol=1e-5)
    np.testing.assert_allclose(outs[:, 1].sum(), full[1], rtol=1e-5)
    g = torch.cat([gr for _, gr in res]).cpu().numpy()
    np.testing.assert_array_equal(g, ld.grad.cpu().numpy())


@pytest.mark.parametrize('sel,nms,top_k,keep', [(0.1, 0.4, 400, 200), (0.3, 0.4, 400, 200), (0.02, 0.45, 64, 16)])
def test_select_topk_nms_bit_exact(dev, sel, nms, top_k, keep):
    rng, anchors, tab, A = _setup(300, 300, 2, 5)
    B = 2
    logits = rng.normal(0, 2.0, (B, A, 11)).astype(f32)
    e, s, _ = op.softmax_rows(logits)
    probs_ref = (e / s).astype(f32)
    pd = ops.softmax(torch.from_numpy(logits).to(dev), 11)
    np.testing.assert_array_equal(pd.cpu().numpy(), probs_ref)
    off = rng.normal(0, 0.2, (B, A, 4)).astype(f32)
    boxes = op.decode_corner(tab.center_np, off)
    s_ref, b_ref, kept = op.detected_bboxes(probs_ref, boxes, sel, nms, top_k, keep)
    for compact in (True, False):   # candidate-list and direct implementations
        sd, bd = ops.select_topk_nms(pd, torch.from_numpy(boxes).to(dev), sel, top_k, keep, nms, compact=compact)
        np.testing.assert_array_equal(sd.cpu().numpy(), s_ref)
        np.testing.assert_array_equal(bd.cpu().numpy(), b_ref)
    assert sum(len(v) for v in kept.values()) > 0


@pytest.mark.parametrize('case', ['many', 'ties', 'few', 'none'])
def test_select_topk_nms_candidate_lists(dev, case):
    """The candidate-list NMS (radix-select path past 4096 candidates per class, tied
    scores, fewer candidates than top_k, no candidate at all) against the oracle."""
    rng, anchors, tab, A = _setup(300, 300, 2, 5)
    B, K = 2, 11
    if case == 'many':      # most scores pass 0.1 in classes 1-2: lists far over 4096
        logits = rng.normal(0, 0.3, (B, A, K)).astype(f32)
        logits[..., 1:3] += 2.0
    elif case == 'ties':    # quantised logits: massive exact ties in score
        logits = np.round(rng.normal(0, 1.5, (B, A, K))).astype(f32)
    elif case == 'few':
        logits = rng.normal(0, 1.0, (B, A, K)).astype(f32)
        logits[..., 0] += 4.0
    else:
        logits = np.zeros((B, A, K), f32)
        logits[..., 0] = 10.0
    e, s, _ = op.softmax_rows(logits)
    probs_ref = (e / s).astype(f32)
    pd = ops.softmax(torch.from_numpy(logits).to(dev), K)
    off = rng.normal(0, 0.2, (B, A, 4)).astype(f32)
    boxes = op.decode_corner(tab.center_np, off)
    s_ref, b_ref, kept = op.detected_bboxes(probs_ref, boxes, 0.1, 0.4, 400, 200)
    sd, bd = ops.select_topk_nms(pd, torch.from_numpy(boxes).to(dev), 0.1, 400, 200, 0.4)
    np.testing.assert_array_equal(sd.cpu().numpy(), s_ref)
    np.testing.assert_array_equal(bd.cpu().numpy(), b_ref)
    n_sel = int((probs_ref[..., 1:] >= 0.1).sum(1).max())
    if case == 'many':
        assert n_sel > 4096
    if case == 'none':
        assert n_sel == 0 and not sd.any()
