"""Parity at the BASELINE.json sizes (1280x720), against the
oracle on the same seeded inputs:

  (a) C2 targets: anchor matching over all 129,915 anchors x B=8 (G <= 40 per image), ODM
      targets and the hard-negative selection — bit-exact (positive masks, argmax labels,
      offsets, matched boxes, IoU, k, the k-th value, the negative mask);
  (b) C2 step: one fp32 REFINE training step at B=8, 720x1280 — loss within 1e-4 relative of
      the float64 oracle; head outputs within max(1e-4, 4x the float32 floor) normwise per level
      (the floor: the oracle's own fp32 evaluation of the same step against float64; only the
      3x5 map, 24 layers + head deep, has one above 1e-4 — measured 1.25e-4); the errors are
      written to gpurun_out/parity_errors.json (kept under profiles/); moving statistics
      within 1e-4 (fixed bounds); parameter gradients within max(2e-3, 4x the error of an
      independent float32 evaluation) — float32 backprop through the deep BatchNorms is
      itself 1e-2..1e-1 off float64 there;
  (c) C4 inference: predict.py's Predictor at B=32 (softmax, decode of refine+det, per-class
      select / top-400 / NMS 0.4 / keep 200) with the clf head biased so that ~2 % of the
      class scores pass the 0.1 selection threshold — probabilities, boxes, NMS keep lists
      and outputs bit-exact against oracle.post given the network's logits and offsets;
  (d) C1 plumbing: train.py main() at 300x300, batch 1, two steps (ALL), then evaluate.py and
      predict.py main() on its checkpoint — all on the committed BDD100K-schema TFRecord
      fixture (tests/golden/tfrecord), torch and TF-bundle checkpoints.
"""
import json
import os

import numpy as np
import pytest
import torch

import config
from oracle import net as onet
from oracle import post as op
from oracle import targets as ot
from rod import ops

pytestmark = pytest.mark.gpu
f32 = np.float32
H, W = 720, 1280
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _anchors(h=H, w=W):
    import utils.net_tools as nt
    config.img_size = (h, w)
    return nt.anchors_all_layer((h, w), config.feat_sizes((h, w)), nt.init_anchor(6))


_PARITY = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out', 'parity_errors.json')


def _record(key, value):
    """Keep the measured errors of the full-size parity tests (copied to profiles/ per round)."""
    os.makedirs(os.path.dirname(_PARITY), exist_ok=True)
    d = json.load(open(_PARITY)) if os.path.exists(_PARITY) else {}
    d[key] = value
    with open(_PARITY, 'w') as f:
        json.dump(d, f, indent=1)


def _nerr(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


# ------------------------------------------------------------------------------- (a)
def test_targets_and_hard_negatives_720p_b8(dev):
    import utils.net_tools as nt
    from rod.data import synthetic_boxes
    from utils.common_tools import cornerBboxes_2_centerBboxes
    B = 8
    anchors = _anchors()
    corner, labels, n = synthetic_boxes(B, seed=31)
    assert n.max() <= 40 and n.min() >= 1
    tg = nt.refine_groundtruth(anchors, cornerBboxes_2_centerBboxes(torch.from_numpy(corner).to(dev)),
                               torch.from_numpy(labels).to(dev), config.refine_method.JACCARD_BIGGER,
                               n_boxes=torch.from_numpy(n).to(dev))
    off, cbox, lbl, pos = (t.cpu().numpy() for t in tg.flat)
    tab = tg.table
    assert tab.A == 129915
    thr = config.refine_pos_jac_val_all_layers
    for b in range(B):
        g, cb, lb, pm = ot.refine_groundtruth(anchors, ot.corner_to_center(corner[b, :n[b]]), labels[b, :n[b]], thr)
        cat = lambda xs, k: np.concatenate([x.reshape(-1, k) for x in xs])
        np.testing.assert_array_equal(pos[b], cat(pm, 1)[:, 0])
        np.testing.assert_array_equal(lbl[b], cat(lb, 1)[:, 0])
        np.testing.assert_array_equal(cbox[b], cat(cb, 4))
        np.testing.assert_array_equal(off[b], cat(g, 4))
    assert pos.sum() > 100 * B

    rng = np.random.default_rng(32)
    ro = (off + rng.normal(0, 0.15, off.shape)).astype(f32)
    dthr = config.det_pos_jac_val_all_layers
    dgt, dpos, dlbl, iou = ops.det_targets(tab.center, torch.from_numpy(ro).to(dev), *tg.flat, tab.lvl_off, dthr)
    r_gt, r_pos, r_lbl, r_iou = op.det_groundtruth(tab.center_np, tab.lvl_off, dthr, ro, off, cbox, lbl, pos)
    np.testing.assert_array_equal(iou.cpu().numpy(), r_iou)
    np.testing.assert_array_equal(dpos.cpu().numpy(), r_pos)
    np.testing.assert_array_equal(dlbl.cpu().numpy(), r_lbl)
    np.testing.assert_array_equal(dgt.cpu().numpy(), r_gt)
    assert r_pos.sum() > 50

    logits = rng.normal(0, 2.0, (B, tab.A, 11)).astype(f32)
    ld = torch.from_numpy(logits).to(dev).requires_grad_(True)
    out, clf = ops.softmax_ce_hnm(ld, dlbl, dpos, iou, tab.lvl_off, float(B))
    clf.backward()
    ref = op.det_clf_loss(np.zeros_like(ro), r_gt, r_pos, logits, r_lbl, r_iou, tab.lvl_off, B)
    o = out.detach().cpu().numpy()
    assert int(o[4]) == ref['n_pos'] and int(o[5]) == ref['k']
    assert o[3] == f32(ref['max_hard_pred'])
    assert int(o[6]) == ref['n_neg_selected'] and ref['n_neg_selected'] > 0
    g = ld.grad.cpu().numpy().reshape(-1, 11)
    pm = r_pos.reshape(-1) != 0
    neg_sel = (np.abs(g).sum(1) != 0) & ~pm                      # rows the selection kept
    np.testing.assert_array_equal(neg_sel, ref['negmask'])
    np.testing.assert_allclose(o[0], ref['pos_loss'], rtol=1e-5)
    np.testing.assert_allclose(o[1], ref['neg_loss'], rtol=1e-5)
    np.testing.assert_allclose(g, ref['g_logits'].reshape(-1, 11), rtol=1e-5, atol=1e-9)


# ------------------------------------------------------------------------------- (b)
def _oracle_refine_step(tr, snap, img, corner, labels, n, B, dt, device='cpu'):
    """The REFINE step in the oracle from the parameter / moving-statistic snapshot taken
    before the HIP step (which updates the moving statistics).  device='cuda' runs the
    oracle's PyTorch ops on the GPU: a second, independent float32 evaluation."""
    P = {k: v.clone().to(device, dt).requires_grad_(True) for k, v in snap[0].items()}
    Bf = {k: v.clone().to(device, dt) for k, v in snap[1].items()}
    x = torch.from_numpy(f32(2.0 / 255.0) * img.cpu().numpy().astype(f32) - f32(1.0)).to(device, dt)
    x = onet._st(x)          # the normalised input is stored too (bf16-storage emulation only)
    mov = {}
    refine = onet.forward(x, P, Bf, True, moving=mov)
    center = ot.corner_to_center(corner.cpu().numpy())
    gts, pms = [[] for _ in range(6)], [[] for _ in range(6)]
    for b in range(B):
        nb = int(n[b])
        g, _, _, p = ot.refine_groundtruth(tr.anchors, center[b, :nb], labels.cpu().numpy()[b, :nb],
                                           config.refine_pos_jac_val_all_layers)
        for l in range(6):
            gts[l].append(g[l])
            pms[l].append(p[l])
    loss = 0.
    for l in range(6):
        d = (torch.from_numpy(np.stack(gts[l])).to(device, dt) - refine[l]) * \
            torch.from_numpy(np.stack(pms[l])).to(device, dt)
        ad = d.abs()
        loss = loss + (0.5 * ((ad - 1) * torch.clamp(ad, max=1.0) + ad)).sum() / B
    loss.backward()
    return P, mov, refine, loss


_TRUTH = {}


def _c2_truth(tr, snap, img, corner, labels, n, B):
    """The float64 oracle REFINE step from bench.py's initial state (rod.data.C2_WEIGHT_SEED /
    C2_BATCH_SEED), computed once per module: (parameter gradients, moving statistics, outputs,
    loss).  ~3 CPU-minutes at 720x1280 b8; shared by the fp32 and the bf16 step tests."""
    if 'c2' not in _TRUTH:
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        P64, mov64, ref64, loss64 = _oracle_refine_step(tr, snap, img, corner, labels, n, B, torch.float64)
        _TRUTH['c2'] = ({k: v.grad.detach().clone() if v.grad is not None else None for k, v in P64.items()},
                        {k: v.detach().clone() for k, v in mov64.items()},
                        [r.detach().clone() for r in ref64], float(loss64.item()),
                        {k: v.clone() for k, v in snap[0].items()})
    g64, mov64, ref64, loss64, snap0 = _TRUTH['c2']
    assert all(torch.equal(snap0[k], v) for k, v in snap[0].items()), 'not the C2 initial weights'
    return g64, mov64, ref64, loss64


class _Grad(object):   # a parameter-like holder of a cached oracle gradient
    def __init__(self, g):
        self.grad = g


def test_refine_step_fp32_720p_b8(dev):
    import utils.net_tools as nt
    from nets.catch_net import factory
    from rod.data import C2_BATCH_SEED, C2_WEIGHT_SEED, synthetic_batch
    from rod.trainer import Trainer
    from utils.common_tools import cornerBboxes_2_centerBboxes
    B = 8     # C2: BDD100K 1280x720 fp32 batch 8 (at B=2 the 3x5 level's BatchNorms see 30 rows and
    #           float32 itself — PyTorch's CPU evaluation as much as this one — lands at 1.25e-4)
    tr = Trainer((H, W), B, dtype=torch.float32, device=dev, learning_rate=1e-3, seed=C2_WEIGHT_SEED)
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=C2_BATCH_SEED)
    snap = ({k: v.detach().cpu().clone() for k, v in tr.net.store.params.items()},
            {k: v.detach().cpu().clone() for k, v in tr.net.store.buffers.items()})
    x = ops.normalize_image(img, torch.float32)
    tg = nt.refine_groundtruth(tr.anchors, cornerBboxes_2_centerBboxes(corner), labels,
                               config.refine_method.JACCARD_BIGGER, n_boxes=n)
    outs = factory(x, 'mobilenet_v2', True, tr.config_dict, torch.float32, net=tr.net).get_output()
    loss = nt.refine_loss(outs, tg[0], tg[3], targets=tg)
    loss.backward()
    torch.cuda.synchronize()
    g64, mov64, ref64, l64 = _c2_truth(tr, snap, img, corner, labels, n, B)
    P64 = {k: _Grad(v) for k, v in g64.items()}
    # an independent float32 evaluation of the same step (the oracle, PyTorch-CPU fp32): its
    # own distance from float64 is the float32 conditioning floor of each output
    P32, _, ref32, _ = _oracle_refine_step(tr, snap, img, corner, labels, n, B, torch.float32)
    rep = [(l, _nerr(a, o64), _nerr(o32, o64)) for l, (a, o32, o64) in enumerate(zip(outs, ref32, ref64))]
    print('per-level normwise error vs fp64 (HIP fp32, oracle fp32):', rep)
    lrel = abs(loss.item() - l64) / abs(l64)
    print('loss', loss.item(), 'fp64', l64, 'rel', lrel)
    # north_star: fp32 logits / boxes within 1e-4 relative; where float32 itself (the oracle's
    # own fp32 evaluation) is further than that from float64 — the deepest level sits 24
    # backbone layers + 4 head convs deep — within 4x that float32 floor
    bars = [max(1e-4, 4 * e32) for _, _, e32 in rep]
    _record('c2_refine_step_fp32_720p_b8', {'levels': [{'level': l, 'err': e, 'oracle_fp32_err': e32, 'bar': bar}
                                                      for (l, e, e32), bar in zip(rep, bars)],
                                           'loss_rel_err': lrel})
    assert all(e <= bar for (_, e, _), bar in zip(rep, bars)), (rep, bars)
    assert lrel <= 1e-4
    # moving means are judged on the scale of their update, (1 - decay) x the batch std: the
    # mean of a conv fed by a linear-BN output (project -> expand) is 0 up to rounding
    bad_mov = []
    for k, v in mov64.items():
        got = tr.net.store.buffers[k].double().cpu()
        scale = v.abs().max()
        if k.endswith('moving_mean'):
            decay = 0.997 if k.startswith('backbone/') else 0.999
            var_b = (mov64[k[:-len('moving_mean')] + 'moving_variance'] - decay) / (1 - decay)
            scale = max(float(scale), (1 - decay) * float(var_b.clamp_min(0).sqrt().max()))
        e = float((got - v).abs().max()) / float(scale)
        if e > 1e-4:
            bad_mov.append((k, e))
    assert not bad_mov, bad_mov[:5]
    # Parameter gradients: float32 backprop through 24 BatchNorm'd layers is ill-conditioned
    # in the deep backbone (the deepest expand / depthwise gradients of ANY float32 evaluation
    # are 1e-2..1.5e-1 off float64 here, measured), so they are held to the float32 scatter:
    # within max(2e-3, 4x) the error of an independent float32 evaluation of the same step (the
    # oracle, PyTorch-CPU fp32).  Measured: worst ratio 3.7 (expanded_conv_22/expand/BatchNorm/
    # beta 0.152 vs 0.041); a third evaluation (the oracle's ops on the GPU) did not widen it.
    Pg = P32
    # gradients that are zero by construction (a bias or beta feeding a BatchNorm directly:
    # shift invariance) are judged on the scale of the step's gradients, not their own
    gscale = float(np.median([float(P64[k].grad.abs().max()) for k in tr.net.store.params]))
    bad, worst = [], 0.0
    rows, zero_rows = [], []
    for name, p in tr.net.store.params.items():
        g64 = P64[name].grad
        if float(g64.abs().max()) < 1e-6 * gscale:
            z = float(p._rod_grad.abs().max()) / gscale
            z32 = max(float(P32[name].grad.abs().max()), float(Pg[name].grad.abs().max())) / gscale
            zero_rows.append((z, z32, name))
            if z > max(1e-4, 4 * z32):
                bad.append((name, 'zero-by-construction', z, z32))
            continue
        e = _nerr(p._rod_grad, g64)
        e32 = max(_nerr(P32[name].grad, g64), _nerr(Pg[name].grad, g64))
        rows.append((e, e32, name))
        worst = max(worst, e)
        if e > max(2e-3, 4 * e32):
            bad.append((name, e, e32))
    rows.sort(reverse=True)
    zero_rows.sort(reverse=True)
    for r in rows[:12]:
        print('grad err %.3e  fp32 scatter %.3e  %s' % r)
    for r in zero_rows[:3]:
        print('zero-by-construction grad |g|/scale %.3e  fp32 %.3e  %s' % r)
    print('worst parameter-gradient normwise error:', worst, 'over', len(tr.net.store.params), 'tensors')
    d = json.load(open(_PARITY)) if os.path.exists(_PARITY) else {}
    d.setdefault('c2_refine_step_fp32_720p_b8', {})['grads'] = {
        'tensors': len(tr.net.store.params), 'worst_err': worst,
        'top': [{'name': nm, 'err': e, 'oracle_fp32_err': e32} for e, e32, nm in rows[:12]]}
    _record('c2_refine_step_fp32_720p_b8', d['c2_refine_step_fp32_720p_b8'])
    assert not bad, bad[:10]


def _cosd(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return 1.0 - float(torch.nn.functional.cosine_similarity(a, b, dim=0))


def test_refine_step_bf16_720p_b8_bench_config(dev):
    """The configuration bench.py times (BASELINE metric: bf16, 720x1280, 8 images, REFINE,
    ref train.py:250-327 / net_tools.py:492-516), from bench.py's own initial state: Trainer
    seed C2_WEIGHT_SEED, lr 1e-3, rod.data.synthetic_batch(seed=C2_BATCH_SEED).  Its loss is
    bench.py's "loss_first_step".  Truth: the oracle step in float64 (shared with the fp32
    test).  Baseline for what bf16 storage can reach: the same oracle step in fp32 arithmetic
    with every tensor the product stores (conv / depthwise outputs, BatchNorm + activation
    outputs, residual sums, and the gradients w.r.t. them) rounded to bf16 (oracle.net
    set_storage; PyTorch-CPU, an independent implementation of bf16 storage).  Bars:
      loss             within max(1e-2, 4x the bf16 baseline's) relative of float64;
      head outputs /   angular error (1 - cos) vs float64 within max(0.02, 3x) the bf16
      moving stats     baseline's, where that baseline keeps cos >= 0.95;
      gradients        within max(0.02, 3x) where the baseline keeps cos >= 0.7, and the
                       median over all tensors within 1.25x the baseline's;
      SGD + clip       bit-exact given the gradient (net_tools.py:645-651)."""
    import utils.net_tools as nt
    from nets.catch_net import factory
    from rod.data import C2_BATCH_SEED, C2_WEIGHT_SEED, synthetic_batch
    from rod.trainer import Trainer
    from utils.common_tools import cornerBboxes_2_centerBboxes
    B, bf16 = 8, torch.bfloat16
    tr = Trainer((H, W), B, dtype=bf16, device=dev, seed=C2_WEIGHT_SEED)     # as bench.py builds it
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=C2_BATCH_SEED)
    snap = ({k: v.detach().cpu().clone() for k, v in tr.net.store.params.items()},
            {k: v.detach().cpu().clone() for k, v in tr.net.store.buffers.items()})
    p0 = tr.net.store.flat.detach().clone()
    x = ops.normalize_image(img, bf16)
    tg = nt.refine_groundtruth(tr.anchors, cornerBboxes_2_centerBboxes(corner), labels,
                               config.refine_method.JACCARD_BIGGER, n_boxes=n)
    outs = factory(x, 'mobilenet_v2', True, tr.config_dict, bf16, net=tr.net).get_output()
    loss = nt.refine_loss(outs, tg[0], tg[3], targets=tg)
    loss.backward()
    torch.cuda.synchronize()
    # the same step through Trainer.step (bench.py's path) gives the same loss bit for bit
    tr2 = Trainer((H, W), B, dtype=bf16, device=dev, seed=C2_WEIGHT_SEED)
    l_bench = tr2.step(img, corner, labels, n)[0]
    assert torch.equal(l_bench, loss.detach().reshape(l_bench.shape)), (l_bench.item(), loss.item())
    del tr2
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    prev = onet.set_storage(bf16)            # fp32 arithmetic, every stored tensor rounded to bf16
    try:
        Pb, movb, refb, lossb = _oracle_refine_step(tr, snap, img, corner, labels, n, B, torch.float32)
    finally:
        onet.set_storage(prev)
    Pb = {k: v.grad.float() if v.grad is not None else None for k, v in Pb.items()}
    refb = [r.detach().float() for r in refb]
    movb = {k: v.float() for k, v in movb.items()}
    lossb = float(lossb.item())
    g64, mov64, ref64, l64 = _c2_truth(tr, snap, img, corner, labels, n, B)
    P64 = {k: _Grad(v) for k, v in g64.items()}
    lrel, lrel_b = abs(loss.item() - l64) / abs(l64), abs(lossb - l64) / abs(l64)
    print('bf16 720p b8 loss', loss.item(), 'fp64', l64, 'rel', lrel, '| bf16-storage oracle', lossb, 'rel', lrel_b)
    assert lrel <= max(1e-2, 4 * lrel_b)
    rep = [(l, _cosd(a, o), _cosd(b_, o)) for l, (a, b_, o) in enumerate(zip(outs, refb, ref64))]
    print('per-level 1-cos vs fp64 (hip, bf16-storage oracle):', rep)
    for l, e_h, e_b in rep:
        if e_b <= 0.05:
            assert e_h <= max(0.02, 3 * e_b), rep
    bad_mov = []
    for k, v in mov64.items():
        if _cosd(movb[k], v) <= 0.05 and _cosd(tr.net.store.buffers[k], v) > max(0.02, 3 * _cosd(movb[k], v)):
            bad_mov.append((k, _cosd(tr.net.store.buffers[k], v), _cosd(movb[k], v)))
    assert not bad_mov, bad_mov[:5]
    # gradients: the random-init network is chaotic in depth (a bf16-sized perturbation grows
    # layer by layer: the forward outputs above decorrelate from float64 level by level, for the
    # bf16-storage oracle as much as for this path), so the deep tensors' gradients of ANY bf16
    # evaluation keep little correlation with the truth.  Bar: on every tensor where the
    # bf16-storage oracle keeps cos >= 0.7, within max(0.02, 3x) its angular error; and over all
    # tensors the median angular error within 1.25x the oracle's
    bad, rows, allrows = [], [], []
    for name, p in tr.net.store.params.items():
        g64, gb = P64[name].grad, Pb[name]
        if gb is None or float(g64.abs().max()) == 0:
            continue   # zero by construction
        e_h, e_b = _cosd(p._rod_grad, g64), _cosd(gb, g64)
        allrows.append((e_h, e_b))
        if e_b > 0.3:
            continue
        rows.append((e_h, e_b, name))
        if e_h > max(0.02, 3 * e_b):
            bad.append((name, e_h, e_b))
    rows.sort(reverse=True)
    for r in rows[:8]:
        print('grad 1-cos %.3e  bf16-storage oracle %.3e  %s' % r)
    med_h = float(np.median([r[0] for r in allrows]))
    med_b = float(np.median([r[1] for r in allrows]))
    print('checked', len(rows), 'of', len(allrows), 'parameter gradients; median 1-cos hip', med_h, 'oracle', med_b)
    assert len(rows) >= 20 and not bad, bad[:10]
    assert med_h <= 1.25 * med_b + 1e-3, (med_h, med_b)
    flat_g = tr.net.store.flat_grad.detach().clone()
    tr.opt.step()
    ref = (p0.cpu().numpy() - np.float32(1e-3) * np.clip(flat_g.cpu().numpy(), -5, 5)).astype(np.float32)
    np.testing.assert_array_equal(tr.net.store.flat.detach().cpu().numpy(), ref)


# ------------------------------------------------------------------------------- (c)
def test_predict_b32_nms_bit_exact(dev):
    import predict
    from rod.data import synthetic_batch
    pr = predict.Predictor((H, W), dev, torch.bfloat16, seed=41)
    pr.keep_intermediates = True
    probe = synthetic_batch(4, H, W, dev, seed=42)[0]
    # random init + initial moving statistics give vanishing eval activations (uniform
    # softmax, nothing selected): calibrate BatchNorm on a probe batch and shift the background
    # logit so that ~2 % of the class scores pass select_threshold 0.1
    from rod.data import detector_like_scores
    f_probe = detector_like_scores(pr, probe, rate=0.02)
    img = synthetic_batch(32, H, W, dev, seed=43)[0]
    scores, bboxes = pr(img)
    logits, probs, boxes, roff, doff = pr.last
    f_pass = float((probs[..., 1:] >= 0.1).float().mean())
    print('fraction of class scores >= 0.1:', f_pass, '(probe batch:', f_probe, ')')
    assert 0.005 <= f_pass <= 0.06
    lg = logits.float().cpu().numpy()
    e, s, _ = op.softmax_rows(lg)
    probs_ref = (e / s).astype(f32)
    P = probs.cpu().numpy()
    np.testing.assert_array_equal(P, probs_ref)
    import utils.net_tools as nt
    tab = nt.anchor_table(pr.anchors, dev)
    bx_ref = op.decode_corner(tab.center_np, roff.float().cpu().numpy() + doff.float().cpu().numpy())
    BX = boxes.cpu().numpy()
    np.testing.assert_array_equal(BX, bx_ref)
    s_ref, b_ref, kept = op.detected_bboxes_vec(P, BX, 0.1, 0.4, 400, 200)
    S = np.stack([scores[c].cpu().numpy() for c in range(1, 11)], 1)
    Bo = np.stack([bboxes[c].cpu().numpy() for c in range(1, 11)], 1)
    np.testing.assert_array_equal(S, s_ref)
    np.testing.assert_array_equal(Bo, b_ref)
    n_kept = sum(len(v) for v in kept.values())
    print('kept detections over 32 images x 10 classes:', n_kept)
    assert n_kept > 320 and max(len(v) for v in kept.values()) > 20
    # the HIP-graph replay (the default predict path) gives the same detections, twice
    pr.keep_intermediates = False
    assert pr.use_graph
    for _ in range(2):
        sg, bg = pr(img)
        for c in range(1, 11):
            assert torch.equal(sg[c], scores[c]) and torch.equal(bg[c], bboxes[c])
    assert pr._graph is not None


def test_predict_1080p_fused_blocks_match_oracle(dev):
    """C5 (BASELINE configs[4]): predict.py's inference path at 1920x1080, batch 2, with the
    fused inverted-residual blocks (rod_ir_block_fwd, ref conv_blocks.py:163-312) on, BatchNorm
    calibrated so the heads give a detector-like score distribution.
      * the fused kernel actually runs (probe);
      * fp32 (the unfused path): head outputs (refine / det offsets, clf logits) within
        max(1e-4, 4x the oracle's own float32 distance from float64)
        normwise of the float64 oracle network in eval mode (ref predict.py:127-137);
      * bf16 with the fused blocks: no less accurate than the unfused bf16 chain (1.5x + 1e-3),
        and within 3x + 1e-2 of what bf16 storage allows — the oracle in fp32 arithmetic with
        every stored tensor rounded to bf16 (oracle.net.set_storage).  (The calibrated random
        network amplifies a bf16-sized perturbation layer by layer, so bf16 outputs of ANY
        implementation sit far from float64 on the deep levels: the storage-rounded oracle
        measures that conditioning);
      * softmax, decode and the per-class select / top-k / NMS keep lists and outputs bit-exact
        against oracle.post given the network's logits and offsets (~2 % of the class scores
        pass select_threshold 0.1)."""
    import predict
    import utils.net_tools as nt
    from nets.catch_net import factory
    from rod import _abi
    from rod.data import detector_like_scores, synthetic_batch
    from rod.dataio import network_input
    Hc, Wc, B = 1080, 1920, 2
    pr = predict.Predictor((Hc, Wc), dev, torch.bfloat16, seed=51)
    probe = synthetic_batch(2, Hc, Wc, dev, seed=52)[0]
    f_probe = detector_like_scores(pr, probe, rate=0.02)
    img = synthetic_batch(B, Hc, Wc, dev, seed=53)[0]
    pr.keep_intermediates = True
    _abi.PROBE.arm('rod_ir_block_fwd')
    ops._DISABLE.add('rcinf')   # the 16..32-channel blocks otherwise take the recompute chain
    try:
        scores, bboxes = pr(img)
    finally:
        ops._DISABLE.discard('rcinf')
    torch.cuda.synchronize()
    _abi.PROBE.disarm()
    n_fused = _abi.PROBE.table().get('rod_ir_block_fwd', (0,))[0]
    print('fused blocks launched:', n_fused, 'probe pass fraction', f_probe)
    assert n_fused >= 4
    logits, probs, boxes, roff, doff = (t.clone() for t in pr.last)
    ops._DISABLE.add('irblock')
    try:
        pr(img)
        u_logits, _, _, u_roff, u_doff = pr.last
    finally:
        ops._DISABLE.discard('irblock')
    # the same calibrated network in fp32 (the unfused fp32 kernels)
    with torch.no_grad():
        f_out = factory(network_input(img, torch.float32), 'mobilenet_v2', False, pr.config_dict, torch.float32,
                        net=pr.net).get_output()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    P = {k: v.detach().double().cpu() for k, v in pr.net.store.params.items()}
    Bf = {k: v.detach().double().cpu() for k, v in pr.net.store.buffers.items()}
    x32 = torch.from_numpy(f32(2.0 / 255.0) * img.cpu().numpy().astype(f32) - f32(1.0))
    with torch.no_grad():
        r64, d64, c64 = onet.forward(x32.double(), P, Bf, False, all_mode=True)
        prev = onet.set_storage(torch.bfloat16)
        try:
            rq, dq, cq = onet.forward(onet._st(x32), {k: v.float() for k, v in P.items()},
                                      {k: v.float() for k, v in Bf.items()}, False, all_mode=True)
        finally:
            onet.set_storage(prev)
        # the oracle's own float32 evaluation: the float32 conditioning floor of each output
        r32, d32, c32 = onet.forward(x32, {k: v.float() for k, v in P.items()}, {k: v.float() for k, v in Bf.items()},
                                     False, all_mode=True)
    cat = lambda ts, k: torch.cat([t.reshape(B, -1, k) for t in ts], 1)
    rep = []
    recs = []
    for name, got, unf, f32o, q, o32, want, k in (('refine', roff, u_roff, f_out[0], rq, r32, r64, 4),
                                                 ('det', doff, u_doff, f_out[1], dq, d32, d64, 4),
                                                 ('clf', logits, u_logits, f_out[2], cq, c32, c64, 11)):
        want = cat(want, k)
        ef, eu, e32, eq = _nerr(got.float(), want), _nerr(unf.float(), want), _nerr(cat(f32o, k), want), \
            _nerr(cat(q, k), want)
        eo = _nerr(cat(o32, k), want)
        rep.append((name, ef, eu, e32, eq, eo))
        # north_star: fp32 logits / boxes within 1e-4 relative, or within 4x the float32 floor
        # (the oracle's own fp32 evaluation) where float32 itself is further from float64
        bar = max(1e-4, 4 * eo)
        recs.append({'output': name, 'hip_fp32_err': e32, 'oracle_fp32_err': eo, 'bar': bar, 'bf16_fused_err': ef,
                     'bf16_unfused_err': eu, 'bf16_storage_oracle_err': eq})
        assert e32 <= bar, rep
        assert ef <= 1.5 * eu + 1e-3 and ef <= 3 * eq + 1e-2, rep
    _record('c5_predict_1080p_b2', recs)
    print('1080p head outputs, normwise error vs fp64 (bf16 fused, bf16 unfused, fp32, bf16-storage oracle, '
          'oracle fp32):', rep)
    lg = logits.float().cpu().numpy()
    e, s_, _ = op.softmax_rows(lg)
    P_ = probs.cpu().numpy()
    np.testing.assert_array_equal(P_, (e / s_).astype(f32))
    tab = nt.anchor_table(pr.anchors, dev)
    BX = boxes.cpu().numpy()
    np.testing.assert_array_equal(BX, op.decode_corner(tab.center_np, roff.float().cpu().numpy() +
                                                       doff.float().cpu().numpy()))
    s_ref, b_ref, kept = op.detected_bboxes_vec(P_, BX, 0.1, 0.4, 400, 200)
    S = np.stack([scores[c].cpu().numpy() for c in range(1, 11)], 1)
    Bo = np.stack([bboxes[c].cpu().numpy() for c in range(1, 11)], 1)
    np.testing.assert_array_equal(S, s_ref)
    np.testing.assert_array_equal(Bo, b_ref)
    n_kept = sum(len(v) for v in kept.values())
    print('1080p kept detections over', B, 'images x 10 classes:', n_kept)
    assert n_kept > 20 * B


# ------------------------------------------------------------------------------- (d)
def _cli(mod, argv):
    import importlib
    m = importlib.import_module(mod)
    return m.main(argv)


def test_cli_train_evaluate_predict_on_tfrecords(dev, tmp_path):
    ds = os.path.join(GOLD, 'tfrecord')
    tdir, sdir, edir = str(tmp_path / 'ckpt'), str(tmp_path / 'summ'), str(tmp_path / 'eval')
    common = ['--img_height=300', '--img_width=300', '--dataset_dir=' + ds]
    _cli('train', common + ['--batch_size=1', '--train_range=ALL', '--checkpoint_refine=None', '--fix_refine=False',
                            '--max_number_of_steps=1', '--save_every_n_steps=2', '--log_every_n_steps=1',
                            '--summary_every_n_steps=1', '--train_dir=' + tdir, '--summary_dir=' + sdir])
    ck = os.path.join(tdir, 'mobilenet_v2.model')
    assert os.path.isfile(ck)
    recs = [json.loads(l) for l in open(os.path.join(sdir, 'train_rank0.jsonl'))]
    assert [r['step'] for r in recs] == [0, 1] and all(np.isfinite(r['loss']).all() for r in recs)
    m07, m12 = _cli('evaluate', common + ['--batch_size=4', '--num_images=8', '--checkpoint_path=' + tdir,
                                          '--eval_dir=' + edir])
    ev = json.load(open(os.path.join(edir, 'eval.json')))
    assert ev['num_batches'] == 2 and not ev['synthetic'] and ev['checkpoint'] == ck
    assert np.isfinite(m07) and np.isfinite(m12) and 0 <= m07 <= 1 and 0 <= m12 <= 1
    scores, boxes = _cli('predict', common + ['--batch_size=2', '--checkpoint_all=' + ck,
                                              '--output=' + str(tmp_path / 'det.json'),
                                              '--vis_dir=' + str(tmp_path / 'vis')])
    assert set(scores) == set(range(1, 11)) and scores[1].shape == (2, 200)
    from PIL import Image   # predict.py:151-196 drawings, written instead of shown
    for name in ('pred_0000.png', 'gt_0000.png'):
        with Image.open(str(tmp_path / 'vis' / name)) as im:
            assert im.size == (1080, 720)
    # the same weights as a TF-1.x tensor bundle: evaluate restores it and gives the same mAP
    from rod.checkpoint import load_variables, save_variables
    from nets.catch_net import CatchNet
    cfg = {'train_range': config.train_range.ALL, 'process_backbone_method': config.process_backbone_method.NONE,
           'deconv_method': config.deconv_method.LEARN_HALF, 'merge_method': config.merge_method.ADD}
    net = CatchNet('mobilenet_v2', cfg, dev)
    load_variables(net.store, ck)
    tfdir = str(tmp_path / 'tfck')
    save_variables(net.store, os.path.join(tfdir, 'mobilenet_v2.model'), 2, fmt='tf')
    t07, t12 = _cli('evaluate', common + ['--batch_size=4', '--num_images=8', '--checkpoint_path=' + tfdir,
                                          '--eval_dir=' + edir])
    assert (t07, t12) == (m07, m12)
    # no dataset and no --synthetic: an error, as in the reference
    with pytest.raises(FileNotFoundError):
        _cli('predict', ['--img_height=300', '--img_width=300', '--dataset_dir=' + str(tmp_path),
                         '--checkpoint_all=' + ck])


def test_tfrecord_source_batches(dev):
    """TFRecordSource on the fixture: the eval path is the legacy bilinear resize of the
    decoded JPEG (oracle.augment) normalised; the train path yields boxes inside [0, 1]."""
    from oracle import augment as oaug
    from rod.dataio import TFRecordSource, tfrecord_files
    exp = np.load(os.path.join(GOLD, 'tfrecord', 'expected.npz'))
    files = tfrecord_files(os.path.join(GOLD, 'tfrecord'))
    src = TFRecordSource(files, 3, (96, 160), dev, torch.float32, train=False)
    x, bo, lo, n = next(src)
    for b in range(3):
        ref = oaug.process_image(exp['image_%d' % b], (0, 0) + exp['image_%d' % b].shape[:2], False, -1, None,
                                 96, 160, True)
        np.testing.assert_array_equal(x[b].cpu().numpy(), ref)
        g = int(n[b])
        np.testing.assert_array_equal(bo[b, :g].cpu().numpy(), exp['boxes_%d' % b])
        np.testing.assert_array_equal(lo[b, :g].cpu().numpy(), exp['labels_%d' % b])
    tr = TFRecordSource(files, 4, (96, 160), dev, torch.bfloat16, train=True, seed=5)
    seen = 0
    for _ in range(3):                       # crosses an epoch boundary (8 records)
        x, bo, lo, n = next(tr)
        assert x.dtype == torch.bfloat16 and x.shape == (4, 96, 160, 3)
        assert float(x.float().abs().max()) <= 1.0 + 1e-6
        for b in range(4):
            g = int(n[b])
            bb = bo[b, :g].cpu().numpy()
            assert ((bb >= 0) & (bb <= 1)).all()
            seen += g
    assert seen > 0 and tr.epoch == 1


def test_tfrecord_fed_graphed_steps_bit_identical(dev):
    """train.py's path: TFRecord batches (fixed box padding, prefetching source, GPU
    augmentation) through Trainer.step_graphed are bit-identical to the eager step on the same
    batches, and ONE graph serves batches whose real box counts differ (no re-capture)."""
    from rod.dataio import GMAX, TFRecordSource, tfrecord_files
    from rod.trainer import Trainer
    files = tfrecord_files(os.path.join(GOLD, 'tfrecord'))
    H, W, B = 160, 288, 2
    sa = TFRecordSource(files, B, (H, W), dev, torch.bfloat16, train=True, seed=7, prefetch=False)
    sb = TFRecordSource(files, B, (H, W), dev, torch.bfloat16, train=True, seed=7)
    ta = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=2)
    tb = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=2)
    counts = set()
    for _ in range(6):
        a, b = next(sa), next(sb)
        assert a[1].shape == (B, GMAX, 4)
        for x, y in zip(a, b):
            assert torch.equal(x, y)
        counts.add(tuple(a[3].tolist()))
        la = ta.step(*a)
        lb = tb.step_graphed(*b)
    torch.cuda.synchronize()
    assert len(counts) > 2, counts
    assert len(tb._graphs) == 1
    assert torch.equal(ta.net.store.flat, tb.net.store.flat)
    for k, v in ta.net.store.buffers.items():
        assert torch.equal(v, tb.net.store.buffers[k]), k
    assert torch.equal(la[0], lb[0])
    assert ta.opt.global_step == tb.opt.global_step == 6
    sa.close()
    sb.close()
