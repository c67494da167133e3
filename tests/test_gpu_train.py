"""End-to-end parity of one REFINE training step (train.py:250-327) against the oracle:
network outputs, moving statistics, loss, every parameter gradient and the SGD update.

Tolerance design (normwise error e(a, b) = max|a-b| / max|b|, measured against the
oracle evaluated in float64 = "truth"):
  fp32 outputs:  e(hip, truth) <= max(1e-4, 4 * e(oracle_fp32, truth))   per level
  fp32 grads:    e(hip, truth) <= max(2e-3, 4 * e(oracle_fp32, truth), 4 * s) per tensor,
                 s = e(truth under 1e-6 relative input noise, truth): activation kinks near
                 zero on the few-row levels make single gradient entries jump under ANY
                 fp32 evaluation order (measured: swapping only the stem conv's summation
                 order moves refine/block_5 grads by 5-20 %)
The second term matters only where fp32 itself is ill-conditioned: BatchNorm over the
few rows of the deepest feature maps (2-30 values at these test sizes) amplifies any
rounding difference (the oracle's own fp32 error there reaches 1e-3..1), so no fp32
implementation can be closer to the truth than fp32 allows.
bf16 storage: loss within 3 %; outputs / moving statistics / gradients: angular error vs
truth (1 - cosine) within max(0.02, 3x) that of a plain bf16 evaluation of the oracle, on
tensors where bf16 can represent the answer (bf16-oracle cosine >= 0.95) and fp32 is well
conditioned (oracle fp32 error < 1e-2).
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


def _oracle_step(tr, img, corner, labels, n, H, W, B, dt, perturb=0.0, seed=0, msf=False):
    P = {k: v.detach().cpu().clone().to(dt).requires_grad_(v.requires_grad) for k, v in tr.net.store.params.items()}
    Bf = {k: v.detach().cpu().clone().to(dt) for k, v in tr.net.store.buffers.items()}
    x = torch.from_numpy(np.float32(2.0 / 255.0) * img.cpu().numpy().astype(np.float32) - np.float32(1.0)).to(dt)
    if perturb:  # fp32-sized relative noise on the input (sensitivity probe of the fp64 truth)
        g = torch.Generator().manual_seed(seed)
        x = x * (1 + perturb * torch.randn(x.shape, generator=g, dtype=dt))
    mov = {}
    refine = onet.forward(x, P, Bf, True, moving=mov, msf=msf)
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
        y = torch.from_numpy(np.stack(gts[l])).to(dt)
        m = torch.from_numpy(np.stack(pms[l])).to(dt)
        d = (y - refine[l]) * m
        ad = d.abs()
        loss = loss + (0.5 * ((ad - 1) * torch.clamp(ad, max=1.0) + ad)).sum() / B
    loss.backward()
    return P, mov, refine, loss


def _cos(a, b):
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    return float(torch.nn.functional.cosine_similarity(a, b, dim=0))


BF16_SPREAD = 3.0   # bf16: angular error (1 - cos vs fp64) within 3x that of a plain bf16 evaluation


def _bf16_ok(got, ref_bf16, truth, floor=0.02):
    """Conditioning-aware bf16 bound, the bf16 analogue of the fp32 '4x the fp32 oracle's
    spread' rule: 1 - cos(got, truth) <= max(floor, BF16_SPREAD * (1 - cos(ref_bf16, truth)))."""
    return 1.0 - _cos(got, truth) <= max(floor, BF16_SPREAD * (1.0 - _cos(ref_bf16, truth)))


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_refine_step_matches_oracle(dev, dtype):
    H, W, B = 160, 288, 2
    tr = Trainer((H, W), B, dtype=dtype, device=dev, learning_rate=1e-2, seed=1)
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=4)
    p0 = tr.net.store.flat.detach().clone()
    P32, mov32, ref32, loss32 = _oracle_step(tr, img, corner, labels, n, H, W, B, torch.float32)
    P64, mov64, ref64, loss64 = _oracle_step(tr, img, corner, labels, n, H, W, B, torch.float64)
    if dtype == torch.float32:
        # sensitivity of the fp64 truth itself to fp32-level noise (2 draws of 1e-6 relative
        # input noise): activation kinks (relu6 / leaky) near zero on the few-row pyramid
        # levels make some gradients legitimately jump under any fp32 evaluation order
        Pp = [_oracle_step(tr, img, corner, labels, n, H, W, B, torch.float64, perturb=1e-6, seed=s_)[0]
              for s_ in (11, 12)]
    if dtype == torch.bfloat16:
        # baseline: the same oracle step evaluated with every tensor in bf16 (PyTorch CPU)
        Pb, movb, refb, _ = _oracle_step(tr, img, corner, labels, n, H, W, B, torch.bfloat16)

    from nets.catch_net import factory
    import utils.net_tools as nt
    from utils.common_tools import cornerBboxes_2_centerBboxes
    x = ops.normalize_image(img, dtype)
    tg = nt.refine_groundtruth(tr.anchors, cornerBboxes_2_centerBboxes(corner), labels,
                               config.refine_method.JACCARD_BIGGER, n_boxes=n)
    out = factory(x, 'mobilenet_v2', True, tr.config_dict, dtype, net=tr.net).get_output()
    loss = nt.refine_loss(out, tg[0], tg[3], targets=tg)
    loss.backward()
    report = []
    for l, (a, o32, o64) in enumerate(zip(out, ref32, ref64)):
        e_h, e_o = _nerr(a, o64), _nerr(o32, o64)
        report.append((l, e_h, e_o))
        if dtype == torch.float32:
            assert e_h <= max(1e-4, 4 * e_o), report
        elif e_o < 1e-2 and _cos(refb[l], o64) >= 0.95:
            # where bf16 can represent the answer at all (a plain bf16 evaluation of the same
            # network reaches cos >= 0.95), stay within 3x its angular error
            assert _bf16_ok(a, refb[l], o64), (l, _cos(a, o64), _cos(refb[l], o64))
    print('per-level (hip err, oracle-fp32 err):', report)
    lt = 1e-4 if dtype == torch.float32 else 3e-2
    assert abs(loss.item() - loss64.item()) <= max(lt, 4 * abs(loss32.item() - loss64.item()) / abs(loss64.item())) * \
        abs(loss64.item()), (loss.item(), loss32.item(), loss64.item())
    for k, v in mov64.items():
        got = tr.net.store.buffers[k]
        e_o = _nerr(mov32[k], v)
        if dtype == torch.float32:
            assert _nerr(got, v) <= max(1e-4, 4 * e_o), k
        elif e_o < 1e-2 and _cos(movb[k].float(), v) >= 0.95:
            assert _bf16_ok(got, movb[k].float(), v), (k, _cos(got, v), _cos(movb[k].float(), v))
    bad = []
    for name, p in tr.net.store.params.items():
        g64, g32, gd = P64[name].grad, P32[name].grad, p._rod_grad
        e_o = _nerr(g32, g64)
        if dtype == torch.float32:
            e_h = _nerr(gd, g64)
            e_s = max(_nerr(pp[name].grad, g64) for pp in Pp)
            if e_h > max(2e-3, 4 * e_o, 4 * e_s):
                bad.append((name, e_h, e_o, e_s))
        elif e_o < 1e-2 and g64.abs().max() > 0 and _cos(Pb[name].grad.float(), g64) >= 0.95 and \
                not _bf16_ok(gd, Pb[name].grad.float(), g64):
            bad.append((name, _cos(gd, g64), _cos(Pb[name].grad.float(), g64), e_o))
    for b_ in bad:
        print('BAD', b_)
    assert not bad, [b_[0] for b_ in bad]
    # SGD with clip (net_tools.py:645-651), bit-exact given the gradient
    flat_g = tr.net.store.flat_grad.detach().clone()
    tr.opt.step()
    ref = (p0.cpu().numpy() - np.float32(1e-2) * np.clip(flat_g.cpu().numpy(), -5, 5)).astype(np.float32)
    np.testing.assert_array_equal(tr.net.store.flat.detach().cpu().numpy(), ref)


_DM, _MM = config.deconv_method, config.merge_method


@pytest.mark.parametrize('dm,mm,hw', [(_DM.LEARN_HALF, _MM.ADD, (320, 576)), (_DM.LEARN_ALL, _MM.ADD, (320, 576)),
                                      (_DM.LEARN_HALF, _MM.CONCAT, (320, 576)),
                                      (_DM.LEARN_ALL, _MM.CONCAT, (288, 512))],
                         ids=['half-add', 'all-add', 'half-concat', 'all-concat'])
def test_all_mode_step_matches_oracle(dev, dm, mm, hw):
    """train_range=ALL, fix_refine=True (train.py:140-249): outputs, det/clf losses and the
    gradients of every trainable (deconv / clf / det) parameter, for each deconv method
    (LEARN_HALF / LEARN_ALL, catch_net.py:177-230) and merge method (ADD / CONCAT, 237-273)."""
    from oracle import post as op
    import utils.net_tools as nt
    from nets.catch_net import factory
    from utils.common_tools import cornerBboxes_2_centerBboxes
    (H, W), B = hw, 2
    tr = Trainer((H, W), B, dtype=torch.float32, device=dev, train_range=config.train_range.ALL, seed=5,
                 deconv_method=dm, merge_method=mm)
    kw = dict(all_mode=True, learn_all=dm is _DM.LEARN_ALL, concat=mm is _MM.CONCAT)
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=6)
    P32 = {k: v.detach().cpu().clone().requires_grad_(v.requires_grad) for k, v in tr.net.store.params.items()}
    B32 = {k: v.detach().cpu().clone() for k, v in tr.net.store.buffers.items()}
    P64 = {k: v.detach().double().requires_grad_(v.requires_grad) for k, v in P32.items()}
    B64 = {k: v.double() for k, v in B32.items()}
    x = torch.from_numpy(np.float32(2.0 / 255.0) * img.cpu().numpy().astype(np.float32) - np.float32(1.0))
    o32 = onet.forward(x, P32, B32, True, moving={}, **kw)
    o64 = onet.forward(x.double(), P64, B64, True, moving={}, **kw)
    # a second fp32 evaluation with a different convolution algorithm (oneDNN off): the
    # spread between fp32 implementations bounds what any fp32 implementation can achieve
    P32b = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in P32.items()}
    torch.backends.mkldnn.enabled = False
    try:
        o32b = onet.forward(x, P32b, {k: v.clone() for k, v in B32.items()}, True, moving={}, **kw)
    finally:
        torch.backends.mkldnn.enabled = True

    xd = ops.normalize_image(img, torch.float32)
    tg = nt.refine_groundtruth(tr.anchors, cornerBboxes_2_centerBboxes(corner), labels,
                               config.refine_method.JACCARD_BIGGER, n_boxes=n)
    refine_out, det_out, clf_out = factory(xd, 'mobilenet_v2', True, tr.config_dict, torch.float32,
                                           net=tr.net).get_output()
    for got, r32, r64 in zip(refine_out + det_out + clf_out, o32[0] + o32[1] + o32[2], o64[0] + o64[1] + o64[2]):
        assert _nerr(got, r64) <= max(1e-4, 4 * _nerr(r32, r64))
    dgt = nt.det_groundtruth(refine_out, tg[0], tg[1], tg[2], tg[3], tr.anchors, targets=tg)
    d_loss, c_loss = nt.det_clf_loss(refine_out, clf_out, det_out, dgt, dgt[1], dgt[2], dgt[3])
    from rod import graph
    graph.backward(graph.scalar_sum(d_loss, c_loss))

    # oracle targets + losses evaluated on the HIP outputs, so that both backward passes see
    # the same hard-negative decisions (their bit-exactness given identical logits is
    # test_gpu_detect.py::test_det_targets_and_hnm_loss); this isolates the network backward
    tab = dgt.table
    cat = lambda ts, k: np.concatenate([t.detach().cpu().numpy().reshape(B, -1, k) for t in ts], 1)
    ro, do, co = cat(refine_out, 4), cat(det_out, 4), cat(clf_out, 11)
    rgt, cbox, lbl, pos = (t.cpu().numpy() for t in tg.flat)
    r_gt, r_pos, r_lbl, r_iou = op.det_groundtruth(tab.center_np, tab.lvl_off, config.det_pos_jac_val_all_layers,
                                                   ro, rgt, cbox, lbl, pos)
    ref = op.det_clf_loss(do, r_gt, r_pos, co, r_lbl, r_iou, tab.lvl_off, B)
    assert abs(d_loss.item() - ref['det_loss']) <= 1e-5 * abs(ref['det_loss'])
    assert abs(c_loss.item() - ref['clf_loss']) <= 1e-5 * abs(ref['clf_loss'])
    st = nt.det_clf_loss.last_stats.detach().cpu().numpy()
    assert st[3] == np.float32(ref['max_hard_pred']) and int(st[6]) == ref['n_neg_selected']
    # same upstream gradients into both oracle graphs; fp64 graph is the truth
    gd = torch.from_numpy(ref['g_det'])
    gc = torch.from_numpy(ref['g_logits'])

    def split(g, outs, k):
        res, off = [], 0
        for t in outs:
            nn_ = t[0].numel() // k
            res.append(g[:, off:off + nn_].reshape(t.shape))
            off += nn_
        return res
    torch.autograd.backward(list(o32[1]) + list(o32[2]), split(gd, o32[1], 4) + split(gc, o32[2], 11))
    torch.backends.mkldnn.enabled = False
    try:
        torch.autograd.backward(list(o32b[1]) + list(o32b[2]), split(gd, o32b[1], 4) + split(gc, o32b[2], 11))
    finally:
        torch.backends.mkldnn.enabled = True
    torch.autograd.backward(list(o64[1]) + list(o64[2]),
                            [t.double() for t in split(gd, o64[1], 4) + split(gc, o64[2], 11)])
    # sensitivity of the fp64 truth itself to fp32-level noise, as in the REFINE test (2 draws of
    # 1e-6 relative input noise, the same upstream gradients): activation kinks (leaky / relu6)
    # at zero in the heads move single gradient entries under ANY fp32 evaluation order
    Pp = []
    for s_ in (11, 12):
        gen = torch.Generator().manual_seed(s_)
        xp = x.double() * (1 + 1e-6 * torch.randn(x.shape, generator=gen, dtype=torch.float64))
        Pq = {k: v.detach().double().requires_grad_(v.requires_grad) for k, v in P32.items()}
        oq = onet.forward(xp, Pq, {k: v.double() for k, v in B32.items()}, True, moving={}, **kw)
        torch.autograd.backward(list(oq[1]) + list(oq[2]),
                                [t.double() for t in split(gd, oq[1], 4) + split(gc, oq[2], 11)])
        Pp.append(Pq)
    bad, checked = [], 0
    for name, p in tr.net.store.params.items():
        if not p.requires_grad:
            continue
        checked += 1
        g64, g32, g32b = P64[name].grad, P32[name].grad, P32b[name].grad
        if _bias_before_bn(name, g64, P64):
            # conv bias followed by a training-mode BatchNorm: its gradient is exactly zero
            # (the batch mean absorbs it), so only rounding residue is left on both sides
            wscale = float(P64[name.replace('/biases', '/weights')].grad.abs().max())
            if float(p._rod_grad.abs().max()) > 1e-4 * wscale:
                bad.append((name, float(p._rod_grad.abs().max()), wscale))
            continue
        e = _nerr(p._rod_grad, g64)
        spread = max(_nerr(g32, g64), _nerr(g32b, g64))
        e_s = max(_nerr(pq[name].grad, g64) for pq in Pp)
        if e > max(2e-3, 4 * spread, 4 * e_s):
            bad.append((name, e, spread, e_s))
        elif e > max(2e-3, 4 * spread):
            print('within the fp64 truth\'s own input-noise sensitivity:', name, e, spread, e_s)
    assert checked > 50 and not bad, bad[:10]


def _bias_before_bn(name, g64, P64):
    """A slim.conv2d bias whose conv feeds a training-mode BatchNorm (every head / deconv conv,
    catch_net.py:301-303): d loss / d bias = sum over rows of d loss / d (BN input) = 0 exactly."""
    w = name.replace('/biases', '/weights')
    if not name.endswith('/biases') or w not in P64 or P64[w].grad is None:
        return False
    return float(g64.abs().max()) <= 1e-6 * float(P64[w].grad.abs().max())


def test_all_mode_train_refine_matches_oracle(dev):
    """train_range=ALL, fix_refine=False (train.py:164-166: every variable trained, total_loss =
    refine + det + clf): the gradient reaches refine_out through the refine loss, through
    det_gt = (refine_gt - refine_out)*pos and through the IoU focal factor (net_tools.py:459-471,
    590-607; no stop-gradient).  Every parameter gradient (backbone and refine heads included)
    against the oracle's differentiable restatement (oracle.post.odm_losses_torch) in float64,
    with the integer decisions (ODM positives, hard negatives) taken from the HIP outputs as in
    test_all_mode_step_matches_oracle."""
    from oracle import post as op
    from rod import graph
    H, W, B = 320, 576, 2
    tr = Trainer((H, W), B, dtype=torch.float32, device=dev, train_range=config.train_range.ALL, seed=5,
                 fix_refine=False)
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=6)
    P32 = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in tr.net.store.params.items()}
    B32 = {k: v.detach().cpu().clone() for k, v in tr.net.store.buffers.items()}
    P64 = {k: v.detach().double().requires_grad_(True) for k, v in P32.items()}
    B64 = {k: v.double() for k, v in B32.items()}
    x = torch.from_numpy(np.float32(2.0 / 255.0) * img.cpu().numpy().astype(np.float32) - np.float32(1.0))
    o32 = onet.forward(x, P32, B32, True, all_mode=True, moving={})
    o64 = onet.forward(x.double(), P64, B64, True, all_mode=True, moving={})
    P32b = {k: v.detach().clone().requires_grad_(True) for k, v in P32.items()}
    torch.backends.mkldnn.enabled = False
    try:
        o32b = onet.forward(x, P32b, {k: v.clone() for k, v in B32.items()}, True, all_mode=True, moving={})
    finally:
        torch.backends.mkldnn.enabled = True
    # a third float32 implementation (PyTorch on the GPU): with the CPU runs it measures how far
    # independent float32 evaluations of this step scatter around float64 (the deep BatchNorms
    # see only a few dozen rows per channel at this size, so some sums cancel heavily)
    P32g = {k: v.detach().to(dev).requires_grad_(True) for k, v in P32.items()}
    o32g = onet.forward(x.to(dev), P32g, {k: v.to(dev) for k, v in B32.items()}, True, all_mode=True, moving={})

    losses = tr.losses(img, corner, labels, n)
    outs = [t for lv in tr.last_out for t in lv]
    g_out = torch.autograd.grad(losses[0], outs, retain_graph=True)
    graph.backward(losses[0])
    tg, dgt = tr.last_targets
    tab = dgt.table
    cat = lambda ts, k: torch.cat([t.reshape(B, -1, k) for t in ts], 1)
    np_ = lambda t: t.detach().cpu().numpy()
    # integer decisions from the HIP step (bit-exact with the numpy oracle given these outputs)
    rgt, cbox, lbl, rpos = (np_(t) for t in tg.flat)
    det_pos, det_lbl = np_(dgt.flat[1]), np_(dgt.flat[2])
    from utils import net_tools as nt
    stats = np_(nt.det_clf_loss.last_stats)
    # the hard-negative mask: recomputed by the numpy oracle from the HIP logits and positives
    clf_hip = np_(cat(tr.last_out[2], 11))
    ref = op.det_clf_loss(np.zeros((B, tab.A, 4), np.float32), np.zeros((B, tab.A, 4), np.float32), det_pos,
                          clf_hip, det_lbl, np_(dgt.flat[3]), tab.lvl_off, B)
    negmask = ref['negmask']
    assert stats[3] == np.float32(ref['max_hard_pred']) and int(stats[6]) == ref['n_neg_selected']

    def oracle_losses(o):
        return op.odm_losses_torch(tab.center_np, tab.lvl_off, cat(o[0], 4), cat(o[1], 4), cat(o[2], 11),
                                   rgt, cbox, rpos, det_pos, det_lbl, negmask, float(B))

    # 1) the loss backward alone, on the HIP outputs themselves (float64 oracle): gradients at
    #    refine_out (refine loss + det_gt + IoU factor), det_out and clf_out
    leaves = [[t.detach().double().cpu().requires_grad_(True) for t in lv] for lv in tr.last_out]
    rl, dl, cl = oracle_losses(leaves)
    for got, want in zip((losses[1], losses[2], losses[3]), (rl, dl, cl)):
        assert abs(got.item() - want.item()) <= 1e-5 * abs(want.item()), (got.item(), want.item())
    g_ref = torch.autograd.grad(rl + dl + cl, [t for lv in leaves for t in lv])
    for k, (gh, gr) in enumerate(zip(g_out, g_ref)):
        assert _nerr(gh, gr) < 1e-4, (k, _nerr(gh, gr))
    # 2) every parameter gradient through the network, against float64 / float32 oracle runs
    l64 = [float(v.detach()) for v in oracle_losses(o64)]
    (sum(oracle_losses(o64))).backward()
    (sum(oracle_losses(o32))).backward()
    torch.backends.mkldnn.enabled = False
    try:
        (sum(oracle_losses(o32b))).backward()
    finally:
        torch.backends.mkldnn.enabled = True
    og = [[t.cpu() for t in lv] for lv in o32g]
    gg = torch.autograd.grad(sum(oracle_losses(og)), [t for lv in og for t in lv])
    torch.autograd.backward([t for lv in o32g for t in lv], [g.to(dev) for g in gg])
    # the fp64 truth under 1e-6 relative input noise (2 draws, the same integer decisions), as in
    # the other step tests: leaky / relu6 gates at zero move single gradients under any fp32 order
    Pp = []
    for s_ in (11, 12):
        gen = torch.Generator().manual_seed(s_)
        xp = x.double() * (1 + 1e-6 * torch.randn(x.shape, generator=gen, dtype=torch.float64))
        Pq = {k: v.detach().double().requires_grad_(True) for k, v in P32.items()}
        oq = onet.forward(xp, Pq, {k: v.double() for k, v in B32.items()}, True, all_mode=True, moving={})
        (sum(oracle_losses(oq))).backward()
        Pp.append(Pq)
    assert abs(losses[2].item() - l64[1]) <= 1e-4 * abs(l64[1])
    assert abs(losses[3].item() - l64[2]) <= 1e-4 * abs(l64[2])
    # Tolerance: 4x the float32 scatter, as in the other step tests.  One exception is allowed in
    # the deepest backbone blocks: at 320x576 their BatchNorms see 30-360 rows per channel and a
    # ReLU6 input within float32 noise of the clamp (e.g. seed 5/6, expanded_conv_18/depthwise
    # channel 532: -2.2e-5 in float64) flips its mask in one float32 evaluation and not in
    # another, moving that channel's gradient by one element's contribution.  Backbone tensors
    # may therefore exceed the bound only by such isolated flips: at most 3% of them, and still
    # within 0.25 normwise.  Heads, deconv and every loss gradient at the outputs stay strict.
    bad, flips, checked = [], [], 0
    for name, p in tr.net.store.params.items():
        g64, g32, g32b, g32g = P64[name].grad, P32[name].grad, P32b[name].grad, P32g[name].grad
        if g64 is None:
            continue
        checked += 1
        e = _nerr(p._rod_grad, g64)
        spread = max(_nerr(g32, g64), _nerr(g32b, g64), _nerr(g32g, g64))
        e_s = max(_nerr(pq[name].grad, g64) for pq in Pp if pq[name].grad is not None)
        if e > max(2e-3, 4 * spread, 4 * e_s):
            (flips if name.startswith('backbone/') and e < 0.25 else bad).append((name, e, spread, e_s))
        elif e > max(2e-3, 4 * spread):
            print('within the fp64 truth\'s own input-noise sensitivity:', name, e, spread, e_s)
    n_backbone = sum(1 for k in tr.net.store.params if k.startswith('backbone/'))
    assert checked > 200 and not bad, bad[:10]
    assert len(flips) <= 0.03 * n_backbone, flips


def test_trainer_steps_reduce_loss(dev):
    H, W, B = 96, 160, 2
    tr = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, learning_rate=5e-2, seed=2)
    batch = synthetic_batch(B, H, W, dev, seed=5)
    losses = [tr.step(*batch)[0].item() for _ in range(8)]
    assert np.isfinite(losses).all()
    assert losses[-1] < losses[0], losses


def test_step_graphed_bit_identical(dev):
    """Trainer.step_graphed (the step captured once as a HIP graph and replayed) runs exactly
    the eager step: parameters, moving statistics and losses bit-identical after 4 steps."""
    H, W, B = 160, 288, 2
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=21)
    ta = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=2)
    tb = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=2)
    for _ in range(4):
        la = ta.step(img, corner, labels, n)
        lb = tb.step_graphed(img, corner, labels, n)
    torch.cuda.synchronize()
    assert tb._graph is not None
    assert torch.equal(ta.net.store.flat, tb.net.store.flat)
    for k, v in ta.net.store.buffers.items():
        assert torch.equal(v, tb.net.store.buffers[k]), k
    assert torch.equal(la[0], lb[0])
    # host-side step state advances once per replay, as it does per eager step
    assert ta.opt.global_step == tb.opt.global_step == 4
    assert tb.net.store.version == ta.net.store.version


@pytest.mark.parametrize('train_range', ['REFINE', 'ALL'])
def test_deferred_slab_sums_bit_identical(dev, train_range):
    """Trainer.step batches the weight-gradient slab sums into a few launches (rod_slab_defer /
    rod_slab_flush, ABI 11): parameters, moving statistics and losses after two steps are
    bit-identical to the immediate per-entry sums (ROD_DISABLE=slabdefer), and nothing is left
    queued after a step."""
    from rod import _abi
    H, W, B = 160, 288, 2
    rng = getattr(config.train_range, train_range)
    img, corner, labels, n = synthetic_batch(B, H, W, dev, seed=23)
    runs, queued = [], []
    real_flush = ops.SLAB.flush

    def counting_flush():   # how many sums were queued when the flush ran
        queued.append(_abi.lib().rod_slab_pending())
        real_flush()
    for off in (True, False):
        if off:
            ops._DISABLE.add('slabdefer')
        ops.SLAB.flush = counting_flush
        try:
            tr = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=2, train_range=rng, fix_refine=False)
            ls = [tr.step(img, corner, labels, n)[0].clone() for _ in range(2)]
        finally:
            ops._DISABLE.discard('slabdefer')
            ops.SLAB.flush = real_flush
        if not off:
            assert max(queued) > 50, queued   # the step's weight-gradient sums were batched
        torch.cuda.synchronize()
        assert _abi.lib().rod_slab_pending() == 0
        runs.append((tr.net.store.flat.clone(), {k: v.clone() for k, v in tr.net.store.buffers.items()}, ls))
    (fa, ba, la), (fb, bb, lb) = runs
    assert torch.equal(fa, fb)
    assert all(torch.equal(v, bb[k]) for k, v in ba.items())
    assert all(torch.equal(x, y) for x, y in zip(la, lb))
