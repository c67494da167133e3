"""ORACLE (test infrastructure only): ODM targets, classification loss with hard-negative
mining, per-class NMS and VOC AP — numpy restatements of the reference:

  det_groundtruth        utils/net_tools.py:431-475
  det_clf_loss           utils/net_tools.py:519-623
  detected_bboxes        utils/net_tools.py:658-758 + tf_extended/bboxes.py:60-232
                         (tf.image.non_max_suppression semantics of TF 1.x CPU kernel)
  bboxes_matching        tf_extended/bboxes.py:246-334, 452-479 (bboxes_jaccard)
  streaming_ap           evaluate.py:146-208 + tf_extended/metrics.py:100-258 (TP/FP arrays,
                         precision / recall, VOC07 / VOC12 AP)

float32 per-op arithmetic; exp/log correctly rounded via float64 (same convention as the
kernels); sums of losses in float64."""
import numpy as np

from .targets import center_to_corner, exp_cr, log_cr

f32 = np.float32


def decode_corner(anc_center, off):
    """corner(decode(anchor, off)); anc_center [A,4] (cy,cx,h,w), off [..., A, 4]."""
    acy, acx, ah, aw = (anc_center[:, i] for i in range(4))
    o = np.asarray(off, f32)
    cy = o[..., 0] * ah + acy
    cx = o[..., 1] * aw + acx
    h = exp_cr(o[..., 2]) * ah
    w = exp_cr(o[..., 3]) * aw
    return np.stack([cy - h / f32(2), cx - w / f32(2), cy + h / f32(2), cx + w / f32(2)], -1)


def pair_jaccard(a, g):
    """jaccard (net_tools.py:237-267) of corresponding boxes a[..., 4], g[..., 4]."""
    vol_a = (a[..., 3] - a[..., 1]) * (a[..., 2] - a[..., 0])
    ih = np.maximum(np.minimum(a[..., 2], g[..., 2]) - np.maximum(a[..., 0], g[..., 0]), f32(0))
    iw = np.maximum(np.minimum(a[..., 3], g[..., 3]) - np.maximum(a[..., 1], g[..., 1]), f32(0))
    inter = ih * iw
    union = vol_a - inter + (g[..., 2] - g[..., 0]) * (g[..., 3] - g[..., 1])
    with np.errstate(all='ignore'):
        return inter / union


def det_groundtruth(anc_center, lvl_off, thr, refine_out, refine_gt, cbox, label, refine_pos):
    """All arrays concatenated over levels: refine_out/refine_gt/cbox [B,A,4], label/pos [B,A]."""
    adj = decode_corner(anc_center, refine_out)
    gc = center_to_corner(cbox)
    iou = pair_jaccard(adj, gc)
    A = anc_center.shape[0]
    lvl = np.searchsorted(np.asarray(lvl_off[1:-1]), np.arange(A), side='right')
    t = np.asarray(thr, f32)[lvl]
    pos = (iou >= t[None, :]).astype(np.int32) * np.asarray(refine_pos, np.int32)
    det_gt = (np.asarray(refine_gt, f32) - np.asarray(refine_out, f32)) * pos[..., None].astype(f32)
    return det_gt, pos, np.asarray(label, np.int32) * pos, iou


def softmax_rows(logits):
    x = np.asarray(logits, f32)
    m = x.max(-1, keepdims=True)
    e = exp_cr(x - m)
    s = np.zeros(x.shape[:-1] + (1,), f32)
    for k in range(x.shape[-1]):  # sequential float32 sum, class order
        s = s + e[..., k:k + 1]
    return e, s, m


def iou_factor(iou, B, lvl_off):
    """net_tools.py:590-600 per (image, level) group."""
    out = np.zeros_like(iou, dtype=f32)
    for b in range(B):
        for l in range(len(lvl_off) - 1):
            u = iou[b, lvl_off[l]:lvl_off[l + 1]].astype(f32)
            mean = f32(np.mean(u, dtype=np.float64))
            var = f32(np.mean(((u - mean) * (u - mean)).astype(np.float64)))
            sd = np.sqrt(var + f32(1e-8)).astype(f32)
            z = (u - mean) / sd
            z = z + (f32(0) - z.min())
            z = z / (z.max() + f32(1e-8))
            out[b, lvl_off[l]:lvl_off[l + 1]] = np.power(z, f32(4)).astype(f32)
    return out


def det_clf_loss(det_out, det_gt, det_pos, clf_logits, det_lbl, iou, lvl_off, bs):
    """Returns dict of losses/stats and gradients wrt det_out and clf_logits (flattened
    [B, A, .] layouts)."""
    B, A, K = clf_logits.shape
    m = det_pos.astype(f32)[..., None]
    d = (det_gt - np.asarray(det_out, f32)) * m
    ad = np.abs(d)
    sl1 = f32(0.5) * ((ad - f32(1)) * np.minimum(ad, f32(1)) + ad)
    det_loss = float(np.sum(sl1, dtype=np.float64)) / bs
    g_det = (-m * np.clip(d, -1, 1) / f32(bs)).astype(f32)

    logits = np.asarray(clf_logits, f32).reshape(-1, K)
    pmask = det_pos.reshape(-1) != 0
    e, s, mx = softmax_rows(logits)
    p0 = (e[:, 0:1] / s)[:, 0]
    nvalues = np.where(~pmask, p0, f32(1.0)).astype(f32)
    n_pos = int(pmask.sum())
    n_neg_tot = int((~pmask).sum())
    k = min(int(f32(3.0) * f32(n_pos)) + B, n_neg_tot)
    thr = np.sort(nvalues)[k - 1] if k > 0 else f32(0)
    negmask = np.logical_and(~pmask, nvalues < thr)
    iouf = iou_factor(iou, B, lvl_off).reshape(-1)
    lse = log_cr(s[:, 0])
    lab = det_lbl.reshape(-1)
    ce_lab = lse - (logits[np.arange(logits.shape[0]), lab] - mx[:, 0])
    ce0 = lse - (logits[:, 0] - mx[:, 0])
    pos_loss = float(np.sum(np.where(pmask, ce_lab * iouf, 0), dtype=np.float64)) / bs
    neg_loss = float(np.sum(np.where(negmask, ce0, 0), dtype=np.float64)) / bs
    p = e / s
    onehot = np.eye(K, dtype=f32)
    g = np.where(pmask[:, None], (iouf / f32(bs))[:, None] * (p - onehot[lab]), 0) + \
        np.where(negmask[:, None], f32(0.5 / bs) * (p - onehot[0]), 0)
    return {'det_loss': det_loss, 'pos_loss': pos_loss, 'neg_loss': neg_loss,
            'clf_loss': neg_loss / 2 + pos_loss, 'max_hard_pred': float(thr), 'n_pos': n_pos, 'k': k,
            'n_neg_selected': int(negmask.sum()), 'negmask': negmask, 'g_det': g_det,
            'g_logits': g.reshape(B, A, K).astype(f32), 'iouf': iouf}


def tf_nms_iou(bi, bj):
    """IOU of tensorflow/core/kernels/non_max_suppression_op.cc (TF 1.x)."""
    ymin_i, xmin_i = min(bi[0], bi[2]), min(bi[1], bi[3])
    ymax_i, xmax_i = max(bi[0], bi[2]), max(bi[1], bi[3])
    ymin_j, xmin_j = min(bj[0], bj[2]), min(bj[1], bj[3])
    ymax_j, xmax_j = max(bj[0], bj[2]), max(bj[1], bj[3])
    area_i = f32(ymax_i - ymin_i) * f32(xmax_i - xmin_i)
    area_j = f32(ymax_j - ymin_j) * f32(xmax_j - xmin_j)
    if area_i <= 0 or area_j <= 0:
        return f32(0)
    ih = max(f32(min(ymax_i, ymax_j) - max(ymin_i, ymin_j)), f32(0))
    iw = max(f32(min(xmax_i, xmax_j) - max(xmin_i, xmin_j)), f32(0))
    inter = f32(ih * iw)
    return f32(inter / f32(f32(area_i + area_j) - inter))


def detected_bboxes(probs, boxes, select_threshold, nms_threshold, top_k, keep_top_k):
    """probs [B,A,K], corner boxes [B,A,4] -> scores [B,K-1,keep], boxes [B,K-1,keep,4],
    and the kept anchor indices per (b, c)."""
    probs = np.asarray(probs, f32)
    boxes = np.asarray(boxes, f32)
    B, A, K = probs.shape
    out_s = np.zeros((B, K - 1, keep_top_k), f32)
    out_b = np.zeros((B, K - 1, keep_top_k, 4), f32)
    kept_idx = {}
    for b in range(B):
        for c in range(1, K):
            p = probs[b, :, c]
            fm = (p >= f32(select_threshold)).astype(f32)
            s = p * fm
            bx = boxes[b] * fm[:, None]
            order = np.argsort(-s, kind='stable')[:min(top_k, A)]  # top_k: desc, ties by index
            sel = []
            for i in order:
                ok = True
                for j in reversed(sel):
                    v = tf_nms_iou(bx[i], bx[j])
                    if v == 0:
                        continue
                    if v > f32(nms_threshold):
                        ok = False
                        break
                if ok:
                    sel.append(i)
                    if len(sel) == keep_top_k:
                        break
            kept_idx[(b, c)] = sel
            out_s[b, c - 1, :len(sel)] = s[sel]
            out_b[b, c - 1, :len(sel)] = bx[sel]
    return out_s, out_b, kept_idx


def bboxes_jaccard_one(ref, g):
    """bboxes_jaccard (tf_extended/bboxes.py:452-479) of ONE detection against each ground
    truth box, float32 per op in TF's evaluation order; safe_divide -> 0 when union <= 0."""
    int_ymin = max(g[0], ref[0])
    int_xmin = max(g[1], ref[1])
    int_ymax = min(g[2], ref[2])
    int_xmax = min(g[3], ref[3])
    h = max(f32(int_ymax - int_ymin), f32(0))
    w = max(f32(int_xmax - int_xmin), f32(0))
    inter = f32(h * w)
    union = f32(f32(-inter + f32(f32(g[2] - g[0]) * f32(g[3] - g[1]))) + f32(f32(ref[2] - ref[0]) * f32(ref[3] - ref[1])))
    return f32(inter / union) if union > 0 else f32(0)


def bboxes_matching(label, scores, bboxes, glabels, gbboxes, gdifficults, thr=0.5):
    """bboxes_matching (tf_extended/bboxes.py:246-334), one image, a plain loop over the
    score-sorted detections: best ground truth of the same label by IoU (argmax: first
    maximum), TP if above `thr` (strict) and not yet matched, FP if matched already or below;
    difficult ground truth records neither.  Returns (n_gt, tp list, fp list)."""
    n_gt = sum(1 for lb, d in zip(glabels, gdifficults) if lb == label and not d)
    gmatch = [False] * len(glabels)
    tp, fp = [], []
    for i in range(len(scores)):
        if len(glabels) == 0:
            tp.append(False)
            fp.append(True)
            continue
        jac = [bboxes_jaccard_one(bboxes[i], gbboxes[j]) * f32(1.0 if glabels[j] == label else 0.0)
               for j in range(len(glabels))]
        idx = max(range(len(jac)), key=lambda j: (jac[j], -j))
        match = jac[idx] > thr
        nd = not gdifficults[idx]
        tp.append(nd and match and not gmatch[idx])
        fp.append(nd and (gmatch[idx] or not match))
        if nd and match:
            gmatch[idx] = True
    return n_gt, tp, fp


def streaming_ap(batches, classes, thr=0.5, counts=False):
    """evaluate.py:146-208 over a list of batches, each (scores {c: [B, N]}, boxes {c: [B, N, 4]},
    glabels [B, G], gboxes [B, G, 4], gcount [B]): matching per image and class, the streaming
    TP/FP arrays (metrics.py:133-206: rows with tp or fp and score > 1e-4 are kept, in batch
    order), then VOC07 / VOC12 AP per class (voc_ap).  Returns ({c: ap07}, {c: ap12}) (and
    {c: (n_tp, n_fp, n_gt)} with counts=True)."""
    acc = {c: ([], [], [], 0) for c in classes}
    for scores, boxes, glabels, gboxes, gcount in batches:
        for c in classes:
            tps, fps, scs, ng = acc[c]
            for b in range(len(gcount)):
                g = int(gcount[b])
                n, tp, fp = bboxes_matching(c, scores[c][b], boxes[c][b], list(glabels[b, :g]), gboxes[b, :g],
                                            [False] * g, thr)
                ng += n
                for t, f_, sc in zip(tp, fp, scores[c][b]):
                    if (t or f_) and sc > f32(1e-4):
                        tps.append(t)
                        fps.append(f_)
                        scs.append(float(sc))
            acc[c] = (tps, fps, scs, ng)
    ap07 = {c: voc_ap(a[0], a[1], a[2], a[3], True) for c, a in acc.items()}
    ap12 = {c: voc_ap(a[0], a[1], a[2], a[3], False) for c, a in acc.items()}
    if counts:
        return ap07, ap12, {c: (sum(a[0]), sum(a[1]), a[3]) for c, a in acc.items()}
    return ap07, ap12


def voc_ap(tp, fp, scores, n_gt, voc07=True):
    """Independent restatement of precision_recall + average_precision_voc07/12."""
    order = sorted(range(len(scores)), key=lambda i: (-scores[i], i))
    ctp = cfp = 0.0
    prec, rec = [], []
    for i in order:
        ctp += float(tp[i])
        cfp += float(fp[i])
        rec.append(ctp / n_gt if n_gt > 0 else 0.0)
        prec.append(ctp / (ctp + cfp) if ctp + cfp > 0 else 0.0)
    if voc07:
        ap = 0.0
        for t in np.arange(0., 1.1, 0.1):  # the reference's thresholds, float64 arange values
            cands = [p for p, r in zip(prec + [0.0], rec + [float('inf')]) if r >= t]
            ap += max(cands) / 11.0
        return ap
    p = [0.0] + prec + [0.0]
    r = [0.0] + rec + [1.0]
    for i in range(len(p) - 2, -1, -1):
        p[i] = max(p[i], p[i + 1])
    return sum(p[i + 1] * (r[i + 1] - r[i]) for i in range(len(p) - 1))


def odm_losses_torch(anc_center, lvl_off, refine_out, det_out, logits, refine_gt, cbox, refine_pos, det_pos, det_lbl,
                     negmask, bs):
    """Differentiable restatement (PyTorch-CPU, any float dtype; test infrastructure) of the
    ALL-mode losses when the refine net is trained (train.py:144-166, fix_refine=False):
    refine_loss (net_tools.py:492-516), det_groundtruth (431-475: det_gt and iou depend on
    refine_out, no stop-gradient) and det_clf_loss (519-623: smooth-L1, sparse softmax CE,
    IoU focal factor through tf.nn.moments / reduce_min / reduce_max / pow).  The integer
    decisions (det_pos, det_lbl, the hard-negative mask) are inputs (constants), as they are
    non-differentiable in the reference.  TF gradient rules are kept: maximum / minimum send
    the gradient to their first argument on ties (where), reduce_min / reduce_max split it
    evenly over ties (torch amin / amax do the same), moments' variance uses
    stop_gradient(mean).  Tensors [B, A, .]; returns (refine_loss, det_loss, clf_loss)."""
    import torch
    T = refine_out.dtype
    ro, do, lg = refine_out, det_out, logits
    B, A, K = lg.shape
    ac = torch.from_numpy(np.asarray(anc_center)).to(T)
    t = lambda a: torch.from_numpy(np.asarray(a)).to(T)
    rgt, cb = t(refine_gt), t(cbox)
    rpos, dpos = t(refine_pos)[..., None], t(det_pos)[..., None]

    def tmax(a, b):
        return torch.where(a >= b, a, b)

    def tmin(a, b):
        return torch.where(a <= b, a, b)

    def smooth_l1(x):
        ax = torch.abs(x)
        return 0.5 * ((ax - 1) * tmin(ax, torch.ones_like(ax)) + ax)
    refine_loss = smooth_l1((rgt - ro) * rpos).sum() / bs
    # decode -> corners -> jaccard against the matched GT box
    cy = ro[..., 0] * ac[:, 2] + ac[:, 0]
    cx = ro[..., 1] * ac[:, 3] + ac[:, 1]
    h = torch.exp(ro[..., 2]) * ac[:, 2]
    w = torch.exp(ro[..., 3]) * ac[:, 3]
    ay0, ax0, ay1, ax1 = cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2
    gy0, gx0 = cb[..., 0] - cb[..., 2] / 2, cb[..., 1] - cb[..., 3] / 2
    gy1, gx1 = cb[..., 0] + cb[..., 2] / 2, cb[..., 1] + cb[..., 3] / 2
    vol_a = (ax1 - ax0) * (ay1 - ay0)
    zero = torch.zeros_like(ay0)
    ih = tmax(tmin(ay1, gy1) - tmax(ay0, gy0), zero)
    iw = tmax(tmin(ax1, gx1) - tmax(ax0, gx0), zero)
    inter = ih * iw
    iou = inter / (vol_a - inter + (gy1 - gy0) * (gx1 - gx0))
    det_gt = (rgt - ro) * dpos
    det_loss = smooth_l1((det_gt - do) * dpos).sum() / bs
    # IoU focal factor per (image, level)
    fs = []
    for l in range(len(lvl_off) - 1):
        u = iou[:, lvl_off[l]:lvl_off[l + 1]]
        mean = u.mean(1, keepdim=True)
        var = ((u - mean.detach()) ** 2).mean(1, keepdim=True)
        z = (u - mean) / torch.sqrt(var + 1e-8)
        z = z + (0. - z.amin(1, keepdim=True))
        z = z / (z.amax(1, keepdim=True) + 1e-8)
        fs.append(z ** 4)
    iouf = torch.cat(fs, 1)
    lsm = torch.log_softmax(lg, -1)
    lab = torch.from_numpy(np.asarray(det_lbl, np.int64))
    ce_lab = -lsm.gather(-1, lab[..., None])[..., 0]
    ce0 = -lsm[..., 0]
    pm = t(det_pos)
    nm = t(np.asarray(negmask).reshape(B, A))
    pos_loss = (ce_lab * pm * iouf).sum() / bs
    neg_loss = (ce0 * nm).sum() / bs
    return refine_loss, det_loss, neg_loss / 2 + pos_loss


def _nms_iou_vec(bi, bj):
    """tf_nms_iou of box bi [4] against boxes bj [n, 4], same float32 operations."""
    ymin_i, xmin_i = min(bi[0], bi[2]), min(bi[1], bi[3])
    ymax_i, xmax_i = max(bi[0], bi[2]), max(bi[1], bi[3])
    ymin_j, xmin_j = np.minimum(bj[:, 0], bj[:, 2]), np.minimum(bj[:, 1], bj[:, 3])
    ymax_j, xmax_j = np.maximum(bj[:, 0], bj[:, 2]), np.maximum(bj[:, 1], bj[:, 3])
    area_i = f32(ymax_i - ymin_i) * f32(xmax_i - xmin_i)
    area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j)
    ih = np.maximum(np.minimum(ymax_i, ymax_j) - np.maximum(ymin_i, ymin_j), f32(0))
    iw = np.maximum(np.minimum(xmax_i, xmax_j) - np.maximum(xmin_i, xmin_j), f32(0))
    inter = ih * iw
    with np.errstate(all='ignore'):
        v = inter / ((area_i + area_j) - inter)
    return np.where((area_i <= 0) | (area_j <= 0), f32(0), v).astype(f32)


def detected_bboxes_vec(probs, boxes, select_threshold, nms_threshold, top_k, keep_top_k):
    """detected_bboxes with the greedy NMS vectorised over the kept set (identical float32
    operations and decisions; for the full-size B=32 parity test)."""
    probs = np.asarray(probs, f32)
    boxes = np.asarray(boxes, f32)
    B, A, K = probs.shape
    out_s = np.zeros((B, K - 1, keep_top_k), f32)
    out_b = np.zeros((B, K - 1, keep_top_k, 4), f32)
    kept_idx = {}
    for b in range(B):
        for c in range(1, K):
            p = probs[b, :, c]
            fm = (p >= f32(select_threshold)).astype(f32)
            s = p * fm
            bx = boxes[b] * fm[:, None]
            order = np.argsort(-s, kind='stable')[:min(top_k, A)]
            sel = []
            kb = np.zeros((0, 4), f32)
            for i in order:
                if len(sel) and (_nms_iou_vec(bx[i], kb) > f32(nms_threshold)).any():
                    continue
                sel.append(int(i))
                kb = np.concatenate([kb, bx[i][None]], 0)
                if len(sel) == keep_top_k:
                    break
            kept_idx[(b, c)] = sel
            out_s[b, c - 1, :len(sel)] = s[sel]
            out_b[b, c - 1, :len(sel)] = bx[sel]
    return out_s, out_b, kept_idx
