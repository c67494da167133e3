"""utils/tf_extended/bboxes.py — box algebra and detection <-> ground-truth matching.

Host numpy float32 (the reference evaluates these on the CPU, evaluate.py:146).  The
sort/NMS entry points (bboxes_sort, bboxes_nms_batch) run on the GPU through
rod_select_topk_nms (one launch per class; net_tools.detected_bboxes fuses select + sort +
NMS of all classes into one).
"""
import numpy as np

from utils.tf_extended.math import safe_divide

__all__ = ['bboxes_sort', 'bboxes_nms_batch', 'bboxes_clip', 'bboxes_resize', 'bboxes_matching',
           'bboxes_matching_batch', 'bboxes_filter_overlap', 'bboxes_jaccard', 'bboxes_intersection',
           'bboxes_flip_left_right']

f32 = np.float32


def bboxes_jaccard(bbox_ref, bboxes, name=None):
    """IoU of a reference box with boxes, safe-divided (bboxes.py:452-479)."""
    r = np.asarray(bbox_ref, f32).T
    b = np.asarray(bboxes, f32).T
    int_ymin = np.maximum(b[0], r[0])
    int_xmin = np.maximum(b[1], r[1])
    int_ymax = np.minimum(b[2], r[2])
    int_xmax = np.minimum(b[3], r[3])
    h = np.maximum(int_ymax - int_ymin, f32(0.))
    w = np.maximum(int_xmax - int_xmin, f32(0.))
    inter = h * w
    union = -inter + (b[2] - b[0]) * (b[3] - b[1]) + (r[2] - r[0]) * (r[3] - r[1])
    return safe_divide(inter, union).astype(f32)


def bboxes_intersection(bbox_ref, bboxes, name=None):
    """Intersection / area of each box (bboxes.py:482-508)."""
    r = np.asarray(bbox_ref, f32).T
    b = np.asarray(bboxes, f32).T
    h = np.maximum(np.minimum(b[2], r[2]) - np.maximum(b[0], r[0]), f32(0.))
    w = np.maximum(np.minimum(b[3], r[3]) - np.maximum(b[1], r[1]), f32(0.))
    return safe_divide(h * w, (b[2] - b[0]) * (b[3] - b[1])).astype(f32)


def bboxes_clip(bbox_ref, bboxes, scope=None):
    """bboxes.py:103-136."""
    if isinstance(bboxes, dict):
        return {c: bboxes_clip(bbox_ref, b) for c, b in bboxes.items()}
    r = np.asarray(bbox_ref, f32)
    b = np.asarray(bboxes, f32)
    ymin = np.maximum(b[..., 0], r[0])
    xmin = np.maximum(b[..., 1], r[1])
    ymax = np.minimum(b[..., 2], r[2])
    xmax = np.minimum(b[..., 3], r[3])
    return np.stack([np.minimum(ymin, ymax), np.minimum(xmin, xmax), ymax, xmax], -1)


def bboxes_resize(bbox_ref, bboxes, name=None):
    """Re-normalise boxes to a crop window bbox_ref (bboxes.py:139-163)."""
    if isinstance(bboxes, dict):
        return {c: bboxes_resize(bbox_ref, b) for c, b in bboxes.items()}
    r = np.asarray(bbox_ref, f32)
    b = np.asarray(bboxes, f32) - np.array([r[0], r[1], r[0], r[1]], f32)
    s = np.array([r[2] - r[0], r[3] - r[1], r[2] - r[0], r[3] - r[1]], f32)
    return b / s


def bboxes_filter_overlap(labels, bboxes, threshold=0.5, assign_negative=False, scope=None):
    """Drop boxes whose fraction inside [0,0,1,1] is <= threshold (bboxes.py:408-428)."""
    scores = bboxes_intersection(np.array([0, 0, 1, 1], f32), bboxes)
    mask = scores > threshold
    if assign_negative:
        return np.where(mask, labels, -np.asarray(labels)), bboxes
    return np.asarray(labels)[mask], np.asarray(bboxes)[mask]


def bboxes_flip_left_right(bboxes):
    """Box part of random_flip_left_right (tf_image.py:284-290)."""
    b = np.asarray(bboxes, f32)
    return np.stack([b[..., 0], 1 - b[..., 3], b[..., 2], 1 - b[..., 1]], -1)


def _select_one_class(scores, bboxes, top_k, keep_top_k, nms_threshold):
    """rod_select_topk_nms on ONE class's [B, N] scores and [B, N, 4] boxes (device tensors):
    the scores become column 1 of a [B, N, 2] table (column 0, the background, is ignored by
    the kernel), select threshold 0 keeps every row (scores are probabilities, >= 0), so the
    kernel runs top-k (descending, ties to the lower index) and greedy NMS only."""
    import torch
    from rod import ops
    s = torch.as_tensor(scores)
    b = torch.as_tensor(bboxes)
    if s.device.type != 'cuda':
        raise ValueError('bboxes_sort / bboxes_nms_batch run on the GPU: pass cuda tensors')
    B, N = s.shape
    probs = torch.zeros((B, N, 2), dtype=torch.float32, device=s.device)
    probs[..., 1] = s.float()
    out_s, out_b = ops.select_topk_nms(probs, b.float().contiguous(), 0.0, top_k, keep_top_k, nms_threshold,
                                       compact=False)
    return out_s[:, 0], out_b[:, 0]


def bboxes_sort(scores, bboxes, top_k=400, scope=None):
    """bboxes.py:60-100: the top_k scores of every image in decreasing order (tf.nn.top_k,
    ties to the lower index) with their boxes gathered — [B, top_k], [B, top_k, 4]; dict
    inputs (one entry per class) give dicts.  Scores must be >= 0 (class probabilities, as at
    the reference's only call site, net_tools.py:750) and top_k <= min(N, 1024)."""
    if isinstance(scores, dict) or isinstance(bboxes, dict):
        out = {c: bboxes_sort(scores[c], bboxes[c], top_k) for c in scores}
        return {c: v[0] for c, v in out.items()}, {c: v[1] for c, v in out.items()}
    if top_k > scores.shape[-1]:
        raise ValueError('bboxes_sort: top_k %d > %d scores (tf.nn.top_k fails the same way)'
                         % (top_k, scores.shape[-1]))
    # no suppression: an IoU is never > +inf
    return _select_one_class(scores, bboxes, top_k, top_k, float('inf'))


def bboxes_nms_batch(scores, bboxes, nms_threshold=0.5, keep_top_k=200, scope=None):
    """bboxes.py:192-232: tf.image.non_max_suppression per image (greedy in score order, a box
    is dropped when its IoU with a kept one is > nms_threshold), the kept scores / boxes in
    score order, zero-padded to keep_top_k — [B, keep_top_k], [B, keep_top_k, 4]; dicts per
    class as in the reference.  N <= 1024 candidates per image (the output of bboxes_sort)."""
    if isinstance(scores, dict) or isinstance(bboxes, dict):
        out = {c: bboxes_nms_batch(scores[c], bboxes[c], nms_threshold, keep_top_k) for c in scores}
        return {c: v[0] for c, v in out.items()}, {c: v[1] for c, v in out.items()}
    return _select_one_class(scores, bboxes, scores.shape[-1], keep_top_k, nms_threshold)


def bboxes_matching(label, scores, bboxes, glabels, gbboxes, gdifficults, matching_threshold=0.5, scope=None):
    """Greedy matching of score-sorted detections of class `label` with ground truth
    (bboxes.py:246-334).  Returns (n_gbboxes, tp [N] bool, fp [N] bool)."""
    scores = np.asarray(scores)
    bboxes = np.asarray(bboxes, f32)
    glabels = np.asarray(glabels)
    gbboxes = np.asarray(gbboxes, f32)
    gdiff = np.asarray(gdifficults).astype(bool)
    n_g = int(np.count_nonzero(np.logical_and(glabels == label, ~gdiff)))
    gmatch = np.zeros(glabels.shape, bool)
    tp = np.zeros(scores.shape, bool)
    fp = np.zeros(scores.shape, bool)
    same = (glabels == label).astype(f32)
    for i in range(scores.shape[0]):
        jac = bboxes_jaccard(bboxes[i], gbboxes) * same
        idx = int(np.argmax(jac)) if jac.size else 0
        if jac.size == 0:
            fp[i] = True
            continue
        match = jac[idx] > matching_threshold
        existing = gmatch[idx]
        nd = not gdiff[idx]
        tp[i] = nd and match and not existing
        fp[i] = nd and (existing or not match)
        if nd and match:
            gmatch[idx] = True
    return n_g, tp, fp


def bboxes_matching_batch(labels, scores, bboxes, glabels, gbboxes, gdifficults, matching_threshold=0.5,
                          scope=None, gt_counts=None):
    """Batched matching (bboxes.py:337-380).  With dict inputs (one entry per class) returns
    dicts (n_gbboxes [B], tp [B, N], fp [B, N]) and the scores, like the reference."""
    if isinstance(scores, dict) or isinstance(bboxes, dict):
        d_n, d_tp, d_fp = {}, {}, {}
        for c in labels:
            n, tp, fp, _ = bboxes_matching_batch(c, scores[c], bboxes[c], glabels, gbboxes, gdifficults,
                                                 matching_threshold, gt_counts=gt_counts)
            d_n[c], d_tp[c], d_fp[c] = n, tp, fp
        return d_n, d_tp, d_fp, scores
    scores = _np(scores)
    bboxes = _np(bboxes)
    glabels, gbboxes, gdifficults = _np(glabels), _np(gbboxes), _np(gdifficults)
    B = scores.shape[0]
    ns, tps, fps = [], [], []
    for b in range(B):
        g = glabels.shape[1] if gt_counts is None else int(gt_counts[b])
        n, tp, fp = bboxes_matching(labels, scores[b], bboxes[b], glabels[b, :g], gbboxes[b, :g],
                                    gdifficults[b, :g], matching_threshold)
        ns.append(n)
        tps.append(tp)
        fps.append(fp)
    return np.array(ns, np.int64), np.stack(tps), np.stack(fps), scores


def _np(t):
    if hasattr(t, 'detach'):
        return t.detach().cpu().numpy()
    return np.asarray(t)
