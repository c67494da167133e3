"""ORACLE (test infrastructure only): target assignment and losses, restated from the
reference's utils/net_tools.py and utils/common_tools.py with numpy float32 arithmetic
(one rounding per op, like the chain of separate TF ops)."""
import numpy as np

from .anchors import anchor_centers, anchor_corners

f32 = np.float32


def log_cr(x):
    return np.log(np.asarray(x, np.float64)).astype(np.float32)


def exp_cr(x):
    return np.exp(np.asarray(x, np.float64)).astype(np.float32)


def corner_to_center(b):
    """common_tools.py:38-56."""
    b = np.asarray(b, np.float32)
    return np.stack([(b[..., 0] + b[..., 2]) / f32(2.), (b[..., 1] + b[..., 3]) / f32(2.),
                     b[..., 2] - b[..., 0], b[..., 3] - b[..., 1]], -1)


def center_to_corner(b):
    """common_tools.py:16-35."""
    b = np.asarray(b, np.float32)
    return np.stack([b[..., 0] - b[..., 2] / f32(2), b[..., 1] - b[..., 3] / f32(2),
                     b[..., 0] + b[..., 2] / f32(2), b[..., 1] + b[..., 3] / f32(2)], -1)


def jaccard(anchors, box):
    """net_tools.py:237-267: anchors [..., 4] corner, box [4] (or [..., 4]) corner."""
    a = np.asarray(anchors, np.float32)
    g = np.asarray(box, np.float32)
    vol_a = (a[..., 3] - a[..., 1]) * (a[..., 2] - a[..., 0])
    iy0 = np.maximum(a[..., 0], g[..., 0])
    ix0 = np.maximum(a[..., 1], g[..., 1])
    iy1 = np.minimum(a[..., 2], g[..., 2])
    ix1 = np.minimum(a[..., 3], g[..., 3])
    h = np.maximum(iy1 - iy0, f32(0.))
    w = np.maximum(ix1 - ix0, f32(0.))
    inter = h * w
    union = vol_a - inter + (g[..., 2] - g[..., 0]) * (g[..., 3] - g[..., 1])
    with np.errstate(all='ignore'):
        return inter / union


def encode(layer, cbox):
    """net_tools.py:147-179 — offsets of centre box cbox [4] against every anchor."""
    acy, acx, ah, aw = anchor_centers(layer)
    with np.errstate(all='ignore'):
        return np.stack([(f32(cbox[0]) - acy) / ah, (f32(cbox[1]) - acx) / aw,
                         log_cr(f32(cbox[2]) / ah), log_cr(f32(cbox[3]) / aw)], -1)


def decode(layer, offsets):
    """net_tools.py:182-234 — offsets [B, fh, fw, A, 4] -> centre boxes."""
    acy, acx, ah, aw = anchor_centers(layer)
    o = np.asarray(offsets, np.float32)
    return np.stack([o[..., 0] * ah + acy, o[..., 1] * aw + acx,
                     exp_cr(o[..., 2]) * ah, exp_cr(o[..., 3]) * aw], -1)


def refine_groundtruth(anchors_all, center_bboxes, labels, thresholds):
    """JACCARD_BIGGER (net_tools.py:382-421) for ONE image, reference loop structure:
    jac [G, fh, fw, A] -> pos = max >= thr, idx = argmax (first), then the masked sum
    over boxes (which is where non-finite encodings turn into NaN, as in TF)."""
    cb = np.asarray(center_bboxes, np.float32)
    lab = np.asarray(labels)
    gt_l, cb_l, lb_l, pm_l = [], [], [], []
    with np.errstate(all='ignore'):
        for layer, thr in zip(anchors_all, thresholds):
            corners = np.stack(anchor_corners(layer), -1)
            jac = np.stack([jaccard(corners, center_to_corner(cb[i])) for i in range(cb.shape[0])], 0)
            pos = (jac.max(0) >= f32(thr)).astype(np.int32)[..., None]
            idx = jac.argmax(0)
            shp = corners.shape[:-1]
            gt = np.zeros(shp + (4,), np.float32)
            cbox = np.zeros(shp + (4,), np.float32)
            lbl = np.zeros(shp + (1,), np.int32)
            for i in range(cb.shape[0]):
                mask = (idx == i).astype(np.float32)[..., None] * pos.astype(np.float32)
                cbox = cbox + mask * cb[i]
                gt = gt + mask * encode(layer, cb[i])
                lbl = lbl + mask.astype(np.int32) * np.int32(lab[i])
            gt_l.append(gt)
            cb_l.append(cbox)
            lb_l.append(lbl)
            pm_l.append(pos)
    return gt_l, cb_l, lb_l, pm_l


def refine_groundtruth_nn(anchors_all, center_bboxes, labels):
    """NEAREST_NEIGHBOR (net_tools.py:354-380) for ONE image: per anchor, the box with the
    least sum of squared encoded offsets (argmin, first minimum; the 4-term sum in index order),
    the masked sum over boxes, pos_mask = ones."""
    cb = np.asarray(center_bboxes, np.float32)
    lab = np.asarray(labels)
    gt_l, cb_l, lb_l, pm_l = [], [], [], []
    with np.errstate(all='ignore'):
        for layer in anchors_all:
            loc = np.stack([encode(layer, cb[i]) for i in range(cb.shape[0])], 0)   # [G, fh, fw, A, 4]
            sq = loc * loc
            dist = ((sq[..., 0] + sq[..., 1]) + sq[..., 2]) + sq[..., 3]
            idx = dist.argmin(0)
            shp = idx.shape
            gt = np.zeros(shp + (4,), np.float32)
            cbox = np.zeros(shp + (4,), np.float32)
            lbl = np.zeros(shp + (1,), np.int32)
            for i in range(cb.shape[0]):
                mask = (idx == i).astype(np.float32)[..., None]
                cbox = cbox + mask * cb[i]
                gt = gt + mask * loc[i]
                lbl = lbl + mask.astype(np.int32) * np.int32(lab[i])
            gt_l.append(gt)
            cb_l.append(cbox)
            lb_l.append(lbl)
            pm_l.append(np.ones(shp + (1,), np.int32))
    return gt_l, cb_l, lb_l, pm_l


def smooth_l1(x):
    """net_tools.py:478-489."""
    x = np.asarray(x, np.float32)
    ax = np.abs(x)
    return f32(0.5) * ((ax - f32(1)) * np.minimum(ax, f32(1)) + ax)


def refine_loss(refine_out, refine_gt, refine_pos, bs):
    """net_tools.py:492-516 — per-layer loss values (float64 sums) and their total."""
    per = []
    for y, x, m in zip(refine_gt, refine_out, refine_pos):
        per.append(float(np.sum(smooth_l1((np.asarray(y, np.float32) - np.asarray(x, np.float32))
                                          * np.asarray(m, np.float32)), dtype=np.float64)) / bs)
    return per, sum(per)


def refine_loss_grad(refine_out, refine_gt, refine_pos, bs):
    """d refine_loss / d refine_out (TF's composed gradient, evaluated in closed form)."""
    out = []
    for y, x, m in zip(refine_gt, refine_out, refine_pos):
        m = np.asarray(m, np.float32)
        d = (np.asarray(y, np.float32) - np.asarray(x, np.float32)) * m
        out.append((-m * np.clip(d, -1, 1) / bs).astype(np.float32))
    return out
