"""Targets, losses, optimiser and post-processing — drop-in for the reference's
utils/net_tools.py (lines 1-758).  Host-side anchor tables are numpy exactly as in the
reference; everything per-anchor / per-pixel runs as librod kernels on the GPU.

Batched API: where the reference works on one image inside the TF input pipeline
(refine_groundtruth), these functions take a batch [B, G, 4] plus the number of valid
boxes per image, and return per-layer views shaped like the reference's batched
tensors ([B, fh, fw, A, 4] / [B, fh, fw, A, 1]).
"""
from __future__ import annotations

import collections
import math

import numpy as np
import torch

import config
from rod import ops


# ================================================================ anchors (host, numpy)
def init_anchor(n_layers):
    """Anchor (height, width) in pixels of config.img_size per layer (net_tools.py:21-82)."""
    boxes = collections.OrderedDict()
    lo, hi = config.normal_anchor_range
    step = (hi - lo) / (n_layers - 1)
    range_min, range_max = lo, lo + step
    H, W = config.img_size[0], config.img_size[1]
    r3 = math.sqrt(3)
    for i in range(n_layers):
        if i == 0:
            scales = list(config.special_anchor_range)
        else:
            scales = [range_min, (2 * range_min + range_max) / 3, (range_min + 2 * range_max) / 3]
            range_min, range_max = range_max, range_max + step
        rows = []
        for s in scales:
            rows += [[s * H, s * W], [s * H / r3, s * W * r3], [s * H * r3, s * W / r3]]
        a = np.array(rows)
        a[:, 0] = np.minimum(a[:, 0], H)
        a[:, 1] = np.minimum(a[:, 1], W)
        boxes['layer_%d' % (i + 1)] = a
    return boxes


def n_anchor_each_layer(backbone_name):
    assert backbone_name in list(config.extract_feat_name.keys())
    return [v.shape[0] for v in init_anchor(len(config.extract_feat_name[backbone_name])).values()]


def anchors_one_layer(img_shape, feat_shape, anchors_one_layer, dtype=np.float32):
    """(yc [fh,fw,1], xc [fh,fw,1], h [A], w [A]) normalised (net_tools.py:98-122)."""
    y, x = np.mgrid[0:feat_shape[0], 0:feat_shape[1]]
    xc = (x + 0.5) / feat_shape[1]
    yc = (y + 0.5) / feat_shape[0]
    h = anchors_one_layer[:, 0] / img_shape[0]
    w = anchors_one_layer[:, 1] / img_shape[1]
    return (yc[..., None].astype(dtype), xc[..., None].astype(dtype), h.astype(dtype), w.astype(dtype))


def anchors_all_layer(img_shape, feats_shape, anchors_all_layer):
    return [list(anchors_one_layer(img_shape, feats_shape[k], v)) for k, v in anchors_all_layer.items()]


class AnchorTable:
    """Flattened anchors of all layers in (fh, fw, A) order, on the device.

    corner = (ymin, xmin, ymax, xmax) = (yref - href/2., ...) in float32 and
    center = ((ymax+ymin)/2., (xmax+xmin)/2., ymax-ymin, xmax-xmin) from those corners,
    both exactly as numpy computes them in net_tools.py:156-171 / 385-395.
    """

    def __init__(self, anchors_all, device):
        corners, centers, off = [], [], [0]
        self.shapes = []
        for yref, xref, href, wref in anchors_all:
            ymin = yref - href / 2.
            xmin = xref - wref / 2.
            ymax = yref + href / 2.
            xmax = xref + wref / 2.
            ymin, xmin, ymax, xmax = (np.float32(v) for v in (ymin, xmin, ymax, xmax))
            cy = (ymax + ymin) / 2.
            cx = (xmax + xmin) / 2.
            h = ymax - ymin
            w = xmax - xmin
            fh, fw, A = ymin.shape
            self.shapes.append((fh, fw, A))
            corners.append(np.stack([ymin, xmin, ymax, xmax], -1).reshape(-1, 4))
            centers.append(np.stack([cy, cx, h, w], -1).reshape(-1, 4))
            off.append(off[-1] + fh * fw * A)
        self.corner_np = np.ascontiguousarray(np.concatenate(corners).astype(np.float32))
        self.center_np = np.ascontiguousarray(np.concatenate(centers).astype(np.float32))
        self.lvl_off = np.array(off, dtype=np.int32)
        self.A = int(off[-1])
        self.corner = torch.from_numpy(self.corner_np).to(device)
        self.center = torch.from_numpy(self.center_np).to(device)

    def split(self, t: torch.Tensor, k):
        """[B, A_total, ...] -> list of per-layer views [B, fh, fw, A(, k)]."""
        outs = []
        for l, (fh, fw, A) in enumerate(self.shapes):
            v = t[:, self.lvl_off[l]:self.lvl_off[l + 1]]
            outs.append(v.view(t.shape[0], fh, fw, A, *([k] if k else [])) if v.is_contiguous()
                        else v.unflatten(1, (fh, fw, A)))
        return outs


_TABLES = {}


def anchor_table(anchors_all, device) -> AnchorTable:
    key = (id(anchors_all), str(device))
    if key not in _TABLES:
        _TABLES[key] = (anchors_all, AnchorTable(anchors_all, device))
    return _TABLES[key][1]


# ================================================================ targets
def refine_groundtruth(anchors_all_layer, center_bboxes, labels, method, n_boxes=None, scope="refine_encode"):
    """Target assignment (net_tools.py:270-428) on the GPU: JACCARD_BIGGER (382-421) or
    NEAREST_NEIGHBOR (354-380, every anchor positive).

    center_bboxes: [B, G, 4] (or [G, 4]) (yc, xc, h, w); labels [B, G]; n_boxes [B]
    valid boxes per image (default: G).  Returns (gt_list, cbboxes_list, labels_list,
    pos_mask_list) of per-layer views [B, fh, fw, A, 4|1].
    """
    if method == config.refine_method.JACCARD_TOPK:
        raise ValueError('Not support now')
    if method not in (config.refine_method.JACCARD_BIGGER, config.refine_method.NEAREST_NEIGHBOR):
        raise ValueError('Function parameter "method" wrong')
    single = center_bboxes.dim() == 2
    if single:
        center_bboxes, labels = center_bboxes[None], labels[None]
    B, G, _ = center_bboxes.shape
    dev = center_bboxes.device
    if n_boxes is None:
        n_boxes = torch.full((B,), G, dtype=torch.int32, device=dev)
    tab = anchor_table(anchors_all_layer, dev)
    off, cbox, lbl, pos = ops.match_anchors(tab.corner, tab.center, tab.lvl_off,
                                            config.refine_pos_jac_val_all_layers[:len(tab.shapes)],
                                            center_bboxes.float(), labels.to(torch.int32),
                                            n_boxes.to(torch.int32),
                                            nearest=method == config.refine_method.NEAREST_NEIGHBOR)
    res = (tab.split(off, 4), tab.split(cbox, 4), tab.split(lbl[..., None], 1), tab.split(pos[..., None], 1))
    res = RefineTargets(*res)
    res.flat = (off, cbox, lbl, pos)
    res.table = tab
    return res


class RefineTargets(tuple):
    """(gt_list, cbboxes_list, labels_list, pos_mask_list) + the concatenated buffers."""

    def __new__(cls, *parts):
        return super().__new__(cls, parts)


# ================================================================ losses
def smooth_l1(x):
    raise NotImplementedError('smooth_l1 is fused into refine_loss / det_clf_loss kernels')


def refine_loss(refine_out, refine_groundtruth, refine_pos_mask, dtype=torch.float32, targets=None, scale=None,
                refine_flat=None):
    """sum_l sum smooth_l1((gt - out) * mask) / bs (net_tools.py:492-516).

    `targets` (the RefineTargets returned by refine_groundtruth) lets the kernel read
    the concatenated target buffers directly; otherwise the per-layer lists are used.
    `scale` overrides bs (data-parallel runs divide by the global batch).
    Returns the scalar loss tensor; the per-layer values (the reference's
    "layer_%d_each_sample" summaries) are left in refine_loss.last_per_layer.
    """
    B = refine_out[0].shape[0]
    scale = float(B) if scale is None else float(scale)
    # refine_flat: the concatenated refine_out when the caller shares it between losses
    pred = ops.levels_concat(refine_out, 4) if refine_flat is None else refine_flat
    if targets is not None:
        gt_flat, _, _, pos_flat = targets.flat
        lvl_off = targets.table.lvl_off
    else:
        gt_flat = ops.levels_concat([g.contiguous() for g in refine_groundtruth], 4).float()
        pos_flat = ops.levels_concat([m.contiguous() for m in refine_pos_mask], 1).view(B, -1)
        sizes = [g[0].numel() // 4 for g in refine_groundtruth]
        lvl_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    vec, total = ops.smooth_l1_masked(pred, gt_flat, pos_flat, lvl_off, scale)
    refine_loss.last_per_layer = vec
    return total


# ================================================================ optimiser
class optimizer(object):
    """Plain SGD, clip-by-value +-5, undecayed learning rate (net_tools.py:626-654).

    The exponential decay the reference builds is only logged (net_tools.py:638-641,
    quirk 1 in SURVEY); `decayed_lr(step)` reproduces that logged value.
    """

    def __init__(self, store, batch_szie, learning_rate=1e-3, fix_learning_rate=True, clip=5.0):
        self.store = store
        self.lr = float(learning_rate)
        self.batch_size = batch_szie
        self.fix = fix_learning_rate
        self.clip = clip
        self.global_step = 0

    def decayed_lr(self, step=None):
        step = self.global_step if step is None else step
        return self.lr * 0.97 ** (step // (20000 / self.batch_size))

    def step(self):
        ops.sgd_clip_(self.store.flat, self.store.flat_grad, self.lr, self.clip)
        self.store.version += 1   # derived weight layouts are refreshed (one batched launch) on next use
        self.global_step += 1


# ================================================================ ODM targets and loss
def _flat_levels(tensors, k, table):
    """Per-layer tensors [B, fh, fw, A(, k)] -> concatenated [B, A_total(, k)] (no copy when
    they are already views of one buffer laid out that way)."""
    return ops.levels_concat([t.contiguous() for t in tensors], k)


def det_groundtruth(refine_out, offset_gt, cbboxes, refine_labels, refine_pos_mask, anchors, scope="det_encode",
                    targets=None, refine_flat=None):
    """ODM targets (net_tools.py:431-475).  Returns (det_gt, det_pos_mask, det_labels, iou)
    as per-layer views [B, fh, fw, A, 4|1] / iou [B, fh, fw, A]; the concatenated buffers
    are attached as `.flat` for the fused loss kernels."""
    tab = targets.table if targets is not None else anchor_table(anchors, refine_out[0].device)
    ro = ops.levels_concat(refine_out, 4) if refine_flat is None else refine_flat
    if targets is not None:
        rgt, cbox, lbl, rpos = targets.flat
    else:
        B = refine_out[0].shape[0]
        rgt = _flat_levels(offset_gt, 4, tab).float()
        cbox = _flat_levels(cbboxes, 4, tab).float()
        lbl = _flat_levels(refine_labels, 1, tab).view(B, -1)
        rpos = _flat_levels(refine_pos_mask, 1, tab).view(B, -1)
    # differentiable wrt refine_out (det_gt and iou; no stop-gradient in the reference) when it
    # requires grad, i.e. when the refine net is trained (train.py fix_refine=False)
    det_gt, det_pos, det_lbl, iou = ops.det_targets(tab.center, ro, rgt, cbox, lbl, rpos, tab.lvl_off,
                                                    config.det_pos_jac_val_all_layers[:len(tab.shapes)])
    res = RefineTargets(tab.split(det_gt, 4), tab.split(det_pos[..., None], 1), tab.split(det_lbl[..., None], 1),
                        tab.split(iou, 0))
    res.flat = (det_gt, det_pos, det_lbl, iou)
    res.table = tab
    return res


# Data-parallel exchange for the hard-negative selection: None (single process) or
# (allreduce(list of device int32 tensors, in-place SUM over ranks), world_size); set by
# rod.trainer.Trainer when it runs under torch.distributed.
HNM_EXCHANGE = None


def det_clf_loss(refine_out, clf_out, det_out, det_groundtruth, det_pos_mask, det_labels, iou_all_layers,
                 dtype=torch.float32, scale=None, targets=None):
    """(det_loss, clf_loss) (net_tools.py:519-623): masked smooth-L1 on the ODM offsets and
    softmax cross-entropy with global hard-negative mining and the IoU focal factor.

    `det_groundtruth` may be the object returned by det_groundtruth() (fast path).  The
    summaries the reference logs (pos/neg/clf loss, max hard prediction, positives) are
    left in det_clf_loss.last_stats ([8] device tensor, see rod_softmax_ce_hnm)."""
    B = clf_out[0].shape[0]
    scale = float(B) if scale is None else float(scale)
    tg = det_groundtruth if isinstance(det_groundtruth, RefineTargets) and hasattr(det_groundtruth, 'flat') \
        else targets
    if tg is None:
        raise ValueError('det_clf_loss needs the det_groundtruth() result (per-layer lists are views of it)')
    det_gt, det_pos, det_lbl, iou = tg.flat
    lvl_off = tg.table.lvl_off
    pred = ops.levels_concat(det_out, 4)
    dvec, det_loss_one = ops.smooth_l1_masked(pred, det_gt, det_pos, lvl_off, scale)
    logits = ops.levels_concat(clf_out, config.total_obj_n)
    if HNM_EXCHANGE is not None:   # data parallel: hard negatives over the global batch (§8e)
        allreduce, world = HNM_EXCHANGE
        cvec, clf_loss = ops.softmax_ce_hnm_dp(logits, det_lbl, det_pos, iou, lvl_off, scale, B * world, allreduce)
    else:
        cvec, clf_loss = ops.softmax_ce_hnm(logits, det_lbl, det_pos, iou, lvl_off, scale)
    det_clf_loss.last_stats = cvec
    det_clf_loss.last_det_per_layer = dvec
    return det_loss_one, clf_loss


# ================================================================ decode / post-processing
def decode_locations_one_layer(anchors_one_layer, offset_bboxes):
    """Centre boxes from [B, fh, fw, A, 4] offsets (net_tools.py:182-234)."""
    tab = AnchorTable([anchors_one_layer], offset_bboxes.device)
    B = offset_bboxes.shape[0]
    out = ops.decode(tab.center, offset_bboxes.reshape(B, -1, 4))
    return out.view(offset_bboxes.shape)


def decode_all_layers(anchors_all, refine_out, det_out=None, to_corner=True):
    """predict.py:130-134 / evaluate.py:139-143 for all layers at once: corner boxes of
    decode(anchor, refine_out + det_out), concatenated [B, A_total, 4] fp32."""
    tab = anchor_table(anchors_all, refine_out[0].device)
    a = ops.levels_concat(refine_out, 4)
    b = ops.levels_concat(det_out, 4) if det_out is not None else None
    return ops.decode(tab.center, a, b, to_corner=to_corner)


def class_probabilities(clf_out):
    """slim.softmax over every layer's logits, concatenated [B, A_total, K] fp32."""
    logits = ops.levels_concat(clf_out, config.total_obj_n)
    return ops.softmax(logits, config.total_obj_n)


def detected_bboxes(predictions, localisations, select_threshold=None, nms_threshold=0.5, clipping_bbox=None,
                    top_k=800, keep_top_k=200):
    """Per-class select -> top_k -> NMS -> pad (net_tools.py:739-758) in one kernel.

    predictions: [B, A_total, K] probabilities (or the per-layer list of them);
    localisations: [B, A_total, 4] corner boxes (or the per-layer list).
    Returns dicts {c: scores [B, keep_top_k]}, {c: boxes [B, keep_top_k, 4]} for c = 1..K-1."""
    if isinstance(predictions, (list, tuple)):
        predictions = ops.levels_concat([p.float() for p in predictions], config.total_obj_n)
    if isinstance(localisations, (list, tuple)):
        localisations = ops.levels_concat([l.float() for l in localisations], 4)
    thr = 0.0 if select_threshold is None else select_threshold
    scores, boxes = ops.select_topk_nms(predictions, localisations, thr, top_k, keep_top_k, nms_threshold)
    if clipping_bbox is not None:
        raise NotImplementedError('clipping_bbox is never used by the reference CLIs (predict.py:136)')
    K = predictions.shape[-1]
    return ({c: scores[:, c - 1] for c in range(1, K)}, {c: boxes[:, c - 1] for c in range(1, K)})


# ================================================================ visualisation (net_tools.py:761-1106)
from utils.visualization import (STANDARD_COLORS, draw_bounding_box_on_image,  # noqa: E402,F401
                                 draw_bounding_box_on_image_array, draw_keypoints_on_image,
                                 draw_keypoints_on_image_array, draw_mask_on_image_array,
                                 visualize_boxes_and_labels_on_image_array)
