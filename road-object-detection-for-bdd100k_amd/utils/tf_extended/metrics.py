"""utils/tf_extended/metrics.py — streaming TP/FP arrays, precision/recall, VOC07/VOC12 AP
(metrics.py:100-258), host numpy float64 as in the reference."""
import numpy as np

from utils.tf_extended.math import cummax

__all__ = ['streaming_tp_fp_arrays', 'StreamingTPFP', 'precision_recall', 'average_precision_voc07',
           'average_precision_voc12']


class StreamingTPFP(object):
    """Accumulator of (n_gt, n_det, tp, fp, scores) for one class (metrics.py:133-206)."""

    def __init__(self, remove_zero_scores=True):
        self.remove_zero_scores = remove_zero_scores
        self.num_gbboxes = 0
        self.num_detections = 0
        self.tp = np.zeros(0, bool)
        self.fp = np.zeros(0, bool)
        self.scores = np.zeros(0, np.float32)

    def update(self, num_gbboxes, tp, fp, scores):
        scores = np.asarray(scores, np.float32).reshape(-1)
        tp = np.asarray(tp, bool).reshape(-1)
        fp = np.asarray(fp, bool).reshape(-1)
        mask = np.logical_or(tp, fp)
        if self.remove_zero_scores:
            mask = np.logical_and(mask, scores > 1e-4)
        self.num_gbboxes += int(np.sum(num_gbboxes))
        self.num_detections += int(mask.sum())
        self.scores = np.concatenate([self.scores, scores[mask]])
        self.tp = np.concatenate([self.tp, tp[mask]])
        self.fp = np.concatenate([self.fp, fp[mask]])

    def value(self):
        return self.num_gbboxes, self.num_detections, self.tp, self.fp, self.scores


def streaming_tp_fp_arrays(num_gbboxes, tp, fp, scores, remove_zero_scores=True, state=None):
    """Dict-aware update: returns {c: StreamingTPFP} (created on first use) updated with
    this batch; `value()` of each gives the reference's metric tuple."""
    if isinstance(scores, dict) or isinstance(fp, dict):
        state = {} if state is None else state
        for c in num_gbboxes.keys():
            state[c] = streaming_tp_fp_arrays(num_gbboxes[c], tp[c], fp[c], scores[c], remove_zero_scores,
                                              state.get(c))
        return state
    st = StreamingTPFP(remove_zero_scores) if state is None else state
    st.update(num_gbboxes, tp, fp, scores)
    return st


def _safe_div(a, b):
    with np.errstate(divide='ignore', invalid='ignore'):
        q = np.asarray(a, np.float64) / np.asarray(b, np.float64)
    return np.where(np.asarray(b) > 0, q, 0.0)


def precision_recall(num_gbboxes, num_detections, tp, fp, scores, dtype=np.float64, scope=None):
    """Sort by score (top_k order: desc, ties by index), cumulative TP/FP -> P, R."""
    scores = np.asarray(scores)
    idx = np.argsort(-scores, kind='stable')[:num_detections]
    tp = np.cumsum(np.asarray(tp)[idx].astype(dtype))
    fp = np.cumsum(np.asarray(fp)[idx].astype(dtype))
    recall = _safe_div(tp, dtype(num_gbboxes))
    precision = _safe_div(tp, tp + fp)
    return precision, recall


def average_precision_voc12(precision, recall, name=None):
    """Area under the cummax precision envelope (metrics.py:212-234)."""
    p = np.concatenate([[0.], np.asarray(precision, np.float64), [0.]])
    r = np.concatenate([[0.], np.asarray(recall, np.float64), [1.]])
    p = cummax(p, reverse=True)
    return float(np.sum(p[1:] * (r[1:] - r[:-1])))


def average_precision_voc07(precision, recall, name=None):
    """11-point interpolated AP (metrics.py:237-258)."""
    p = np.concatenate([np.asarray(precision, np.float64), [0.]])
    r = np.concatenate([np.asarray(recall, np.float64), [np.inf]])
    ap = 0.
    for t in np.arange(0., 1.1, 0.1):
        v = p[r >= t]
        ap += (v.max() if v.size else -np.inf) / 11.
    return float(ap)
