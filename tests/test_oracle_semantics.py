"""Known-answer tests that pin the oracle's restatement of TF-1.x op semantics where no
reference fixture exists, plus the product's host-side evaluation code
(utils/tf_extended) against the oracle's independent restatement."""
import numpy as np
import pytest

from oracle import post as op
from oracle import targets as ot
from rod.ops import same_pad

f32 = np.float32


def test_tf_same_padding_table():
    # (out, pad_before): stride-2 on an even extent pads 0 before / 1 after
    assert same_pad(720, 2) == (360, 0)
    assert same_pad(45, 2) == (23, 1)
    assert same_pad(1280, 2) == (640, 0)
    assert same_pad(13, 1) == (13, 1)
    assert same_pad(3, 2) == (2, 1)


def test_jaccard_known_answers():
    box = np.array([0.1, 0.2, 0.5, 0.6], f32)
    assert ot.jaccard(box[None], box)[0] == 1.0
    assert ot.jaccard(np.array([[0.6, 0.6, 0.9, 0.9]], f32), box)[0] == 0.0
    half = np.array([[0.1, 0.2, 0.5, 0.4]], f32)  # half of the box
    np.testing.assert_allclose(ot.jaccard(half, box)[0], 0.5, rtol=1e-6)


def test_smooth_l1_known_answers():
    x = np.array([0.5, -0.5, 2.0, -2.0, 0.0, 1.0], f32)
    np.testing.assert_array_equal(ot.smooth_l1(x), np.array([0.125, 0.125, 1.5, 1.5, 0.0, 0.5], f32))


def test_encode_decode_round_trip():
    rng = np.random.default_rng(0)
    from oracle import anchors as oa
    init = oa.init_anchor(6, (300, 300))
    layer = oa.anchors_one_layer((300, 300), (10, 10), init[2])
    cb = np.array([0.4, 0.6, 0.2, 0.3], f32)
    enc = ot.encode(layer, cb)
    dec = ot.decode(layer, enc[None])[0]
    np.testing.assert_allclose(dec, np.broadcast_to(cb, dec.shape), rtol=2e-6, atol=2e-7)


def test_nms_hand_cases():
    # three boxes: B overlaps A strongly (suppressed), C disjoint (kept); ties by index
    boxes = np.array([[[0, 0, 1, 1], [0, 0.05, 1, 1.05], [2, 2, 3, 3], [0, 0, 0, 0]]], f32) / 4
    probs = np.zeros((1, 4, 3), f32)
    probs[0, :, 1] = [0.9, 0.8, 0.7, 0.0]
    s, b, kept = op.detected_bboxes(probs, boxes, 0.1, 0.5, 400, 3)
    assert kept[(0, 1)] == [0, 2, 3]  # zero-score, zero-area box is kept as filler (IoU 0)
    np.testing.assert_array_equal(s[0, 0], np.array([0.9, 0.7, 0.0], f32))
    # IoU exactly at threshold is NOT suppressed (strict >)
    bx = np.array([[[0, 0, 1, 1], [0, 0.5, 1, 1.5]]], f32)  # IoU = 1/3
    pr = np.zeros((1, 2, 2), f32)
    pr[0, :, 1] = [0.9, 0.9]
    _, _, kept = op.detected_bboxes(pr, bx, 0.1, f32(1) / f32(3), 400, 2)
    assert kept[(0, 1)] == [0, 1]
    assert op.tf_nms_iou(bx[0, 0], bx[0, 1]) == f32(1) / f32(3)


def test_voc_ap_known_answers():
    # perfect detector
    assert op.voc_ap([1, 1], [0, 0], [0.9, 0.8], 2, True) == pytest.approx(1.0)
    assert op.voc_ap([1, 1], [0, 0], [0.9, 0.8], 2, False) == pytest.approx(1.0)
    # one TP then one FP, 2 GT: recall 0.5 at precision 1
    assert op.voc_ap([1, 0], [0, 1], [0.9, 0.8], 2, False) == pytest.approx(0.5)
    assert op.voc_ap([1, 0], [0, 1], [0.9, 0.8], 2, True) == pytest.approx(6 / 11)


def test_product_metrics_match_oracle():
    from utils.tf_extended import metrics as M
    rng = np.random.default_rng(3)
    for _ in range(20):
        n = int(rng.integers(1, 60))
        scores = rng.random(n).astype(f32)
        scores[rng.random(n) < 0.2] = scores[0]  # ties
        tp = rng.random(n) < 0.4
        fp = ~tp
        n_gt = int(tp.sum() + rng.integers(0, 5))
        p, r = M.precision_recall(n_gt, n, tp, fp, scores)
        assert M.average_precision_voc07(p, r) == pytest.approx(op.voc_ap(tp, fp, scores, n_gt, True), abs=1e-12)
        assert M.average_precision_voc12(p, r) == pytest.approx(op.voc_ap(tp, fp, scores, n_gt, False), abs=1e-12)


def test_product_matching_known_case():
    from utils.tf_extended import bboxes as tb
    g = np.array([[0, 0, .5, .5], [.5, .5, 1, 1], [0, 0, .5, .5]], f32)
    gl = np.array([1, 1, 2])
    det = np.array([[0, 0, .5, .5], [0, 0, .5, .5], [.5, .5, 1, .9], [.2, .2, .3, .3]], f32)
    n, tp, fp = tb.bboxes_matching(1, np.array([.9, .8, .7, .6]), det, gl, g, np.zeros(3))
    assert n == 2
    assert tp.tolist() == [True, False, True, False]   # second hit on an already matched GT is FP
    assert fp.tolist() == [False, True, False, True]


def test_vectorised_nms_oracle_equals_scalar():
    """oracle.post.detected_bboxes_vec (used at B=32 full size) takes the same decisions and
    float32 values as the scalar restatement, including ties, zero-area filler boxes and
    scores below the selection threshold."""
    from oracle import post as op
    rng = np.random.default_rng(7)
    B, A, K = 2, 300, 4
    logits = rng.normal(0, 2.0, (B, A, K)).astype(np.float32)
    logits[:, 10:20] = logits[:, 10:11]                   # exact score ties
    e, s, _ = op.softmax_rows(logits)
    probs = (e / s).astype(np.float32)
    c = rng.uniform(0.2, 0.8, (B, A, 2)).astype(np.float32)
    hw = rng.uniform(0.0, 0.3, (B, A, 2)).astype(np.float32)
    hw[:, 50:55] = 0                                       # zero-area boxes
    boxes = np.concatenate([c - hw / 2, c + hw / 2], -1).astype(np.float32)
    for sel, nms, tk, keep in [(0.1, 0.4, 100, 30), (0.0, 0.5, 300, 200), (0.3, 0.2, 64, 8)]:
        a = op.detected_bboxes(probs, boxes, sel, nms, tk, keep)
        b = op.detected_bboxes_vec(probs, boxes, sel, nms, tk, keep)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
        assert a[2] == b[2]


def test_product_matching_and_streaming_ap_match_oracle():
    """utils.tf_extended matching + streaming TP/FP + VOC AP (the host half of evaluate.py:
    146-208) against oracle.post.bboxes_matching / streaming_ap (a plain-loop restatement of
    tf_extended/bboxes.py:246-334 and metrics.py:100-258) on random batches with shared labels,
    duplicate detections, ties and padded (zero-score) rows."""
    import utils.tf_extended as tfe
    from oracle import post as op
    rng = np.random.default_rng(11)
    classes = [1, 2, 3]
    batches, state = [], None
    for _ in range(4):
        B, N, G = 3, 12, 6
        gcount = rng.integers(0, G + 1, B)
        gl = rng.integers(1, 4, (B, G)).astype(np.int64)
        c0 = rng.uniform(0.1, 0.9, (B, G, 2))
        hw = rng.uniform(0.05, 0.4, (B, G, 2))
        gb = np.concatenate([c0 - hw / 2, c0 + hw / 2], -1).astype(f32)
        scores, boxes = {}, {}
        for c in classes:
            s = np.sort(rng.random((B, N)).astype(f32), 1)[:, ::-1].copy()
            s[:, -3:] = 0                                   # padded rows of the NMS output
            s[:, 2] = s[:, 1]                               # a tie
            jit = rng.normal(0, 0.03, (B, N, 4)).astype(f32)
            pick = rng.integers(0, G, (B, N))
            bx = np.take_along_axis(gb, pick[..., None], 1) + jit   # near (some) ground truth
            bx[:, 3] = bx[:, 1]                                       # a duplicate detection
            scores[c], boxes[c] = s, bx.astype(f32)
        batches.append((scores, boxes, gl, gb, gcount))
        n_g, tp, fp, _ = tfe.bboxes_matching_batch(classes, scores, boxes, gl, gb, np.zeros_like(gl),
                                                   matching_threshold=0.5, gt_counts=gcount)
        for c in classes:
            for b in range(B):
                g = int(gcount[b])
                n, t, f_ = op.bboxes_matching(c, scores[c][b], boxes[c][b], list(gl[b, :g]), gb[b, :g], [False] * g)
                assert n == n_g[c][b] and list(tp[c][b]) == t and list(fp[c][b]) == f_
        state = tfe.streaming_tp_fp_arrays(n_g, tp, fp, scores, state=state)
    ap07, ap12 = op.streaming_ap(batches, classes)
    hits = 0
    for c in classes:
        p, r = tfe.precision_recall(*state[c].value())
        hits += int(state[c].value()[2].sum())
        assert tfe.average_precision_voc07(p, r) == pytest.approx(ap07[c], abs=1e-12)
        assert tfe.average_precision_voc12(p, r) == pytest.approx(ap12[c], abs=1e-12)
    assert hits > 10 and 0 < min(ap12.values()) < 1
