"""A16: evaluate.py's AP numbers against the oracle (ref evaluate.py:100-208,
tf_extended/bboxes.py:246-380, metrics.py:100-258).

evaluate.main runs on the committed BDD100K-schema TFRecord fixture at 300x300 with a
checkpoint whose detector has a realistic score distribution (BatchNorm calibrated on the
fixture, background logit shifted so ~10 % of the class scores pass evaluate.py's
select_threshold 0.3: the per-class NMS keeps many boxes and some match the ground truth).
The oracle path takes the same network outputs (the HIP forward is deterministic) and does
everything after them on its own: the per-class select / top-k 400 / NMS 0.4 / keep 200
(oracle.post.detected_bboxes_vec, also checked bit-exact against the kernel here), the greedy
matching at IoU 0.5 and the streaming VOC07 / VOC12 AP (oracle.post.streaming_ap).  Every
class's AP printed by evaluate.py must equal the oracle's (1e-12), and the mAPs their means."""
import json
import os

import numpy as np
import pytest
import torch

import config
from oracle import post as op

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def test_evaluate_ap_matches_oracle(dev, tmp_path):
    import evaluate
    import predict
    from nets.catch_net import factory
    from rod.checkpoint import save_variables
    from rod.data import detector_like_scores
    from rod.dataio import make_source, network_input
    from utils import net_tools
    ds = os.path.join(GOLD, 'tfrecord')
    hw, bs, n_img = (300, 300), 4, 8
    pr = predict.Predictor(hw, dev, torch.float32, seed=61, select_threshold=0.3)
    probe = next(make_source(ds, 8, hw, dev, dtype=torch.float32, max_images=n_img))[0]
    frac = detector_like_scores(pr, probe, rate=0.10)
    ck = str(tmp_path / 'ck' / 'mobilenet_v2.model')
    save_variables(pr.net.store, ck, 0)
    edir = str(tmp_path / 'eval')
    m07, m12 = evaluate.main(['--img_height=300', '--img_width=300', '--dataset_dir=' + ds, '--batch_size=%d' % bs,
                              '--num_images=%d' % n_img, '--checkpoint_path=' + os.path.dirname(ck),
                              '--eval_dir=' + edir])
    ev = json.load(open(os.path.join(edir, 'eval.json')))

    classes = list(range(1, config.total_obj_n))
    src = make_source(ds, bs, hw, dev, dtype=torch.float32, max_images=n_img)
    batches = []
    with torch.no_grad():
        for _ in range(n_img // bs):
            img, gb, gl, gn = next(src)
            refine_out, det_out, clf_out = factory(network_input(img, torch.float32), 'mobilenet_v2', False,
                                                   pr.config_dict, torch.float32, net=pr.net).get_output()
            probs = net_tools.class_probabilities(clf_out)
            boxes = net_tools.decode_all_layers(pr.anchors, refine_out, det_out, to_corner=True)
            rs, rb = net_tools.detected_bboxes(probs, boxes, select_threshold=0.3, nms_threshold=0.4, top_k=400,
                                               keep_top_k=200)
            s_ref, b_ref, _ = op.detected_bboxes_vec(probs.cpu().numpy(), boxes.cpu().numpy(), 0.3, 0.4, 400, 200)
            for c in classes:   # the kernel's NMS is the oracle's, bit for bit
                np.testing.assert_array_equal(rs[c].cpu().numpy(), s_ref[:, c - 1])
                np.testing.assert_array_equal(rb[c].cpu().numpy(), b_ref[:, c - 1])
            batches.append(({c: s_ref[:, c - 1] for c in classes}, {c: b_ref[:, c - 1] for c in classes},
                            gl.cpu().numpy(), gb.cpu().numpy(), gn.cpu().numpy()))
    ap07, ap12, cnt = op.streaming_ap(batches, classes, 0.5, counts=True)
    print('probe pass fraction', frac, '| (tp, fp, n_gt) per class', cnt)
    print('AP07', ap07, '\nAP12', ap12, '\nevaluate.py mAP', m07, m12)
    for c in classes:
        assert ev['AP_VOC07'][str(c)] == pytest.approx(ap07[c], abs=1e-12), c
        assert ev['AP_VOC12'][str(c)] == pytest.approx(ap12[c], abs=1e-12), c
    assert m07 == pytest.approx(sum(ap07.values()) / len(classes), abs=1e-12)
    assert m12 == pytest.approx(sum(ap12.values()) / len(classes), abs=1e-12)
    assert sum(v[0] for v in cnt.values()) > 0 and sum(v[1] for v in cnt.values()) > 0   # TPs and FPs


def test_tfe_bboxes_sort_and_nms_batch_match_oracle(dev):
    """The drop-in tf_extended sort / NMS pair (ref tf_extended/bboxes.py:60-100, 192-232, as
    net_tools.py:750-754 chains them): bboxes_sort = tf.nn.top_k (descending, ties to the lower
    index) + gather; bboxes_nms_batch = greedy tf.image.non_max_suppression over the sorted
    candidates, zero-padded to keep_top_k.  Per class (dict inputs), against numpy top-k and
    oracle.post.detected_bboxes_vec, bit-exact, with exact ties and zero scores in the input."""
    import utils.tf_extended as tfe
    rng = np.random.default_rng(17)
    B, N, top_k, keep = 3, 700, 400, 150
    sc, bx = {}, {}
    for c in (1, 2):
        s = rng.random((B, N)).astype(np.float32) ** 3
        s[:, 100:140] = s[:, 100:101]          # ties
        s[:, 500:] = 0                         # not selected upstream
        ctr = rng.uniform(0.1, 0.9, (B, N, 2)).astype(np.float32)
        hw = rng.uniform(0.02, 0.3, (B, N, 2)).astype(np.float32)
        sc[c], bx[c] = s, np.concatenate([ctr - hw / 2, ctr + hw / 2], -1).astype(np.float32)
    ds, db = tfe.bboxes_sort({c: torch.from_numpy(v).to(dev) for c, v in sc.items()},
                             {c: torch.from_numpy(v).to(dev) for c, v in bx.items()}, top_k=top_k)
    ns, nb = tfe.bboxes_nms_batch(ds, db, nms_threshold=0.45, keep_top_k=keep)
    for c in (1, 2):
        order = np.argsort(-sc[c], axis=1, kind='stable')[:, :top_k]
        want_s = np.take_along_axis(sc[c], order, 1)
        want_b = np.take_along_axis(bx[c], order[..., None], 1)
        np.testing.assert_array_equal(ds[c].cpu().numpy(), want_s)
        np.testing.assert_array_equal(db[c].cpu().numpy(), want_b)
        probs = np.stack([np.zeros_like(want_s), want_s], -1)
        s_ref, b_ref, kept = op.detected_bboxes_vec(probs, want_b, 0.0, 0.45, top_k, keep)
        np.testing.assert_array_equal(ns[c].cpu().numpy(), s_ref[:, 0])
        np.testing.assert_array_equal(nb[c].cpu().numpy(), b_ref[:, 0])
        print('kept per image (class %d):' % c, [len(kept[(b, 1)]) for b in range(B)])
        assert all(10 < len(kept[(b, 1)]) <= keep for b in range(B))
    with pytest.raises(ValueError):
        tfe.bboxes_sort(torch.from_numpy(sc[1]).to(dev), torch.from_numpy(bx[1]).to(dev), top_k=N + 1)
