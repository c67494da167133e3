"""Host tools of SURVEY §8f rank 4: the BDD100K JSON -> VOC XML -> TFRecord converters
(reference convert/json2xml/*.py, dataset/pascalvoc_to_tfrecords.py, tf_convert_data.py) and the
detection drawing of predict.py (net_tools.py:761-1106).  CPU only."""
import io
import json
import os

import numpy as np
from PIL import Image

import config
from convert import bdd2voc
from dataset.bdd100k import BDD100K_LABELS
from rod.tfrecord import TFRecordFile, decode_detection_example
import tf_convert_data
from utils import net_tools


def _frame(objs):
    return {'name': 'x', 'frames': [{'objects': [{'category': c, 'box2d': {'x1': x1, 'y1': y1, 'x2': x2, 'y2': y2}}
                                                 for c, (x1, y1, x2, y2) in objs]}]}


def test_json_to_voc_to_tfrecord_round_trip(tmp_path):
    jd, root = tmp_path / 'json', tmp_path / 'voc'
    jd.mkdir()
    frames = {
        'a0': [('car', (10.7, 20.2, 300.9, 200.0)), ('bike', (1, 2, 3, 4)), ('traffic light', (600, 30, 640, 90))],
        'b1': [('motor', (5, 5, 50, 50))],                        # nothing kept: no XML written
        'c2': [('person', (0, 0, 1279, 719)), ('rider', (100, 100, 140, 200))],
    }
    for k, objs in frames.items():
        (jd / (k + '.json')).write_text(json.dumps(_frame(objs)))
    n, skipped = bdd2voc.convert_dir(str(jd), str(root / 'Annotations'))
    assert n == 2 and skipped == ['b1.json']
    (root / 'JPEGImages').mkdir()
    jpegs = {}
    for k in ('a0', 'c2'):
        buf = io.BytesIO()
        Image.fromarray(np.full((72, 128, 3), 40, np.uint8)).save(buf, format='JPEG')
        jpegs[k] = buf.getvalue()
        (root / 'JPEGImages' / (k + '.jpg')).write_bytes(jpegs[k])
    shards = tf_convert_data.main(['--dataset_dir', str(root) + '/', '--output_dir', str(tmp_path / 'tf'),
                                   '--output_name', 'bdd100k_train'])
    assert [os.path.basename(s) for s in shards] == ['bdd100k_train_000.tfrecord']
    recs = [decode_detection_example(p) for p in TFRecordFile(shards[0])]
    assert len(recs) == 2
    for (enc, fmt, shape, boxes, lab, dif, tru), k in zip(recs, ('a0', 'c2')):
        kept = [(c, b) for c, b in frames[k] if c in bdd2voc.CATEGORIES]
        assert enc == jpegs[k] and list(shape) == [720, 1280, 3]
        want = np.array([[int(b[1]) / 720, int(b[0]) / 1280, int(b[3]) / 720, int(b[2]) / 1280] for _, b in kept],
                        np.float32)
        np.testing.assert_array_equal(boxes, want)
        assert list(lab) == [BDD100K_LABELS[c][0] for c, _ in kept]
        assert not dif.any() and not tru.any()


def test_visualize_boxes_draws_class_colours():
    img = np.zeros((120, 200, 3), np.uint8)
    boxes = np.array([[0.2, 0.1, 0.8, 0.5], [0.1, 0.6, 0.5, 0.9]], np.float32)
    out = net_tools.visualize_boxes_and_labels_on_image_array(img, boxes, np.array([8, 2]), np.array([0.9, 0.1]),
                                                              config.category_index, line_thickness=2)
    assert out is img
    from PIL import ImageColor
    car = ImageColor.getrgb(net_tools.STANDARD_COLORS[8 % len(net_tools.STANDARD_COLORS)])
    assert tuple(img[96, 50]) == car            # bottom edge of the scored box (y = 0.8 * 120)
    assert not img[12:60, 120:180].any()         # the second box is below min_score_thresh
    gt = np.zeros((120, 200, 3), np.uint8)
    net_tools.visualize_boxes_and_labels_on_image_array(gt, boxes[:1], np.array([8]), None, config.category_index)
    assert tuple(gt[96, 50]) == (255, 0, 0)      # ground truth: one colour, no labels
