"""A17 host side and oracle (no GPU): the numpy restatement of the augmentation chain on
known answers, and the sampler's constraints (tf.image.sample_distorted_bounding_box with the
reference's arguments, data_pileline_tools.py:95-98) as properties."""
import random

import numpy as np

from oracle import augment as oa
from utils.augmentation import process

f32 = np.float32


def test_resize_identity_and_constant():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (13, 17, 3)).astype(np.uint8)
    np.testing.assert_array_equal(oa.resize_bilinear_legacy(img, 13, 17), img.astype(f32))
    const = np.full((9, 11, 3), 77, np.uint8)
    np.testing.assert_array_equal(oa.resize_bilinear_legacy(const, 20, 31), np.full((20, 31, 3), 77, f32))
    # legacy scaling: output row o samples input o * in/out (no half-pixel offset)
    ramp = np.tile(np.arange(8, dtype=np.uint8)[None, :, None], (2, 1, 3))
    out = oa.resize_bilinear_legacy(ramp, 2, 16)
    np.testing.assert_allclose(out[0, :, 0], np.minimum(np.arange(16) * 0.5, 7), atol=0)


def test_saturation_known_answers():
    rng = np.random.default_rng(1)
    px = rng.uniform(0, 255, (1000, 3)).astype(f32)
    gray = np.repeat(rng.uniform(0, 255, (50, 1)).astype(f32), 3, 1)
    # grey pixels carry no saturation: unchanged for any factor
    np.testing.assert_array_equal(oa.adjust_saturation(gray, 0.3), gray)
    # factor 1: the HSV round trip only (a few ulps)
    np.testing.assert_allclose(oa.adjust_saturation(px, 1.0), px, rtol=0, atol=2e-4)
    # factor 0: every pixel becomes grey at its max channel (v)
    np.testing.assert_allclose(oa.adjust_saturation(px, 0.0), np.repeat(px.max(1, keepdims=True), 3, 1), atol=0)
    # value (max channel) is preserved for factors <= 1 and the hue ordering of channels too
    out = oa.adjust_saturation(px, 0.6)
    np.testing.assert_allclose(out.max(1), px.max(1), rtol=0, atol=2e-4)
    assert (np.argsort(out, 1, kind='stable')[:, -1] == np.argsort(px, 1, kind='stable')[:, -1]).mean() > 0.99


def test_contrast_and_orderings():
    rng = np.random.default_rng(2)
    img = rng.uniform(0, 255, (6, 7, 3)).astype(f32)
    np.testing.assert_allclose(oa.adjust_contrast(img, 1.0), img, atol=3e-5)
    half = oa.adjust_contrast(img, 0.5)
    np.testing.assert_allclose(half.reshape(-1, 3).mean(0), img.reshape(-1, 3).mean(0), rtol=1e-5)
    np.testing.assert_allclose(half.reshape(-1, 3).std(0), 0.5 * img.reshape(-1, 3).std(0), rtol=1e-4)
    # ordering 2 is contrast first; 0 is contrast last: different results in general
    a = oa.distort_color(img, 0, 0.4, 0.7, 0.6)
    b = oa.distort_color(img, 2, 0.4, 0.7, 0.6)
    assert np.abs(a - b).max() > 1e-3
    assert set(oa.ORDERINGS) == {0, 1, 2, 3}


def test_boxes_resize_filter_flip_clip():
    boxes = np.array([[0.1, 0.1, 0.5, 0.5],      # 56% inside the crop -> kept, clipped
                      [0.0, 0.0, 0.22, 0.22],    # mostly outside -> dropped
                      [0.4, 0.4, 0.9, 0.95],     # partly outside -> kept, clipped
                      [0.3, 0.3, 0.3, 0.6]], f32)  # zero area -> safe_divide 0 -> dropped
    labels = np.array([1, 2, 3, 4], np.int32)
    ref = np.array([0.2, 0.2, 0.8, 0.8], f32)
    b, lab = oa.process_boxes(boxes, labels, 4, ref, flip=False)
    np.testing.assert_array_equal(lab, [1, 3])
    np.testing.assert_allclose(b[0], np.clip((boxes[0] - [.2, .2, .2, .2]) / f32(0.6), 0, 1), rtol=1e-6)
    assert b.min() >= 0 and b.max() <= 1 and b[1, 2] == 1 and b[1, 3] == 1
    bf, labf = oa.process_boxes(boxes, labels, 4, ref, flip=True)
    np.testing.assert_array_equal(labf, lab)
    np.testing.assert_allclose(bf[:, 1], 1 - b[:, 3], atol=1e-7)
    np.testing.assert_allclose(bf[:, 3], 1 - b[:, 1], atol=1e-7)


def test_sampler_constraints():
    rng = np.random.default_rng(3)
    H, W = 720, 1280
    n_crop = 0
    for trial in range(300):
        k = int(rng.integers(0, 6))
        c = rng.uniform(0.1, 0.9, (k, 2))
        s = rng.uniform(0.02, 0.3, (k, 2))
        boxes = np.clip(np.concatenate([c - s / 2, c + s / 2], 1)[:, [0, 1, 2, 3]], 0, 1).astype(f32)
        crop, ref = process.distorted_bounding_box_crop(rng, H, W, boxes, min_object_covered=0.4,
                                                        aspect_ratio_range=(0.6, 1.67))
        y, x, h, w = (int(v) for v in crop)
        assert 0 <= y and 0 <= x and y + h <= H and x + w <= W and h > 0 and w > 0
        np.testing.assert_array_equal(ref, np.array([f32(y) / f32(H), f32(x) / f32(W), f32(y + h) / f32(H),
                                                     f32(x + w) / f32(W)], f32))
        if (h, w) == (H, W):
            continue                             # fallback after max_attempts: the whole image
        n_crop += 1
        assert 0.2 * H * W <= h * w <= H * W     # area_range (0.2, 1.0)
        assert 0.6 - 1.0 / h <= w / h <= 1.67 + 1.0 / h   # aspect ratio, up to lrint of the width
        assert process._covers((y, x, h, w), boxes, H, W, 0.4)
    assert n_crop > 200


def test_color_magnitudes_per_process():
    cd = process.ColorDistorter(random.Random(7))
    assert len(cd.magnitudes) == 4
    for lower, bright, hue in cd.magnitudes:
        assert 0.5 <= lower <= 1 and 0 <= bright <= 200 and 0 <= hue <= 0.5
    rng = np.random.default_rng(0)
    seen = set()
    for _ in range(200):
        o, (d, s, c) = cd.sample(rng)
        lower, bright, _ = cd.magnitudes[o]
        assert abs(d) <= bright / 255. and lower <= s <= 1 and lower <= c <= 1
        seen.add(o)
    assert seen == {0, 1, 2, 3}
