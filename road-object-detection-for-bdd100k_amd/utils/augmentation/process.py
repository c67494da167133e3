"""Host mirror of the reference's utils/augmentation/process.py.

The reference builds these as per-image TF graph ops; here the random choices are drawn on
the host per image (they are tiny) and the pixel / box work runs batched in librod:

  distort_color                 process.py:27-80  -> ColorDistorter (magnitudes drawn once per
                                process with Python `random`, as the reference draws them at graph
                                build, one set per colour ordering) + per-image factors
  apply_with_random_selector    process.py:8-24   -> ordering ~ U{0..3} per image
  distorted_bounding_box_crop   process.py:83-139 -> sample_distorted_bounding_box (the TF op's
                                published sampling rules, restated below) + rod_augment_boxes
"""
import math
import random

import numpy as np

BBOX_CROP_OVERLAP = 0.3     # process.py:6


class ColorDistorter(object):
    """distort_color(fast_mode=False) for the four orderings (process.py:27-80).

    apply_with_random_selector builds distort_color once per ordering (case 0..3) at graph
    build, and each build draws `lower`, `bright`, `hue` from Python's `random`
    (process.py:46-48): four fixed magnitude sets per process.  Per image: the ordering, then
    random_brightness delta ~ U(-bright/255, bright/255) (on the 0-255 image: a tiny shift),
    random_saturation / random_contrast factors ~ U(lower, 1).  Hue is disabled in the
    reference (commented out) and here."""

    def __init__(self, py_random=random):
        self.magnitudes = []
        for _ in range(4):
            lower = py_random.uniform(0.5, 1.)
            bright = py_random.uniform(0., 200.)
            hue = py_random.uniform(0., 0.5)
            self.magnitudes.append((lower, bright, hue))

    def sample(self, rng):
        """(ordering, [brightness delta, saturation factor, contrast factor]) for one image."""
        ordering = int(rng.integers(0, 4))          # apply_with_random_selector, process.py:19
        lower, bright, _ = self.magnitudes[ordering]
        max_delta = bright / 255.
        delta = rng.uniform(-max_delta, max_delta)  # tf.image.random_brightness
        sat = rng.uniform(lower, 1.)                # tf.image.random_saturation
        con = rng.uniform(lower, 1.)                # tf.image.random_contrast
        return ordering, np.array([delta, sat, con], np.float32)


def _generate_random_crop(rng, W, H, min_area_frac, max_area_frac, aspect):
    """GenerateRandomCrop of TF's sample_distorted_bounding_box kernel: height from the area
    range and aspect ratio (rounded with lrint), width = lrint(height * aspect), nudged by one
    row into the area range, then a uniform offset.  Returns (y, x, h, w) or None."""
    min_area = min_area_frac * W * H
    max_area = max_area_frac * W * H
    height = int(np.rint(math.sqrt(min_area / aspect)))
    max_height = int(np.rint(math.sqrt(max_area / aspect)))
    if int(np.rint(max_height * aspect)) > W:
        max_height = int((W + 0.5 - 1e-7) / aspect)
    max_height = min(max_height, H)
    height = min(height, max_height)
    if height < max_height:
        height += int(rng.integers(0, max_height - height + 1))
    width = int(np.rint(height * aspect))
    area = float(width * height)
    if area < min_area:
        height += 1
        width = int(np.rint(height * aspect))
        area = float(width * height)
    if area > max_area:
        height -= 1
        width = int(np.rint(height * aspect))
        area = float(width * height)
    if area < min_area or area > max_area or width > W or height > H or width <= 0 or height <= 0:
        return None
    y = int(rng.integers(0, H - height)) if height < H else 0
    x = int(rng.integers(0, W - width)) if width < W else 0
    return y, x, height, width


def _covers(crop, boxes, H, W, min_object_covered):
    """SatisfiesOverlapConstraints: some box (in integer pixels) has >= min_object_covered of
    its area inside the crop.  With no boxes the whole image is the box
    (use_image_if_no_bounding_boxes=True)."""
    y, x, h, w = crop
    if len(boxes) == 0:
        boxes = np.array([[0., 0., 1., 1.]], np.float32)
    for b in boxes:
        bx0, by0 = int(b[1] * W), int(b[0] * H)
        bx1, by1 = int(b[3] * W), int(b[2] * H)
        area = (bx1 - bx0) * (by1 - by0)
        if area <= 0:
            continue
        iw = max(0, min(bx1, x + w) - max(bx0, x))
        ih = max(0, min(by1, y + h) - max(by0, y))
        if iw * ih / area >= min_object_covered:
            return True
    return False


def sample_distorted_bounding_box(rng, H, W, boxes, min_object_covered=0.5, aspect_ratio_range=(0.9, 1.1),
                                  area_range=(0.2, 1.0), max_attempts=200):
    """tf.image.sample_distorted_bounding_box (process.py:117-124): up to max_attempts draws of
    an aspect ratio ~ U(range) and a crop (GenerateRandomCrop) until one covers
    min_object_covered of some box; else the whole image.  Returns (begin_yx, size_hw,
    distort_bbox [ymin, xmin, ymax, xmax] as float32 fractions)."""
    crop = None
    for _ in range(max_attempts):
        aspect = rng.uniform(aspect_ratio_range[0], aspect_ratio_range[1])
        c = _generate_random_crop(rng, W, H, area_range[0], area_range[1], aspect)
        if c is not None and _covers(c, boxes, H, W, min_object_covered):
            crop = c
            break
    if crop is None:
        crop = (0, 0, H, W)
    y, x, h, w = crop
    f = np.float32
    ref = np.array([f(y) / f(H), f(x) / f(W), f(y + h) / f(H), f(x + w) / f(W)], np.float32)
    return (y, x), (h, w), ref


def distorted_bounding_box_crop(rng, H, W, boxes, min_object_covered=0.5, aspect_ratio_range=(0.9, 1.1),
                                area_range=(0.2, 1.0), max_attempts=200):
    """The sampling half of process.distorted_bounding_box_crop (process.py:83-139): the crop
    window (y, x, h, w) and distort_bbox.  tf.slice, bboxes_resize and
    bboxes_filter_overlap(BBOX_CROP_OVERLAP) run batched in librod
    (utils.data_pileline_tools.process_raw_data_train)."""
    (y, x), (h, w), ref = sample_distorted_bounding_box(rng, H, W, boxes, min_object_covered, aspect_ratio_range,
                                                        area_range, max_attempts)
    return np.array([y, x, h, w], np.int32), ref
