"""Host mirror of the reference's utils/data_pileline_tools.py (same module name, typo kept).

The reference decodes one image at a time on 4 CPU threads and runs the TF image ops per
image.  Here a batch of decoded uint8 images already on the device goes through two librod
launches per step (rod_augment_images, rod_augment_boxes); only the random parameters are
drawn on the host:

  prepare_data_train / process_raw_data_train  data_pileline_tools.py:45-108
  prepare_data_test                            data_pileline_tools.py:18-43
"""
import numpy as np
import torch

from rod import ops
from utils.augmentation import process


class TrainAugmenter(object):
    """process_raw_data_train for batches (data_pileline_tools.py:76-108):

        distorted_bounding_box_crop(min_object_covered=0.4, aspect_ratio_range=(0.6, 1.67))
        -> resize_image(out_shape, BILINEAR, align_corners=False)
        -> random_flip_left_right
        -> apply_with_random_selector(distort_color(fast_mode=False), 4 orderings)
        -> clip boxes to [0, 1]

    and, fused when `dtype` is given, train.py:126 `(2/255) * imgs - 1` cast to DTYPE.
    `seed` drives the per-image draws (numpy); the colour magnitudes come from Python's
    `random`, once per augmenter, as the reference draws them once per graph."""

    def __init__(self, out_shape, seed=0, py_random=None):
        import random
        self.out_shape = tuple(out_shape)
        self.rng = np.random.default_rng(seed)
        self.color = process.ColorDistorter(py_random if py_random is not None else random.Random(seed))

    def sample(self, src_hw, boxes, n):
        """Per-image parameters: crop [B,4], distort_bbox [B,4], mode [B,2], colour [B,3]."""
        B = len(src_hw)
        crop = np.zeros((B, 4), np.int32)
        ref = np.zeros((B, 4), np.float32)
        mode = np.zeros((B, 2), np.int32)
        colour = np.zeros((B, 3), np.float32)
        for b in range(B):
            H, W = int(src_hw[b][0]), int(src_hw[b][1])
            crop[b], ref[b] = process.distorted_bounding_box_crop(self.rng, H, W, boxes[b][:int(n[b])],
                                                                  min_object_covered=0.4,
                                                                  aspect_ratio_range=(0.6, 1.67))
            mode[b, 0] = int(self.rng.uniform(0, 1) < .5)       # random_flip_left_right
            mode[b, 1], colour[b] = self.color.sample(self.rng)  # apply_with_random_selector
        return crop, ref, mode, colour

    def __call__(self, images, boxes, labels, n, dtype=None, params=None):
        """images: uint8 [B, H, W, 3] device tensor; boxes [B, G, 4] / labels [B, G] / n [B] as
        HOST arrays (annotations come from the reader on the host).  Returns device tensors
        (image, boxes, labels, n): image float 0-255 [B, Ho, Wo, 3], or the normalised
        network input in `dtype`."""
        boxes = np.asarray(boxes, np.float32)
        B, H, W, _ = images.shape
        src_hw = np.tile(np.array([H, W], np.int32), (B, 1))
        crop, ref, mode, colour = params if params is not None else self.sample(src_hw, boxes, n)
        img = ops.augment_images(images, crop, mode, colour, self.out_shape,
                                 dtype=dtype if dtype is not None else torch.float32, normalize=dtype is not None)
        bo, lo, no = ops.augment_boxes(boxes, labels, n, ref, mode, threshold=process.BBOX_CROP_OVERLAP)
        self.last_params = (crop, ref, mode, colour)
        return img, bo, lo, no


def process_raw_data_train(images, labels, bboxes, n, out_shape, seed=0, dtype=None):
    """One-shot form of TrainAugmenter (argument order of the reference: image, labels, bboxes)."""
    return TrainAugmenter(out_shape, seed)(images, bboxes, labels, n, dtype=dtype)


def prepare_data_test(images, out_shape, dtype=None):
    """resize_image(config.img_size, BILINEAR, align_corners=False) only (data_pileline_tools.py:39-40);
    boxes are unchanged.  With `dtype`, fused (2/255)x - 1 (evaluate.py / predict.py:98)."""
    B, H, W, _ = images.shape
    crop = np.tile(np.array([0, 0, H, W], np.int32), (B, 1))
    mode = np.tile(np.array([0, -1], np.int32), (B, 1))
    return ops.augment_images(images, crop, mode, np.zeros((B, 3), np.float32), out_shape,
                              dtype=dtype if dtype is not None else torch.float32, normalize=dtype is not None)
