"""Host mirror of the reference's utils/augmentation/tf_image.py (the two functions the
training / test pipelines call), batched on the GPU through rod_augment_images /
rod_augment_boxes:

  resize_image            tf_image.py:266-278 (legacy bilinear, align_corners=False; float out)
  random_flip_left_right  tf_image.py:281-305 (coin < 0.5; image reverse_v2 + box flip)
"""
import numpy as np
import torch

from rod import ops


def resize_image(images, size, dtype=torch.float32):
    """images uint8 [B, H, W, 3] (device) -> float [B, size[0], size[1], 3] on the 0-255 scale."""
    B, H, W, _ = images.shape
    crop = np.tile(np.array([0, 0, H, W], np.int32), (B, 1))
    mode = np.tile(np.array([0, -1], np.int32), (B, 1))
    return ops.augment_images(images, crop, mode, np.zeros((B, 3), np.float32), size, dtype=dtype)


def random_flip_left_right(rng, images, bboxes, labels=None, n=None):
    """Flip each image with probability 1/2 (uniform < .5, tf_image.py:293-294).  images uint8
    [B, H, W, 3]; bboxes [B, G, 4] (device or host).  Returns (float images, boxes, flips)."""
    B, H, W, _ = images.shape
    flips = (rng.uniform(0, 1, B) < .5).astype(np.int32)
    crop = np.tile(np.array([0, 0, H, W], np.int32), (B, 1))
    mode = np.stack([flips, np.full(B, -1, np.int32)], 1)
    out = ops.augment_images(images, crop, mode, np.zeros((B, 3), np.float32), (H, W))
    G = bboxes.shape[1]
    if labels is None:
        labels = np.ones((B, G), np.int32)
    if n is None:
        n = np.full(B, G, np.int32)
    ref = np.tile(np.array([0, 0, 1, 1], np.float32), (B, 1))
    # threshold -1: the overlap filter keeps every box (flip and clip only)
    bo, _, _ = ops.augment_boxes(bboxes, labels, n, ref, mode, threshold=-1.0)
    return out, bo, flips
