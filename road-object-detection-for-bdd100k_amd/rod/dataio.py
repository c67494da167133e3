"""Batch sources for the CLIs.

The reference reads BDD100K TFRecords through slim's DatasetDataProvider
(dataset/bdd100k.py, utils/data_pileline_tools.py).  TFRecord + JPEG ingest is the
first "next" row of SURVEY.md §8(f) and is not built yet; until then every CLI runs on
synthetic BDD-shaped batches (rod.data) and says so in its log.  The source yields
device tensors already at the network resolution:
    img uint8 [B, H, W, 3], corner boxes fp32 [B, G, 4], labels int32 [B, G], n int32 [B]
"""
import glob
import logging
import os

import numpy as np
import torch

from rod.data import SEED, synthetic_batch, synthetic_boxes

log = logging.getLogger(__name__)


def tfrecord_files(dataset_dir, split='train'):
    return sorted(glob.glob(os.path.join(dataset_dir, 'bdd100k_%s_*.tfrecord' % split)))


class SyntheticSource(object):
    def __init__(self, batch_size, img_size, device, seed=SEED, n_distinct=4):
        self.batch_size = batch_size
        self.img_size = img_size
        self.device = device
        self.batches = [synthetic_batch(batch_size, img_size[0], img_size[1], device, seed=seed + i)
                        for i in range(n_distinct)]
        self.i = 0

    def __iter__(self):
        return self

    def __next__(self):
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b


class AugmentedSource(object):
    """Training batches through process_raw_data_train (data_pileline_tools.py:76-108) on the GPU:
    synthetic decoded BDD100K frames (uint8 720x1280, the dataset's native size) with host-side
    annotations, augmented per step by utils.data_pileline_tools.TrainAugmenter (random crop /
    resize / flip / colour on the device) and normalised into `dtype` (train.py:126)."""

    def __init__(self, batch_size, img_size, device, dtype, seed=SEED, n_distinct=4, raw_hw=(720, 1280)):
        from utils.data_pileline_tools import TrainAugmenter
        self.dtype = dtype
        self.raw = []
        for i in range(n_distinct):
            g = torch.Generator(device='cpu').manual_seed(seed + i)
            img = torch.randint(0, 256, (batch_size, raw_hw[0], raw_hw[1], 3), dtype=torch.uint8, generator=g)
            corner, labels, n = synthetic_boxes(batch_size, seed=seed + i)
            self.raw.append((img.to(device), corner, labels, n))
        self.aug = TrainAugmenter(img_size, seed=seed)
        self.i = 0

    def __iter__(self):
        return self

    def __next__(self):
        img, corner, labels, n = self.raw[self.i % len(self.raw)]
        self.i += 1
        return self.aug(img, corner, labels, n, dtype=self.dtype)


def make_source(dataset_dir, batch_size, img_size, device, split='train', seed=SEED, augment_dtype=None):
    """augment_dtype: training batches go through the GPU augmentation pipeline and come out
    normalised in this dtype; None = network-resolution uint8 batches (eval / predict / bench)."""
    files = tfrecord_files(dataset_dir, split) if dataset_dir else []
    if files:
        raise NotImplementedError('TFRecord/JPEG ingest (SURVEY.md §8f rank 1) is not built yet; found %d files in %s'
                                  % (len(files), dataset_dir))
    log.warning('no BDD100K TFRecords under %r: using synthetic BDD-shaped batches (rod.data)', dataset_dir)
    if augment_dtype is not None:
        return AugmentedSource(batch_size, img_size, device, augment_dtype, seed)
    return SyntheticSource(batch_size, img_size, device, seed)
