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

from rod.data import SEED, synthetic_batch

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


def make_source(dataset_dir, batch_size, img_size, device, split='train', seed=SEED):
    files = tfrecord_files(dataset_dir, split) if dataset_dir else []
    if files:
        raise NotImplementedError('TFRecord/JPEG ingest (SURVEY.md §8f rank 1) is not built yet; found %d files in %s'
                                  % (len(files), dataset_dir))
    log.warning('no BDD100K TFRecords under %r: using synthetic BDD-shaped batches (rod.data)', dataset_dir)
    return SyntheticSource(batch_size, img_size, device, seed)
