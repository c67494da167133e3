"""Batch sources for the CLIs.

The reference reads BDD100K TFRecords through slim's DatasetDataProvider
(dataset/bdd100k.py, dataset/pascalvoc_common.py:40-107, utils/data_pileline_tools.py:18-69).
`TFRecordSource` is that reader: the record scan and checksums are native (librodio), JPEG
decode runs on a host thread pool (`num_readers` threads, as the reference's reader threads),
and the per-image preprocessing runs on the GPU (rod_augment_images / rod_augment_boxes):
process_raw_data_train for training, the bilinear resize of prepare_data_test otherwise.

Every source yields device tensors at the network resolution:
    img [B, H, W, 3] (uint8, or already (2/255)x-1 normalised in the compute dtype — see
    `network_input`), corner boxes fp32 [B, G, 4], labels int32 [B, G], n int32 [B]
Synthetic BDD-shaped batches (rod.data) only with an explicit `synthetic=True`.
"""
import glob
import logging
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from rod.data import SEED, synthetic_batch, synthetic_boxes

GMAX = 64   # padded ground-truth boxes per training image; larger batches: next multiple

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


def network_input(img, dtype):
    """(2/255)*img - 1 in `dtype` (train.py:126, evaluate.py:117) of a source batch."""
    from rod import ops
    if img.is_floating_point():   # the GPU preprocessing already normalised it
        return ops.cast(img, dtype)
    return ops.normalize_image(img, dtype)


class TFRecordSource(object):
    """DatasetDataProvider + prepare_data_train / prepare_data_test over TFRecord files of the
    schema of dataset/pascalvoc_common.py:75-88.

    train=True: records in a seeded random order, reshuffled every epoch (shuffle=True at
    train.py:106), each image through process_raw_data_train (random crop / resize / flip /
    colour, data_pileline_tools.py:71-108) on the GPU, normalised into `dtype`.
    train=False: file order (shuffle=False, evaluate.py:103), resize to img_size only
    (data_pileline_tools.py:39-40), normalised into `dtype`; boxes unchanged.  The number of
    ground-truth boxes varies per image: batches are zero-padded to the largest count
    (dynamic_pad=True, evaluate.py:109-114) with the counts in n.

    Training batches are padded to a FIXED box count instead: `gmax` (64), or the
    next multiple of 64 above it for a batch that holds more.  The batch shapes then do not
    change from step to step, so the captured training step (Trainer.step_graphed) replays
    without re-capture; the matching kernel reads only the first n[b] boxes of each row, so
    the padding changes no result.

    prefetch (default: on for training): the host half of the NEXT batch (record reads,
    JPEG decode on the reader pool, pinned staging, augmentation sampling) runs on a
    background thread while the current step runs on the GPU; the device half (upload,
    augmentation kernels) is issued from the caller's thread, stream-ordered behind it."""

    def __init__(self, files, batch_size, img_size, device, dtype, train=True, seed=SEED, num_readers=4,
                 verify=True, max_images=None, rank=0, world=1, gmax=GMAX, prefetch=None):
        from rod import tfrecord
        if not files:
            raise FileNotFoundError('no TFRecord files')
        self.files = [tfrecord.TFRecordFile(f, verify=verify) for f in files]
        self.index = [(fi, ri) for fi, f in enumerate(self.files) for ri in range(len(f))]
        if max_images is not None:
            self.index = self.index[:max_images]
        if not self.index:
            raise ValueError('the TFRecord files hold no records')
        self.batch_size, self.img_size, self.device, self.dtype = batch_size, tuple(img_size), device, dtype
        self.train = train
        # data parallel: every rank draws the SAME permutation (same seed) and reads its own
        # disjoint slice of it, so one global batch holds no image twice and an epoch is one
        # pass over the data set (the reference reads it on one device); each rank keeps
        # len // world records per epoch (the remainder is dropped, as DistributedSampler's
        # drop_last) so the ranks' epochs stay in step
        # (evaluation is never sharded: every record is read once, in file order)
        self.rank, self.world = (int(rank), max(1, int(world))) if train else (0, 1)
        self.gmax = int(gmax) if train else 0
        self.rng = np.random.default_rng(seed)
        self.order = self._shard(self.rng.permutation(len(self.index)) if train else np.arange(len(self.index)))
        self.pos = 0
        self.epoch = 0
        self.pool = ThreadPoolExecutor(max_workers=max(1, int(num_readers)))
        self.aug = None
        if train:
            from utils.data_pileline_tools import TrainAugmenter
            self.aug = TrainAugmenter(self.img_size, seed=seed + 1000 * self.rank)   # per-rank augmentation draws
        self.prefetch = train if prefetch is None else bool(prefetch)
        self._ahead = ThreadPoolExecutor(max_workers=1) if self.prefetch else None
        self._next_host = None
        # prefetching on a GPU: the background thread also uploads the batch's pixels on its own
        # copy stream, so the ~20 MB host->device copy overlaps the previous step instead of
        # sitting on the compute stream in front of the augmentation kernels
        self._copy_stream = torch.cuda.Stream(device) if self.prefetch and self.device.type == 'cuda' else None

    def __len__(self):
        """Records this rank reads per epoch."""
        return len(self.order)

    def close(self):
        if self._ahead is not None:
            self._ahead.shutdown(wait=True)
        self.pool.shutdown(wait=True)

    def __iter__(self):
        return self

    def _shard(self, perm):
        if self.world == 1:
            return perm
        if len(perm) < self.world:   # fewer records than ranks: one record each, reused
            return perm[self.rank % len(perm):self.rank % len(perm) + 1]
        return perm[self.rank::self.world][:len(perm) // self.world]

    def _load(self, k):
        from rod import tfrecord
        fi, ri = self.index[k]
        enc, fmt, shape, boxes, labels, _, _ = tfrecord.decode_detection_example(self.files[fi][ri])
        img = tfrecord.decode_image(enc, fmt)
        return img, boxes, labels

    def _take(self):
        ks = []
        for _ in range(self.batch_size):
            if self.pos == len(self.order):
                self.pos = 0
                self.epoch += 1
                if self.train:
                    self.order = self._shard(self.rng.permutation(len(self.index)))
            ks.append(int(self.order[self.pos]))
            self.pos += 1
        return ks

    def _host(self):
        """Host half of a batch: record reads + JPEG decode (reader pool), the padded box arrays,
        the pinned staging buffer and, for training, the augmentation draws (in batch order, so
        the sequence of batches does not depend on prefetching)."""
        items = list(self.pool.map(self._load, self._take()))
        B = len(items)
        G = max(1, max(len(b) for _, b, _ in items))
        if self.gmax:
            G = max(self.gmax, -(-G // GMAX) * GMAX)
        boxes = np.zeros((B, G, 4), np.float32)
        labels = np.zeros((B, G), np.int32)
        n = np.zeros(B, np.int32)
        hw = np.zeros((B, 2), np.int32)
        offs = np.zeros(B, np.int64)
        tot = 0
        for b, (img, bx, lb) in enumerate(items):
            g = len(bx)
            boxes[b, :g], labels[b, :g], n[b] = bx, lb, g
            hw[b] = img.shape[:2]
            offs[b] = tot
            tot += img.size
        flat = torch.empty(tot, dtype=torch.uint8, pin_memory=self.device.type == 'cuda')
        fl = flat.numpy()
        for b, (img, _, _) in enumerate(items):
            fl[offs[b]:offs[b] + img.size] = img.reshape(-1)
        draws = self.aug.sample(hw, boxes, n) if self.train else None
        up = None
        if self._copy_stream is not None:   # the upload, on the copy stream (see __init__)
            with torch.cuda.stream(self._copy_stream):
                src = flat.to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._copy_stream)
            up = (src, ev)
        return flat, boxes, labels, n, hw, offs, draws, up

    def _device(self, host):
        from rod import ops
        flat, boxes, labels, n, hw, offs, draws, up = host
        B = len(n)
        if up is not None:
            src, ev = up
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            src.record_stream(cur)   # the copy stream's allocation is used on this stream
        else:
            src = flat.to(self.device, non_blocking=True)
        if self.train:
            crop, ref, mode, colour = draws
            x = ops.augment_images(src, crop, mode, colour, self.img_size, dtype=self.dtype, normalize=True,
                                   src_hw=hw, src_off=offs)
            bo, lo, no = ops.augment_boxes(boxes, labels, n, ref, mode, threshold=0.3)
            return x, bo, lo, no
        crop = np.concatenate([np.zeros((B, 2), np.int32), hw], 1)
        mode = np.tile(np.array([0, -1], np.int32), (B, 1))
        x = ops.augment_images(src, crop, mode, np.zeros((B, 3), np.float32), self.img_size, dtype=self.dtype,
                               normalize=True, src_hw=hw, src_off=offs)
        dev = lambda a: torch.from_numpy(a).to(self.device)
        return x, dev(boxes), dev(labels), dev(n)

    def __next__(self):
        if self._ahead is None:
            return self._device(self._host())
        fut = self._next_host if self._next_host is not None else self._ahead.submit(self._host)
        host = fut.result()
        self._next_host = self._ahead.submit(self._host)   # decode the next batch during this step
        return self._device(host)


def make_source(dataset_dir, batch_size, img_size, device, split='train', seed=SEED, augment_dtype=None,
                synthetic=False, dtype=torch.float32, num_readers=4, max_images=None, rank=0, world=1):
    """augment_dtype: training batches go through the GPU augmentation pipeline and come out
    normalised in this dtype; None = network-resolution uint8 batches (eval / predict / bench).
    synthetic: run on synthetic BDD-shaped batches (rod.data) — only when asked for explicitly;
    a missing dataset is an error, as in the reference (its reader fails on an empty pattern).
    rank / world: data parallel — TFRecords are read as disjoint per-rank slices of one shared
    shuffle; synthetic sources draw per-rank batches (seed + 1000 * rank)."""
    if synthetic:
        log.warning('--synthetic: using synthetic BDD-shaped batches (rod.data), not %r', dataset_dir)
    else:
        files = tfrecord_files(dataset_dir, split) if dataset_dir else []
        if files:
            log.info('reading %d TFRecord file(s) from %s', len(files), dataset_dir)
            train = augment_dtype is not None
            return TFRecordSource(files, batch_size, img_size, torch.device(device),
                                  augment_dtype if train else dtype, train=train, seed=seed, num_readers=num_readers,
                                  max_images=max_images, rank=rank, world=world)
        raise FileNotFoundError('no bdd100k_%s_*.tfrecord under %r (pass --synthetic to run on synthetic '
                                'BDD-shaped batches)' % (split, dataset_dir))
    seed = seed + 1000 * rank
    if augment_dtype is not None:
        return AugmentedSource(batch_size, img_size, device, augment_dtype, seed)
    return SyntheticSource(batch_size, img_size, device, seed)
