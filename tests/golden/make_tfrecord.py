"""Generate the tiny BDD100K-schema TFRecord fixture used by the ingest tests
(tests/golden/tfrecord/bdd100k_train_000.tfrecord + expected.npz).

Writes records exactly as the reference's converter lays them out
(dataset/pascalvoc_to_tfrecords.py:131-171, file pattern dataset/bdd100k.py:9): JPEG bytes,
shape, per-box (ymin, xmin, ymax, xmax) normalised floats, BDD labels (dataset/bdd100k.py:23-35).
Images are small smooth synthetic scenes (gradients + filled boxes, so JPEG stays small);
the boxes are the filled rectangles.  expected.npz keeps the annotations and the pixels PIL
decodes from each record (pins the decoder across machines).  Run from the repo root:
    python tests/golden/make_tfrecord.py
"""
import io
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'tfrecord')
SIZES = [(72, 128), (90, 160), (72, 128), (60, 100), (90, 160), (72, 128), (81, 144), (72, 128)]
LABELS = np.array([1, 2, 3, 4, 6, 8, 10])


def scene(rng, H, W):
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.stack([60 + 120 * yy / H, 80 + 100 * xx / W, 120 + 60 * (yy + xx) / (H + W)], -1)
    G = int(rng.integers(1, 6))
    boxes, labels = [], []
    for _ in range(G):
        h, w = rng.uniform(0.15, 0.5), rng.uniform(0.1, 0.4)
        y0, x0 = rng.uniform(0, 1 - h), rng.uniform(0, 1 - w)
        r0, c0, r1, c1 = int(y0 * H), int(x0 * W), int(np.ceil((y0 + h) * H)), int(np.ceil((x0 + w) * W))
        img[r0:r1, c0:c1] = rng.uniform(0, 255, 3)
        boxes.append((r0 / H, c0 / W, r1 / H, c1 / W))
        labels.append(int(rng.choice(LABELS)))
    return np.clip(img, 0, 255).astype(np.uint8), np.array(boxes, np.float32), np.array(labels, np.int64)


def main():
    from PIL import Image
    from rod import tfrecord
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20261016)
    exp = {}
    path = os.path.join(OUT, 'bdd100k_train_000.tfrecord')
    with tfrecord.TFRecordWriter(path) as w:
        for i, (H, W) in enumerate(SIZES):
            img, boxes, labels = scene(rng, H, W)
            buf = io.BytesIO()
            Image.fromarray(img).save(buf, format='JPEG', quality=92)
            data = buf.getvalue()
            w.write(tfrecord.encode_detection_example(data, (H, W, 3), boxes, labels,
                                                      labels_text=[b'obj'] * len(labels)))
            exp['image_%d' % i] = tfrecord.decode_image(data)
            exp['boxes_%d' % i] = boxes
            exp['labels_%d' % i] = labels
    np.savez_compressed(os.path.join(OUT, 'expected.npz'), n=len(SIZES), **exp)
    print('wrote', path, os.path.getsize(path), 'bytes')


if __name__ == '__main__':
    main()
