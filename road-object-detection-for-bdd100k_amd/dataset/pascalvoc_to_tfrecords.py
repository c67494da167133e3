"""Pascal-VOC layout (Annotations/*.xml + JPEGImages/*.jpg) -> TFRecord shards of
tf.train.Example in the schema the reader decodes (reference dataset/pascalvoc_to_tfrecords.py,
keys at pascalvoc_common.py:75-88), written by rod.tfrecord (no TensorFlow).

Semantics kept from the reference:
  * boxes normalised by the XML's size: (ymin/h, xmin/w, ymax/h, xmax/w) (lines 122-127);
  * labels through the BDD100K label map (LABELS = BDD100K_LABELS, line 63);
  * `difficult` / `truncated` come out 0 whatever the XML says: the reference tests the
    Element's truthiness (`if obj.find('difficult'):`, an element without children is falsy,
    lines 110-117) — SURVEY appendix A quirk 10;
  * SAMPLES_PER_FILES = 5000 examples per shard named <output_dir>/<name>_%03d.tfrecord,
    files in sorted order, optional shuffle with RANDOM_SEED 4242.
"""
import os
import random
import sys
import xml.etree.ElementTree as ET

from dataset.bdd100k import BDD100K_LABELS
from rod.tfrecord import TFRecordWriter, encode_detection_example

LABELS = BDD100K_LABELS
DIRECTORY_ANNOTATIONS = 'Annotations/'
DIRECTORY_IMAGES = 'JPEGImages/'
RANDOM_SEED = 4242
SAMPLES_PER_FILES = 5000


def process_image(directory, name):
    """(jpeg bytes, shape [h, w, c], boxes, labels, labels_text, difficult, truncated)."""
    with open(os.path.join(directory, DIRECTORY_IMAGES, name + '.jpg'), 'rb') as f:
        image_data = f.read()
    root = ET.parse(os.path.join(directory, DIRECTORY_ANNOTATIONS, name + '.xml')).getroot()
    size = root.find('size')
    shape = [int(size.find('height').text), int(size.find('width').text), int(size.find('depth').text)]
    boxes, labels, labels_text, difficult, truncated = [], [], [], [], []
    for obj in root.findall('object'):
        label = obj.find('name').text
        labels.append(int(LABELS[label][0]))
        labels_text.append(label.encode('ascii'))
        d, t = obj.find('difficult'), obj.find('truncated')
        # the reference's `if obj.find(...)`: True only for an element WITH children
        difficult.append(int(d.text) if d is not None and len(d) else 0)
        truncated.append(int(t.text) if t is not None and len(t) else 0)
        bb = obj.find('bndbox')
        boxes.append((float(bb.find('ymin').text) / shape[0], float(bb.find('xmin').text) / shape[1],
                      float(bb.find('ymax').text) / shape[0], float(bb.find('xmax').text) / shape[1]))
    return image_data, shape, boxes, labels, labels_text, difficult, truncated


def output_filename(output_dir, name, idx):
    return '%s/%s_%03d.tfrecord' % (output_dir, name, idx)


def run(dataset_dir, output_dir, name='voc_train', shuffling=False):
    """Convert every annotation under dataset_dir/Annotations; returns the shard paths."""
    os.makedirs(output_dir, exist_ok=True)
    names = sorted(os.listdir(os.path.join(dataset_dir, DIRECTORY_ANNOTATIONS)))
    if shuffling:
        random.seed(RANDOM_SEED)
        random.shuffle(names)
    shards, i, fidx = [], 0, 0
    while i < len(names):
        path = output_filename(output_dir, name, fidx)
        with TFRecordWriter(path) as w:
            j = 0
            while i < len(names) and j < SAMPLES_PER_FILES:
                sys.stdout.write('\r>> Converting image %d/%d' % (i + 1, len(names)))
                sys.stdout.flush()
                img, shape, boxes, labels, text, diff, trunc = process_image(dataset_dir, names[i][:-4])
                w.write(encode_detection_example(img, shape, boxes, labels, text, diff, trunc))
                i += 1
                j += 1
        shards.append(path)
        fidx += 1
    print('\nFinished converting the dataset!')
    return shards
