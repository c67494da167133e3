"""BDD100K dataset description (reference dataset/bdd100k.py): the TFRecord file pattern, the
split size, and the label map the converter and the evaluation use."""
FILE_PATTERN = 'bdd100k_%s_*.tfrecord'
SPLITS_TO_SIZES = {'train': 70000}
NUM_CLASSES = 10
# name -> (label id, super-category) (bdd100k.py:23-35)
BDD100K_LABELS = {
    'none': (0, 'Background'), 'bus': (1, 'Vehicle'), 'traffic light': (2, 'Flag'), 'traffic sign': (3, 'Flag'),
    'person': (4, 'Human'), 'bike': (5, 'Vehicle'), 'truck': (6, 'Vehicle'), 'motor': (7, 'Vehicle'),
    'car': (8, 'Vehicle'), 'train': (9, 'Vehicle'), 'rider': (10, 'Human'),
}
