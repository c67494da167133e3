"""Detector configuration — the reference's config.py surface (same names, same enums).

Reference: config.py:13-100.  Differences (additions only):
  * ``feat_sizes(img_size)`` derives the six tapped feature-map sizes of any input
    resolution from the backbone's TF-SAME stride chain; the reference hard-codes
    the 418x418 row only (config.py:33-38).
  * ``feat_size_all_layers`` is kept for drop-in use and equals feat_sizes((418, 418)).
"""
from enum import Enum, unique

import numpy as np

# ---- anchors (config.py:14-16) ----------------------------------------------------------
normal_anchor_range = [0.05, 0.7]    # layers 2..6 share [0.05, 0.70]
special_anchor_range = [0.02, 0.03]  # layer 1 anchor sizes

img_size = (418, 418)  # default (height, width); BDD100K runs use (720, 1280)

supported_backbone_name = ['vgg_16', 'mobilenet_v2']

# endpoints tapped from each backbone (config.py:25-31)
extract_feat_name = {
    'vgg_16': ['backbone/vgg_16/conv4/conv4_3', 'backbone/vgg_16/conv5/conv5_3',
               'backbone/vgg_16/block7/conv7', 'backbone/vgg_16/block8/conv3x3',
               'backbone/vgg_16/block9/conv3x3', 'backbone/vgg_16/block10/conv3x3'],
    'mobilenet_v2': ['layer_11', 'layer_15', 'layer_18', 'layer_20', 'layer_22', 'layer_24'],
}

# strides of the 24 MobileNet-v2 spec entries (nets/backbone/mobilenet/mobilenet_v2.py:58-86)
MOBILENET_V2_STRIDES = [1, 1, 2, 1, 2, 1, 1, 2, 1, 1, 1, 2, 1, 1, 1, 2, 1, 1, 2, 1, 2, 1, 2, 1]


def feat_sizes(size, backbone_name='mobilenet_v2'):
    """{'layer_1': (fh, fw), ...} for an input of size (H, W): the TF-SAME ceil chain of the
    MobileNet-v2 strides, or VGG-16's chain (VALID 2x2 pools, pad2d + VALID 3x3 s2, VALID 3x3)."""
    if backbone_name == 'vgg_16':
        from nets.backbone.vgg import feat_sizes as vgg_sizes
        sizes = vgg_sizes(size)
        return {'layer_%d' % (j + 1): sizes[name] for j, name in enumerate(extract_feat_name['vgg_16'])}
    if backbone_name != 'mobilenet_v2':
        raise ValueError('unknown backbone %r' % backbone_name)
    h, w = int(size[0]), int(size[1])
    per_layer = {}
    for i, s in enumerate(MOBILENET_V2_STRIDES):
        h, w = -(-h // s), -(-w // s)
        per_layer['layer_%d' % (i + 1)] = (h, w)
    return {'layer_%d' % (j + 1): per_layer[name]
            for j, name in enumerate(extract_feat_name['mobilenet_v2'])}


feat_size_all_layers = {
    'mobilenet_v2': feat_sizes((418, 418)),
    'vgg_16': {'layer_1': (52, 52), 'layer_2': (26, 26), 'layer_3': (13, 13),
               'layer_4': (7, 7), 'layer_5': (4, 4), 'layer_6': (2, 2)},
}


# ---- network-building switches (config.py:44-71) -------------------------------------------
class process_backbone_method(Enum):
    NONE = 0
    PREORDER_MSF = 1
    RESIZE = 2
    MSF = 3


class train_range(Enum):
    REFINE = 0  # train the backbone + refine (ARM) heads only
    ALL = 1     # train deconv + det/clf (ODM) heads (and optionally the rest)


@unique
class merge_method(Enum):
    CONCAT = 0
    ADD = 1


@unique
class deconv_method(Enum):
    LEARN_HALF = 0
    LEARN_ALL = 1


# ---- target assignment (config.py:75-80) --------------------------------------------------
@unique
class refine_method(Enum):
    NEAREST_NEIGHBOR = 0
    JACCARD_BIGGER = 1
    JACCARD_TOPK = 2


refine_pos_jac_val_all_layers = [0.2, 0.3, 0.4, 0.4, 0.3, 0.3]
det_pos_jac_val_all_layers = [0.5, 0.6, 0.7, 0.7, 0.6, 0.6]

clf_weights = np.ones(11)

# ---- dataset (config.py:87-100) -------------------------------------------------------------
total_obj_n = 11  # 10 classes + background

category_index = {i: {'name': n} for i, n in enumerate(
    ['Background', 'Bus', 'Light', 'Sign', 'Person', 'Bike', 'Truck', 'Motor', 'Car', 'Train', 'Rider'])}
