"""VGG-16 backbone with the SSD extra blocks (reference nets/backbone/vgg.py:67-137), the
second entry of config.supported_backbone_name.

Structure (vgg_arg_scope: every conv SAME, bias, ReLU, xavier weights, zero biases):
  conv1 2x64, pool1, conv2 2x128, pool2, conv3 3x256, pool3, conv4 3x512 [tap conv4_3], pool4,
  conv5 3x512 [tap conv5_3], pool5 (2x2/2 VALID max pools, vgg.py:93-101);
  block6: conv6 3x3 1024 + dropout; block7: conv7 1x1 1024 [tap] + dropout;
  block8: conv1x1 256, pad2d(1), conv3x3 512 stride 2 VALID [tap];
  block9: conv1x1 128, pad2d(1), conv3x3 256 stride 2 VALID [tap];
  block10: conv1x1 128, conv3x3 256 VALID [tap].
Dropout is tf.layers.dropout(rate=dropout_keep_prob=0.5, training=is_training) as the
reference calls it (vgg.py:106, 111: the keep probability is passed as the drop RATE).

MI355X mapping: every SAME stride-1 conv is the implicit-GEMM rod_conv_fwd (3x3 / 1x1, the
ReLU of the previous conv applied in its load prologue: ops.conv2d_act returns an owned
Pending); the strided / VALID 3x3s of blocks 8-10 run on maps <= 1/16 of the input through
rod_im2col3x3 + the ksize-1 GEMM; pools and dropout are rod_maxpool2x2 / rod_dropout.
"""
from __future__ import annotations

import numpy as np

from rod import graph, ops
from rod.params import xavier_uniform

SCOPE = 'backbone/vgg_16'
# (scope, Cout, ksize, stride, padding, explicit pad) in execution order; 'pool' / 'dropout' markers
PLAN = [('conv1/conv1_1', 64, 3), ('conv1/conv1_2', 64, 3), 'pool',
        ('conv2/conv2_1', 128, 3), ('conv2/conv2_2', 128, 3), 'pool',
        ('conv3/conv3_1', 256, 3), ('conv3/conv3_2', 256, 3), ('conv3/conv3_3', 256, 3), 'pool',
        ('conv4/conv4_1', 512, 3), ('conv4/conv4_2', 512, 3), ('conv4/conv4_3', 512, 3), 'pool',
        ('conv5/conv5_1', 512, 3), ('conv5/conv5_2', 512, 3), ('conv5/conv5_3', 512, 3), 'pool',
        ('block6/conv6', 1024, 3), 'dropout',
        ('block7/conv7', 1024, 1), 'dropout',
        ('block8/conv1x1', 256, 1), ('block8/conv3x3', 512, 3, 2, 'VALID', 1),
        ('block9/conv1x1', 128, 1), ('block9/conv3x3', 256, 3, 2, 'VALID', 1),
        ('block10/conv1x1', 128, 1), ('block10/conv3x3', 256, 3, 1, 'VALID', 0)]
DROPOUT_RATE = 0.5   # vgg_16(dropout_keep_prob=0.5) passed as tf.layers.dropout(rate=...)


def _spec(e):
    name, cout, k = e[:3]
    stride, padding, pad = (e[3], e[4], e[5]) if len(e) > 3 else (1, 'SAME', 0)
    return name, cout, k, stride, padding, pad


def feat_sizes(size):
    """Spatial sizes of the six tapped endpoints for an input of size (H, W)."""
    h, w = int(size[0]), int(size[1])
    out = {}
    for e in PLAN:
        if e == 'pool':
            h, w = h // 2, w // 2
        elif e != 'dropout':
            name, _, k, s, padding, pad = _spec(e)
            if padding == 'VALID':
                h, w = (h + 2 * pad - k) // s + 1, (w + 2 * pad - k) // s + 1
            out['%s/%s' % (SCOPE, name)] = (h, w)
    return out


class VGG16:
    def __init__(self, store, rng, scope=SCOPE):
        self.store = store
        self.scope = scope
        self.channels = {}
        cin = 3
        for e in PLAN:
            if isinstance(e, str):
                continue
            name, cout, k, _, _, _ = _spec(e)
            base = '%s/%s' % (scope, name)
            store.add(base + '/weights', xavier_uniform(rng, (cout, k, k, cin)))
            store.add(base + '/biases', np.zeros(cout, np.float32))
            self.channels[base] = cout
            cin = cout
        self.last_dropout_masks = []

    def endpoint_channels(self, names):
        return [self.channels[n] for n in names]

    def __call__(self, x, is_training, taps=None, final_endpoint=None):
        """Returns the endpoint dict {'backbone/vgg_16/conv1/conv1_1': ..., ...} (the reference's
        outputs collection, vgg.py:134); tapped endpoints are handed out as relu outputs
        (graph.fork aliases when the backbone consumes them too)."""
        P = self.store.params
        taps = set(taps or ())
        end_points = {}
        self.last_dropout_masks = []
        last = '%s/%s' % (self.scope, _spec(PLAN[-1])[0])
        for e in PLAN:
            if e == 'pool':
                x = ops.max_pool2x2(x)
                continue
            if e == 'dropout':
                x, mask = ops.dropout(x, DROPOUT_RATE, is_training)
                self.last_dropout_masks.append(mask)
                continue
            name, cout, k, s, padding, pad = _spec(e)
            base = '%s/%s' % (self.scope, name)
            x = ops.conv2d_act(x, P[base + '/weights'], P[base + '/biases'], k, ops.ROD_ACT_RELU, s, padding, pad,
                               is_training)
            if base in taps:
                x = ops.materialize(x)
                if base != last and final_endpoint != base:
                    end_points[base], x = graph.fork(x, 2)
                else:
                    end_points[base] = x
            else:
                end_points[base] = x
            if base == last or final_endpoint == base:
                break
        return end_points
