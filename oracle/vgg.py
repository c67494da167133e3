"""ORACLE (test infrastructure only): VGG-16 + SSD extra blocks (reference
nets/backbone/vgg.py:67-137) restated with PyTorch-CPU ops on NCHW tensors.

slim.conv2d under vgg_arg_scope: SAME padding (TF-SAME, oracle.net.conv), bias, ReLU;
slim.max_pool2d([2, 2]): stride 2, VALID (floor); custom_layers.pad2d(1) + VALID stride-2 3x3
(blocks 8, 9); VALID 3x3 (block 10); tf.layers.dropout(rate=0.5): x / keep * binary with the
binary masks the product drew (`masks`, NHWC uint8, in call order) — the mask is random, the
arithmetic around it is what parity checks.
"""
import torch
import torch.nn.functional as F

from . import net as onet

SCOPE = 'backbone/vgg_16'
PLAN = [('conv1/conv1_1', 3), ('conv1/conv1_2', 3), 'pool', ('conv2/conv2_1', 3), ('conv2/conv2_2', 3), 'pool',
        ('conv3/conv3_1', 3), ('conv3/conv3_2', 3), ('conv3/conv3_3', 3), 'pool',
        ('conv4/conv4_1', 3), ('conv4/conv4_2', 3), ('conv4/conv4_3', 3), 'pool',
        ('conv5/conv5_1', 3), ('conv5/conv5_2', 3), ('conv5/conv5_3', 3), 'pool',
        ('block6/conv6', 3), 'dropout', ('block7/conv7', 1), 'dropout',
        ('block8/conv1x1', 1), ('block8/conv3x3', 3, 2, 1), ('block9/conv1x1', 1), ('block9/conv3x3', 3, 2, 1),
        ('block10/conv1x1', 1), ('block10/conv3x3', 3, 1, 0)]
TAPS = [SCOPE + '/conv4/conv4_3', SCOPE + '/conv5/conv5_3', SCOPE + '/block7/conv7', SCOPE + '/block8/conv3x3',
        SCOPE + '/block9/conv3x3', SCOPE + '/block10/conv3x3']   # config.py:23-25
KEEP = 0.5


def backbone(x, P, masks=None):
    """Returns the tapped endpoints (NCHW).  masks: the dropout binaries (training) or None."""
    eps = {}
    mi = 0
    for e in PLAN:
        if e == 'pool':
            x = F.max_pool2d(x, 2, 2)
            continue
        if e == 'dropout':
            if masks is not None:
                m = masks[mi].permute(0, 3, 1, 2).to(x.dtype)
                x = x / KEEP * m
            mi += 1
            continue
        name, k = e[0], e[1]
        w, b = P['%s/%s/weights' % (SCOPE, name)], P['%s/%s/biases' % (SCOPE, name)]
        if len(e) > 2:   # custom_layers.pad2d(pad) then VALID (stride s)
            s, pad = e[2], e[3]
            x = F.conv2d(F.pad(x, (pad, pad, pad, pad)), w.permute(0, 3, 1, 2), b, s)
        else:
            x = onet.conv(x, w, b)
        x = torch.relu(x)
        full = '%s/%s' % (SCOPE, name)
        if full in TAPS:
            eps[full] = x
    return [eps[t] for t in TAPS]


def forward(img_nhwc, P, B, training, masks=None, moving=None):
    """REFINE network on VGG-16: refine_out, six [B, fh, fw, A, 4]."""
    feats = backbone(img_nhwc.permute(0, 3, 1, 2), P, masks if training else None)
    return onet.head(feats, P, B, 'refine', 4, training, moving)
