"""ORACLE (test infrastructure only): anchor generation, restated from
utils/net_tools.py:21-142 of the reference."""
import math

import numpy as np

NORMAL_RANGE = (0.05, 0.7)    # config.py:15
SPECIAL_RANGE = (0.02, 0.03)  # config.py:16


def init_anchor(n_layers, img_size):
    """net_tools.py:21-82 — (h, w) in pixels of img_size for each layer."""
    out = []
    amin, amax = NORMAL_RANGE
    per = (amax - amin) / (n_layers - 1)
    lo, hi = amin, amin + per
    H, W = img_size
    for i in range(n_layers):
        if i == 0:
            f = list(SPECIAL_RANGE)
        else:
            f = [lo, (2 * lo + hi) / 3, (lo + 2 * hi) / 3]
            lo = hi
            hi = lo + per
        rows = []
        for s in f:
            rows.append([s * H, s * W])
            rows.append([s * H / math.sqrt(3), s * W * math.sqrt(3)])
            rows.append([s * H * math.sqrt(3), s * W / math.sqrt(3)])
        a = np.array(rows)
        a[:, 0] = np.minimum(a[:, 0], H)
        a[:, 1] = np.minimum(a[:, 1], W)
        out.append(a)
    return out


def anchors_one_layer(img_shape, feat_shape, anchors):
    """net_tools.py:98-122."""
    y, x = np.mgrid[0:feat_shape[0], 0:feat_shape[1]]
    xc = ((x + 0.5) / feat_shape[1])[..., None].astype(np.float32)
    yc = ((y + 0.5) / feat_shape[0])[..., None].astype(np.float32)
    h = (anchors[:, 0] / img_shape[0]).astype(np.float32)
    w = (anchors[:, 1] / img_shape[1]).astype(np.float32)
    return yc, xc, h, w


def anchor_corners(layer):
    """net_tools.py:385-395 / 156-165: float32 corners of every anchor [fh, fw, A]."""
    yref, xref, href, wref = layer
    return (np.float32(yref - href / 2.), np.float32(xref - wref / 2.),
            np.float32(yref + href / 2.), np.float32(xref + wref / 2.))


def anchor_centers(layer):
    """net_tools.py:168-171 (from the float32 corners)."""
    ymin, xmin, ymax, xmax = anchor_corners(layer)
    return (ymax + ymin) / 2., (xmax + xmin) / 2., ymax - ymin, xmax - xmin


def feat_sizes(img_size, strides):
    h, w = img_size
    out = []
    for s in strides:
        h, w = -(-h // s), -(-w // s)
        out.append((h, w))
    return out
