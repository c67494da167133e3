"""Modified MobileNet-v2 backbone (reference nets/backbone/mobilenet/mobilenet_v2.py:41-87,
built by mobilenet.py:149-294 from conv_blocks.expanded_conv, conv_blocks.py:163-312).

Spec differences from stock MobileNet-v2, kept as in the reference: the stem conv has
stride 1, layers 19-20 have 320 outputs, and four x2-expansion blocks (256 outputs) are
appended.  Every conv is followed by BatchNorm (center+scale, decay 0.997, eps 1e-3)
and ReLU6, except the linear projection; no conv has a bias.
"""
from __future__ import annotations

import numpy as np
import torch

from rod import graph, ops
from rod.params import trunc_normal


def make_divisible(v, divisor, min_value=None):
    """Channel rounding of conv_blocks._make_divisible (conv_blocks.py:50-57)."""
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


# (kind, stride, num_outputs, expansion factor, divisible_by); kind 'conv' = 3x3 stem
V2_SPEC = [('conv', 1, 32, None, None), ('ir', 1, 16, 1, 1)] + \
    [('ir', s, c, 6, 8) for s, c in [(2, 24), (1, 24), (2, 32), (1, 32), (1, 32), (2, 64), (1, 64), (1, 64),
                                     (1, 64), (2, 96), (1, 96), (1, 96), (1, 96), (2, 160), (1, 160), (1, 160),
                                     (2, 320), (1, 320)]] + \
    [('ir', s, 256, 2, 8) for s in (2, 1, 2, 1)]

BN_DECAY = 0.997   # mobilenet.training_scope bn_decay (mobilenet.py:390)
BN_EPS = 1e-3      # slim.batch_norm default
W_STD = 0.09       # trunc-normal stddev (mobilenet.py:388)


def layer_plan(in_ch=3):
    """[(index, kind, stride, cin, inner, cout, residual, scope)] for the 24 spec entries."""
    plan, cin, n_ir = [], in_ch, 0
    for i, (kind, s, cout, exp, div) in enumerate(V2_SPEC):
        if kind == 'conv':
            plan.append((i + 1, 'conv', s, cin, None, cout, False, 'Conv'))
        else:
            inner = make_divisible(cin * exp, div)
            scope = 'expanded_conv' if n_ir == 0 else 'expanded_conv_%d' % n_ir
            n_ir += 1
            plan.append((i + 1, 'ir', s, cin, inner, cout, s == 1 and cin == cout, scope))
        cin = cout
    return plan


class MobilenetV2:
    def __init__(self, store, rng, scope='backbone/MobilenetV2'):
        self.store = store
        self.plan = layer_plan()
        self.scope = scope
        for (idx, kind, s, cin, inner, cout, res, sc) in self.plan:
            base = '%s/%s' % (scope, sc)
            if kind == 'conv':
                store.add(base + '/weights', trunc_normal(rng, (cout, 3, 3, cin), W_STD))
                self._bn(base + '/BatchNorm', cout)
                continue
            if inner > cin:  # conv_blocks.py:263
                store.add(base + '/expand/weights', trunc_normal(rng, (inner, 1, 1, cin), W_STD))
                self._bn(base + '/expand/BatchNorm', inner)
            store.add(base + '/depthwise/depthwise_weights', trunc_normal(rng, (3, 3, inner), W_STD))
            self._bn(base + '/depthwise/BatchNorm', inner)
            store.add(base + '/project/weights', trunc_normal(rng, (cout, 1, 1, inner), W_STD))
            self._bn(base + '/project/BatchNorm', cout)

    def endpoint_channels(self, names):
        outs = {'layer_%d' % idx: cout for (idx, _, _, _, _, cout, _, _) in self.plan}
        return [outs[n] for n in names]

    def _bn(self, name, c):
        self.store.add(name + '/gamma', np.ones(c, np.float32))
        self.store.add(name + '/beta', np.zeros(c, np.float32))
        self.store.add_buffer(name + '/moving_mean', np.zeros(c, np.float32))
        self.store.add_buffer(name + '/moving_variance', np.ones(c, np.float32))

    def _bn_args(self, name):
        P, B = self.store.params, self.store.buffers
        return P[name + '/gamma'], P[name + '/beta'], B[name + '/moving_mean'], B[name + '/moving_variance']

    def _eval_bn(self, name):
        """(mean, rstd, gamma, beta) of an eval-mode BatchNorm (moving statistics)."""
        g, b, mm, mv = self._bn_args(name)
        return (*ops.eval_stats(mm, mv, BN_EPS), g, b)

    def _conv_bn(self, x, w, ks, name, act, training, dw_stride=0):
        """conv + BatchNorm(+act) as one node (ops.conv2d_bn), left Pending (owned).  dw_stride: an
        expand conv feeding a depthwise of that stride (stride 2: its output may stay unwritten, the
        consumers recomputing it from x — ops._nostore_ok)."""
        return ops.conv2d_bn(x, w, None, ks, *self._bn_args(name), act, training, BN_DECAY, BN_EPS,
                             dw_stride=dw_stride)

    def __call__(self, x, is_training, final_endpoint=None, taps=None):
        """Returns the endpoint dict {'layer_1': ..., 'layer_24': ...} (mobilenet.py:275-281).

        Endpoints named in `taps` are consumed outside the backbone: they are handed out as
        a graph.fork alias, so their gradient meets the backbone's own with rod_add."""
        P = self.store.params
        end_points = {}
        self.tap_events = {}
        taps = set(taps or ())
        # The stem, expand and depthwise BatchNorms each feed exactly one consumer (the next
        # depthwise or project conv), so they stay Pending and are applied in that consumer's
        # load prologue; the project BatchNorm (+ residual) is written out as the endpoint.
        # Each conv and its BatchNorm are one autograd node (ops.conv2d_bn / dw3x3_bn) whose
        # backward runs the BatchNorm backward with the conv's own (fused for 1x1 where it pays).
        fuse = 'bnpro' not in ops._DISABLE
        keep = (lambda p: p) if fuse else ops.materialize
        # training with explicit taps (the detector): a project output that is no endpoint, has
        # no residual and feeds only the next block's expand (itself without a residual: block 1
        # -> block 2) stays Pending too — the expand applies it in its prologue and its backward
        # hands that BatchNorm its sums (rod_pw_bwd_gred), so neither the 720p x 16 BatchNorm
        # output nor its backward reduce crosses HBM
        chain = fuse and is_training and bool(taps) and 'chainpro' not in ops._DISABLE
        for i, (idx, kind, s, cin, inner, cout, res, sc) in enumerate(self.plan):
            base = '%s/%s' % (self.scope, sc)
            name = 'layer_%d' % idx
            tapped = name in taps or final_endpoint == name
            if kind == 'conv':
                x = self._conv_bn(x, P[base + '/weights'], 3, base + '/BatchNorm', ops.ROD_ACT_RELU6, is_training)
                x = ops.materialize(x) if tapped else keep(x)
            elif (not is_training and inner > cin and torch.is_tensor(x) and x.dtype == torch.bfloat16 and
                  ops.ir_block_preferred(cin, inner, cout, s, res, x.dtype)):
                # inference: the whole block in one kernel, the expanded tensor never in HBM
                x = ops.ir_block_fwd(x, P[base + '/expand/weights'], self._eval_bn(base + '/expand/BatchNorm'),
                                     P[base + '/depthwise/depthwise_weights'],
                                     self._eval_bn(base + '/depthwise/BatchNorm'), P[base + '/project/weights'],
                                     self._eval_bn(base + '/project/BatchNorm'), s, res)
            else:
                inp = None
                if res:
                    inp, x = graph.fork(x, 2)
                if inner > cin:
                    x = keep(self._conv_bn(x, P[base + '/expand/weights'], 1, base + '/expand/BatchNorm',
                                           ops.ROD_ACT_RELU6, is_training, dw_stride=s))
                x = keep(ops.dw3x3_bn(x, P[base + '/depthwise/depthwise_weights'], s,
                                      *self._bn_args(base + '/depthwise/BatchNorm'), ops.ROD_ACT_RELU6, is_training,
                                      BN_DECAY, BN_EPS))
                nxt = self.plan[i + 1] if i + 1 < len(self.plan) else None
                pend = (chain and not res and not tapped and final_endpoint != name and nxt is not None and
                        nxt[1] != 'conv' and nxt[4] > nxt[3] and not nxt[6])
                if pend:
                    x = self._conv_bn(x, P[base + '/project/weights'], 1, base + '/project/BatchNorm',
                                      ops.ROD_ACT_NONE, is_training)
                else:   # written out (+ the residual): in inference one launch (ops.conv2d_bn_act)
                    x = ops.conv2d_bn_act(x, P[base + '/project/weights'], None, 1,
                                          *self._bn_args(base + '/project/BatchNorm'), ops.ROD_ACT_NONE, is_training,
                                          BN_DECAY, BN_EPS, residual=inp)
            last = final_endpoint == name or idx == self.plan[-1][0]
            if name in taps and not last:
                end_points[name], x = graph.fork(x, 2)
            else:
                end_points[name] = x
            if name in taps and ops.LEVELS.active(end_points[name]):
                # where a consumer on another stream (a detector head, ops.LEVELS) may start
                ev = torch.cuda.Event()
                ev.record()
                self.tap_events[name] = ev
            if last:
                break
        return end_points


def mobilenet_v2(inputs, is_training, net):
    """Functional form mirroring mobilenet_v2(inputs, is_training=...) -> end_points."""
    return net(inputs, is_training)
