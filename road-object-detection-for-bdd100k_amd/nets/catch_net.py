"""Detector assembly — drop-in for the reference's nets/catch_net.py (factory, 37-363).

``factory(inputs, backbone_name, is_training, config_dict, dtype)`` builds (once, cached
per configuration) and runs the network on NHWC `inputs` and exposes ``get_output()``
exactly as the reference: REFINE -> refine_out; ALL -> (refine_out, det_out, clf_out),
each a list of six [B, fh, fw, A, 4 | 11] tensors.

Structure (reference line numbers):
  backbone endpoints layer_11/15/18/20/22/24 (__feats_aug_block NONE, 111-114)
  ALL: deconv pyramid LEARN_HALF (160-212) or LEARN_ALL (214-230) + ADD / CONCAT merge (237-273)
  heads: per level, for ch in [128, k*A]: conv1x1(+bias) -> BN -> leaky(0.2) ->
         conv3x3(+bias) -> BN -> leaky (276-342); head BN is slim's default
         (center, no scale, decay 0.999, eps 1e-3); weights xavier, biases zero.
"""
from __future__ import annotations

import collections
import contextlib

import numpy as np
import torch

import config
from nets.backbone.mobilenet_v2 import MobilenetV2
from nets.backbone.vgg import VGG16
from rod import graph, ops
from rod.params import ParamStore, trunc_normal, xavier_uniform

HEAD_BN_DECAY = 0.999
HEAD_BN_EPS = 1e-3


def n_anchor_each_layer(backbone_name):
    import utils.net_tools as net_tools
    return net_tools.n_anchor_each_layer(backbone_name)


class CatchNet:
    """Parameters + forward of the whole detector for one configuration."""

    def __init__(self, backbone_name, config_dict, device, seed=0, build_all=None):
        if backbone_name not in config.supported_backbone_name:
            raise ValueError('backbone %r is not supported (config.supported_backbone_name)' % backbone_name)
        self.msf = config_dict['process_backbone_method'] is config.process_backbone_method.PREORDER_MSF
        if not self.msf and config_dict['process_backbone_method'] is not config.process_backbone_method.NONE:
            raise ValueError('Not support the method(%s) now' % str(config_dict['process_backbone_method']))
        if self.msf and backbone_name != 'mobilenet_v2':
            raise ValueError('Sorry, not support the method(%s) for mobilenet_v2 now ~_~!!' %
                             str(config_dict['process_backbone_method']))
        self.backbone_name = backbone_name
        self.config_dict = dict(config_dict)
        self.train_range = config_dict['train_range']
        all_mode = self.train_range is config.train_range.ALL if build_all is None else build_all
        self.all_mode = all_mode
        rng = np.random.default_rng(seed)
        self.store = ParamStore()
        self.backbone = MobilenetV2(self.store, rng) if backbone_name == 'mobilenet_v2' else VGG16(self.store, rng)
        self.feat_ch = self._endpoint_channels()
        if self.msf:
            self._msf_params(rng)
        self.n_anchor = n_anchor_each_layer(backbone_name)
        self._head('refine', self.feat_ch, 4, rng)
        self.deconv_method = config_dict.get('deconv_method', config.deconv_method.LEARN_HALF)
        self.merge_method = config_dict.get('merge_method', config.merge_method.ADD)
        if all_mode:
            if self.deconv_method not in (config.deconv_method.LEARN_HALF, config.deconv_method.LEARN_ALL):
                raise ValueError('Parameter "method(%s)" wrong' % str(self.deconv_method))
            if self.merge_method not in (config.merge_method.ADD, config.merge_method.CONCAT):
                raise ValueError('parameter "method(%s)" wrong...' % str(self.merge_method))
            self._deconv(rng)
            # the deconv pyramid returns every level at the backbone tap's channel count
            # (LEARN_HALF: 2 * (C // 2), LEARN_ALL: C), so CONCAT doubles the head input
            merged_ch = self.feat_ch if self.merge_method is config.merge_method.ADD else \
                [c + d for c, d in zip(self.feat_ch, self.deconv_ch)]
            self._head('clf', merged_ch, config.total_obj_n, rng)
            self._head('det', merged_ch, 4, rng)
        self.store.finalize(device)

    # ------------------------------------------------------------------ parameters
    def _endpoint_channels(self):
        return self.backbone.endpoint_channels(config.extract_feat_name[self.backbone_name])

    # ------------------------------------------------------------------ PREORDER_MSF (catch_net.py:115-152)
    MSF_BLOCKS = [['layer_4', 'layer_7'], ['layer_7', 'layer_11']]
    MSF_COMPRESS = [[4, 16], [3, 12]]
    # space_to_depth blocks round(h / s_h), fixed by the stride chain (layer_4 / layer_7 are 4x / 2x
    # the size of layer_11, layer_7 / layer_11 4x / 2x that of layer_15); they set the SE widths
    MSF_RATIOS = [[4, 2], [4, 2]]

    def _msf_params(self, rng):
        """slim.conv2d 1x1 (+bias; outside the mobilenet arg_scope: xavier, no normaliser) and
        slim.batch_norm (beta only) per augmented endpoint, named in creation order under the
        'backbone' scope (Conv, Conv_1, ... / BatchNorm, BatchNorm_1, ...); se_block dense layers
        'backbone/se_aug_layer_%d/{bottleneck_fc, recover_fc}/{kernel, bias}'."""
        from nets.backbone.mobilenet_v2 import layer_plan
        outs = {'layer_%d' % idx: cout for (idx, _, _, _, _, cout, _, _) in layer_plan()}
        names = config.extract_feat_name['mobilenet_v2']
        ratios = self.MSF_RATIOS
        k = 0
        for index, blocks in enumerate(self.MSF_BLOCKS):
            ch = outs[names[index]]
            for (b, cc), r in zip(zip(blocks, self.MSF_COMPRESS[index]), ratios[index]):
                sfx = '' if k == 0 else '_%d' % k
                self._conv_params('backbone/Conv' + sfx, cc, 1, outs[b], rng)
                self._head_bn('backbone/BatchNorm' + sfx, cc)
                ch += cc * r * r
                k += 1
            se = 'backbone/se_aug_layer_%d' % (index + 1)
            # tf.contrib.layers.variance_scaling_initializer(): truncated normal, 2 / fan_in
            self.store.add(se + '/bottleneck_fc/kernel', trunc_normal(rng, (ch, ch // 8), float(np.sqrt(2.0 / ch))))
            self.store.add(se + '/bottleneck_fc/bias', np.zeros(ch // 8, np.float32))
            self.store.add(se + '/recover_fc/kernel', trunc_normal(rng, (ch // 8, ch), float(np.sqrt(2.0 / (ch // 8)))))
            self.store.add(se + '/recover_fc/bias', np.zeros(ch, np.float32))
            self.feat_ch[index] = ch

    def feats_aug(self, endpoints, training):
        """__feats_aug_block PREORDER_MSF (catch_net.py:115-152) -> the six backbone features."""
        P = self.store.params
        names = config.extract_feat_name['mobilenet_v2']
        uses = {}
        for index, blocks in enumerate(self.MSF_BLOCKS):
            for n in blocks + [names[index]]:
                uses[n] = uses.get(n, 0) + 1
        pool = {n: list(graph.fork(endpoints[n], k)) if k > 1 else [endpoints[n]] for n, k in uses.items()}
        feats = []
        k = 0
        for index, name in enumerate(names):
            if index >= len(self.MSF_BLOCKS):
                feats.append(endpoints[name])
                continue
            s_feat = pool[name].pop()
            s_h, s_w = s_feat.shape[1], s_feat.shape[2]
            aug = []
            for b, cc, r in zip(self.MSF_BLOCKS[index], self.MSF_COMPRESS[index], self.MSF_RATIOS[index]):
                feat = pool[b].pop()
                h, w = feat.shape[1], feat.shape[2]
                rh, rw = round(h / s_h), round(w / s_w)
                if rh != r or rw != r:
                    raise ValueError('PREORDER_MSF: %s is %dx%d, %s %dx%d: block %d expected' % (b, h, w, name, s_h, s_w, r))
                feat = ops.pad_top_left(feat, abs(h - rh * s_h), abs(w - rw * s_w))
                sfx = '' if k == 0 else '_%d' % k
                x = ops.materialize(self._conv_bn(feat, P['backbone/Conv%s/weights' % sfx],
                                                  P['backbone/Conv%s/biases' % sfx], 1, 'backbone/BatchNorm' + sfx,
                                                  training))
                if rh > 1:
                    x = ops.space_to_depth(x, rh)
                aug.append(x)
                k += 1
            aug.append(s_feat)
            se = 'backbone/se_aug_layer_%d' % (index + 1)
            feats.append(ops.se_block(ops.channel_concat(aug), P[se + '/bottleneck_fc/kernel'],
                                      P[se + '/bottleneck_fc/bias'], P[se + '/recover_fc/kernel'],
                                      P[se + '/recover_fc/bias']))
        return feats

    def _head_bn(self, name, c):
        self.store.add(name + '/beta', np.zeros(c, np.float32))
        self.store.add_buffer(name + '/moving_mean', np.zeros(c, np.float32))
        self.store.add_buffer(name + '/moving_variance', np.ones(c, np.float32))

    def _conv_params(self, name, cout, k, cin, rng, bias=True):
        self.store.add(name + '/weights', xavier_uniform(rng, (cout, k, k, cin)))
        if bias:
            self.store.add(name + '/biases', np.zeros(cout, np.float32))

    def _head(self, scope, in_chs, k, rng):
        for i, cin in enumerate(in_chs):
            base = '%s/block_%d' % (scope, i + 1)
            n = 0
            for ch in [128, k * self.n_anchor[i]]:
                for ks in (1, 3):
                    cname = base + ('/Conv' if n == 0 else '/Conv_%d' % n)
                    bname = base + ('/BatchNorm' if n == 0 else '/BatchNorm_%d' % n)
                    self._conv_params(cname, ch, ks, cin, rng)
                    self._head_bn(bname, ch)
                    cin = ch
                    n += 1

    def _deconv(self, rng):
        """__deconv_bone parameters (catch_net.py:177-230); self.deconv_ch = output channels
        per level in backbone order."""
        chs = list(reversed(self.feat_ch))
        out_ch = []
        i_c = chs[0]
        for i in range(len(chs)):
            base = 'deconv/block_%d' % (i + 1)
            if i == 0:
                self._conv_params(base + '/Conv', chs[0], 1, chs[0], rng)
                self._head_bn(base + '/BatchNorm', chs[0])
                o_c = chs[0]
            elif self.deconv_method is config.deconv_method.LEARN_HALF:
                f_c = chs[i] // 2
                # tf.get_variable('weight_%d', [2, 2, f_c, i_c], trunc-normal 0.02) (catch_net.py:189)
                self.store.add(base + '/weight_%d' % i, trunc_normal(rng, (2, 2, f_c, i_c), 0.02))
                self._conv_params(base + '/Conv', f_c, 1, i_c, rng)
                self._head_bn(base + '/BatchNorm', 2 * f_c)
                o_c = 2 * f_c
            else:   # LEARN_ALL (catch_net.py:214-230): [2, 2, f_c = C_target, i_c], BN over f_c
                f_c = chs[i]
                self.store.add(base + '/weight_%d' % i, trunc_normal(rng, (2, 2, f_c, i_c), 0.02))
                self._head_bn(base + '/BatchNorm', f_c)
                o_c = f_c
            out_ch.append(o_c)
            i_c = o_c
        self.deconv_ch = list(reversed(out_ch))

    # ------------------------------------------------------------------ forward
    def _bn(self, x, name, training, act=ops.ROD_ACT_LEAKY, parts=None, pending=False):
        """BatchNorm (beta only) + leaky; pending: applied in the next conv's load prologue."""
        P, B = self.store.params, self.store.buffers
        p = ops.bn_pending(x, None, P[name + '/beta'], B[name + '/moving_mean'], B[name + '/moving_variance'],
                           act, training, HEAD_BN_DECAY, HEAD_BN_EPS, parts)
        return p if pending and 'bnpro' not in ops._DISABLE else ops.materialize(p)

    def _conv_bn(self, x, w, b, ks, name, training, act=ops.ROD_ACT_LEAKY):
        """conv(+bias) + BatchNorm (beta only) + leaky as one node (ops.conv2d_bn), Pending."""
        P, B = self.store.params, self.store.buffers
        return ops.conv2d_bn(x, w, b, ks, None, P[name + '/beta'], B[name + '/moving_mean'],
                             B[name + '/moving_variance'], act, training, HEAD_BN_DECAY, HEAD_BN_EPS)

    def _conv_bn_out(self, x, w, b, ks, name, training, act=ops.ROD_ACT_LEAKY):
        """_conv_bn written out (inference: the BatchNorm and leaky in the conv's epilogue)."""
        P, B = self.store.params, self.store.buffers
        return ops.conv2d_bn_act(x, w, b, ks, None, P[name + '/beta'], B[name + '/moving_mean'],
                                 B[name + '/moving_variance'], act, training, HEAD_BN_DECAY, HEAD_BN_EPS)

    def head_out(self, feats, scope, k, training, ready=None):
        """__det_out / __clf_out (catch_net.py:276-342).  The levels' chains are independent:
        each runs on its own stream (ops.LEVELS), forked where its feature was produced
        (`ready`: events recorded by the backbone at its taps) and joined before returning."""
        P = self.store.params
        lv = ops.LEVELS if ops.LEVELS.active(feats[0]) else None
        outs = []
        for i, x in enumerate(feats):
            base = '%s/block_%d' % (scope, i + 1)
            n = 0
            s = lv.fork(i, x, ready[i] if ready else None) if lv is not None else None
            with torch.cuda.stream(s) if s is not None else contextlib.nullcontext():
                for ch in [128, k * self.n_anchor[i]]:
                    for ks in (1, 3):
                        cname = base + ('/Conv' if n == 0 else '/Conv_%d' % n)
                        bname = base + ('/BatchNorm' if n == 0 else '/BatchNorm_%d' % n)
                        # the first three BatchNorms feed only the next conv of the head (its prologue);
                        # the last one is written out
                        if n == 3:
                            x = self._conv_bn_out(x, P[cname + '/weights'], P[cname + '/biases'], ks, bname,
                                                  training)
                        else:
                            x = self._conv_bn(x, P[cname + '/weights'], P[cname + '/biases'], ks, bname, training)
                            if 'bnpro' in ops._DISABLE:
                                x = ops.materialize(x)
                        n += 1
            B_, fh, fw, _ = x.shape
            outs.append(x.view(B_, fh, fw, self.n_anchor[i], k))
        if lv is not None:
            lv.join(outs)
        return outs

    def deconv_bone(self, feats, training):
        """Deconvolution pyramid (catch_net.py:160-230), LEARN_HALF or LEARN_ALL; returns the
        levels in reversed (deepest-first) order."""
        P = self.store.params
        half = self.deconv_method is config.deconv_method.LEARN_HALF
        layers = list(reversed(feats))
        out = []
        x = layers[0]
        n = len(layers)
        for i in range(n):
            base = 'deconv/block_%d' % (i + 1)
            if i == 0:
                x = self._conv_bn_out(x, P[base + '/Conv/weights'], P[base + '/Conv/biases'], 1, base + '/BatchNorm',
                                      training)
            elif half:
                B_, h, w, _ = layers[i].shape
                x_out, x_up, x_rs = xs
                up = ops.deconv2x2(x_up, P[base + '/weight_%d' % i], (h, w))        # conv2d_transpose
                rs = ops.resize_bilinear(x_rs, (h, w))                               # resize_images
                rh = ops.conv2d(rs, P[base + '/Conv/weights'], P[base + '/Conv/biases'], 1)
                out.append(x_out)
                cat = ops.channel_concat([up, rh])                                   # tf.concat(-1)
                x = self._bn(cat, base + '/BatchNorm', training)
            else:
                B_, h, w, _ = layers[i].shape
                x_out, x_up = xs
                up = ops.deconv2x2(x_up, P[base + '/weight_%d' % i], (h, w))        # conv2d_transpose
                out.append(x_out)
                x = self._bn(up, base + '/BatchNorm', training)
            if i < n - 1:
                # output list + transpose conv (+ resize for LEARN_HALF)
                xs = graph.fork(x, 3 if half else 2)
        out.append(x)
        return out

    @torch.no_grad()
    def calibrate_batchnorm(self, inputs):
        """Set every BatchNorm's moving statistics to the batch statistics of `inputs` (one
        training-mode forward with decay 0).  For synthetic-weight runs only (bench / tests):
        random weights with the initial moving statistics (0, 1) make eval-mode activations
        vanish layer by layer (logits ~1e-7, uniform softmax), which is not what a trained
        detector's inference path sees."""
        import nets.backbone.mobilenet_v2 as mb
        global HEAD_BN_DECAY
        saved = (mb.BN_DECAY, HEAD_BN_DECAY)
        mb.BN_DECAY, HEAD_BN_DECAY = 0.0, 0.0
        try:
            self.forward(inputs, True)
        finally:
            mb.BN_DECAY, HEAD_BN_DECAY = saved

    def forward(self, inputs, is_training):
        if is_training:
            return self._forward(inputs, is_training)
        # inference: every BatchNorm's eval statistics from one launch (ParamStore.eval_refresh)
        self.store.eval_refresh(HEAD_BN_EPS)
        try:
            return self._forward(inputs, is_training)
        finally:
            self.store.eval_release()

    def _forward(self, inputs, is_training):
        names = config.extract_feat_name[self.backbone_name]
        if self.msf:
            taps = sorted(set(names) | {n for b in self.MSF_BLOCKS for n in b}, key=lambda n: int(n.split('_')[1]))
            feats = self.feats_aug(self.backbone(inputs, is_training, taps=taps), is_training)
        else:
            ep = self.backbone(inputs, is_training, taps=names)
            feats = [ep[n] for n in names]
        ready = [getattr(self.backbone, 'tap_events', {}).get(n) for n in names] if not self.msf else None
        self.backbone_feats = collections.OrderedDict(('layer_%d' % (i + 1), f) for i, f in enumerate(feats))
        if not self.all_mode:
            return self.head_out(feats, 'refine', 4, is_training, ready)
        # multi-consumer tensors are forked so their gradients are summed by rod_add:
        # every feature feeds the refine head and the merge; the deepest one also the deconv
        forks = [graph.fork(f, 3 if i == len(feats) - 1 else 2) for i, f in enumerate(feats)]
        refine_out = self.head_out([f[0] for f in forks], 'refine', 4, is_training, ready)
        deconv_in = feats[:-1] + [forks[-1][2]]     # the shallower ones contribute only their shape
        deconv = self.deconv_bone(deconv_in, is_training)
        self.deconv_feats = deconv
        if self.merge_method is config.merge_method.ADD:
            merged = [ops.add(f[1], d) for f, d in zip(forks, reversed(deconv))]
        else:   # CONCAT: tf.concat([backbone, deconv], -1) (catch_net.py:258-263)
            merged = [ops.channel_concat([f[1], d]) for f, d in zip(forks, reversed(deconv))]
        self.merge_feats = merged
        mf = [graph.fork(m, 2) for m in merged]
        clf_out = self.head_out([m[0] for m in mf], 'clf', config.total_obj_n, is_training)
        det_out = self.head_out([m[1] for m in mf], 'det', 4, is_training)
        return refine_out, det_out, clf_out


_NET_CACHE = {}


def get_net(backbone_name, config_dict, device='cuda', seed=0):
    key = (backbone_name, config_dict['train_range'], config_dict.get('deconv_method'), config_dict.get('merge_method'),
           config_dict['process_backbone_method'], str(device), seed)
    if key not in _NET_CACHE:
        _NET_CACHE[key] = CatchNet(backbone_name, config_dict, device, seed)
    return _NET_CACHE[key]


class factory(object):
    """Drop-in for catch_net.factory: runs the network on `inputs` at construction."""

    def __init__(self, inputs, backbone_name, is_training, config_dict, dtype=torch.float32, net=None):
        assert backbone_name in config.supported_backbone_name
        self.backbone_name = backbone_name
        self.is_training = is_training
        self.train_range = config_dict['train_range']
        self.net = net if net is not None else get_net(backbone_name, config_dict, inputs.device)
        x = inputs if inputs.dtype == dtype else ops.cast(inputs, dtype)
        out = self.net.forward(x, is_training)
        self.backbone_feats = self.net.backbone_feats
        if self.net.all_mode:
            self.refine_out, self.det_out, self.clf_out = out
            self.deconv_feats = self.net.deconv_feats
            self.merge_feats = self.net.merge_feats
        else:
            self.refine_out = out

    def get_output(self):
        if self.train_range is config.train_range.ALL:
            return self.refine_out, self.det_out, self.clf_out
        elif self.train_range is config.train_range.REFINE:
            return self.refine_out
        raise ValueError('Error')
