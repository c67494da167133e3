"""Generate golden fixtures from the reference itself (run only in the build container,
where /root/reference exists).  Never imported by tests; its outputs are committed:

  ref_anchors_<H>x<W>.npz   init_anchor + anchors_all_layer outputs (net_tools.py:21-142)
  ref_anchor_geom_<H>x<W>.npz  the float32 anchor corners and recomputed centres / sizes the
                            reference itself builds inside refine_groundtruth (JACCARD_BIGGER,
                            net_tools.py:385-395) and decode_locations_one_layer
                            (net_tools.py:202-223), captured from the stub's call records
  ref_spec.json             MobileNet-v2 spec params (mobilenet_v2.py:57-86) and
                            _make_divisible samples (conv_blocks.py:50-57)

TensorFlow is not installable here; a stub module that answers every `tensorflow.*`
import with a MagicMock lets the reference's *pure numpy/python* functions run for real.
Only undecorated functions and data tables are trusted (slim-decorated functions become
mocks).  Usage:  python tests/golden/make_golden.py
"""
import importlib.abc
import importlib.machinery
import json
import os
import sys
from unittest import mock

import numpy as np

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


class _TFStub(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, name, path, target=None):
        if name == 'tensorflow' or name.startswith('tensorflow.'):
            return importlib.machinery.ModuleSpec(name, self, is_package=True)
        return None

    def create_module(self, spec):
        m = mock.MagicMock(name=spec.name)
        m.__path__ = []
        m.__spec__ = spec
        return m

    def exec_module(self, module):
        pass


def tf_same_chain(h, w, strides):
    out = []
    for s in strides:
        h, w = -(-h // s), -(-w // s)
        out.append((h, w))
    return out


def capture_geometry(nt, anc, H, W):
    """Run the reference's refine_groundtruth (JACCARD_BIGGER) and decode_locations_one_layer
    under the stub: their numpy anchor arithmetic runs for real and its results arrive as
    arguments of the mocked tf calls (tf.stack of the corners; the offset-tensor mock's
    __mul__ / __add__ with anchor_h / anchor_w / anchor_cy / anchor_cx)."""
    from unittest import mock as _m
    import config as ref_config
    tf = nt.tf
    tf.reset_mock()
    tf.while_loop.side_effect = lambda cond, body, loop_vars, **kw: tuple(_m.MagicMock() for _ in loop_vars)
    center = _m.MagicMock()          # a [G, 4] tensor in the graph; only the anchors are numpy
    nt.refine_groundtruth(anc, center, np.array([1]), ref_config.refine_method.JACCARD_BIGGER)
    corners = [c.args[0] for c in tf.stack.call_args_list
               if isinstance(c.args[0], (list, tuple)) and len(c.args[0]) == 4 and
               all(isinstance(a, np.ndarray) for a in c.args[0])]
    assert len(corners) == len(anc), len(corners)
    arrs = {}
    for l, layer in enumerate(anc):
        arrs['corner_%d' % l] = np.stack(corners[l], -1)
        tf.reset_mock()
        off = _m.MagicMock()
        off.get_shape.return_value.as_list.return_value = [1, -1, 4]
        nt.decode_locations_one_layer(layer, off)
        r = tf.reshape.return_value.__getitem__.return_value
        muls = [c.args[0] for c in r.__mul__.call_args_list]
        adds = [c.args[0] for c in r.__mul__.return_value.__add__.call_args_list]
        assert len(muls) == 2 and len(adds) == 2
        arrs['center_%d' % l] = np.stack([adds[0], adds[1], muls[0], muls[1]], -1)   # (cy, cx, h, w)
    tf.while_loop.side_effect = None
    np.savez_compressed(os.path.join(OUT, 'ref_anchor_geom_%dx%d.npz' % (H, W)), **arrs)


def main():
    sys.meta_path.insert(0, _TFStub())
    sys.path.insert(0, REF)
    import config as ref_config
    import utils.net_tools as nt
    from nets.backbone.mobilenet import conv_blocks, mobilenet_v2

    # --- spec table -------------------------------------------------------------
    spec = []
    for op in mobilenet_v2.V2_DEF['spec']:
        p = dict(op.params)
        entry = {'stride': int(p.get('stride', 1)), 'num_outputs': int(p['num_outputs'])}
        if 'kernel_size' in p:
            entry['kernel_size'] = list(p['kernel_size'])
        exp = p.get('expansion_size')
        if exp is not None:
            entry['expansion_for_inputs'] = {str(c): int(exp(num_inputs=c)) for c in
                                             (16, 24, 32, 64, 96, 160, 256, 320)}
        spec.append(entry)
    default_exp = None
    for v in mobilenet_v2.V2_DEF['defaults'].values():
        if isinstance(v, dict) and 'expansion_size' in v:
            default_exp = {str(c): int(v['expansion_size'](num_inputs=c)) for c in (16, 24, 32, 64, 96, 160, 320)}
    strides = [e['stride'] for e in spec]
    md = {f'{v}_{d}': int(conv_blocks._make_divisible(v, d)) for v in (3, 17, 32, 96, 100, 144, 200, 960, 1920)
          for d in (1, 8)}
    json.dump({'spec': spec, 'make_divisible': md, 'default_expansion_for_inputs': default_exp,
               'extract_feat_name': ref_config.extract_feat_name['mobilenet_v2'],
               'feat_size_418': {k: list(v) for k, v in ref_config.feat_size_all_layers['mobilenet_v2'].items()},
               'refine_pos_jac_val_all_layers': ref_config.refine_pos_jac_val_all_layers,
               'det_pos_jac_val_all_layers': ref_config.det_pos_jac_val_all_layers,
               'total_obj_n': ref_config.total_obj_n},
              open(os.path.join(OUT, 'ref_spec.json'), 'w'), indent=1)

    # --- anchors at several resolutions ----------------------------------------------
    taps = [11, 15, 18, 20, 22, 24]
    for (H, W) in [(300, 300), (418, 418), (720, 1280), (1080, 1920)]:
        ref_config.img_size = (H, W)  # init_anchor reads config.img_size (net_tools.py:37-38)
        chain = tf_same_chain(H, W, strides)
        feats = {'layer_%d' % (i + 1): chain[t - 1] for i, t in enumerate(taps)}
        init = nt.init_anchor(6)
        anc = nt.anchors_all_layer((H, W), feats, init)
        arrs = {}
        for i, (k, v) in enumerate(init.items()):
            arrs['init_%d' % i] = np.asarray(v)
        for i, (y, x, h, w) in enumerate(anc):
            arrs['y_%d' % i], arrs['x_%d' % i], arrs['h_%d' % i], arrs['w_%d' % i] = y, x, h, w
            arrs['feat_%d' % i] = np.array(feats['layer_%d' % (i + 1)])
        arrs['n_anchor'] = np.array([v.shape[0] for v in init.values()])
        np.savez_compressed(os.path.join(OUT, 'ref_anchors_%dx%d.npz' % (H, W)), **arrs)
        capture_geometry(nt, anc, H, W)
    print('golden fixtures written to', OUT)


if __name__ == '__main__':
    main()
