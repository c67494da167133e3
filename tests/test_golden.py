"""Oracle and product host code against fixtures produced by the reference itself
(tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import pytest

from oracle import anchors as oa
from oracle import net as onet

SIZES = [(300, 300), (418, 418), (720, 1280), (1080, 1920)]


def _load(golden_dir, H, W):
    return np.load(os.path.join(golden_dir, 'ref_anchors_%dx%d.npz' % (H, W)))


@pytest.mark.parametrize('H,W', SIZES)
def test_oracle_anchors_match_reference(golden_dir, H, W):
    g = _load(golden_dir, H, W)
    spec = json.load(open(os.path.join(golden_dir, 'ref_spec.json')))
    strides = [e['stride'] for e in spec['spec']]
    chain = oa.feat_sizes((H, W), strides)
    init = oa.init_anchor(6, (H, W))
    for i in range(6):
        np.testing.assert_array_equal(init[i], g['init_%d' % i])
        feat = chain[onet.TAPS[i] - 1]
        assert tuple(g['feat_%d' % i]) == feat
        y, x, h, w = oa.anchors_one_layer((H, W), feat, init[i])
        for name, arr in zip('yxhw', (y, x, h, w)):
            ref = g['%s_%d' % (name, i)]
            assert arr.dtype == ref.dtype and arr.shape == ref.shape
            np.testing.assert_array_equal(arr, ref)


@pytest.mark.parametrize('H,W', SIZES)
def test_product_anchors_match_reference(golden_dir, H, W):
    import config
    import utils.net_tools as nt
    g = _load(golden_dir, H, W)
    old = config.img_size
    config.img_size = (H, W)
    try:
        feats = config.feat_sizes((H, W))
        init = nt.init_anchor(6)
        anc = nt.anchors_all_layer((H, W), feats, init)
    finally:
        config.img_size = old
    assert nt.n_anchor_each_layer('mobilenet_v2') == list(g['n_anchor'])
    for i, (y, x, h, w) in enumerate(anc):
        np.testing.assert_array_equal(list(init.values())[i], g['init_%d' % i])
        for name, arr in zip('yxhw', (y, x, h, w)):
            np.testing.assert_array_equal(arr, g['%s_%d' % (name, i)])
        assert tuple(g['feat_%d' % i]) == feats['layer_%d' % (i + 1)]


def test_spec_table_matches_reference(golden_dir):
    spec = json.load(open(os.path.join(golden_dir, 'ref_spec.json')))
    from nets.backbone.mobilenet_v2 import V2_SPEC, layer_plan, make_divisible
    assert len(spec['spec']) == len(V2_SPEC) == len(onet.SPEC)
    for ref, mine, orc in zip(spec['spec'], V2_SPEC, onet.SPEC):
        assert ref['stride'] == mine[1] == orc[1]
        assert ref['num_outputs'] == mine[2] == orc[2]
    for key, val in spec['make_divisible'].items():
        v, d = map(int, key.split('_'))
        assert make_divisible(v, d) == val == onet.make_divisible(v, d)
    # expansion sizes as the reference computes them (defaults: expand_input(6))
    plan = layer_plan()
    for (idx, kind, s, cin, inner, cout, res, sc), ref in zip(plan, spec['spec']):
        if kind != 'ir':
            continue
        table = ref.get('expansion_for_inputs', spec['default_expansion_for_inputs'])
        assert inner == table[str(cin)], (idx, cin, inner)
    assert [p for p in onet.layer_plan()] == [tuple(p) for p in plan]


def test_config_surface(golden_dir):
    import config
    spec = json.load(open(os.path.join(golden_dir, 'ref_spec.json')))
    assert config.extract_feat_name['mobilenet_v2'] == spec['extract_feat_name']
    assert {k: list(v) for k, v in config.feat_size_all_layers['mobilenet_v2'].items()} == spec['feat_size_418']
    assert config.refine_pos_jac_val_all_layers == spec['refine_pos_jac_val_all_layers']
    assert config.det_pos_jac_val_all_layers == spec['det_pos_jac_val_all_layers']
    assert config.total_obj_n == spec['total_obj_n']
    assert config.train_range.REFINE.value == 0 and config.train_range.ALL.value == 1
    assert config.refine_method.JACCARD_BIGGER.value == 1


def _geom(golden_dir, H, W):
    return np.load(os.path.join(golden_dir, 'ref_anchor_geom_%dx%d.npz' % (H, W)))


@pytest.mark.parametrize('H,W', SIZES)
def test_anchor_geometry_matches_reference(golden_dir, H, W):
    """The float32 anchor corners and the centres / sizes recomputed from them, as the
    reference computes them inside refine_groundtruth (net_tools.py:385-395) and
    decode_locations_one_layer (202-223): oracle and product tables bit-identical."""
    import config
    import utils.net_tools as nt
    g = _geom(golden_dir, H, W)
    old = config.img_size
    config.img_size = (H, W)
    try:
        anc = nt.anchors_all_layer((H, W), config.feat_sizes((H, W)), nt.init_anchor(6))
    finally:
        config.img_size = old
    tab = nt.AnchorTable(anc, 'cpu')
    ref_corner = np.concatenate([g['corner_%d' % l].reshape(-1, 4) for l in range(6)])
    ref_center = np.concatenate([g['center_%d' % l] for l in range(6)])
    np.testing.assert_array_equal(tab.corner_np, ref_corner)
    np.testing.assert_array_equal(tab.center_np, ref_center)
    for l, layer in enumerate(anc):
        np.testing.assert_array_equal(np.stack(oa.anchor_corners(layer), -1), g['corner_%d' % l])
        np.testing.assert_array_equal(np.stack(oa.anchor_centers(layer), -1).reshape(-1, 4), g['center_%d' % l])


@pytest.mark.gpu
@pytest.mark.parametrize('H,W', SIZES)
def test_device_anchor_tables_match_reference(golden_dir, dev, H, W):
    """The anchor tables the kernels read (uploaded to HBM once per resolution) against the
    reference's own numbers: anchors_all_layer and the JACCARD_BIGGER / decode geometry."""
    import config
    import utils.net_tools as nt
    g, gg = _load(golden_dir, H, W), _geom(golden_dir, H, W)
    old = config.img_size
    config.img_size = (H, W)
    try:
        anc = nt.anchors_all_layer((H, W), config.feat_sizes((H, W)), nt.init_anchor(6))
    finally:
        config.img_size = old
    for l, (y, x, h, w) in enumerate(anc):
        for name, arr in zip('yxhw', (y, x, h, w)):
            np.testing.assert_array_equal(arr, g['%s_%d' % (name, l)])
    tab = nt.AnchorTable(anc, dev)
    np.testing.assert_array_equal(tab.corner.cpu().numpy(),
                                  np.concatenate([gg['corner_%d' % l].reshape(-1, 4) for l in range(6)]))
    np.testing.assert_array_equal(tab.center.cpu().numpy(), np.concatenate([gg['center_%d' % l] for l in range(6)]))
