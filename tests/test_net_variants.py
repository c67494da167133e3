"""CPU: the parameter set the product builds for every deconv / merge method (catch_net.py:
160-273) is exactly what the oracle network consumes — names and shapes — so the GPU parity
test (test_gpu_train.py::test_all_mode_step_matches_oracle) compares like with like."""
import pytest
import torch

import config
from nets.catch_net import CatchNet
from oracle import net as onet

_DM, _MM = config.deconv_method, config.merge_method


@pytest.mark.parametrize('dm', [_DM.LEARN_HALF, _DM.LEARN_ALL])
@pytest.mark.parametrize('mm', [_MM.ADD, _MM.CONCAT])
def test_all_mode_params_match_oracle(dm, mm):
    cfg = {'train_range': config.train_range.ALL, 'process_backbone_method': config.process_backbone_method.NONE,
           'deconv_method': dm, 'merge_method': mm}
    net = CatchNet('mobilenet_v2', cfg, 'cpu', 0)
    P = {k: v.detach().clone().double() for k, v in net.store.params.items()}
    B = {k: v.detach().clone().double() for k, v in net.store.buffers.items()}
    used = set()

    class Tracker(dict):
        def __getitem__(self, k):
            used.add(k)
            return dict.__getitem__(self, k)
    x = torch.zeros((1, 64, 96, 3), dtype=torch.float64)
    refine, det, clf = onet.forward(x, Tracker(P), B, True, all_mode=True, moving={},
                                    learn_all=dm is _DM.LEARN_ALL, concat=mm is _MM.CONCAT)
    assert used == set(P), (sorted(set(P) - used)[:5], sorted(used - set(P))[:5])
    assert [tuple(t.shape[-2:]) for t in clf] == [(a, 11) for a in onet.N_ANCHOR]
    if mm is _MM.CONCAT:
        assert net.store.params['clf/block_1/Conv/weights'].shape[-1] == 2 * net.feat_ch[0]
    if dm is _DM.LEARN_ALL:
        assert 'deconv/block_2/Conv/weights' not in P
        assert tuple(P['deconv/block_2/weight_1'].shape) == (2, 2, net.feat_ch[-2], net.feat_ch[-1])


def test_unknown_methods_raise():
    cfg = {'train_range': config.train_range.ALL, 'process_backbone_method': config.process_backbone_method.NONE,
           'deconv_method': 'bogus', 'merge_method': _MM.ADD}
    with pytest.raises(ValueError):
        CatchNet('mobilenet_v2', cfg, 'cpu', 0)


def test_vgg_params_and_sizes_match_reference_and_oracle():
    """VGG-16 (vgg.py:67-137): the tapped sizes at 418x418 equal the reference's own table
    (config.feat_size_all_layers['vgg_16'], config.py:36-37), and the oracle consumes exactly
    the product's backbone + refine-head parameters."""
    from oracle import vgg as ovgg
    assert config.feat_sizes((418, 418), 'vgg_16') == config.feat_size_all_layers['vgg_16']
    cfg = {'train_range': config.train_range.REFINE, 'process_backbone_method': config.process_backbone_method.NONE,
           'deconv_method': _DM.LEARN_HALF, 'merge_method': _MM.ADD}
    net = CatchNet('vgg_16', cfg, 'cpu', 0)
    assert net.feat_ch == [512, 512, 1024, 512, 256, 256]
    P = {k: v.detach().clone().double() for k, v in net.store.params.items()}
    B = {k: v.detach().clone().double() for k, v in net.store.buffers.items()}
    used = set()

    class Tracker(dict):
        def __getitem__(self, k):
            used.add(k)
            return dict.__getitem__(self, k)
    out = ovgg.forward(torch.zeros((1, 288, 512, 3), dtype=torch.float64), Tracker(P), B, False)
    assert used == set(P)
    sizes = config.feat_sizes((288, 512), 'vgg_16')
    assert [tuple(o.shape[1:3]) for o in out] == [sizes['layer_%d' % (i + 1)] for i in range(6)]


def test_preorder_msf_params_match_oracle():
    """PREORDER_MSF + SE (catch_net.py:115-152, attention_module.py:3-33): product parameters ==
    oracle consumption; the augmented levels are 192 channels wide."""
    cfg = {'train_range': config.train_range.ALL, 'process_backbone_method': config.process_backbone_method.PREORDER_MSF,
           'deconv_method': _DM.LEARN_HALF, 'merge_method': _MM.ADD}
    net = CatchNet('mobilenet_v2', cfg, 'cpu', 0)
    assert net.feat_ch[:2] == [192, 192]
    P = {k: v.detach().clone().double() for k, v in net.store.params.items()}
    B = {k: v.detach().clone().double() for k, v in net.store.buffers.items()}
    used = set()

    class Tracker(dict):
        def __getitem__(self, k):
            used.add(k)
            return dict.__getitem__(self, k)
    onet.forward(torch.zeros((1, 160, 288, 3), dtype=torch.float64), Tracker(P), B, False, all_mode=True, msf=True)
    assert used == set(P)
