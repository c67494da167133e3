"""A17 on the GPU: rod_augment_images / rod_augment_boxes against the numpy oracle
(oracle/augment.py) on the same sampled parameters.

Bar: boxes, labels and counts bit-exact; images bit-exact without colour ops (crop, legacy
resize, flip are the same float32 op sequence); with colour ops within 1e-3 on the 0-255
scale (the contrast mean is an f64 sum in a different order; every other op is float32 per
operation in both); bf16 normalised output within one bf16 rounding of the oracle."""
import numpy as np
import pytest
import torch

from oracle import augment as oa
from rod import ops
from utils import data_pileline_tools as dpt
from utils.augmentation import tf_image

pytestmark = pytest.mark.gpu


def _params(rng, hw, B, colour=True):
    crop, mode, col = [], [], []
    for b in range(B):
        H, W = hw[b]
        h = int(rng.integers(1, H + 1))
        w = int(rng.integers(1, W + 1))
        crop.append([int(rng.integers(0, H - h + 1)), int(rng.integers(0, W - w + 1)), h, w])
        mode.append([int(rng.integers(0, 2)), int(rng.integers(0, 4)) if colour else -1])
        col.append([rng.uniform(-0.8, 0.8), rng.uniform(0.5, 1.0), rng.uniform(0.5, 1.0)])
    return np.array(crop, np.int32), np.array(mode, np.int32), np.array(col, np.float32)


def _oracle(srcs, crop, mode, col, Ho, Wo, normalize):
    return np.stack([oa.process_image(srcs[b], crop[b], mode[b, 0], mode[b, 1], col[b], Ho, Wo, normalize)
                     for b in range(len(srcs))])


@pytest.mark.parametrize('colour', [False, True])
@pytest.mark.parametrize('Ho,Wo', [(72, 128), (45, 81), (7, 5)])
def test_augment_images_uniform_batch(dev, colour, Ho, Wo):
    rng = np.random.default_rng(Ho * 7 + colour)
    B, H, W = 5, 90, 160
    src = rng.integers(0, 256, (B, H, W, 3)).astype(np.uint8)
    crop, mode, col = _params(rng, [(H, W)] * B, B, colour)
    if colour:
        mode[:4, 1] = [0, 1, 2, 3]
    out = ops.augment_images(torch.from_numpy(src).to(dev), crop, mode, col, (Ho, Wo)).cpu().numpy()
    ref = _oracle(src, crop, mode, col, Ho, Wo, False)
    if colour:
        np.testing.assert_allclose(out, ref, rtol=0, atol=1e-3)
    else:
        np.testing.assert_array_equal(out, ref)


def test_augment_images_ragged_sources_and_bf16(dev):
    """Images of different sizes packed in one buffer; normalised bf16 output."""
    rng = np.random.default_rng(11)
    hw = [(37, 53), (64, 48), (5, 9), (120, 200)]
    srcs = [rng.integers(0, 256, (h, w, 3)).astype(np.uint8) for h, w in hw]
    off = np.cumsum([0] + [s.size for s in srcs])[:-1].astype(np.int64)
    flat = torch.from_numpy(np.concatenate([s.reshape(-1) for s in srcs])).to(dev)
    crop, mode, col = _params(rng, hw, len(hw))
    Ho, Wo = 33, 47
    out32 = ops.augment_images(flat, crop, mode, col, (Ho, Wo), src_hw=np.array(hw, np.int32), src_off=off,
                               normalize=True).cpu().numpy()
    out16 = ops.augment_images(flat, crop, mode, col, (Ho, Wo), dtype=torch.bfloat16, normalize=True,
                               src_hw=np.array(hw, np.int32), src_off=off)
    ref = _oracle(srcs, crop, mode, col, Ho, Wo, True)
    np.testing.assert_allclose(out32, ref, rtol=0, atol=1e-5)
    np.testing.assert_array_equal(out16.float().cpu().numpy(), torch.from_numpy(out32).bfloat16().float().numpy())


def test_augment_images_rejects_bad_crop(dev):
    src = torch.zeros((1, 10, 10, 3), dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        ops.augment_images(src, np.array([[5, 0, 6, 10]]), np.array([[0, -1]]), np.zeros((1, 3)), (4, 4))


@pytest.mark.parametrize('G', [8, 64, 100])
def test_augment_boxes_bit_exact(dev, G):
    rng = np.random.default_rng(G)
    B = 6
    n = rng.integers(0, G + 1, B).astype(np.int32)
    n[0], n[1] = 0, G
    c = rng.uniform(0, 1, (B, G, 2))
    s = rng.uniform(0, 0.5, (B, G, 2))
    boxes = np.concatenate([c - s / 2, c + s / 2], -1).astype(np.float32)
    boxes[:, ::7, 2] = boxes[:, ::7, 0]            # zero-height boxes: safe_divide -> score 0
    labels = rng.integers(1, 11, (B, G)).astype(np.int32)
    y0 = rng.uniform(0, 0.5, B)
    x0 = rng.uniform(0, 0.5, B)
    ref = np.stack([y0, x0, y0 + rng.uniform(0.3, 0.5, B), x0 + rng.uniform(0.3, 0.5, B)], 1).astype(np.float32)
    ref[2] = [0, 0, 1, 1]
    mode = np.stack([rng.integers(0, 2, B), np.zeros(B)], 1).astype(np.int32)
    bo, lo, no = ops.augment_boxes(torch.from_numpy(boxes).to(dev), torch.from_numpy(labels).to(dev),
                                   torch.from_numpy(n).to(dev), ref, mode)
    bo, lo, no = bo.cpu().numpy(), lo.cpu().numpy(), no.cpu().numpy()
    for b in range(B):
        rb, rl = oa.process_boxes(boxes[b], labels[b], n[b], ref[b], mode[b, 0])
        assert no[b] == len(rb)
        np.testing.assert_array_equal(bo[b, :no[b]], rb)
        np.testing.assert_array_equal(lo[b, :no[b]], rl)
        assert (bo[b, no[b]:] == 0).all() and (lo[b, no[b]:] == 0).all()


def test_train_augmenter_end_to_end(dev):
    """TrainAugmenter (process_raw_data_train) = the oracle chain on its own sampled parameters;
    the result feeds the anchor matcher as the reference's pipeline does."""
    from rod.data import synthetic_boxes
    rng = np.random.default_rng(5)
    B, H, W = 4, 72, 128
    src = rng.integers(0, 256, (B, H, W, 3)).astype(np.uint8)
    corner, labels, n = synthetic_boxes(B, seed=3)
    aug = dpt.TrainAugmenter((64, 96), seed=9)
    img, bo, lo, no = aug(torch.from_numpy(src).to(dev), corner, labels, n)
    crop, ref, mode, col = aug.last_params
    np.testing.assert_allclose(img.cpu().numpy(), _oracle(src, crop, mode, col, 64, 96, False), rtol=0, atol=1e-3)
    for b in range(B):
        rb, rl = oa.process_boxes(corner[b], labels[b], n[b], ref[b], mode[b, 0])
        np.testing.assert_array_equal(bo[b, :len(rb)].cpu().numpy(), rb)
        np.testing.assert_array_equal(lo[b, :len(rb)].cpu().numpy(), rl)
    # normalised bf16 network input from the same parameters
    x, _, _, _ = aug(torch.from_numpy(src).to(dev), corner, labels, n, dtype=torch.bfloat16, params=aug.last_params)
    ref_x = torch.from_numpy(_oracle(src, crop, mode, col, 64, 96, True)).bfloat16()
    assert (x.float().cpu() - ref_x.float()).abs().max().item() <= 2 ** -7


def test_prepare_data_test_and_flip(dev):
    rng = np.random.default_rng(6)
    src = rng.integers(0, 256, (3, 40, 60, 3)).astype(np.uint8)
    t = torch.from_numpy(src).to(dev)
    out = dpt.prepare_data_test(t, (30, 50)).cpu().numpy()
    np.testing.assert_array_equal(out, np.stack([oa.resize_bilinear_legacy(s, 30, 50) for s in src]))
    np.testing.assert_array_equal(tf_image.resize_image(t, (30, 50)).cpu().numpy(), out)
    boxes = np.array([[[0.1, 0.2, 0.5, 0.7]]] * 3, np.float32)
    img, bo, flips = tf_image.random_flip_left_right(np.random.default_rng(1), t, boxes)
    for b in range(3):
        exp = src[b, :, ::-1] if flips[b] else src[b]
        np.testing.assert_array_equal(img[b].cpu().numpy(), exp.astype(np.float32))
        eb = [0.1, 1 - np.float32(0.7), 0.5, 1 - np.float32(0.2)] if flips[b] else boxes[b, 0]
        np.testing.assert_array_equal(bo[b, 0].cpu().numpy(), np.asarray(eb, np.float32))


def test_augmented_source_trains(dev):
    """The CLI's training source: augmented batches through one Trainer step."""
    from rod.dataio import AugmentedSource
    from rod.trainer import Trainer
    H, W, B = 96, 160, 2
    src = AugmentedSource(B, (H, W), dev, torch.bfloat16, seed=4, n_distinct=1, raw_hw=(120, 200))
    tr = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=1)
    x, bo, lo, no = next(src)
    assert x.dtype == torch.bfloat16 and x.shape == (B, H, W, 3)
    assert float(x.float().abs().max()) < 1.5
    loss = tr.step(x, bo, lo, no)[0]
    assert np.isfinite(loss.item())
