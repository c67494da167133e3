"""Synthetic BDD100K-shaped batches — there is no dataset on the box.

Images: uint8 [B, H, W, 3] i.i.d. U{0..255}; GT per image: G ~ U{1..40} boxes padded
to Gmax=64, centres U(0.05, 0.95), h, w log-uniform in [0.01, 0.6], corners clipped to
[0, 1]; labels uniform over the 7 classes the BDD converter keeps {1,2,3,4,6,8,10}
(reference convert/json2xml/parseJson.py:8-10, dataset/bdd100k.py:23-35).
"""
import numpy as np
import torch

BDD_LABELS = np.array([1, 2, 3, 4, 6, 8, 10], np.int32)
SEED = 20261015
# bench.py's training step starts from Trainer(seed=C2_WEIGHT_SEED) on synthetic_batch(seed=
# C2_BATCH_SEED (+ rank)); tests/test_gpu_fullsize.py checks that very first step (fp32 and
# bf16) against the float64 oracle, so bench.py's "loss_first_step" is a pinned number
C2_WEIGHT_SEED = 21
C2_BATCH_SEED = 22


def synthetic_boxes(B, gmax=64, gmin=1, gmax_draw=40, seed=SEED):
    rng = np.random.default_rng(seed)
    n = rng.integers(gmin, gmax_draw + 1, size=B).astype(np.int32)
    corner = np.zeros((B, gmax, 4), np.float32)
    labels = np.zeros((B, gmax), np.int32)
    for b in range(B):
        k = 0
        while k < n[b]:
            cy, cx = rng.uniform(0.05, 0.95, 2)
            h, w = np.exp(rng.uniform(np.log(0.01), np.log(0.6), 2))
            box = np.clip([cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2], 0, 1)
            if box[2] - box[0] <= 1e-4 or box[3] - box[1] <= 1e-4:
                continue  # degenerate boxes rejected
            corner[b, k] = box
            labels[b, k] = rng.choice(BDD_LABELS)
            k += 1
    return corner, labels, n


def synthetic_batch(B, H, W, device, seed=SEED):
    g = torch.Generator(device='cpu').manual_seed(seed)
    img = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, generator=g)
    corner, labels, n = synthetic_boxes(B, seed=seed)
    return (img.to(device), torch.from_numpy(corner).to(device), torch.from_numpy(labels).to(device),
            torch.from_numpy(n).to(device))


def detector_like_scores(predictor, probe, rate=0.02, iters=14):
    """Make a randomly initialised Predictor (predict.py) produce a detector-like score
    distribution: BatchNorm moving statistics calibrated on `probe` (uint8 batch), then the
    background logit of the clf heads shifted until about `rate` of the class scores pass
    the selection threshold (bench / tests: NMS then has real work).  Returns the
    fraction reached on the probe."""
    import config
    from rod.dataio import network_input
    net = predictor.net
    net.calibrate_batchnorm(network_input(probe, predictor.dtype))
    betas = [net.store.params['clf/block_%d/BatchNorm_3/beta' % (i + 1)] for i in range(6)]
    thr = predictor.kw['select_threshold']
    keep = predictor.keep_intermediates
    predictor.keep_intermediates = True

    def frac(shift):
        with torch.no_grad():
            for b in betas:
                b.data[0::config.total_obj_n] = shift
        predictor(probe)
        return float((predictor.last[1][..., 1:] >= thr).float().mean())
    lo, hi = -8.0, 8.0
    for _ in range(iters):
        mid = 0.5 * (lo + hi)
        if frac(mid) > rate:
            lo = mid
        else:
            hi = mid
    f = frac(hi)
    predictor.keep_intermediates = keep
    return f
