"""ORACLE (test infrastructure only): the deterministic part of the training data pipeline
(SURVEY §8 row A17), numpy float32 per operation:

  crop (tf.slice)                 utils/augmentation/process.py:117-127
  resize_image (legacy bilinear)  utils/augmentation/tf_image.py:266-278 -> TF ResizeBilinear,
                                  align_corners=False (LegacyScaler: src = dst * in/out)
  random_flip_left_right          utils/augmentation/tf_image.py:281-305 (image + boxes)
  distort_color, fast_mode=False  utils/augmentation/process.py:27-80 (4 orderings; hue disabled)
  bboxes_resize                   utils/tf_extended/bboxes.py:139-163
  bboxes_filter_overlap(0.3)      utils/tf_extended/bboxes.py:408-428 + 482-508 (safe_divide)
  clip to [0, 1]                  utils/data_pileline_tools.py:106-107
  (2/255) x - 1                   train.py:126

The colour ops live in TensorFlow 1.x (absent here, as is every TF op the reference calls):
adjust_brightness = x + delta; adjust_saturation = TF's AdjustSaturationOp CPU kernel
(rgb_to_hsv / hsv_to_rgb in float, the 2/6 and 4/6 hue offsets added as double literals);
adjust_contrast = (x - mean) * factor + mean with the per-image channel mean.  These are
restated from TF's published kernels; the reference holds no fixtures for them, so their
parity is UNPINNED against TF itself (the kernel is checked against this restatement).
Sampling (crop window, flip coin, colour order and magnitudes) is random in the reference and
parity-free; the sampler's constraints are checked as properties in the tests."""
import numpy as np

f32 = np.float32


def _lerp_axis(n_out, n_in):
    scale = f32(n_in) / f32(n_out)
    src = np.arange(n_out, dtype=f32) * scale
    fl = np.floor(src)
    lo = np.maximum(fl.astype(np.int64), 0)
    hi = np.minimum(np.ceil(src).astype(np.int64), n_in - 1)
    return lo, hi, (src - fl).astype(f32)


def resize_bilinear_legacy(img, Ho, Wo):
    """[H, W, C] (any dtype) -> float32 [Ho, Wo, C]; compute_lerp order of resize_bilinear_op.cc."""
    x = np.asarray(img).astype(f32)
    H, W = x.shape[:2]
    y0, y1, fy = _lerp_axis(Ho, H)
    x0, x1, fx = _lerp_axis(Wo, W)
    tl, tr = x[y0][:, x0], x[y0][:, x1]
    bl, br = x[y1][:, x0], x[y1][:, x1]
    fx = fx[None, :, None]
    fy = fy[:, None, None]
    top = tl + (tr - tl) * fx
    bot = bl + (br - bl) * fx
    return (top + (bot - top) * fy).astype(f32)


def adjust_saturation(rgb, scale):
    """TF AdjustSaturationOp (CPU) per pixel, float32; rgb [..., 3]."""
    with np.errstate(divide='ignore', invalid='ignore'):
        r, g, b = (rgb[..., i].astype(f32) for i in range(3))
        vv = np.maximum(r, np.maximum(g, b))
        rng = (vv - np.minimum(r, np.minimum(g, b))).astype(f32)
        s = np.where(vv > 0, rng / vv, f32(0)).astype(f32)
        norm = (f32(1) / (f32(6) * rng)).astype(f32)
        h_r = (norm * (g - b)).astype(f32)
        h_g = ((norm * (b - r)).astype(np.float64) + 2.0 / 6.0).astype(f32)
        h_b = ((norm * (r - g)).astype(np.float64) + 4.0 / 6.0).astype(f32)
        h = np.where(r == vv, h_r, np.where(g == vv, h_g, h_b)).astype(f32)
        h = np.where(rng <= 0, f32(0), h)
        h = np.where(h < 0, h + f32(1), h).astype(f32)
        s = np.minimum(f32(1), np.maximum(f32(0), (s * f32(scale)).astype(f32)))
        c = (s * vv).astype(f32)
        m = (vv - c).astype(f32)
        dh = (h * f32(6)).astype(f32)
        cat = dh.astype(np.int32)
        fm = dh.copy()
        for _ in range(4):
            fm = np.where(fm <= 0, fm + f32(2), fm).astype(f32)
        for _ in range(4):
            fm = np.where(fm >= 2, fm - f32(2), fm).astype(f32)
        x = (c * (f32(1) - np.abs(fm - f32(1)))).astype(f32)
        z = np.zeros_like(c)
        table = {0: (c, x, z), 1: (x, c, z), 2: (z, c, x), 3: (z, x, c), 4: (x, z, c), 5: (c, z, x)}
        out = [z.copy(), z.copy(), z.copy()]
        for k, trip in table.items():
            sel = cat == k
            for i in range(3):
                out[i] = np.where(sel, trip[i], out[i])
        return np.stack([(o + m).astype(f32) for o in out], -1)


def adjust_contrast(img, factor):
    """(x - mean) * factor + mean, mean per channel over H, W (float64 sum, rounded once)."""
    mean = (img.astype(np.float64).reshape(-1, img.shape[-1]).sum(0) / (img.shape[0] * img.shape[1])).astype(f32)
    return ((img - mean) * f32(factor) + mean).astype(f32)


ORDERINGS = {0: 'BSC', 1: 'SBC', 2: 'CBS', 3: 'SCB'}   # process.py:59-77


def distort_color(img, ordering, delta, sat, con):
    for op in ORDERINGS[ordering]:
        if op == 'B':
            img = (img + f32(delta)).astype(f32)
        elif op == 'S':
            img = adjust_saturation(img, sat)
        else:
            img = adjust_contrast(img, con)
    return img


def process_image(src, crop, flip, ordering, colour, Ho, Wo, normalize):
    """One image of process_raw_data_train; src uint8 [H, W, 3]; crop (y0, x0, h, w)."""
    y0, x0, h, w = (int(v) for v in crop)
    img = resize_bilinear_legacy(src[y0:y0 + h, x0:x0 + w], Ho, Wo)
    if flip:
        img = img[:, ::-1]
    if ordering >= 0:
        img = distort_color(img, ordering, *colour)
    if normalize:
        img = (f32(2.0 / 255.0) * img - f32(1)).astype(f32)
    return np.ascontiguousarray(img)


def process_boxes(boxes, labels, n, ref, flip, threshold=0.3):
    """bboxes_resize -> bboxes_filter_overlap -> flip -> clip for one image's first n boxes."""
    b = np.asarray(boxes[:n], f32)
    r = np.asarray(ref, f32)
    v = np.array([r[0], r[1], r[0], r[1]], f32)
    s = np.array([r[2] - r[0], r[3] - r[1], r[2] - r[0], r[3] - r[1]], f32)
    b = ((b - v) / s).astype(f32)
    iy0, ix0 = np.maximum(b[:, 0], f32(0)), np.maximum(b[:, 1], f32(0))
    iy1, ix1 = np.minimum(b[:, 2], f32(1)), np.minimum(b[:, 3], f32(1))
    hh = np.maximum(iy1 - iy0, f32(0))
    ww = np.maximum(ix1 - ix0, f32(0))
    inter = (hh * ww).astype(f32)
    vol = ((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])).astype(f32)
    with np.errstate(divide='ignore', invalid='ignore'):
        score = np.where(vol > 0, inter / vol, f32(0)).astype(f32)
    keep = score > f32(threshold)
    b, lab = b[keep], np.asarray(labels[:n])[keep]
    if flip:
        b = np.stack([b[:, 0], f32(1) - b[:, 3], b[:, 2], f32(1) - b[:, 1]], -1).astype(f32)
    b = np.minimum(np.maximum(b, f32(0)), f32(1)).astype(f32)
    return b, lab
