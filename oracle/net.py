"""ORACLE (test infrastructure only): the detector network restated with PyTorch-CPU
fp32 ops (autograd gives the reference gradients).

Restates nets/backbone/mobilenet/mobilenet_v2.py:41-87 (spec), conv_blocks.py:163-312
(expanded_conv), mobilenet.py:417-420 (BN defaults), nets/catch_net.py:160-342 (deconv
pyramid, ADD merge, heads).  TF 'SAME' padding is applied explicitly (asymmetric for
stride 2 on even extents), BatchNorm in training mode normalises with the biased batch
variance and feeds the Bessel-corrected one to the moving average (FusedBatchNorm).
Parameters are taken by the same slim-style names the product uses; weights are
[Cout, kh, kw, Cin] (depthwise [3, 3, C], deconv [2, 2, f_c, i_c] as in TF).
"""
import math

import torch
import torch.nn.functional as F

# (kind, stride, cout, expansion, divisible_by) — mobilenet_v2.py:58-86
SPEC = [('conv', 1, 32, None, None), ('ir', 1, 16, 1, 1)] + \
    [('ir', s, c, 6, 8) for s, c in [(2, 24), (1, 24), (2, 32), (1, 32), (1, 32), (2, 64), (1, 64), (1, 64),
                                     (1, 64), (2, 96), (1, 96), (1, 96), (1, 96), (2, 160), (1, 160), (1, 160),
                                     (2, 320), (1, 320)]] + \
    [('ir', s, 256, 2, 8) for s in (2, 1, 2, 1)]
TAPS = [11, 15, 18, 20, 22, 24]  # config.py:30-31
N_ANCHOR = [6, 9, 9, 9, 9, 9]


# Storage-rounding emulation (test baseline only): with set_storage(torch.bfloat16) every tensor
# the product keeps in HBM — conv / depthwise outputs, BatchNorm + activation outputs, residual
# sums — is rounded to bf16 after fp32 arithmetic, and so is the gradient w.r.t. each of them in
# backward: "bf16 storage, fp32 arithmetic", the product's bf16 mode, as an independent
# PyTorch-CPU evaluation (the plain bf16 evaluation rounds every intermediate op as well).
_STORE = [None]


class _RoundST(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t, dt):
        return t.to(dt).to(t.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(_STORE[0]).to(g.dtype), None


def set_storage(dtype):
    """dtype (e.g. torch.bfloat16) or None (no rounding); returns the previous setting."""
    prev = _STORE[0]
    _STORE[0] = dtype
    return prev


def _st(t):
    return t if _STORE[0] is None else _RoundST.apply(t, _STORE[0])


def make_divisible(v, d, min_value=None):
    """conv_blocks.py:50-57."""
    min_value = d if min_value is None else min_value
    nv = max(min_value, int(v + d / 2) // d * d)
    return nv + d if nv < 0.9 * v else nv


def same_pad(size, stride, k):
    out = -(-size // stride)
    total = max((out - 1) * stride + k - size, 0)
    return total // 2, total - total // 2


def conv(x, w, b=None, stride=1):
    """slim.conv2d SAME on NCHW x with an [O, kh, kw, I] weight."""
    k = w.shape[1]
    pt, pb = same_pad(x.shape[2], stride, k)
    pl, pr = same_pad(x.shape[3], stride, k)
    x = F.pad(x, (pl, pr, pt, pb))
    return _st(F.conv2d(x, w.permute(0, 3, 1, 2), b, stride))


def dwconv(x, w, stride):
    """DepthwiseConv2dNative SAME, w [3, 3, C]."""
    C = x.shape[1]
    pt, pb = same_pad(x.shape[2], stride, 3)
    pl, pr = same_pad(x.shape[3], stride, 3)
    x = F.pad(x, (pl, pr, pt, pb))
    return _st(F.conv2d(x, w.permute(2, 0, 1)[:, None], None, stride, groups=C))


def batch_norm(x, gamma, beta, mm, mv, training, decay, eps=1e-3, moving=None, name=None):
    if training:
        mean = x.mean((0, 2, 3))
        var = x.var((0, 2, 3), unbiased=False)
        n = x.numel() // x.shape[1]
        if moving is not None:
            with torch.no_grad():
                moving[name + '/moving_mean'] = mm - (mm - mean) * (1 - decay)
                moving[name + '/moving_variance'] = mv - (mv - var * n / max(n - 1, 1)) * (1 - decay)
    else:
        mean, var = mm, mv
    sc = torch.rsqrt(var + eps)
    if gamma is not None:
        sc = sc * gamma
    y = (x - mean[None, :, None, None]) * sc[None, :, None, None]
    if beta is not None:
        y = y + beta[None, :, None, None]
    return y


def relu6(x):
    return torch.clamp(x, 0.0, 6.0)


def leaky(x):
    return torch.where(x > 0, x, 0.2 * x)


def layer_plan():
    plan, cin, n_ir = [], 3, 0
    for i, (kind, s, cout, exp, div) in enumerate(SPEC):
        if kind == 'conv':
            plan.append((i + 1, kind, s, cin, None, cout, False, 'Conv'))
        else:
            inner = make_divisible(cin * exp, div)
            sc = 'expanded_conv' if n_ir == 0 else 'expanded_conv_%d' % n_ir
            n_ir += 1
            plan.append((i + 1, kind, s, cin, inner, cout, s == 1 and cin == cout, sc))
        cin = cout
    return plan


def backbone(x, P, B, training, moving=None, scope='backbone/MobilenetV2'):
    """Returns the 24 endpoints (NCHW)."""
    eps = {}

    def bn(t, name, act):
        y = batch_norm(t, P[name + '/gamma'], P[name + '/beta'], B[name + '/moving_mean'],
                       B[name + '/moving_variance'], training, 0.997, 1e-3, moving, name)
        return _st(relu6(y) if act else y)

    for (idx, kind, s, cin, inner, cout, res, sc) in layer_plan():
        base = scope + '/' + sc
        if kind == 'conv':
            x = bn(conv(x, P[base + '/weights'], None, s), base + '/BatchNorm', True)
        else:
            inp = x
            if inner > cin:
                x = bn(conv(x, P[base + '/expand/weights']), base + '/expand/BatchNorm', True)
            x = bn(dwconv(x, P[base + '/depthwise/depthwise_weights'], s), base + '/depthwise/BatchNorm', True)
            x = bn(conv(x, P[base + '/project/weights']), base + '/project/BatchNorm', False)
            if res:
                x = _st(x + inp)
        eps['layer_%d' % idx] = x
    return eps


def head(feats, P, B, scope, k, training, moving=None):
    """__det_out / __clf_out (catch_net.py:276-342); returns NHWC [B, fh, fw, A, k]."""
    outs = []
    for i, x in enumerate(feats):
        base = '%s/block_%d' % (scope, i + 1)
        n = 0
        for ch in [128, k * N_ANCHOR[i]]:
            for ks in (1, 3):
                cn = base + ('/Conv' if n == 0 else '/Conv_%d' % n)
                bn_ = base + ('/BatchNorm' if n == 0 else '/BatchNorm_%d' % n)
                x = conv(x, P[cn + '/weights'], P[cn + '/biases'])
                x = _st(leaky(batch_norm(x, None, P[bn_ + '/beta'], B[bn_ + '/moving_mean'],
                                         B[bn_ + '/moving_variance'], training, 0.999, 1e-3, moving, bn_)))
                n += 1
        Bn, C, fh, fw = x.shape
        outs.append(x.permute(0, 2, 3, 1).reshape(Bn, fh, fw, N_ANCHOR[i], k))
    return outs


def resize_bilinear_legacy(x, size):
    """tf.image.resize_images(BILINEAR, align_corners=False), TF1 legacy scaling:
    src = dst * in/out, no half-pixel offset; NCHW."""
    H, W = x.shape[2], x.shape[3]
    Ho, Wo = size

    def axis(n_in, n_out):
        scale = n_in / n_out
        src = torch.arange(n_out, dtype=torch.float32) * torch.tensor(scale, dtype=torch.float32)
        lo = torch.floor(src).long()
        hi = torch.clamp(lo + 1, max=n_in - 1)
        return lo, hi, (src - lo.float())

    y0, y1, fy = axis(H, Ho)
    x0, x1, fx = axis(W, Wo)
    tl = x[:, :, y0][:, :, :, x0]
    tr = x[:, :, y0][:, :, :, x1]
    bl = x[:, :, y1][:, :, :, x0]
    br = x[:, :, y1][:, :, :, x1]
    fx_ = fx[None, None, None, :].to(x.device, x.dtype)
    fy_ = fy[None, None, :, None].to(x.device, x.dtype)
    top = tl + (tr - tl) * fx_
    bot = bl + (br - bl) * fx_
    return top + (bot - top) * fy_


def conv_transpose_2x2(x, w, out_hw):
    """tf.nn.conv2d_transpose(stride 2, SAME, kernel 2): out[2i+a, 2j+b, f] =
    sum_c x[i, j, c] w[a, b, f, c], cropped to out_hw (pad_before is always 0)."""
    Bn, C, H, W = x.shape
    f = w.shape[2]
    y = torch.einsum('nchw,abfc->nfhawb', x, w).reshape(Bn, f, 2 * H, 2 * W)
    return y[:, :, :out_hw[0], :out_hw[1]]


def deconv_bone(feats, P, B, training, moving=None, learn_all=False):
    """catch_net.py:160-230: LEARN_HALF (transpose conv to C/2 ++ 1x1 conv of the bilinear
    resize) or LEARN_ALL (transpose conv to C), each followed by BN(beta) + leaky."""
    layers = list(reversed(feats))
    out = []
    x = layers[0]
    for i in range(len(layers)):
        base = 'deconv/block_%d' % (i + 1)
        if i == 0:
            x = conv(x, P[base + '/Conv/weights'], P[base + '/Conv/biases'])
        elif learn_all:
            h, w = layers[i].shape[2], layers[i].shape[3]
            x = conv_transpose_2x2(x, P[base + '/weight_%d' % i], (h, w))
        else:
            h, w = layers[i].shape[2], layers[i].shape[3]
            up = conv_transpose_2x2(x, P[base + '/weight_%d' % i], (h, w))
            rh = conv(resize_bilinear_legacy(x, (h, w)), P[base + '/Conv/weights'], P[base + '/Conv/biases'])
            x = torch.cat([up, rh], 1)
        x = leaky(batch_norm(x, None, P[base + '/BatchNorm/beta'], B[base + '/BatchNorm/moving_mean'],
                             B[base + '/BatchNorm/moving_variance'], training, 0.999, 1e-3, moving,
                             base + '/BatchNorm'))
        out.append(x)
    return out


MSF_BLOCKS = [['layer_4', 'layer_7'], ['layer_7', 'layer_11']]
MSF_COMPRESS = [[4, 16], [3, 12]]


def space_to_depth(x, r):
    """tf.space_to_depth on NCHW: out channel (di*r + dj)*C + c."""
    Bn, C, H, W = x.shape
    return x.reshape(Bn, C, H // r, r, W // r, r).permute(0, 3, 5, 1, 2, 4).reshape(Bn, r * r * C, H // r, W // r)


def se_block(x, P, name):
    """attention_module.py:3-33 on NCHW."""
    sq = x.mean((2, 3))
    hid = torch.relu(sq @ P[name + '/bottleneck_fc/kernel'] + P[name + '/bottleneck_fc/bias'])
    e = torch.sigmoid(hid @ P[name + '/recover_fc/kernel'] + P[name + '/recover_fc/bias'])
    return x * e[:, :, None, None]


def feats_aug(ep, P, B, training, moving=None):
    """__feats_aug_block PREORDER_MSF (catch_net.py:115-152)."""
    feats, k = [], 0
    for index, t in enumerate(TAPS):
        s_feat = ep['layer_%d' % t]
        if index >= len(MSF_BLOCKS):
            feats.append(s_feat)
            continue
        aug = []
        for name in MSF_BLOCKS[index]:
            f = ep[name]
            h, w = f.shape[2], f.shape[3]
            rh, rw = round(h / s_feat.shape[2]), round(w / s_feat.shape[3])
            f = F.pad(f, (abs(w - rw * s_feat.shape[3]), 0, abs(h - rh * s_feat.shape[2]), 0))
            sfx = '' if k == 0 else '_%d' % k
            f = conv(f, P['backbone/Conv%s/weights' % sfx], P['backbone/Conv%s/biases' % sfx])
            bn = 'backbone/BatchNorm' + sfx
            f = leaky(batch_norm(f, None, P[bn + '/beta'], B[bn + '/moving_mean'], B[bn + '/moving_variance'],
                                 training, 0.999, 1e-3, moving, bn))
            if rh > 1:
                f = space_to_depth(f, rh)
            aug.append(f)
            k += 1
        feats.append(se_block(torch.cat(aug + [s_feat], 1), P, 'backbone/se_aug_layer_%d' % (index + 1)))
    return feats


def forward(img_nhwc, P, B, training, all_mode=False, moving=None, learn_all=False, concat=False, msf=False):
    """Full network on an NHWC fp32 input; returns refine_out (and det_out, clf_out).
    learn_all: deconv_method LEARN_ALL; concat: merge_method CONCAT (catch_net.py:237-273);
    msf: process_backbone_method PREORDER_MSF (catch_net.py:115-152)."""
    x = img_nhwc.permute(0, 3, 1, 2)
    ep = backbone(x, P, B, training, moving)
    feats = feats_aug(ep, P, B, training, moving) if msf else [ep['layer_%d' % t] for t in TAPS]
    refine = head(feats, P, B, 'refine', 4, training, moving)
    if not all_mode:
        return refine
    dec = deconv_bone(feats, P, B, training, moving, learn_all)
    if concat:
        merged = [torch.cat([u, d], 1) for u, d in zip(feats, reversed(dec))]
    else:
        merged = [u + d for u, d in zip(feats, reversed(dec))]
    clf = head(merged, P, B, 'clf', 11, training, moving)
    det = head(merged, P, B, 'det', 4, training, moving)
    return refine, det, clf
