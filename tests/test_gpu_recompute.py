"""The expanded tensor of an inverted-residual block recomputed instead of read (ABI 23; ref
conv_blocks.py:263-270 expand -> 238-247 depthwise, mobilenet.py:417-420 BatchNorm).

y = bf16(x_act . W^T) is what the expand conv's forward (rod_conv_fwd, the streaming 1x1 kernel)
stores.  The recompute forms re-form it per tile from the narrow block input with the same MFMA and
rounding, so every output must be bit-identical to the form that reads the stored y:
  * rod_pw_bwd_rc vs rod_pw_bwd (the 24 -> 144 expands, plain input; 16 -> 96 with a prologue),
  * rod_pw_bwd_gred_rc vs rod_pw_bwd_gred (block 1's 16 -> 96 expand whose input is block 0's
    project output: linear input BatchNorm, its backward sums handed over),
  * rod_dw3x3_fwd_rc vs rod_dw3x3_fwd over the stored tensor with the BN_e + ReLU6 prologue: y and
    the BatchNorm statistics parts (stride 2 and 1, both pack widths of the tile plan),
  * rod_dw3x3_bwd_fused_rc vs rod_dw3x3_bwd_fused (stride 2): dx, dw and the BN_e backward parts,
  * a REFINE training step with the recompute on / off (ROD_DISABLE=rc), eager and graphed."""
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu
bf16 = torch.bfloat16


def _bn(C, g, dev, mag=1.0):
    return ((torch.randn(C, generator=g) * 0.2 * mag).to(dev), (torch.rand(C, generator=g) + 0.5).to(dev),
            (torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.2).to(dev))


def _forward_y(x, w, xpro, M, Cin, Cout):
    """The stored expand output: rod_conv_fwd exactly as _ConvBN.forward runs it."""
    wt0 = ops._prep(w, 0, bf16, Cout, Cin, 1)
    y = torch.empty((1, 1, M, Cout), dtype=bf16, device=x.device)
    ops.conv_fwd_raw(x.view(1, 1, M, Cin), wt0, None, y, 1, 1, M, Cin, Cout, 1, None, xpro)
    return y.view(M, Cout), wt0


# (M, Cin, Cout, input prologue act or None): the step's streaming expand shapes (720p b8 has
# 7,372,800 rows for 16 -> 96 and 1,843,200 for 24 -> 144) at sizes the streaming forward takes
# (M >= 65536), ragged tails, and a tile-sized case
RC_SHAPES = [(70001, 24, 144, None), (131072, 24, 144, ops.ROD_ACT_RELU6), (65536 + 17, 16, 96, ops.ROD_ACT_NONE),
             (100003, 16, 96, ops.ROD_ACT_RELU6), (65600, 16, 96, None)]


# (M, Cin, Cout, input prologue act or None): every N-group width of the statistics-only forward
# (Cout 32 / 48 / 64 / 96 / 144 / 192: 2 / 3 / 4 / 6 / 9 / 12 MFMA tiles; 12, and 9 with a
# prologue, take MODE 3 of the streaming kernel), tails of 1, 5 and 127 rows, both prologue forms
STATS_SHAPES = [(65536 + 1, 16, 96, ops.ROD_ACT_NONE), (65536 * 2 + 5, 24, 144, None), (70000 + 127, 32, 192, None),
                (65536 + 40, 16, 32, ops.ROD_ACT_RELU6), (65536 * 3, 24, 48, ops.ROD_ACT_NONE), (99999, 32, 64, None),
                (65536 + 3, 24, 144, ops.ROD_ACT_RELU6), (7372800 // 8, 16, 96, ops.ROD_ACT_NONE)]


@pytest.mark.parametrize('M,Cin,Cout,xact', STATS_SHAPES)
def test_conv_fwd_stats_bit_identical(dev, M, Cin, Cout, xact):
    """rod_conv_fwd_stats (the expand's statistics with its output never written) against the
    statistics parts the storing forward (rod_conv_fwd) writes beside y: bit-identical."""
    g = torch.Generator().manual_seed(M + Cin + Cout)
    x = (torch.randn(M, Cin, generator=g) * 1.5).to(dev, bf16)
    w = (torch.randn(Cout, 1, 1, Cin, generator=g) * 0.3).to(dev)
    xpro = None if xact is None else (*_bn(Cin, g, dev), xact)
    code = ops.dtcode(x)
    assert _abi.lib().rod_conv_fwd_stats_supported(M, Cin, Cout, code)
    wt0 = ops._prep(w, 0, bf16, Cout, Cin, 1)
    nparts = -(-M // 128)
    p0 = torch.full((nparts, 3, Cout), -7.0, device=dev)
    p1 = torch.full((nparts, 3, Cout), -9.0, device=dev)
    y = torch.empty((1, 1, M, Cout), dtype=bf16, device=dev)
    ops.conv_fwd_raw(x.view(1, 1, M, Cin), wt0, None, y, 1, 1, M, Cin, Cout, 1, p0, xpro)
    _abi.call('rod_conv_fwd_stats', x, *ops._pro_args(xpro), wt0, p1, M, Cin, Cout, code, ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(p0, p1)


@pytest.mark.parametrize('M,Cin,Cout,xact', RC_SHAPES)
def test_pw_bwd_rc_bit_identical(dev, M, Cin, Cout, xact):
    assert _abi.lib().rod_pw_bwd_rc_supported(M, Cin, Cout, ops.dtcode(torch.empty(1, dtype=bf16)))
    g = torch.Generator().manual_seed(M + 3 * Cin + Cout)
    x = (torch.randn(M, Cin, generator=g) * 1.3 + 0.2).to(dev, bf16)
    w = (torch.randn(Cout, 1, 1, Cin, generator=g) * 0.25).to(dev)
    xpro = None
    if xact is not None:
        xm, xr, xg, xb = _bn(Cin, g, dev)
        xpro = (xm, xr, xg, xb, xact)
    y, wt0 = _forward_y(x, w, xpro, M, Cin, Cout)
    dz = torch.randn(M, Cout, generator=g).to(dev, bf16)
    mean = y.float().mean(0)
    rstd = torch.rsqrt(y.float().var(0, unbiased=False) + 1e-3)
    gamma = (torch.rand(Cout, generator=g) + 0.5).to(dev)
    beta = (torch.randn(Cout, generator=g) * 0.3).to(dev)
    act = ops.ROD_ACT_RELU6
    coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)
    wt1 = ops._prep(w, 1, bf16, Cout, Cin, 1)
    outs = []
    for rc in (False, True):
        dw = torch.zeros(Cout, Cin, device=dev)
        dx = ops.pw_bwd(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, True, dw, None,
                        wt0=wt0 if rc else None)
        outs.append((dx, dw))
    torch.cuda.synchronize()
    (dx0, dw0), (dx1, dw1) = outs
    assert torch.equal(dx0, dx1), float((dx0.float() - dx1.float()).abs().max())
    assert torch.equal(dw0, dw1), float((dw0 - dw1).abs().max())


@pytest.mark.parametrize('M', [65536 + 17, 262144 + 5])
def test_pw_bwd_gred_rc_bit_identical(dev, M):
    Cin, Cout = 16, 96
    g = torch.Generator().manual_seed(M)
    x = (torch.randn(M, Cin, generator=g) * 2.0 - 0.4).to(dev, bf16)
    w = (torch.randn(Cout, 1, 1, Cin, generator=g) * 0.25).to(dev)
    xm, xr, xg, xb = _bn(Cin, g, dev)
    xpro = (xm, xr, xg, xb, ops.ROD_ACT_NONE)     # block 0's linear project BatchNorm
    y, wt0 = _forward_y(x, w, xpro, M, Cin, Cout)
    dz = torch.randn(M, Cout, generator=g).to(dev, bf16)
    mean = y.float().mean(0)
    rstd = torch.rsqrt(y.float().var(0, unbiased=False) + 1e-3)
    gamma = (torch.rand(Cout, generator=g) + 0.5).to(dev)
    beta = (torch.randn(Cout, generator=g) * 0.3).to(dev)
    act = ops.ROD_ACT_RELU6
    coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)
    wt1 = ops._prep(w, 1, bf16, Cout, Cin, 1)
    outs = []
    for rc in (False, True):
        dw = torch.zeros(Cout, Cin, device=dev)
        dx, parts = ops.pw_bwd_gred(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, dw,
                                    wt0=wt0 if rc else None)
        outs.append((dx, dw, parts))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b), float((a.float() - b.float()).abs().max())


@pytest.mark.parametrize('graphed', [False, True])
def test_step_recompute_bit_identical(dev, graphed):
    """REFINE step at 480x864 b2 with every recompute form off (ROD_DISABLE=rc: the expanded
    tensors written and read) and with the defaults (blocks 1 and 3: the expand output never written
    — rod_conv_fwd_stats, rod_dw3x3_fwd_rc, rod_dw3x3_bwd_fused_rc, rod_pw_bwd(_gred)_rc; block 1's
    16 -> 96 backward recompute elsewhere too): losses and parameters bit-identical, eager and
    graphed, and the recompute entries ran."""
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    runs = []
    names = ['rod_pw_bwd_rc', 'rod_pw_bwd_gred_rc', 'rod_dw3x3_fwd_rc', 'rod_dw3x3_bwd_fused_rc', 'rod_conv_fwd_stats',
             'rod_pw_bwd', 'rod_pw_bwd_gred', 'rod_dw3x3_fwd']
    for off in (True, False):
        if off:
            ops._DISABLE.add('rc')
        try:
            tr = Trainer((480, 864), 2, dtype=bf16, device=dev, seed=7)
            batches = [synthetic_batch(2, 480, 864, dev, seed=50 + i) for i in range(2)]
            step = tr.step_graphed if graphed else tr.step
            _abi.PROBE.arm(names)
            losses = [step(*batches[i % 2])[0].detach().clone() for i in range(3)]
            torch.cuda.synchronize()
            calls = _abi.PROBE.table()
            _abi.PROBE.disarm()
            runs.append((tr.net.store.flat.detach().clone(), torch.stack([l.reshape(()) for l in losses]), calls))
        finally:
            ops._DISABLE.discard('rc')
    (f0, l0, c0), (f1, l1, c1) = runs
    assert not any(n in c0 for n in names[:5]), c0
    for n in ('rod_pw_bwd_gred_rc', 'rod_pw_bwd_rc', 'rod_dw3x3_fwd_rc', 'rod_dw3x3_bwd_fused_rc', 'rod_conv_fwd_stats'):
        assert c1.get(n, (0,))[0] >= 1, (n, c1)
    n_eager = 3 if not graphed else 1    # the probe does not see captured calls or replays
    assert c1['rod_conv_fwd_stats'][0] == 2 * n_eager and c1['rod_dw3x3_bwd_fused_rc'][0] == 2 * n_eager, c1
    assert torch.equal(l0, l1), (l0, l1)
    assert torch.equal(f0, f1)


def test_nostore_step_opt_in_dw_recompute(dev):
    """The opt-in recompute of the stride-1 depthwise forwards (ROD_ENABLE=rcdw) on top of the
    defaults: bit-identical step."""
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    runs = []
    for on in (False, True):
        if on:
            ops._ENABLE.add('rcdw')
        try:
            tr = Trainer((480, 864), 2, dtype=bf16, device=dev, seed=8)
            b = synthetic_batch(2, 480, 864, dev, seed=77)
            losses = [tr.step(*b)[0].detach().clone() for _ in range(2)]
            torch.cuda.synchronize()
            runs.append((tr.net.store.flat.detach().clone(), torch.stack([l.reshape(()) for l in losses])))
        finally:
            ops._ENABLE.discard('rcdw')
    assert torch.equal(runs[0][1], runs[1][1])
    assert torch.equal(runs[0][0], runs[1][0])


@pytest.mark.parametrize('graphed', [False, True])
def test_predict_expand_recompute_bit_identical(dev, graphed):
    """Inference (predict.py path, ALL network, 480x864 b2): the blocks with a 16- / 24- / 32-channel
    input (blocks 1-6, strides 1 and 2) leave their expand output unwritten and the depthwise
    forward recomputes it (ops.rc_eval_ok / _nostore_eval_ok); against ROD_DISABLE=rcinf (written
    and read) the head outputs and the detections are bit-identical (the fused block kernel off in
    both: its single rounding differs from the chain's), and rod_dw3x3_fwd_rc ran once per block."""
    import predict
    from rod.data import synthetic_batch
    img = synthetic_batch(2, 480, 864, dev, seed=61)[0]
    runs = []
    for off in (True, False):
        if off:
            ops._DISABLE.add('rcinf')
        ops._DISABLE.add('irblock')
        try:
            pr = predict.Predictor((480, 864), dev, bf16, seed=60)
            pr.keep_intermediates = not graphed
            _abi.PROBE.arm(['rod_dw3x3_fwd_rc', 'rod_ir_block_fwd'])
            scores, boxes = pr(img)
            if graphed:
                scores, boxes = pr(img)   # a replay of the captured graph
            torch.cuda.synchronize()
            calls = _abi.PROBE.table()
            _abi.PROBE.disarm()
            inter = [t.clone() for t in pr.last] if not graphed else []
            runs.append((inter, torch.stack([scores[c] for c in sorted(scores)]),
                         torch.stack([boxes[c] for c in sorted(boxes)]), calls))
        finally:
            ops._DISABLE.discard('rcinf')
            ops._DISABLE.discard('irblock')
    (i0, s0, b0, c0), (i1, s1, b1, c1) = runs
    assert 'rod_dw3x3_fwd_rc' not in c0, c0
    assert c1.get('rod_dw3x3_fwd_rc', (0,))[0] == 6, c1
    assert 'rod_ir_block_fwd' not in c0 and 'rod_ir_block_fwd' not in c1
    for a, b in zip(i0, i1):
        assert torch.equal(a, b)
    assert torch.equal(s0, s1) and torch.equal(b0, b1)


# (N, H, W, Cin, C, stride, input prologue act or None): block 1 (720p, 16 -> 96, stride 2, the
# 16-byte pack plan) on 2 images, block 3 / block 2 shapes (24 -> 144 at 360x640, strides 2 / 1),
# small maps on the 8-byte pack plan with odd sizes (TF-SAME pads 1 / 0), Cin 32
DW_SHAPES = [(2, 720, 1280, 16, 96, 2, ops.ROD_ACT_NONE), (8, 360, 640, 24, 144, 2, None),
             (5, 360, 640, 24, 144, 1, None), (2, 99, 171, 16, 96, 2, ops.ROD_ACT_RELU6),
             (3, 57, 83, 24, 144, 1, ops.ROD_ACT_NONE), (2, 64, 96, 32, 192, 1, None), (1, 37, 45, 32, 192, 2, None)]


@pytest.mark.parametrize('N,H,W,Cin,C,stride,xact', DW_SHAPES)
def test_dw3x3_fwd_rc_bit_identical(dev, N, H, W, Cin, C, stride, xact):
    code = ops.dtcode(torch.empty(1, dtype=bf16))
    assert _abi.lib().rod_dw3x3_fwd_rc_supported(N, H, W, C, Cin, stride, code)
    g = torch.Generator().manual_seed(N * H + W + C + stride)
    M = N * H * W
    x = (torch.randn(N, H, W, Cin, generator=g) * 1.4 + 0.1).to(dev, bf16)
    w_e = (torch.randn(C, 1, 1, Cin, generator=g) * 0.3).to(dev)
    xpro = None
    if xact is not None:
        xm, xr, xg, xb = _bn(Cin, g, dev)
        xpro = (xm, xr, xg, xb, xact)
    ye, wt0 = _forward_y(x.view(M, Cin), w_e, xpro, M, Cin, C)
    ye = ye.view(N, H, W, C)
    em = ye.float().mean((0, 1, 2)) + (torch.randn(C, generator=g) * 0.05).to(dev)
    er = torch.rsqrt(ye.float().var((0, 1, 2), unbiased=False) + 1e-3)
    eg, eb = (torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.5 + 0.5).to(dev)
    epro = (em, er, eg, eb, ops.ROD_ACT_RELU6)
    wd = (torch.randn(3, 3, C, generator=g) * 0.3).to(dev)
    Ho, pt = ops.same_pad(H, stride)
    Wo, pl = ops.same_pad(W, stride)
    nparts = _abi.lib().rod_dw3x3_fwd_stat_parts(N, Ho, Wo, C, stride, code)
    outs = []
    for rc in (False, True):
        y = torch.empty((N, Ho, Wo, C), dtype=bf16, device=dev)
        parts = torch.full((nparts, 3, C), -7.0, device=dev)
        if rc:
            _abi.call('rod_dw3x3_fwd_rc', x, *ops._pro_args(xpro), wt0, Cin, *ops._pro_args(epro), wd, y, parts, N, H,
                      W, C, stride, pt, pl, Ho, Wo, code, ops.stream())
        else:
            _abi.call('rod_dw3x3_fwd', ye, *ops._pro_args(epro), wd, y, parts, N, H, W, C, stride, pt, pl, Ho, Wo, code,
                      ops.stream())
        outs.append((y, parts))
    torch.cuda.synchronize()
    (y0, p0), (y1, p1) = outs
    assert torch.equal(y0, y1), float((y0.float() - y1.float()).abs().max())
    assert torch.equal(p0, p1), float((p0 - p1).abs().max())


def _fused_bwd_inputs(N, H, W, Cin, C, xact, g, dev):
    M = N * H * W
    x = (torch.randn(N, H, W, Cin, generator=g) * 1.4 + 0.1).to(dev, bf16)
    w_e = (torch.randn(C, 1, 1, Cin, generator=g) * 0.3).to(dev)
    xpro = None
    if xact is not None:
        xm, xr, xg, xb = _bn(Cin, g, dev)
        xpro = (xm, xr, xg, xb, xact)
    ye, wt0 = _forward_y(x.view(M, Cin), w_e, xpro, M, Cin, C)
    ye = ye.view(N, H, W, C)
    em = ye.float().mean((0, 1, 2)) + (torch.randn(C, generator=g) * 0.05).to(dev)
    er = torch.rsqrt(ye.float().var((0, 1, 2), unbiased=False) + 1e-3)
    epro = (em, er, (torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.5 + 0.5).to(dev),
            ops.ROD_ACT_RELU6)
    return x, xpro, wt0, ye, epro


# (N, H, W, Cin, C, input prologue act): block 1 at 720p on 2 images, block 3 (24 -> 144 at
# 360x640), odd sizes (TF-SAME pads 1 / 0), Cin 32
BWD_SHAPES = [(2, 720, 1280, 16, 96, ops.ROD_ACT_NONE), (8, 360, 640, 24, 144, None), (2, 99, 171, 16, 96, None),
              (3, 58, 81, 24, 144, ops.ROD_ACT_NONE), (1, 45, 64, 32, 192, None)]


@pytest.mark.parametrize('N,H,W,Cin,C,xact', BWD_SHAPES)
def test_dw3x3_bwd_fused_rc_bit_identical(dev, N, H, W, Cin, C, xact):
    code = ops.dtcode(torch.empty(1, dtype=bf16))
    Ho, pt = ops.same_pad(H, 2)
    Wo, pl = ops.same_pad(W, 2)
    assert _abi.lib().rod_dw3x3_bwd_fused_rc_supported(N, H, W, C, Cin, 2, pt, pl, code)
    g = torch.Generator().manual_seed(N * H + W + C)
    x, xpro, wt0, ye, epro = _fused_bwd_inputs(N, H, W, Cin, C, xact, g, dev)
    wd = (torch.randn(3, 3, C, generator=g) * 0.3).to(dev)
    yd = torch.empty((N, Ho, Wo, C), dtype=bf16, device=dev)
    _abi.call('rod_dw3x3_fwd', ye, *ops._pro_args(epro), wd, yd, None, N, H, W, C, 2, pt, pl, Ho, Wo, code, ops.stream())
    dz = torch.randn(N, Ho, Wo, C, generator=g).to(dev, bf16)
    dm = yd.float().mean((0, 1, 2))
    dr = torch.rsqrt(yd.float().var((0, 1, 2), unbiased=False) + 1e-3)
    dgam, dbet = (torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.3).to(dev)
    coef = ops.bn_bwd_reduce(dz, yd, dm, dr, dgam, dbet, ops.ROD_ACT_RELU6, False, False)
    nparts = _abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, 2, pt, pl)
    wsb = _abi.query('rod_dw3x3_bwd_fused_workspace', N, H, W, C, 2, pt, pl)
    outs = []
    for rc in (False, True):
        dx = torch.empty_like(ye)
        dw = torch.zeros(3, 3, C, device=dev)
        gp = torch.full((nparts, 2, C), -7.0, device=dev)
        ws = ops.workspace(wsb, dev)
        if rc:
            _abi.call('rod_dw3x3_bwd_fused_rc', x, *ops._pro_args(xpro), wt0, Cin, *ops._pro_args(epro), dz, yd, dm, dr,
                      dgam, dbet, ops.ROD_ACT_RELU6, coef, wd, dx, dw, gp, ws, N, H, W, C, 2, pt, pl, Ho, Wo, code,
                      ops.stream())
        else:
            _abi.call('rod_dw3x3_bwd_fused', ye, *ops._pro_args(epro), dz, yd, dm, dr, dgam, dbet, ops.ROD_ACT_RELU6,
                      coef, wd, dx, dw, gp, ws, N, H, W, C, 2, pt, pl, Ho, Wo, code, ops.stream())
        outs.append((dx, dw, gp))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b), float((a.float() - b.float()).abs().max())
