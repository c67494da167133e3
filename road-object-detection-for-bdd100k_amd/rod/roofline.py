"""Algorithmic cost of one librod call (bytes that must cross HBM at minimum, and flops),
from the call's own arguments — the per-unit figures of SURVEY.md §8(d):

  dw3x3 fwd / bwd_data : es*(in + out) + 9*C*4 bytes, 18*N*Ho*Wo*C flops
  dw3x3 fwd_rc         : es*(x + out + We) + 9*C*4 (x the Cin-wide block input: the expanded input
                         is recomputed, ABI 23), 2*N*H*W*Cin*C + 18*N*Ho*Wo*C
  dw3x3 bwd_filter     : es*(x + dy) + 9*C*4, 18*N*Ho*Wo*C
  conv fwd (1x1 / 3x3) : es*(M*Cin + M*Cout + Cout*K) (+4*Cout bias), 2*M*K*Cout; the _bnact form
                         (inference BatchNorm epilogue) + es*M*Cout for a residual
  conv wgrad           : es*(M*Cin + M*Cout) + 4*Cout*K, 2*M*K*Cout
  bn_stats             : es*M*C;  bn_apply: es*M*C*(2 + residual)
  bn_bwd               : es*M*C*3 (read dy, read x, write dx)
  bn_bwd_reduce        : es*M*C*2 (read dz, read y: the first, algorithmic reads)
  bn_bwd_apply         : es*M*C*1 (write dy).  Its reads of dz and y are the SECOND pass of the
                         reduce -> apply split: design traffic, not algorithmic bytes, so the
                         BatchNorm backward as a whole counts 3 passes (read dz, read y, write
                         dy) whichever kernels do them; design_bytes() gives the 5 passes the
                         two-kernel design moves (reduce 2 + apply 3)
  dw3x3_bwd_fused      : es*(x + dx) + 2*9*C*4, 36*N*Ho*Wo*C + 8*N*Ho*Wo*C (+ 6*N*H*W*C with the
                         input BatchNorm's sums).  Its reads of dz and y are the BatchNorm
                         backward's SECOND pass (as for bn_bwd_apply): design traffic; dy is
                         never stored
  dw3x3_bwd_fused_rc   : es*(x + dx) with x the Cin-wide block input (ABI 23: ye recomputed),
                         flops + 2*N*H*W*Cin*C
  conv_fwd_stats       : es*(M*Cin + W) + the parts (ABI 23: y never written)
  dw3x3_bwd_fused_pw   : the same algorithmic bytes (ABI 20: dz is recomputed from the cout-wide dy_p;
                         its reads of yd and dy_p are design traffic), flops + 2*N*H*W*C*cout
  pw_bwd (fused 1x1)   : es*(2*M*Cout + M*Cin [+ M*Cin dx]) + W, 2*M*Cin*Cout per product;
                         the _rc forms (ABI 23) recompute y = x.W^T instead of reading it:
                         es*(M*Cout + M*Cin [+ M*Cin dx]) + 2W, + 2*M*Cin*Cout flops
  pw_bwd_gred (project): es*(2*M*Cout + 2*M*Cin) + W, 4*M*Cin*Cout + 10*M*Cout + 6*M*Cin (the
                         input BatchNorm's sums ride on the x it reads and the dx it writes);
                         the _dyp form writes the Cout-wide dy instead of dx: es*(3*M*Cout + M*Cin) + W
  match_anchors        : B*A*(16 + 16 + 16 + 4 + 4) + anchors, 15*G*A*B flops
  ir_block_fwd (fused) : es*(N*H*W*Cin + N*Ho*Wo*Cout) + weights, 2*N*H*W*Cin*inner +
                         18*N*Ho*Wo*inner + 2*N*Ho*Wo*inner*Cout
"""

_ES = {0: 4, 1: 2}

# Version of the per-call cost model above, carried in every bench / probe JSON.  Figures are
# comparable only within one version:
#   1 (rounds 1-2): rod_bn_bwd_apply 3 passes; rod_dw3x3_bwd_fused es*(ye + dz + yd + dx)
#   2 (round 3 on): rod_bn_bwd_apply 1 pass (write dy) and rod_dw3x3_bwd_fused es*(ye + dx) —
#     their reads of (dz, y) are the BatchNorm backward's second pass, reported as design bytes
COST_MODEL_VERSION = 2

MI355X_HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
MI355X_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (spec, no sparsity)
MI355X_F32_PEAK_TFLOPS = 157.3    # f32 MFMA / vector


def cost(name, a):
    """(bytes, flops) of the call rod_<name>(*a)."""
    # ABI 3: rod_dw3x3_fwd / _bwd_filter / rod_conv_fwd / _wgrad carry the five BatchNorm
    # prologue arguments after x (P = 5 positions); ABI 4: rod_conv_fwd (after stat_parts)
    # and rod_dw3x3_bwd_data (after dx) the seven gred arguments
    if name == "rod_augment_images":
        # written network input + one uint8 sample per output value read (the crop is resampled)
        B, Ho, Wo, dt = a[8], a[9], a[10], a[12]
        return (_ES[dt] + 1) * B * Ho * Wo * 3, 0
    if name == "rod_dw3x3_fwd":
        N, H, W, C, Ho, Wo, dt = a[9], a[10], a[11], a[12], a[16], a[17], a[18]
        es = _ES[dt]
        return es * (N * H * W * C + N * Ho * Wo * C) + 36 * C, 18 * N * Ho * Wo * C
    if name == "rod_dw3x3_fwd_rc":        # ABI 23: the expanded input recomputed from the block input
        N, H, W, C, Ho, Wo, dt, Cin = a[16], a[17], a[18], a[19], a[23], a[24], a[25], a[7]
        es = _ES[dt]
        return es * (N * H * W * Cin + N * Ho * Wo * C + C * Cin) + 36 * C, \
            2 * N * H * W * Cin * C + 18 * N * Ho * Wo * C
    if name == "rod_dw3x3_bwd_data":
        N, H, W, C, Ho, Wo, dt = a[10], a[11], a[12], a[13], a[17], a[18], a[19]
        es = _ES[dt]
        gred = es * N * H * W * C if a[9] is not None else 0   # the epilogue reads y
        return es * (N * H * W * C + N * Ho * Wo * C) + 36 * C + gred, 18 * N * Ho * Wo * C
    if name == "rod_dw3x3_bwd_filter":
        N, H, W, C, Ho, Wo, dt = a[9], a[10], a[11], a[12], a[16], a[17], a[18]
        es = _ES[dt]
        return es * (N * H * W * C + N * Ho * Wo * C) + 36 * C, 18 * N * Ho * Wo * C
    if name == "rod_dw3x3_bwd_fused":
        N, H, W, C, Ho, Wo, dt = a[19], a[20], a[21], a[22], a[26], a[27], a[28]
        es = _ES[dt]
        red = 6 * N * H * W * C if a[17] is not None else 0
        return es * 2 * N * H * W * C + 72 * C, 44 * N * Ho * Wo * C + red
    if name == "rod_dw3x3_bwd_fused_rc":   # ABI 23: the expanded input recomputed from x (Cin wide)
        Cin, N, H, W, C, Ho, Wo, dt = a[7], a[26], a[27], a[28], a[29], a[33], a[34], a[35]
        es = _ES[dt]
        return es * (N * H * W * Cin + N * H * W * C + C * Cin) + 72 * C, \
            44 * N * Ho * Wo * C + 6 * N * H * W * C + 2 * N * H * W * Cin * C
    if name == "rod_dw3x3_bwd_fused_pw":
        N, H, W, C, dt, cout = a[21], a[22], a[23], a[24], a[25], a[8]
        es = _ES[dt]
        red = 6 * N * H * W * C if a[19] is not None else 0
        return es * 2 * N * H * W * C + 72 * C, 44 * N * H * W * C + red + 2 * N * H * W * C * cout
    if name == "rod_conv_fwd":
        N, H, W, Cin, Cout, ks, dt = a[18], a[19], a[20], a[21], a[22], a[23], a[26]
        es = _ES[dt]
        M = N * H * W
        K = ks * ks * Cin
        gred = es * M * Cout if a[17] is not None else 0   # the gred epilogue reads y
        return es * (M * Cin + M * Cout + Cout * K) + (4 * Cout if a[7] is not None else 0) + gred, 2 * M * K * Cout
    if name == "rod_conv_fwd_stats":      # ABI 23: the statistics of y only, y never written
        M, Cin, Cout, dt = a[8], a[9], a[10], a[11]
        es = _ES[dt]
        return es * (M * Cin + Cout * Cin) + 12 * -(-M // 128) * Cout, 2 * M * Cin * Cout + 3 * M * Cout
    if name == "rod_conv_fwd_bnact":      # conv + eval BatchNorm / act (+ residual) epilogue (ABI 21)
        N, H, W, Cin, Cout, ks, dt = a[17], a[18], a[19], a[20], a[21], a[22], a[25]
        es = _ES[dt]
        M = N * H * W
        K = ks * ks * Cin
        res = es * M * Cout if a[15] is not None else 0
        return es * (M * Cin + M * Cout + Cout * K) + (4 * Cout if a[7] is not None else 0) + res, \
            2 * M * K * Cout + 5 * M * Cout
    if name == "rod_conv_bwd_data_bn":    # BatchNorm-backward apply in the backward-data loader (ABI 22)
        M, Cout, Cin, dt = a[12], a[13], a[14], a[15]
        es = _ES[dt]
        return es * (3 * M * Cout + M * Cin + Cin * Cout), 2 * M * Cout * Cin + 8 * M * Cout
    if name == "rod_conv_wgrad":
        N, H, W, Cin, Cout, ks, dt = a[10], a[11], a[12], a[13], a[14], a[15], a[18]
        es = _ES[dt]
        M = N * H * W
        K = ks * ks * Cin
        return es * (M * Cin + M * Cout) + 4 * Cout * K, 2 * M * K * Cout
    if name == "rod_bn_stats":
        M, C, dt = a[1], a[2], a[11]
        return _ES[dt] * M * C, 3 * M * C
    if name == "rod_bn_apply":
        M, C, dt = a[7], a[8], a[13]
        res = a[5] is not None
        return _ES[dt] * M * C * (3 if res else 2), 5 * M * C
    if name == "rod_bn_bwd":
        M, C, dt = a[10], a[11], a[16]
        return _ES[dt] * M * C * 3, 16 * M * C  # algorithmic: read dy, read x, write dx
    if name == "rod_bn_bwd_apply":
        M, C, dt = a[8], a[9], a[11]
        return _ES[dt] * M * C * 1, 8 * M * C   # write dy (dz, y re-read: design traffic)
    if name == "rod_bn_bwd_reduce":
        M, C, dt = a[10], a[11], a[13]
        return _ES[dt] * M * C * 2, 6 * M * C   # read dz, read y
    if name == "rod_pw_bwd":
        M, Cin, Cout, dt = a[19], a[20], a[21], a[22]
        es = _ES[dt]
        want_dx = a[15] is not None
        byts = es * (2 * M * Cout + M * Cin + (M * Cin if want_dx else 0)) + Cout * Cin * (es + 4)
        return byts, 2 * M * Cin * Cout * (2 if want_dx else 1) + 10 * M * Cout
    if name == "rod_pw_bwd_gred":
        M, Cin, Cout, dt = a[19], a[20], a[21], a[22]
        es = _ES[dt]
        return es * (2 * M * Cout + 2 * M * Cin) + Cout * Cin * (es + 4), \
            4 * M * Cin * Cout + 10 * M * Cout + 6 * M * Cin
    if name == "rod_pw_bwd_rc":          # ABI 23: y recomputed from x (never read)
        M, Cin, Cout, dt = a[18], a[19], a[20], a[21]
        es = _ES[dt]
        want_dx = a[15] is not None
        byts = es * (M * Cout + M * Cin + (M * Cin if want_dx else 0)) + Cout * Cin * (2 * es + 4)
        return byts, 2 * M * Cin * Cout * (3 if want_dx else 2) + 10 * M * Cout
    if name == "rod_pw_bwd_gred_rc":
        M, Cin, Cout, dt = a[19], a[20], a[21], a[22]
        es = _ES[dt]
        return es * (M * Cout + 2 * M * Cin) + Cout * Cin * (2 * es + 4), \
            6 * M * Cin * Cout + 10 * M * Cout + 6 * M * Cin
    if name == "rod_pw_bwd_gred_dyp":
        M, Cin, Cout, dt = a[19], a[20], a[21], a[22]
        es = _ES[dt]
        return es * (3 * M * Cout + M * Cin) + Cout * Cin * (es + 4), \
            4 * M * Cin * Cout + 10 * M * Cout + 6 * M * Cin
    if name == "rod_ir_block_fwd":
        # fused inverted residual: x read once (the residual re-read is L2-served by design),
        # out written once, the expanded tensor never in HBM; expand flops over all input
        # pixels, depthwise + project over the output pixels
        N, H, W, Cin, inner, Cout, s, dt = a[18], a[19], a[20], a[21], a[22], a[23], a[24], a[25]
        es = _ES[dt]
        Ho, Wo = -(-H // s), -(-W // s)
        byts = es * (N * H * W * Cin + N * Ho * Wo * Cout) + es * inner * (Cin + Cout) + 36 * inner
        return byts, 2 * N * H * W * Cin * inner + 18 * N * Ho * Wo * inner + 2 * N * Ho * Wo * inner * Cout
    if name == "rod_match_anchors":
        B, A, G = a[12], a[13], a[14]
        return B * A * 56 + A * 32 + B * G * 20, 15 * G * A * B
    # --- the remaining entries of a training / inference step (for the whole-step sum) ---
    if name == "rod_normalize_image":
        n, dt = a[2], a[3]
        return (1 + _ES[dt]) * n, 2 * n
    if name == "rod_cast":
        n = a[4]
        return (_ES[a[1]] + _ES[a[3]]) * n, 0
    if name == "rod_bn_stat_parts":
        M, C, nparts, dt = a[1], a[2], a[4], a[5]
        return _ES[dt] * M * C + 12 * nparts * C, 3 * M * C
    if name == "rod_bn_finalize":
        nparts, C = a[1], a[3]
        return 12 * nparts * C + 16 * C, 10 * nparts * C
    if name == "rod_bn_bwd_parts":
        M, C, nparts, dt = a[9], a[10], a[8], a[11]
        return _ES[dt] * M * C * 2 + 8 * nparts * C, 6 * M * C
    if name == "rod_bn_bwd_finalize":
        nparts, C = a[1], a[3]
        return 8 * nparts * C + 24 * C, 4 * nparts * C
    if name == "rod_bn_eval_stats":
        C = a[5]
        return 16 * C, 3 * C
    if name == "rod_copy2d":
        return 2 * a[4] * a[5], 0
    if name == "rod_add":
        n, dt = a[3], a[4]
        return 3 * _ES[dt] * n, n
    if name == "rod_sgd_clip":
        n = a[2]
        return 12 * n, 3 * n                 # read param, read grad, write param (fp32)
    if name == "rod_conv_weight_prep_batch":
        total, dt = a[2], a[3]
        return (4 + _ES[dt]) * total, 0
    if name == "rod_smoothl1_masked":
        B, A, dt = a[10], a[11], a[12]
        es = _ES[dt]
        wgt = a[8] is not None
        return B * A * (4 * es + 16 + 4 + 4 * es + (16 if wgt else 0)), 12 * B * A * 4
    if name == "rod_decode":
        B, A, dt = a[4], a[5], a[7]
        return B * A * (2 * 4 * _ES[dt] + 16) + 16 * A, 20 * B * A
    if name == "rod_softmax":
        rows, K, dt = a[2], a[3], a[4]
        return rows * K * (_ES[dt] + 4), 4 * rows * K
    if name == "rod_select_topk_nms":
        B, A, K = a[2], a[3], a[4]
        return B * A * (K * 4 + 16), 0
    if name == "rod_det_targets":
        B, A, dt = a[13], a[14], a[15]
        return B * A * (4 * _ES[dt] + 16 + 16 + 4 + 4 + 16 + 4 + 4 + 4), 40 * B * A
    if name in ("rod_resize_bilinear", "rod_resize_bilinear_bwd"):
        N, H, W, C, Ho, Wo, dt = a[2], a[3], a[4], a[5], a[6], a[7], a[8]
        return _ES[dt] * C * N * (H * W + Ho * Wo), 8 * N * Ho * Wo * C
    if name in ("rod_depth_to_space2", "rod_space_to_depth2"):
        N, h, w, Fc, dt = a[2], a[3], a[4], a[5], a[9]
        return 2 * _ES[dt] * N * h * w * 4 * Fc, 0
    return 0, 0


def design_bytes(name, a):
    """Bytes the call's kernels are DESIGNED to move (>= cost()[0]): differs from the
    algorithmic count only where a design re-reads a tensor — the apply pass of the two-kernel
    BatchNorm backward re-reads dz and y (reduce 2 passes + apply 3 = 5 against 3)."""
    if name == "rod_bn_bwd_apply":
        M, C, dt = a[8], a[9], a[11]
        return _ES[dt] * M * C * 3
    if name == "rod_dw3x3_bwd_fused":     # + the re-read of dz and y (BatchNorm backward pass 2)
        N, C, Ho, Wo, dt = a[19], a[22], a[26], a[27], a[28]
        return cost(name, a)[0] + _ES[dt] * 2 * N * Ho * Wo * C
    if name == "rod_dw3x3_bwd_fused_rc":  # + the re-read of dz and y (BatchNorm backward pass 2)
        N, C, Ho, Wo, dt = a[26], a[29], a[33], a[34], a[35]
        return cost(name, a)[0] + _ES[dt] * 2 * N * Ho * Wo * C
    if name == "rod_dw3x3_bwd_fused_pw":  # + the reads of yd and the cout-wide dy_p
        N, H, W, C, dt, cout = a[21], a[22], a[23], a[24], a[25], a[8]
        return cost(name, a)[0] + _ES[dt] * N * H * W * (C + cout)
    return cost(name, a)[0]


def kernel_match(name, pat):
    """pat = 'a&b!c': the kernel name contains a and b and not c (demangled or mangled names: the
    rocprofv3 CSVs hold both forms, e.g. '..., 2, 3, true>(' / '...Li2ELi3ELb1EE...')."""
    inc, *exc = pat.split('!')
    return all(t in name for t in inc.split('&')) and not any(t in name for t in exc)


# template-argument tails that tell apart kernels of one name: the depthwise backward's
# recompute form (PW, ABI 20) and the backward-data BatchNorm prologue (BWD, ABI 22)
_PW = ('2, 3, true>', 'Li2ELi3ELb1EE')
_BWD = ('32, false, true>', 'Li32ELb0ELb1EE')
# pw_bwd_stream_kernel<CIN, COUT, PRO, DX, XG, XL, RC> (round 6 names): XG = the input sums of
# rod_pw_bwd_gred's expand form (PRO, DX, XG all true), RC = the recompute form (last argument);
# pw_bwd_gred_kernel<COUT, NW, FAST, DYP>: DYP = rod_pw_bwd_gred_dyp (last argument)
_XG = (', true, true, true, ', 'Lb1ELb1ELb1E')
_LAST = ('true>(rod::PwBwdArgs', 'Lb1EEEvNS_9PwBwdArgs')
# pw_stream_kernel<NT, KT, MODE, ...>: MODE 3 = statistics only (rod_conv_fwd_stats; KT is 1 there)
_STATS_ONLY = (', 1, 3', 'ELi1ELi3E')


def _forms(base, inc=(), exc=()):
    """Demangled and mangled patterns of the template kernel rod::`base` with the (demangled,
    mangled) pairs of inc / exc: each form's name prefix is part of it, so an exclusion written
    for one form never lets the other form's name through."""
    heads = ('rod::%s<' % base, '_ZN3rod%d%sI' % (len(base), base))
    return tuple('&'.join([heads[i]] + [t[i] for t in inc]) + ''.join('!' + t[i] for t in exc) for i in (0, 1))

# C-ABI entry -> (kernel patterns of which exactly one launches once per entry call, patterns
# of every kernel the entry launches; kernel_match) for attributing rocprofv3 PMC counters
# (tools/pmc_traffic.py); shared helper kernels (slab_sum, splitk_combine) are not attributed.
ENTRY_KERNELS = {
    # rod_bn_bwd runs only on small tensors on the training path (ops.bn_bwd_dy): the one-launch kernel
    "rod_bn_bwd": (("bn_bwd_small_kernel",), ("bn_bwd_small_kernel",)),
    "rod_bn_apply": (("bn_apply_kernel",), ("bn_apply_kernel",)),
    "rod_bn_bwd_reduce": (("bn_bwd_reduce_kernel",), ("bn_bwd_reduce_kernel", "bn_bwd_finalize_kernel")),
    "rod_bn_bwd_apply": (("bn_bwd_apply_kernel",), ("bn_bwd_apply_kernel",)),
    "rod_pw_bwd": (_forms("pw_bwd_kernel") + _forms("pw_bwd_stream_kernel", exc=(_XG, _LAST)),) * 2,
    "rod_pw_bwd_rc": (_forms("pw_bwd_stream_kernel", inc=(_LAST,), exc=(_XG,)),) * 2,
    "rod_pw_bwd_gred": (_forms("pw_bwd_gred_kernel", exc=(_LAST,)) +
                        _forms("pw_bwd_stream_kernel", inc=(_XG,), exc=(_LAST,)),) * 2,
    "rod_pw_bwd_gred_rc": (_forms("pw_bwd_stream_kernel", inc=(_XG, _LAST)),) * 2,
    "rod_pw_bwd_gred_dyp": (_forms("pw_bwd_gred_kernel", inc=(_LAST,)),) * 2,
    "rod_dw3x3_fwd": (("dw3x3_fwd_!dw3x3_fwd_rc",), ("dw3x3_fwd_!dw3x3_fwd_rc",)),
    "rod_dw3x3_fwd_rc": (("dw3x3_fwd_rc_kernel",), ("dw3x3_fwd_rc_kernel",)),
    "rod_dw3x3_bwd_data": (("dw3x3_bwd_data",), ("dw3x3_bwd_data",)),
    "rod_dw3x3_bwd_filter": (("dw3x3_bwdw_lx", "dw3x3_bwd_filter_kernel"), ("dw3x3_bwdw_lx", "dw3x3_bwd_filter_kernel")),
    "rod_dw3x3_bwd_fused": (("dw3x3_bwd_fused!dw3x3_bwd_fused_rc!" + "!".join(_PW),),) * 2,
    "rod_dw3x3_bwd_fused_rc": (("dw3x3_bwd_fused_rc_kernel",),) * 2,
    "rod_dw3x3_bwd_fused_pw": tuple(tuple("dw3x3_bwd_fused2&" + t for t in _PW) for _ in range(2)),
    "rod_conv_wgrad": (("conv_wgrad_kernel",), ("conv_wgrad_kernel", "colsum_kernel")),
    "rod_conv_fwd": (("conv_fwd_kernel!" + "!".join(_BWD), "stem_fwd_mfma_kernel") +
                     _forms("pw_stream_kernel", exc=(_STATS_ONLY,)),) * 2,
    "rod_conv_fwd_stats": (_forms("pw_stream_kernel", inc=(_STATS_ONLY,)),) * 2,
    "rod_conv_bwd_data_bn": tuple(tuple("conv_fwd_kernel&" + t for t in _BWD) for _ in range(2)),
    "rod_bn_finalize": (("bn_parts_merge_kernel",), ("bn_parts_merge_kernel",)),
    "rod_ir_block_fwd": (("ir_block_fwd_kernel",), ("ir_block_fwd_kernel",)),
}
