"""Algorithmic cost of one librod call (bytes that must cross HBM at minimum, and flops),
from the call's own arguments — the per-unit figures of SURVEY.md §8(d):

  dw3x3 fwd / bwd_data : es*(in + out) + 9*C*4 bytes, 18*N*Ho*Wo*C flops
  dw3x3 bwd_filter     : es*(x + dy) + 9*C*4, 18*N*Ho*Wo*C
  conv fwd (1x1 / 3x3) : es*(M*Cin + M*Cout + Cout*K) (+4*Cout bias), 2*M*K*Cout
  conv wgrad           : es*(M*Cin + M*Cout) + 4*Cout*K, 2*M*K*Cout
  bn_stats             : es*M*C;  bn_apply: es*M*C*(2 + residual)
  bn_bwd               : es*M*C*3 (read dy, read x, write dx; the reduce+apply split re-reads
                         dy and x, so achieved/peak also shows that avoidable re-read)
  bn_bwd_reduce        : es*M*C*2 (read dz, read y);  bn_bwd_apply: es*M*C*3
  pw_bwd (fused 1x1)   : es*(2*M*Cout + M*Cin [+ M*Cin dx]) + W, 2*M*Cin*Cout per product
  match_anchors        : B*A*(16 + 16 + 16 + 4 + 4) + anchors, 15*G*A*B flops
  ir_block_fwd (fused) : es*(N*H*W*Cin + N*Ho*Wo*Cout) + weights, 2*N*H*W*Cin*inner +
                         18*N*Ho*Wo*inner + 2*N*Ho*Wo*inner*Cout
"""

_ES = {0: 4, 1: 2}

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
    if name == "rod_dw3x3_bwd_data":
        N, H, W, C, Ho, Wo, dt = a[10], a[11], a[12], a[13], a[17], a[18], a[19]
        es = _ES[dt]
        gred = es * N * H * W * C if a[9] is not None else 0   # the epilogue reads y
        return es * (N * H * W * C + N * Ho * Wo * C) + 36 * C + gred, 18 * N * Ho * Wo * C
    if name == "rod_dw3x3_bwd_filter":
        N, H, W, C, Ho, Wo, dt = a[9], a[10], a[11], a[12], a[16], a[17], a[18]
        es = _ES[dt]
        return es * (N * H * W * C + N * Ho * Wo * C) + 36 * C, 18 * N * Ho * Wo * C
    if name == "rod_conv_fwd":
        N, H, W, Cin, Cout, ks, dt = a[18], a[19], a[20], a[21], a[22], a[23], a[26]
        es = _ES[dt]
        M = N * H * W
        K = ks * ks * Cin
        gred = es * M * Cout if a[17] is not None else 0   # the gred epilogue reads y
        return es * (M * Cin + M * Cout + Cout * K) + (4 * Cout if a[7] is not None else 0) + gred, 2 * M * K * Cout
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
        return _ES[dt] * M * C * 3, 8 * M * C   # read dz, read y, write dy
    if name == "rod_bn_bwd_reduce":
        M, C, dt = a[10], a[11], a[13]
        return _ES[dt] * M * C * 2, 6 * M * C   # read dz, read y
    if name == "rod_pw_bwd":
        M, Cin, Cout, dt = a[19], a[20], a[21], a[22]
        es = _ES[dt]
        want_dx = a[15] is not None
        byts = es * (2 * M * Cout + M * Cin + (M * Cin if want_dx else 0)) + Cout * Cin * (es + 4)
        return byts, 2 * M * Cin * Cout * (2 if want_dx else 1) + 10 * M * Cout
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
    return 0, 0


# C-ABI entry -> (kernel-name substrings of which exactly one launches once per entry call,
# substrings of every kernel the entry launches) for attributing rocprofv3 PMC counters
# (tools/pmc_traffic.py); shared helper kernels (slab_sum, splitk_combine) are not attributed
ENTRY_KERNELS = {
    # rod_bn_bwd runs only on small tensors on the training path (ops.bn_bwd_dy): the one-launch kernel
    "rod_bn_bwd": (("bn_bwd_small_kernel",), ("bn_bwd_small_kernel",)),
    "rod_bn_apply": (("bn_apply_kernel",), ("bn_apply_kernel",)),
    "rod_bn_bwd_reduce": (("bn_bwd_reduce_kernel",), ("bn_bwd_reduce_kernel", "bn_bwd_finalize_kernel")),
    "rod_bn_bwd_apply": (("bn_bwd_apply_kernel",), ("bn_bwd_apply_kernel",)),
    "rod_pw_bwd": (("pw_bwd_kernel",), ("pw_bwd_kernel",)),
    "rod_dw3x3_fwd": (("dw3x3_fwd_",), ("dw3x3_fwd_",)),
    "rod_dw3x3_bwd_data": (("dw3x3_bwd_data",), ("dw3x3_bwd_data",)),
    "rod_dw3x3_bwd_filter": (("dw3x3_bwdw_lx", "dw3x3_bwd_filter_kernel"), ("dw3x3_bwdw_lx", "dw3x3_bwd_filter_kernel")),
    "rod_conv_wgrad": (("conv_wgrad_kernel",), ("conv_wgrad_kernel", "colsum_kernel")),
    "rod_conv_fwd": (("conv_fwd_kernel", "stem_conv_fwd_kernel"), ("conv_fwd_kernel", "stem_conv_fwd_kernel")),
    "rod_bn_finalize": (("bn_parts_merge_kernel",), ("bn_parts_merge_kernel",)),
    "rod_ir_block_fwd": (("ir_block_fwd_kernel",), ("ir_block_fwd_kernel",)),
}
