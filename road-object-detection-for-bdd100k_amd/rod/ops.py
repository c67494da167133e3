"""Differentiable ops backed by librod (HIP kernels for gfx950).

Every op here launches only librod kernels on the current HIP stream; PyTorch provides
device memory, streams and the autograd tape.  Parameter gradients are written by the
kernels straight into the flat gradient buffer of rod.params.ParamStore (the op
returns None for the parameter), so no PyTorch arithmetic touches gradients either.

Tensor conventions: activations NHWC [N, H, W, C] contiguous in fp32 or bf16; conv
weights fp32 [Cout, k, k, Cin]; depthwise weights fp32 [3, 3, C]; BN vectors fp32 [C].
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import _abi
from ._abi import ROD_ACT_LEAKY, ROD_ACT_NONE, ROD_ACT_RELU, ROD_ACT_RELU6  # noqa: F401

_DT = {torch.float32: _abi.ROD_F32, torch.bfloat16: _abi.ROD_BF16}
# debug bisection switches (comma list): splitk, epistats, convstats, dwstats, bnpro, pwgred, stembn, pro3
_DISABLE = set(os.environ.get("ROD_DISABLE", "").split(","))
# opt-in paths (comma list): gred = BatchNorm-backward reduction fused into the backward-data
# epilogues (measured slower than the separate streaming reduce on MI355X: DESIGN.md §6);
# gredpw = the same for the 1x1 convs that take the streaming kernel (measured neutral); dwbn,
# side: DESIGN.md §6
_ENABLE = set(os.environ.get("ROD_ENABLE", "").split(","))


def dtcode(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}") from None


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


class _Side:
    """Weight gradients on a side stream (single process): a conv's / depthwise's filter
    gradient only reads (x, dy) and writes its own slot of the flat gradient buffer, so it can
    run beside the backward-data chain that the rest of the backward waits on.  The side stream
    forks from the main stream where dy is ready and is joined once, before the optimizer step
    (join()); the tensors it reads stay referenced until then, so the caching allocator cannot
    hand their memory to main-stream work in between.  Works under HIP-graph capture (the fork /
    join become graph edges).  Opt-in (ROD_ENABLE=side: measured slower, the overlapped kernels
    contend for the same CUs and HBM — DESIGN.md §6); never under data parallelism (the gradient
    buckets are reduced from inside backward); outside SIDE.backward (tests, other callers of
    .backward()) everything stays on the calling stream."""

    def __init__(self):
        self.on = False
        self.stream = None
        self.keep = []

    def backward(self, loss, device):
        """graph.backward(loss) with the weight gradients on the side stream, joined before
        returning (so every caller after it sees complete gradients on the main stream)."""
        from . import graph
        if "side" in _DISABLE:
            return graph.backward(loss)
        if self.stream is None or self.stream.device != torch.device(device):
            self.stream = torch.cuda.Stream(device=device)
        self.on = True
        try:
            graph.backward(loss)
        finally:
            self.on = False
            torch.cuda.current_stream().wait_stream(self.stream)
            self.keep.clear()

    def run(self, fn, *keep):
        if not self.on:
            return fn()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            r = fn()
        self.keep.extend(keep)
        return r



SIDE = _Side()


class LevelStreams:
    """Independent per-level chains (the detector heads: one chain of small convs per pyramid
    level, catch_net.py:276-342) on their own HIP streams, so the latency-bound launches of the
    small levels overlap each other and the backbone instead of queueing behind them.

    fork(i, ready): the stream of chain i, made to wait for `ready` (an event recorded where the
    chain's input was produced) or for everything the calling stream has queued; join(outs):
    the calling stream waits for every chain stream used.  Tensors crossing streams are marked
    with record_stream, so the caching allocator never hands their memory to another stream
    while the consumer may still read it.  Fork and join are event edges, i.e. graph
    dependencies under HIP-graph capture; autograd runs each backward node on its forward's
    stream and synchronises the edges between streams itself.  ROD_HEAD_STREAMS=n chains
    streams (0: every chain on the calling stream)."""

    def __init__(self):
        self.n = int(os.environ.get("ROD_HEAD_STREAMS", "3"))
        self.pool = {}
        self.used = []

    def active(self, t):
        # not under SyncBatchNorm: its statistics all-gathers would be issued from the chain
        # streams — torch.distributed's would run there, several streams driving one
        # communicator; the library's would fork its communication stream from a chain stream,
        # which crashes the end of a HIP-graph capture (rod.ddp.GradReducer._on_chain_stream)
        return self.n > 0 and SYNC_BN is None and torch.is_tensor(t) and t.is_cuda

    def stream(self, i, device):
        key = (str(device), i % self.n)
        if key not in self.pool:
            self.pool[key] = torch.cuda.Stream(device=device)
        return self.pool[key]

    def fork(self, i, x, ready=None):
        s = self.stream(i, x.device)
        if ready is not None:
            s.wait_event(ready)
        else:
            s.wait_stream(torch.cuda.current_stream(x.device))
        x.record_stream(s)
        if s not in self.used:
            self.used.append(s)
        return s

    def join(self, outs):
        if not self.used:
            return
        cur = torch.cuda.current_stream(self.used[0].device)
        for s in self.used:
            cur.wait_stream(s)
        for o in outs:
            o.record_stream(cur)
        self.used = []


LEVELS = LevelStreams()


class SlabDefer(object):
    """Deferred parameter-gradient sums over one backward (rod_slab_defer / rod_slab_flush,
    include/rod.h ABI 11): the weight-gradient entries queue their final fixed-order slab sums
    instead of launching ~115 tiny kernels per step, and flush() runs them as a few batched
    launches (bit-identical).  The tensors those entries were given stay referenced until the
    flush is enqueued, so the caching allocator cannot hand their memory to later work.
    Everything that reads a parameter gradient runs after flush(): the optimizer, and each
    data-parallel bucket all-reduce (rod.ddp.GradReducer flushes before launching one)."""

    def __init__(self):
        self.active = False

    def begin(self):
        if "slabdefer" in _DISABLE:
            return
        _abi.lib().rod_slab_defer(1)
        _abi.KEEP = []
        self.active = True

    def flush(self):
        """Enqueue every queued sum on the current stream (deferral stays on)."""
        if not self.active:
            return
        _abi.call("rod_slab_flush", stream())
        _abi.KEEP = []    # the flush is enqueued: stream order protects the slabs from here on

    def flush_range(self, t):
        """Enqueue only the queued sums that write into tensor t (a gradient bucket, ABI 15).
        The slabs of the sums left queued stay referenced until the full flush."""
        if not self.active:
            return
        _abi.call("rod_slab_flush_range", t.data_ptr(), t.data_ptr() + t.numel() * t.element_size(), stream())

    def end(self):
        if not self.active:
            return
        try:
            self.flush()
        finally:
            _abi.lib().rod_slab_defer(0)
            _abi.KEEP = None
            self.active = False


SLAB = SlabDefer()


def grad_slot(p):
    """The flat-buffer gradient view registered for parameter tensor p (or None)."""
    return getattr(p, "_rod_grad", None)


def _mark_written(p):
    cb = getattr(p, "_rod_on_grad", None)
    if cb is not None:
        cb(p)


def same_pad(size: int, stride: int, k: int = 3):
    """TF 'SAME' padding: (out, pad_before) for one spatial dim (conv_blocks.py:40-46)."""
    out = -(-size // stride)
    total = max((out - 1) * stride + k - size, 0)
    return out, total // 2


# ----------------------------------------------------------------------------- ingest
def normalize_image(img_u8: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """(2/255)*img - 1 (train.py:126) from a uint8 NHWC tensor."""
    out = torch.empty(img_u8.shape, dtype=dtype, device=img_u8.device)
    _abi.call("rod_normalize_image", img_u8, out, img_u8.numel(), dtcode(out), stream())
    return out


def _device_i(a, dev, dtype):
    """Small host parameter array -> device, pinned + non-blocking (no stream sync)."""
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dtype)
    if dev.type == 'cuda':
        t = t.pin_memory()
    return t.to(dev, non_blocking=True)


def augment_images(src, crop, mode, colour, out_hw, dtype=torch.float32, normalize=False, src_hw=None,
                   src_off=None):
    """rod_augment_images: crop -> legacy bilinear resize -> flip -> colour chain [-> (2/255)x-1]
    (data_pileline_tools.py:76-108, train.py:126).  src: uint8 [B, H, W, 3] device tensor, or a
    flat uint8 buffer with per-image src_hw [B, 2] / src_off [B] (host arrays).  crop [B, 4],
    mode [B, 2], colour [B, 3]: host arrays of the sampled parameters."""
    dev = src.device
    if src_hw is None:
        B, H, W, _ = src.shape
        src_hw = np.tile(np.array([H, W], np.int32), (B, 1))
        src_off = np.arange(B, dtype=np.int64) * (H * W * 3)
    B = len(src_hw)
    Ho, Wo = int(out_hw[0]), int(out_hw[1])
    crop = np.asarray(crop, np.int32).reshape(B, 4)
    hw = np.asarray(src_hw, np.int64).reshape(B, 2)
    if (crop[:, :2] < 0).any() or (crop[:, 2:] <= 0).any() or (crop[:, 0] + crop[:, 2] > hw[:, 0]).any() or \
            (crop[:, 1] + crop[:, 3] > hw[:, 1]).any():
        raise ValueError('augment_images: crop window outside the source image')
    if int((hw[:, 0] * hw[:, 1] * 3).max()) >= 2 ** 31:
        raise ValueError('augment_images: a source image exceeds 2 GiB')
    if int((np.asarray(src_off, np.int64) + hw[:, 0] * hw[:, 1] * 3).max()) > src.numel():
        raise ValueError('augment_images: source offsets exceed the buffer')
    out = torch.empty((B, Ho, Wo, 3), dtype=dtype, device=dev)
    ws = workspace(_abi.query('rod_augment_workspace', B, Ho, Wo), dev)
    _abi.call('rod_augment_images', src, _device_i(src_off, dev, torch.int64), _device_i(src_hw, dev, torch.int32),
              _device_i(crop, dev, torch.int32), _device_i(np.asarray(mode, np.int32), dev, torch.int32),
              _device_i(np.asarray(colour, np.float32), dev, torch.float32), ws, out, B, Ho, Wo,
              int(bool(normalize)), dtcode(out), stream())
    return out


def augment_boxes(boxes, labels, n, ref, mode=None, threshold=0.3):
    """rod_augment_boxes: bboxes_resize -> bboxes_filter_overlap -> flip -> clip (process.py:130-134,
    tf_image.py:284-289, data_pileline_tools.py:106-107).  boxes [B, G, 4] / labels [B, G] / n [B]
    as device tensors or host arrays; ref [B, 4], mode [B, 2] host arrays.  Returns device
    (boxes, labels, n), zero-padded past n."""
    dev = boxes.device if torch.is_tensor(boxes) else torch.device('cuda')
    b = boxes if torch.is_tensor(boxes) else _device_i(np.asarray(boxes, np.float32), dev, torch.float32)
    lab = labels if torch.is_tensor(labels) else _device_i(np.asarray(labels, np.int32), dev, torch.int32)
    nn = n if torch.is_tensor(n) else _device_i(np.asarray(n, np.int32), dev, torch.int32)
    B, G = b.shape[0], b.shape[1]
    bo = torch.empty_like(b)
    lo = torch.empty_like(lab)
    no = torch.empty_like(nn)
    md = None if mode is None else _device_i(np.asarray(mode, np.int32), dev, torch.int32)
    _abi.call('rod_augment_boxes', b.contiguous(), lab.contiguous(), nn, _device_i(np.asarray(ref, np.float32), dev,
              torch.float32), md, bo, lo, no, B, G, float(threshold), stream())
    return bo, lo, no


def cast(x: torch.Tensor, dtype) -> torch.Tensor:
    if x.dtype == dtype:
        return x
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    _abi.call("rod_cast", x, dtcode(x), out, dtcode(out), x.numel(), stream())
    return out


def copy2d(src, src_ld_bytes, dst, dst_ld_bytes, rows, cols_bytes, src_off=0, dst_off=0):
    _abi.call("rod_copy2d", src.data_ptr() + src_off, src_ld_bytes, dst.data_ptr() + dst_off, dst_ld_bytes,
              rows, cols_bytes, stream())


# ----------------------------------------------------------------------------- SyncBN
# Data-parallel BatchNorm over the GLOBAL batch (the reference normalises over its
# whole single-device batch, mobilenet.py:417-420).  None = per-rank statistics (the default);
# otherwise an object with `.world` and `.gather(parts) -> [world * nparts, ...]` (rank order,
# rod.ddp.GradReducer.bn_allgather).  Every rank merges the same gathered partial statistics
# in the same fixed order, so mean / rstd / coefficients are identical on all ranks.
SYNC_BN = None


def _sync_nparts(M):
    return int(max(1, min(1024, M // 256)))


# ----------------------------------------------------------------------------- BatchNorm prologue
class Pending:
    """act(BatchNorm(y)) whose statistics are known but which is NOT materialised.

    A consumer that supports the BatchNorm-apply prologue (conv2d, dw3x3) reads y and forms
    act((y - mean) * rstd*gamma + beta) as it loads it (include/rod.h, ABI 3), and its backward
    runs the BatchNorm backward itself; `materialize` writes the tensor for any other consumer.
    """
    __slots__ = ('y', 'mean', 'rstd', 'gamma', 'beta', 'act', 'training', 'owned')

    def __init__(self, y, mean, rstd, gamma, beta, act, training, owned=False):
        self.y, self.mean, self.rstd, self.gamma, self.beta = y, mean, rstd, gamma, beta
        self.act, self.training = act, training
        # owned: y is the output of a producer node (_ConvBN / _DWBN) that runs this
        # BatchNorm's backward itself; the consumer hands back d/d(act output) unchanged
        self.owned = owned

    @property
    def shape(self):
        return self.y.shape


def _pro_args(p):
    """The five prologue arguments of the ABI-3 entries (NULLs without a prologue)."""
    if p is None:
        return (None, None, None, None, 0)
    mean, rstd, gamma, beta, act = p
    return (mean, rstd, gamma, beta, act)


def _bn_backward(dz, y, mean, rstd, gamma, beta, act, need_g, need_b):
    """rod_bn_bwd: gradient wrt the pre-BatchNorm y from the gradient dz of act(BN(y));
    dgamma / dbeta go to the parameters' flat-buffer slots."""
    if SYNC_BN is not None:   # reduction over the global batch, then the local apply
        coef = bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, need_g, need_b)
        return _bn_bwd_apply(dz, y, mean, rstd, gamma, beta, act, coef)
    N, H, W, C = y.shape
    M = N * H * W
    dz = dz.contiguous()
    dy = torch.empty_like(y)
    dg = grad_slot(gamma) if need_g else None
    db = grad_slot(beta) if need_b else None
    if db is None:
        db = torch.empty(C, dtype=torch.float32, device=y.device)  # the kernel always may write dbeta
    ws = workspace(_abi.query("rod_bn_bwd_workspace", M, C), y.device)
    _abi.call("rod_bn_bwd", dz, y, mean, rstd, gamma, beta, dy, dg, db, ws, M, C, 0, 0, 0, act, dtcode(y),
              stream())
    if need_g:
        _mark_written(gamma)
    if need_b:
        _mark_written(beta)
    return dy


# BatchNorm-backward sums handed from a consumer's backward to the producer's: the fused
# depthwise backward (rod_dw3x3_bwd_fused) computes, beside the gradient dx it returns
# for its input act(BN(y)), that BatchNorm's backward sums over (dx, y).  The producer node
# (_ConvBN) receives exactly that dx as its dz when the depthwise is the only consumer, and then
# finalizes the sums instead of running rod_bn_bwd_reduce over (dz, y).  Entries hold their dx
# (so its memory cannot be reused while listed) and are dropped when the backward ends.
# An entry is accepted only for the very tensor it was made for, or a view of the same storage
# whose version counter is unchanged: a gradient summed IN PLACE into dx (a second consumer of
# the depthwise input) shares dx's pointer and shape but bumps its version, and then the
# producer runs its own reduce over the summed dz instead of picking up stale sums.
_BN_PARTS = {}


def _put_bn_parts(dx, parts):
    _BN_PARTS[dx.data_ptr()] = (dx, parts, dx._version)


def _take_bn_parts(dz):
    e = _BN_PARTS.pop(dz.data_ptr(), None) if dz is not None else None
    if e is None:
        return None
    dx, parts, ver = e
    if dx is dz:
        return parts if dz._version == ver else None
    if dx.shape != dz.shape or dx.dtype != dz.dtype or dz._version != ver or \
            dx.untyped_storage().data_ptr() != dz.untyped_storage().data_ptr():
        return None
    return parts


def clear_bn_parts():
    """End of a backward: drop the hand-offs.  Returns how many unmaterialised depthwise-input
    gradients (the project recipes below) were never consumed by their depthwise node."""
    _BN_PARTS.clear()
    left = len(_DZ_RECIPE)
    _DZ_RECIPE.clear()
    return left


# Unmaterialised depthwise-output gradients (ABI 20).  In an inverted-residual block the gradient
# at the project conv's input is dz = dy_p . W_p; the project node (rod_pw_bwd_gred_dyp) hands the
# depthwise node the cout-wide dy_p and W_p^T instead of writing the C-wide dz, and returns a
# placeholder of dz's shape whose memory is never written.  The depthwise node takes the recipe
# (rod_dw3x3_bwd_fused_pw recomputes dz per tile, or rod_conv_fwd materialises it for any other
# path); a placeholder that reaches anything else is caught at the end of backward (graph.backward).
_DZ_RECIPE = {}


def _put_dz_recipe(dz, recipe):
    _DZ_RECIPE[dz.data_ptr()] = (dz, recipe, dz._version)


def _take_dz_recipe(dz):
    if dz is None:
        return None
    e = _DZ_RECIPE.pop(dz.data_ptr(), None)
    if e is None:
        return None
    ph, recipe, ver = e
    same = ph is dz or (ph.shape == dz.shape and ph.dtype == dz.dtype and
                        ph.untyped_storage().data_ptr() == dz.untyped_storage().data_ptr())
    if not same or dz._version != ver:
        raise RuntimeError("an unmaterialised depthwise-input gradient was modified or aliased before its "
                           "depthwise node consumed it")
    return recipe


def _materialize_dz(recipe, shape, dtype):
    """dz = dy_p . W_p^T with rod_conv_fwd (the MFMA rod_pw_bwd_gred forms it with, k zero-padded:
    the same bf16 values) for a depthwise path other than rod_dw3x3_bwd_fused_pw."""
    dyp, wt1, cout = recipe
    N, H, W, C = shape
    dz = torch.empty(shape, dtype=dtype, device=dyp.device)
    conv_fwd_raw(dyp.view(N, H, W, cout), wt1, None, dz, N, H, W, cout, C, 1)
    return dz


def bn_bwd_coef_from_parts(parts, M, C, rstd, gamma, beta, need_g, need_b):
    """rod_bn_bwd_finalize of [nparts][2][C] backward sums (a consumer kernel's epilogue) ->
    coef [3, C]; dgamma / dbeta to the parameters' slots.  Under SyncBatchNorm the parts are
    all-gathered first (the parameter gradients stay this rank's own sums, as bn_bwd_reduce)."""
    coef = torch.empty(3 * C, dtype=torch.float32, device=parts.device)
    dg = grad_slot(gamma) if need_g else None
    db = grad_slot(beta) if need_b else None
    nparts = parts.shape[0]
    if SYNC_BN is not None:
        if dg is not None or db is not None:
            _abi.call("rod_bn_bwd_finalize", parts, nparts, M, C, rstd, gamma, dg, db,
                      torch.empty(3 * C, dtype=torch.float32, device=parts.device), stream())
        gp = SYNC_BN.gather(parts)
        _abi.call("rod_bn_bwd_finalize", gp, gp.shape[0], M * SYNC_BN.world, C, rstd, gamma, None, None, coef,
                  stream())
    else:
        _abi.call("rod_bn_bwd_finalize", parts, nparts, M, C, rstd, gamma, dg, db, coef, stream())
    if need_g:
        _mark_written(gamma)
    if need_b:
        _mark_written(beta)
    return coef


def bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, need_g, need_b):
    """rod_bn_bwd_reduce: the BatchNorm-backward sums of (dz, y) -> coef [3, C] for a consumer
    that applies dy itself; dgamma / dbeta go to the parameters' flat-buffer slots."""
    C = y.shape[-1]
    M = y.numel() // C
    coef = torch.empty(3 * C, dtype=torch.float32, device=y.device)
    dg = grad_slot(gamma) if need_g else None
    db = grad_slot(beta) if need_b else None
    if SYNC_BN is not None:
        dz = dz.contiguous()
        nparts = _sync_nparts(M)
        parts = torch.empty((nparts, 2, C), dtype=torch.float32, device=y.device)
        _abi.call("rod_bn_bwd_parts", dz, y, mean, rstd, gamma, beta, act, parts, nparts, M, C, dtcode(y), stream())
        if dg is not None or db is not None:
            # parameter gradients from this rank's rows only: the DP reducer sums them
            _abi.call("rod_bn_bwd_finalize", parts, nparts, M, C, rstd, gamma, dg, db,
                      torch.empty(3 * C, dtype=torch.float32, device=y.device), stream())
        gp = SYNC_BN.gather(parts)
        _abi.call("rod_bn_bwd_finalize", gp, gp.shape[0], M * SYNC_BN.world, C, rstd, gamma, None, None, coef,
                  stream())
    else:
        ws = workspace(_abi.query("rod_bn_bwd_workspace", M, C), y.device)
        _abi.call("rod_bn_bwd_reduce", dz, y, mean, rstd, gamma, beta, dg, db, coef, ws, M, C, act, dtcode(y),
                  stream())
    if need_g:
        _mark_written(gamma)
    if need_b:
        _mark_written(beta)
    return coef


def pw_bwd_supported(Cin, Cout, dtype):
    return "pwbwd" not in _DISABLE and bool(_abi.lib().rod_pw_bwd_supported(int(Cin), int(Cout), _DT[dtype]))


def pw_bwd(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, want_dx, dw, db, wt0=None):
    """rod_pw_bwd: dx (or None), dw / db written in place (fp32 [Cout, Cin] / [Cout]).
    wt0 (the forward operand): rod_pw_bwd_rc — y is recomputed from x in the kernel, not read."""
    Cin, Cout = x.shape[-1], dz.shape[-1]
    M = dz.numel() // Cout
    dx = torch.empty_like(x) if want_dx else None
    ws = workspace(_abi.query("rod_pw_bwd_workspace", M, Cin, Cout), x.device)
    if wt0 is not None:
        assert db is None
        _abi.call("rod_pw_bwd_rc", dz, wt0, mean, rstd, gamma, beta, act, coef, x, *_pro_args(xpro),
                  wt1 if want_dx else None, dx, dw, ws, M, Cin, Cout, dtcode(x), stream())
        return dx
    _abi.call("rod_pw_bwd", dz, y, mean, rstd, gamma, beta, act, coef, x, *_pro_args(xpro), wt1 if want_dx else None,
              dx, dw, db, ws, M, Cin, Cout, dtcode(y), stream())
    return dx


def pw_bwd_rc_ok(M, Cin, Cout, dtype):
    """The expand backward recomputes its pre-BatchNorm y from x (ABI 23, rod_pw_bwd_rc /
    rod_pw_bwd_gred_rc) instead of reading it: ROD_DISABLE=rc turns it off (A/B).  Taken for
    block 1's 16 -> 96 (720p b8: 683 -> 549 us); the 24 -> 144 form measured slower (266 -> 310 us
    a call: one wave per SIMD, nothing hides the recompute's LDS round trip) and is opt-in
    (ROD_ENABLE=rc144)."""
    if "rc" in _DISABLE or dtype != torch.bfloat16 or (Cin != 16 and "rc144" not in _ENABLE):
        return False
    return bool(_abi.lib().rod_pw_bwd_rc_supported(int(M), int(Cin), int(Cout), _DT[dtype]))


def dw_rc_ok(xe, N, H, W, C, stride):
    """(x, x prologue, wt0, Cin) when the depthwise input xe is an expand conv's output that
    rod_dw3x3_fwd_rc can recompute (ABI 23), else None.  Opt-in (ROD_ENABLE=rcdw): bit-identical,
    but measured slower than reading the stored tensor at every 720p b8 block shape
    (tools/rc_bench.py: block 1 378 -> 570 us, block 2 288 -> 357) — the per-row MFMA
    and its epilogue sit on the barrier-synchronised row pipeline of a 4-wave block."""
    src = getattr(xe, "_rod_expand", None)
    if src is None or "rc" in _DISABLE or "rcdw" not in _ENABLE or xe.dtype != torch.bfloat16:
        return None
    xin, xpro, wt0, Cin = src
    if not _abi.lib().rod_dw3x3_fwd_rc_supported(N, H, W, C, int(Cin), int(stride), _DT[xe.dtype]):
        return None
    return src


def _nostore_ok(x, ipro, N, H, W, Cin, Cout, dw_stride):
    """The expand conv of an inverted-residual block whose depthwise has stride 2 need not write its
    output at all (ABI 23): every consumer of it can recompute it from the block input x — the
    depthwise forward (rod_dw3x3_fwd_rc), the depthwise backward (rod_dw3x3_bwd_fused_rc) and the
    expand's own backward (rod_pw_bwd_gred_rc for 16 -> 96 with the previous project's BatchNorm
    pending, else rod_pw_bwd_rc) — and its BatchNorm statistics come from rod_conv_fwd_stats.  Taken
    only when every one of those paths applies (no silent read of the unwritten tensor is possible:
    _ConvBN / _DWBN raise if they end up elsewhere).  ROD_DISABLE=nostore or rc turns it off."""
    if dw_stride != 2 or "nostore" in _DISABLE or "rc" in _DISABLE or "epistats" in _DISABLE or "bnpro" in _DISABLE or \
            SYNC_BN is not None or x.dtype != torch.bfloat16:
        return False
    L = _abi.lib()
    M = N * H * W
    dt = _DT[x.dtype]
    _, pt = same_pad(H, 2)
    _, pl = same_pad(W, 2)
    if not (L.rod_conv_fwd_stats_supported(M, Cin, Cout, dt) and L.rod_dw3x3_fwd_rc_supported(N, H, W, Cout, Cin, 2, dt)
            and L.rod_dw3x3_bwd_fused_rc_supported(N, H, W, Cout, Cin, 2, pt, pl, dt)
            and _dw_fused_ok(N, -(-H // 2), -(-W // 2), Cout, x.dtype, 2)):
        return False
    if not L.rod_pw_bwd_rc_supported(M, Cin, Cout, dt):
        return False
    gred = ipro is not None and M >= 65536 and pw_bwd_gred_parts(M, Cin, Cout, x.dtype) > 0
    return gred or _pw_fused_ok(M, Cin, Cout, x.dtype)


def rc_eval_ok(Cin, inner, stride, dtype):
    """Inference: an inverted-residual block whose expand output the depthwise
    forward can recompute from the block input (rod_dw3x3_fwd_rc: Cin 16 / 24 / 32) runs as the
    unfused chain with that output never written, in preference to the fused block kernel
    (ir_block_fwd).  Measured on one box, alternating (profiles/r6_rcinf_ab.txt): 1080p b8 893 / 890
    (fused blocks 1, 2, 4, 5) -> 902 / 904 img/s, 720p b32 2162 / 2160 -> 2172 / 2183.
    ROD_DISABLE=rcinf turns it off, rcinf1 keeps the stride-1 blocks on the fused kernel."""
    if "rcinf" in _DISABLE or "nostore" in _DISABLE or "rc" in _DISABLE or "bnpro" in _DISABLE or \
            dtype != torch.bfloat16 or inner <= Cin or Cin not in (16, 24, 32):
        return False
    return stride == 2 or "rcinf1" not in _DISABLE


def _nostore_eval_ok(x, N, H, W, Cin, Cout, dw_stride):
    """Inference: the expand conv of a block rc_eval_ok takes need not write its output — the
    depthwise forward recomputes it from the block input (rod_dw3x3_fwd_rc, the eval BatchNorm in
    its expand epilogue, no statistics), the same rounded values the stored tensor would hold.
    There is no backward."""
    if dw_stride not in (1, 2) or not rc_eval_ok(Cin, Cout, dw_stride, x.dtype) or \
            torch.is_grad_enabled() and x.requires_grad:
        return False
    return bool(_abi.lib().rod_dw3x3_fwd_rc_supported(N, H, W, Cout, Cin, int(dw_stride), _DT[x.dtype]))


def pw_bwd_gred_parts(M, Cin, Cout, dtype):
    """Part count of rod_pw_bwd_gred for this project shape (0: not taken)."""
    if "pwgred" in _DISABLE:
        return 0
    return int(_abi.lib().rod_pw_bwd_gred_parts(int(M), int(Cin), int(Cout), _DT[dtype]))


def pw_bwd_gred(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, dw, dyp=False, wt0=None):
    """rod_pw_bwd_gred: the project conv's backward through its BatchNorm (dx, dw written in
    place) plus the input BatchNorm's backward sums over (dx, x) -> (dx, [nparts, 2, Cin]).
    dyp=True: rod_pw_bwd_gred_dyp — (dy [M, Cout], parts), dx not written (ABI 20).
    wt0 (the forward operand; the 16 -> 96 expand): rod_pw_bwd_gred_rc — y recomputed, not read."""
    Cin, Cout = x.shape[-1], dz.shape[-1]
    M = dz.numel() // Cout
    nparts = pw_bwd_gred_parts(M, Cin, Cout, x.dtype)
    out = torch.empty((M, Cout), dtype=x.dtype, device=x.device) if dyp else torch.empty_like(x)
    xparts = torch.empty((nparts, 2, Cin), dtype=torch.float32, device=x.device)
    ws = workspace(_abi.query("rod_pw_bwd_gred_workspace", M, Cin, Cout), x.device)
    if wt0 is not None:
        assert not dyp
        _abi.call("rod_pw_bwd_gred_rc", dz, wt0, mean, rstd, gamma, beta, act, coef, x, *_pro_args(xpro), wt1, out, dw,
                  xparts, ws, M, Cin, Cout, dtcode(x), stream())
        return out, xparts
    _abi.call("rod_pw_bwd_gred_dyp" if dyp else "rod_pw_bwd_gred", dz, y, mean, rstd, gamma, beta, act, coef, x,
              *_pro_args(xpro), wt1, out, dw, xparts, ws, M, Cin, Cout, dtcode(y), stream())
    return out, xparts


def dw_pw_ok(src_dw, x, Cout, ipro):
    """The project conv's input x comes from a stride-1 depthwise whose backward can recompute
    its gradient from dy_p (rod_dw3x3_bwd_fused_pw_supported); src_dw = (stride, the depthwise's
    input-prologue activation) recorded by _DWBN.forward."""
    if src_dw is None or "dwpw" in _DISABLE or ipro is None:
        return False
    stride, pro_act = src_dw
    N, H, W, C = x.shape
    return stride == 1 and _dw_fused_ok(N, H, W, C, x.dtype, 1) and \
        bool(_abi.lib().rod_dw3x3_bwd_fused_pw_supported(N, H, W, C, int(Cout), int(pro_act), int(ipro[4]),
                                                         dtcode(x)))


def _bn_backward_parts(dz, y, mean, rstd, gamma, beta, act, parts, need_g, need_b):
    """Finish a BatchNorm backward whose reduction the producer of dz already did in its
    epilogue (gred partial sums): rod_bn_bwd_finalize -> rod_bn_bwd_apply."""
    N, H, W, C = y.shape
    M = N * H * W
    coef = torch.empty(3 * C, dtype=torch.float32, device=y.device)
    dg = grad_slot(gamma) if need_g else None
    db = grad_slot(beta) if need_b else None
    _abi.call("rod_bn_bwd_finalize", parts, parts.shape[0], M, C, rstd, gamma, dg, db, coef, stream())
    dy = torch.empty_like(y)
    _abi.call("rod_bn_bwd_apply", dz, y, mean, rstd, gamma, beta, coef, dy, M, C, act, dtcode(y), stream())
    if need_g:
        _mark_written(gamma)
    if need_b:
        _mark_written(beta)
    return dy


def _gred_args(g):
    """The seven gred arguments (pre-BatchNorm y, mean, rstd, gamma, beta, act, parts)."""
    if g is None:
        return (None, None, None, None, None, 0, None)
    return g


def _split_in(x):
    """(tensor, gamma, beta, mean, rstd, act, training, owned) of a plain tensor or a Pending.
    An owned Pending's gamma / beta are passed detached: its producer writes their gradients."""
    if isinstance(x, Pending):
        if x.owned:
            det = lambda t: None if t is None else t.detach()
            return x.y, det(x.gamma), det(x.beta), x.mean, x.rstd, x.act, x.training, True
        return x.y, x.gamma, x.beta, x.mean, x.rstd, x.act, x.training, False
    return x, None, None, None, None, 0, False, False


# ----------------------------------------------------------------------------- depthwise
class _DW3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, want_stats, gamma, beta, mean, rstd, act, training, owned=False):
        ctx.owned = owned
        N, H, W, C = x.shape
        Ho, pt = same_pad(H, stride)
        Wo, pl = same_pad(W, stride)
        y = torch.empty((N, Ho, Wo, C), dtype=x.dtype, device=x.device)
        parts = None
        if want_stats:  # BatchNorm partial statistics from the epilogue
            nparts = _abi.lib().rod_dw3x3_fwd_stat_parts(N, Ho, Wo, C, stride, dtcode(x))
            parts = torch.empty((nparts, 3, C), dtype=torch.float32, device=x.device)
        pro = (mean, rstd, gamma, beta, act) if mean is not None else None
        _abi.call("rod_dw3x3_fwd", x, *_pro_args(pro), w, y, parts, N, H, W, C, stride, pt, pl, Ho, Wo, dtcode(x),
                  stream())
        ctx.save_for_backward(x, w, gamma, beta, mean, rstd)
        ctx.geo = (N, H, W, C, stride, pt, pl, Ho, Wo)
        ctx.act, ctx.pro, ctx.training = act, pro is not None, training
        if want_stats:
            ctx.mark_non_differentiable(parts)
            ctx.set_materialize_grads(False)
            return y, parts
        return y

    @staticmethod
    def backward(ctx, dy, *_):
        x, w, gamma, beta, mean, rstd = ctx.saved_tensors
        N, H, W, C, s, pt, pl, Ho, Wo = ctx.geo
        dy = dy.contiguous()
        pro = (mean, rstd, gamma, beta, ctx.act) if ctx.pro else None
        need_g = ctx.pro and gamma is not None and ctx.needs_input_grad[4]
        need_b = ctx.pro and beta is not None and ctx.needs_input_grad[5]
        dx = None
        if ctx.needs_input_grad[0] or need_g or need_b:
            if ctx.pro and not ctx.training:
                raise RuntimeError("BatchNorm backward in inference mode is not part of the reference graph")
            dx = torch.empty_like(x)   # gradient wrt the dw input (the BatchNorm output when pro)
            gred = None
            if ctx.pro and "gred" in _ENABLE and not ctx.owned and SYNC_BN is None:   # sums in the epilogue
                nparts = _abi.lib().rod_dw3x3_bwd_data_gred_parts(N, H, W, C, s, dtcode(x))
                parts = torch.empty((nparts, 2, C), dtype=torch.float32, device=x.device)
                gred = (x, mean, rstd, gamma, beta, ctx.act, parts)
            _abi.call("rod_dw3x3_bwd_data", dy, w, dx, *_gred_args(gred), N, H, W, C, s, pt, pl, Ho, Wo, dtcode(x),
                      stream())
        if ctx.needs_input_grad[1]:
            g = grad_slot(w)
            ws = workspace(_abi.query("rod_dw3x3_bwd_filter_workspace", N, Ho, Wo, C), x.device)
            _abi.call("rod_dw3x3_bwd_filter", x, *_pro_args(pro), dy, g, ws, N, H, W, C, s, pt, pl, Ho, Wo,
                      dtcode(x), stream())
            _mark_written(w)
        if ctx.pro and dx is not None and not ctx.owned:
            if gred is not None:
                dx = _bn_backward_parts(dx, x, mean, rstd, gamma, beta, ctx.act, gred[6], need_g, need_b)
            else:
                dx = _bn_backward(dx, x, mean, rstd, gamma, beta, ctx.act, need_g, need_b)
        return dx, None, None, None, None, None, None, None, None, None, None


def dw3x3(x, w, stride=1, want_stats=False):
    """Depthwise 3x3, TF-SAME (conv_blocks.py:238-247).  x: tensor or Pending (the BatchNorm
    of the layer below is then applied in the load prologue).  want_stats: also return the
    BatchNorm partial statistics of the output (for bn_pending(..., parts=))."""
    xt, g, b, m, r, act, tr, own = _split_in(x)
    if want_stats and "dwstats" in _DISABLE:
        return _DW3x3.apply(xt, w, stride, False, g, b, m, r, act, tr, own), None
    return _DW3x3.apply(xt, w, stride, want_stats, g, b, m, r, act, tr, own)


# ----------------------------------------------------------------------------- dense conv
def _prep(w, mode, dtype, Cout, Cin, ks):
    """GEMM operand layout of conv weight w (rod_conv_weight_prep): cached per parameter store
    and refreshed in one batched launch per step; a tensor outside a store is prepared here."""
    store = getattr(w, "_rod_store", None)
    if store is not None and "prepcache" not in _DISABLE:
        return store.prepped(w, mode, dtype, Cout, Cin, ks)
    wt = torch.empty((Cout, ks * ks * Cin) if mode == 0 else (Cin, ks * ks * Cout), dtype=dtype, device=w.device)
    _abi.call("rod_conv_weight_prep", w, wt, Cout, Cin, ks, mode, dtcode(wt), stream())
    return wt


def conv_fwd_raw(x, wt, b, y, N, H, W, Cin, Cout, ksize, stat_parts=None, pro=None, gred=None):
    """rod_conv_fwd with its split-K workspace (allocated only when the plan splits)."""
    nb = 0 if "splitk" in _DISABLE else _abi.query("rod_conv_fwd_workspace", N, H, W, Cin, Cout, ksize)
    ws = workspace(nb, x.device) if nb else None
    _abi.call("rod_conv_fwd", x, *_pro_args(pro), wt, b, y, ws, stat_parts, *_gred_args(gred), N, H, W, Cin, Cout,
              ksize, 0, 0, dtcode(x), stream())


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, ksize, want_stats, gamma, beta, mean, rstd, act, training, owned=False):
        ctx.owned = owned
        N, H, W, Cin = x.shape
        Cout = w.shape[0]
        assert w.shape == (Cout, ksize, ksize, Cin), (tuple(w.shape), ksize, Cin)
        wt = _prep(w, 0, x.dtype, Cout, Cin, ksize)
        y = torch.empty((N, H, W, Cout), dtype=x.dtype, device=x.device)
        parts = None
        if want_stats:  # BatchNorm partial statistics from the epilogue ([ceil(M/128)][3][Cout])
            parts = torch.empty((-(-(N * H * W) // 128), 3, Cout), dtype=torch.float32, device=x.device)
        pro = (mean, rstd, gamma, beta, act) if mean is not None else None
        conv_fwd_raw(x, wt, b, y, N, H, W, Cin, Cout, ksize, parts, pro)
        ctx.save_for_backward(x, w, b, gamma, beta, mean, rstd)
        ctx.ksize = ksize
        ctx.act, ctx.pro, ctx.training = act, pro is not None, training
        if want_stats:
            ctx.mark_non_differentiable(parts)
            ctx.set_materialize_grads(False)
            return y, parts
        return y

    @staticmethod
    def backward(ctx, dy, *_):
        x, w, b, gamma, beta, mean, rstd = ctx.saved_tensors
        ks = ctx.ksize
        N, H, W, Cin = x.shape
        Cout = w.shape[0]
        dy = dy.contiguous()
        pro = (mean, rstd, gamma, beta, ctx.act) if ctx.pro else None
        need_g = ctx.pro and gamma is not None and ctx.needs_input_grad[5]
        need_b = ctx.pro and beta is not None and ctx.needs_input_grad[6]
        dx = None
        if ctx.needs_input_grad[0] or need_g or need_b:
            if ctx.pro and not ctx.training:
                raise RuntimeError("BatchNorm backward in inference mode is not part of the reference graph")
            wt1 = _prep(w, 1, x.dtype, Cout, Cin, ks)
            dx = torch.empty_like(x)   # gradient wrt the conv input (the BatchNorm output when pro)
            gred = None
            if ctx.pro and "gred" in _ENABLE and not ctx.owned and SYNC_BN is None:   # sums in the epilogue
                parts = torch.empty((-(-(N * H * W) // 128), 2, Cin), dtype=torch.float32, device=x.device)
                gred = (x, mean, rstd, gamma, beta, ctx.act, parts)
            conv_fwd_raw(dy, wt1, None, dx, N, H, W, Cout, Cin, ks, gred=gred)
        need_w = ctx.needs_input_grad[1]
        need_bias = b is not None and ctx.needs_input_grad[2]
        if need_w or need_bias:
            gw = grad_slot(w) if need_w else None
            if gw is None:  # bias-only gradient still needs a scratch dW
                gw = torch.empty(w.shape, dtype=torch.float32, device=x.device)
            gb = grad_slot(b) if need_bias else None
            ws = workspace(_abi.query("rod_conv_wgrad_workspace", N, H, W, Cin, Cout, ks), x.device)
            _abi.call("rod_conv_wgrad", x, *_pro_args(pro), dy, gw, gb, ws, N, H, W, Cin, Cout, ks, 0, 0, dtcode(x),
                      stream())
            if need_w:
                _mark_written(w)
            if need_bias:
                _mark_written(b)
        if ctx.pro and dx is not None and not ctx.owned:
            if gred is not None:
                dx = _bn_backward_parts(dx, x, mean, rstd, gamma, beta, ctx.act, gred[6], need_g, need_b)
            else:
                dx = _bn_backward(dx, x, mean, rstd, gamma, beta, ctx.act, need_g, need_b)
        return dx, None, None, None, None, None, None, None, None, None, None, None


def conv2d(x, w, b=None, ksize=1, want_stats=False):
    """slim.conv2d, stride 1, SAME (1x1 or 3x3), NHWC.  x: tensor or Pending (BatchNorm of the
    layer below applied in the load prologue).  want_stats: also return the BatchNorm partial
    statistics of the output (for bn_pending(..., parts=))."""
    xt, g, bb, m, r, act, tr, own = _split_in(x)
    if want_stats and "convstats" in _DISABLE:
        return _Conv.apply(xt, w, b, ksize, False, g, bb, m, r, act, tr, own), None
    return _Conv.apply(xt, w, b, ksize, want_stats, g, bb, m, r, act, tr, own)


# ----------------------------------------------------------------------------- batch norm
def bn_statistics(x, mmean, mvar, training, decay, eps=1e-3, parts=None):
    """(mean, rstd) fp32 [C] of slim.batch_norm: batch statistics (+ moving-average update)
    in training — from the producer's partial statistics when given — else the moving ones."""
    C = x.shape[-1]
    M = x.numel() // C
    mean = torch.empty(C, dtype=torch.float32, device=x.device)
    rstd = torch.empty(C, dtype=torch.float32, device=x.device)
    if "epistats" in _DISABLE:
        parts = None
    if training and SYNC_BN is not None:   # statistics over the global batch (all ranks' parts)
        if parts is None:
            nparts = _sync_nparts(M)
            parts = torch.empty((nparts, 3, C), dtype=torch.float32, device=x.device)
            _abi.call("rod_bn_stat_parts", x.contiguous(), M, C, parts, nparts, dtcode(x), stream())
        gp = SYNC_BN.gather(parts)
        nb = _abi.query("rod_bn_finalize_workspace", gp.shape[0], C)
        ws = workspace(nb, x.device) if nb else None
        _abi.call("rod_bn_finalize", gp, gp.shape[0], M * SYNC_BN.world, C, eps, decay, mean, rstd, mmean, mvar, ws,
                  stream())
    elif training and parts is not None:  # statistics already reduced by the producer's epilogue
        nb = _abi.query("rod_bn_finalize_workspace", parts.shape[0], C)
        ws = workspace(nb, x.device) if nb else None
        _abi.call("rod_bn_finalize", parts, parts.shape[0], M, C, eps, decay, mean, rstd, mmean, mvar, ws, stream())
    elif training:
        ws = workspace(_abi.query("rod_bn_stats_workspace", M, C), x.device)
        _abi.call("rod_bn_stats", x, M, C, 0, eps, decay, mean, rstd, mmean, mvar, ws, dtcode(x), stream())
    else:
        hit = _eval_cached(mmean, mvar, eps)
        if hit is not None:
            return hit
        _abi.call("rod_bn_eval_stats", mmean, mvar, eps, mean, rstd, C, stream())
    return mean, rstd


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, mean, rstd, act, training):
        N, H, W, C = x.shape
        M = N * H * W
        y = torch.empty_like(x)
        _abi.call("rod_bn_apply", x, mean, rstd, gamma, beta, residual, y, M, C, 0, 0, 0, act, dtcode(x),
                  stream())
        ctx.save_for_backward(x, mean, rstd, gamma, beta)
        ctx.act = act
        ctx.training = training
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, gamma, beta = ctx.saved_tensors
        if not ctx.training:
            raise RuntimeError("BatchNorm backward in inference mode is not part of the reference graph")
        need_g = gamma is not None and ctx.needs_input_grad[1]
        need_b = beta is not None and ctx.needs_input_grad[2]
        dx = _bn_backward(dy, x, mean, rstd, gamma, beta, ctx.act, need_g, need_b)
        dres = dy if ctx.has_res else None
        return dx, None, None, dres, None, None, None, None


def bn_pending(x, gamma, beta, mmean, mvar, act, training, decay, eps=1e-3, parts=None):
    """slim.batch_norm (fused) + activation, left for the consumer's load prologue."""
    mean, rstd = bn_statistics(x, mmean, mvar, training, decay, eps, parts)
    return Pending(x, mean, rstd, gamma, beta, act, training)


def materialize(p, residual=None):
    """Write act(BatchNorm(y)) (+ residual after the activation) of a Pending."""
    if isinstance(p, Pending) and getattr(p.y, "_rod_nostore", False):
        raise RuntimeError("an unwritten expand output (ABI 23 recompute) cannot be materialised")
    if not isinstance(p, Pending):
        return p
    if p.owned:
        det = lambda t: None if t is None else t.detach()
        return _BNApplyOwned.apply(p.y, residual, p.mean, p.rstd, det(p.gamma), det(p.beta), p.act)
    return _BNAct.apply(p.y, p.gamma, p.beta, residual, p.mean, p.rstd, p.act, p.training)


def bn_act(x, gamma, beta, mmean, mvar, act, training, decay, eps=1e-3, residual=None, parts=None):
    """slim.batch_norm (fused) + activation (+ residual add after the activation), written out.
    parts: partial statistics of x from its producer (conv2d(..., want_stats=True))."""
    return materialize(bn_pending(x, gamma, beta, mmean, mvar, act, training, decay, eps, parts), residual)


# ----------------------------------------------------------------------------- conv / dw + BatchNorm nodes
# A conv (or depthwise conv) and the slim.batch_norm that follows it are ONE autograd node
# whose output is an owned Pending: consumers apply the BatchNorm in their load prologue and
# hand back d/d(act(BN(y))) untouched; this node's backward runs the BatchNorm backward and
# the conv backward together, so a 1x1 conv can take the fused rod_pw_bwd path (dy never
# written) and the others at least skip nothing they did before.

def _bn_bwd_apply(dz, y, mean, rstd, gamma, beta, act, coef):
    C = y.shape[-1]
    dy = torch.empty_like(y)
    _abi.call("rod_bn_bwd_apply", dz.contiguous(), y, mean, rstd, gamma, beta, coef, dy, y.numel() // C, C, act,
              dtcode(y), stream())
    return dy


def _needs(p):
    return p is not None and p.requires_grad


def bn_bwd_dy(dz, y, mean, rstd, gamma, beta, act, need_g, need_b):
    """d/dy of act(BN(y)) from dz, dgamma / dbeta into their slots.  Small tensors (<= 4096
    rows: the deep maps and the heads' last levels) take rod_bn_bwd, which runs the reduction,
    the coefficients and the apply in one launch; larger ones rod_bn_bwd_reduce (reduce +
    finalize) then rod_bn_bwd_apply."""
    C = y.shape[-1]
    M = y.numel() // C
    if M <= 4096 and SYNC_BN is None:
        return _bn_backward(dz, y, mean, rstd, gamma, beta, act, need_g, need_b)
    coef = bn_bwd_reduce(dz.contiguous(), y, mean, rstd, gamma, beta, act, need_g, need_b)
    return _bn_bwd_apply(dz, y, mean, rstd, gamma, beta, act, coef)


# fused 1x1 backward where it measured faster than the unfused chain (tools/pwbwd_bench.py):
# the expand-shaped convs (Cout >= 2 Cin) on >= 200k rows
def _pw_fused_ok(M, Cin, Cout, dtype):
    return M >= 200_000 and Cout >= 2 * Cin and pw_bwd_supported(Cin, Cout, dtype)


def _bwd_data_bn_ok(M, Cout, Cin, dtype, ipro):
    # the opt-in gred form of the backward-data (ROD_ENABLE=gredpw, below) keeps the two-launch
    # chain, and so do the shapes whose plain backward-data takes the K <= 96 streaming kernel
    return "bnbwd" not in _DISABLE and not (ipro is not None and "gredpw" in _ENABLE) and \
        bool(_abi.lib().rod_conv_bwd_data_bn_supported(int(Cout), int(Cin), _DT[dtype])) and \
        not _abi.lib().rod_conv_fwd_stream_ok(int(M), int(Cout), int(Cin), _DT[dtype])


def conv_bwd_data_bn(dz, y, mean, rstd, gamma, beta, act, coef, w):
    """rod_conv_bwd_data_bn (ABI 22): (dy, dx) of a 1x1 conv + BatchNorm — dy the BatchNorm-
    backward apply of (dz, y) (written), dx = dy . W — bit-identical to rod_bn_bwd_apply followed
    by rod_conv_fwd with the mode-1 weights."""
    N, H, W_, Cout = y.shape
    Cin = w.shape[-1]
    M = N * H * W_
    wt1 = _prep(w, 1, y.dtype, Cout, Cin, 1)
    dy = torch.empty_like(y)
    dx = torch.empty((N, H, W_, Cin), dtype=y.dtype, device=y.device)
    nb = 0 if "splitk" in _DISABLE else _abi.query("rod_conv_fwd_workspace", 1, 1, M, Cout, Cin, 1)
    ws = workspace(nb, y.device) if nb else None
    _abi.call("rod_conv_bwd_data_bn", dz.contiguous(), y, mean, rstd, gamma, beta, act, coef, wt1, dy, dx, ws, M,
              Cout, Cin, dtcode(y), stream())
    return dy, dx


def _conv_bwd_from_dy(x, w, b, ks, dy, pro, need_dx):
    """rod_conv_fwd (mode-1 weights) for dx and rod_conv_wgrad for dw / db from a dense dy
    (the weight gradient on the side stream when SIDE is on)."""
    N, H, W, Cin = x.shape
    Cout = w.shape[0]
    need_w, need_bias = _needs(w), _needs(b)
    if need_w or need_bias:
        gw = grad_slot(w) if need_w else torch.empty(w.shape, dtype=torch.float32, device=x.device)
        gb = grad_slot(b) if need_bias else None

        def wgrad():
            ws = workspace(_abi.query("rod_conv_wgrad_workspace", N, H, W, Cin, Cout, ks), x.device)
            _abi.call("rod_conv_wgrad", x, *_pro_args(pro), dy, gw, gb, ws, N, H, W, Cin, Cout, ks, 0, 0,
                      dtcode(x), stream())
        SIDE.run(wgrad, x, dy, gw, pro)
        if need_w:
            _mark_written(w)
        if need_bias:
            _mark_written(b)
    dx = None
    if need_dx:
        wt1 = _prep(w, 1, x.dtype, Cout, Cin, ks)
        dx = torch.empty_like(x)
        gred = None
        if pro is not None and ks == 1 and "gredpw" in _ENABLE and \
                _abi.lib().rod_conv_fwd_stream_ok(N * H * W, Cout, Cin, dtcode(x)):
            # opt-in (ROD_ENABLE=gredpw): dx is the gradient of the input's BatchNorm output (an
            # owned Pending: the depthwise BatchNorm of the block, conv_blocks.py:238-247); the
            # streaming backward-data also forms that BatchNorm's backward sums over (dx, x),
            # handed to its producer (_DWBN), which then skips its rod_bn_bwd_reduce pass.
            # Correct (tests/test_gpu_gred.py, the step tests) but measured no faster: the
            # reduce passes it removes (-0.8 ms) come back as backward-data time (+0.6-0.8 ms:
            # the extra read of x at ~3 TB/s, narrow N groups re-reading dy), DESIGN.md §6
            parts = torch.empty((-(-(N * H * W) // 128), 2, Cin), dtype=torch.float32, device=x.device)
            gred = (x,) + tuple(pro) + (parts,)
        conv_fwd_raw(dy, wt1, None, dx, N, H, W, Cout, Cin, ks, gred=gred)
        if gred is not None:
            _put_bn_parts(dx, gred[-1])
    return dx


class _ConvBN(torch.autograd.Function):
    """slim.conv2d (1x1 / 3x3, stride 1, SAME, optional bias) + slim.batch_norm as one node.
    obn = (gamma, beta, moving_mean, moving_var, act, training, decay, eps); ipro = the input's
    BatchNorm prologue (mean, rstd, gamma, beta, act) when the input is an owned Pending."""

    @staticmethod
    def forward(ctx, x, w, b, ks, ipro, obn, dw_stride=0):
        gamma, beta, mm, mv, act, training, decay, eps = obn
        N, H, W, Cin = x.shape
        Cout = w.shape[0]
        assert w.shape == (Cout, ks, ks, Cin), (tuple(w.shape), ks, Cin)
        wt = _prep(w, 0, x.dtype, Cout, Cin, ks)
        ctx.nostore = training and ks == 1 and b is None and act == ROD_ACT_RELU6 and \
            _nostore_ok(x, ipro, N, H, W, Cin, Cout, dw_stride)
        if not training and ks == 1 and b is None and act == ROD_ACT_RELU6 and \
                _nostore_eval_ok(x, N, H, W, Cin, Cout, dw_stride):
            # inference: nothing is computed here; the depthwise forms the values from x
            y = torch.empty(1, dtype=x.dtype, device=x.device).expand(N, H, W, Cout)
            y._rod_expand = (x, ipro, wt, Cin)
            y._rod_nostore = True
            mean, rstd = bn_statistics(y, mm, mv, False, decay, eps)
            ctx.training = False
            ctx.mark_non_differentiable(mean, rstd)
            return y, mean, rstd
        if ctx.nostore:
            # the expanded tensor is never written (ABI 23): a placeholder of its shape that no
            # kernel reads (its consumers recompute it from x), the statistics from x alone
            y = torch.empty(1, dtype=x.dtype, device=x.device).expand(N, H, W, Cout)
            parts = torch.empty((-(-(N * H * W) // 128), 3, Cout), dtype=torch.float32, device=x.device)
            _abi.call("rod_conv_fwd_stats", x, *_pro_args(ipro), wt, parts, N * H * W, Cin, Cout, dtcode(x), stream())
            y._rod_expand = (x, ipro, wt, Cin)
            y._rod_nostore = True
            mean, rstd = bn_statistics(y, mm, mv, training, decay, eps, parts)
            ctx.src_dw = None
            ctx.save_for_backward(x, w, b, y, mean, rstd)
            ctx.ks, ctx.ipro, ctx.gb, ctx.act, ctx.training = ks, ipro, (gamma, beta), act, training
            ctx.mark_non_differentiable(mean, rstd)
            ctx.set_materialize_grads(False)
            return y, mean, rstd
        y = torch.empty((N, H, W, Cout), dtype=x.dtype, device=x.device)
        parts = None
        if training:
            parts = torch.empty((-(-(N * H * W) // 128), 3, Cout), dtype=torch.float32, device=x.device)
        if ks == 3 and ipro is not None and N * H * W >= 16384 and "pro3" not in _DISABLE:
            # a 3x3 conv gathers each input element for 9 taps, so its load prologue would apply
            # the input BatchNorm 9 times per element: write act(BN(x)) once instead (the same
            # rounded values) and use it for the forward and the weight gradient
            # (the heads' 128 -> 128 convs, catch_net.py:301-304)
            xb = torch.empty_like(x)
            im, ir, ig, ib, ia = ipro
            _abi.call("rod_bn_apply", x, im, ir, ig, ib, None, xb, N * H * W, Cin, 0, 0, 0, ia, dtcode(x), stream())
            x, ipro = xb, None
        ctx.src_dw = getattr(x, "_rod_dw", None)   # x is a depthwise output (_DWBN.forward)
        conv_fwd_raw(x, wt, b, y, N, H, W, Cin, Cout, ks, parts, ipro)
        if ks == 1 and b is None and training and x.dtype == torch.bfloat16 and Cin <= 32:
            # an expand conv: the consumer depthwise may recompute y from x (dw_rc_ok, ABI 23)
            y._rod_expand = (x, ipro, wt, Cin)
        mean, rstd = bn_statistics(y, mm, mv, training, decay, eps, parts)
        ctx.save_for_backward(x, w, b, y, mean, rstd)
        ctx.ks, ctx.ipro, ctx.gb, ctx.act, ctx.training = ks, ipro, (gamma, beta), act, training
        ctx.mark_non_differentiable(mean, rstd)
        ctx.set_materialize_grads(False)
        return y, mean, rstd

    @staticmethod
    def backward(ctx, dz, *_):
        if dz is None:
            return None, None, None, None, None, None, None
        if not ctx.training:
            raise RuntimeError("BatchNorm backward in inference mode is not part of the reference graph")
        x, w, b, y, mean, rstd = ctx.saved_tensors
        gamma, beta = ctx.gb
        N, H, W, Cin = x.shape
        Cout = w.shape[0]
        M = N * H * W
        dz = dz.contiguous()
        need_dx = ctx.needs_input_grad[0]
        parts = _take_bn_parts(dz)   # the BN sums a fused depthwise backward already formed
        if ctx.nostore and parts is None:
            raise RuntimeError("expand conv without a stored output: its BatchNorm-backward sums must come from the "
                               "depthwise backward (rod_dw3x3_bwd_fused_rc)")
        if ctx.ks == 1 and b is None and ctx.ipro is not None and need_dx and _needs(w) and \
                M >= 65536 and SYNC_BN is None and pw_bwd_gred_parts(M, Cin, Cout, y.dtype) > 0:
            # the project conv of an inverted-residual block (conv_blocks.py:287-294): one pass for
            # its BatchNorm backward apply, dgrad and wgrad, which also forms the backward sums of
            # the depthwise BatchNorm whose output it consumed (ipro) over (dx, x) — handed to that
            # BatchNorm's node (_DWBN), which then skips its rod_bn_bwd_reduce pass.  The expand
            # 16 -> 96 takes the same entry: its input is the previous block's project output, whose
            # linear BatchNorm then gets its sums from here (when dx is that BatchNorm's whole
            # gradient: no residual path adds to it — _take_bn_parts checks)
            if parts is not None:
                coef = bn_bwd_coef_from_parts(parts, M, Cout, rstd, gamma, beta, _needs(gamma), _needs(beta))
            else:
                coef = bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, ctx.act, _needs(gamma), _needs(beta))
            wt1 = _prep(w, 1, x.dtype, Cout, Cin, 1)
            if dw_pw_ok(ctx.src_dw, x, Cout, ctx.ipro):
                # the depthwise recomputes dx = dy . W per tile (rod_dw3x3_bwd_fused_pw): hand it
                # dy and W^T, return an unwritten placeholder of dx's shape (_DZ_RECIPE)
                dyp, xparts = pw_bwd_gred(dz, y, mean, rstd, gamma, beta, ctx.act, coef, x, ctx.ipro, wt1,
                                          grad_slot(w), dyp=True)
                _mark_written(w)
                dx = torch.empty(1, dtype=x.dtype, device=x.device).expand(x.shape)
                _put_dz_recipe(dx, (dyp, wt1, Cout))
                _put_bn_parts(dx, xparts)
                return dx, None, None, None, None, None, None
            # the 16 -> 96 expand: its pre-BatchNorm y recomputed from x in the kernel (ABI 23)
            wt0 = _prep(w, 0, x.dtype, Cout, Cin, 1) if ctx.nostore or pw_bwd_rc_ok(M, Cin, Cout, x.dtype) else None
            dx, xparts = pw_bwd_gred(dz, y, mean, rstd, gamma, beta, ctx.act, coef, x, ctx.ipro, wt1, grad_slot(w),
                                     wt0=wt0)
            _mark_written(w)
            _put_bn_parts(dx, xparts)
            return dx, None, None, None, None, None, None
        if ctx.nostore and not (ctx.ks == 1 and _pw_fused_ok(M, Cin, Cout, y.dtype) and (need_dx or _needs(w))):
            raise RuntimeError("expand conv without a stored output reached a backward path that reads it")
        if ctx.ks == 3 and not need_dx and b is None and ctx.ipro is None and _needs(w) and \
                "stembn" not in _DISABLE and _abi.lib().rod_stem_wgrad_bn_supported(Cin, Cout, 3, dtcode(y)):
            # the stem (mobilenet_v2.py:58 + its batch_norm): the weight gradient forms dy from the
            # BatchNorm's (dz, y) in its loader — the [M, 32] dy is never written (rod_stem_wgrad_bn)
            if parts is not None:
                coef = bn_bwd_coef_from_parts(parts, M, Cout, rstd, gamma, beta, _needs(gamma), _needs(beta))
            else:
                coef = bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, ctx.act, _needs(gamma), _needs(beta))
            ws = workspace(_abi.query("rod_conv_wgrad_workspace", N, H, W, Cin, Cout, 3), x.device)
            _abi.call("rod_stem_wgrad_bn", x, dz, y, mean, rstd, gamma, beta, ctx.act, coef, grad_slot(w), ws, N, H,
                      W, Cin, Cout, 3, dtcode(y), stream())
            _mark_written(w)
            return None, None, None, None, None, None, None
        if ctx.ks == 1 and _pw_fused_ok(M, Cin, Cout, y.dtype) and (need_dx or _needs(w) or _needs(b)):
            if parts is not None:
                coef = bn_bwd_coef_from_parts(parts, M, Cout, rstd, gamma, beta, _needs(gamma), _needs(beta))
            else:
                coef = bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, ctx.act, _needs(gamma), _needs(beta))
            gw = grad_slot(w) if _needs(w) else torch.empty((Cout, Cin), dtype=torch.float32, device=y.device)
            gb = grad_slot(b) if _needs(b) else None
            wt1 = _prep(w, 1, x.dtype, Cout, Cin, 1) if need_dx else None
            # the streaming expand shapes (16 -> 96, 24 -> 144): y recomputed from x (ABI 23)
            wt0 = _prep(w, 0, x.dtype, Cout, Cin, 1) \
                if gb is None and (ctx.nostore or pw_bwd_rc_ok(M, Cin, Cout, x.dtype)) else None
            dx = pw_bwd(dz, y, mean, rstd, gamma, beta, ctx.act, coef, x, ctx.ipro, wt1, need_dx, gw, gb, wt0=wt0)
            if _needs(w):
                _mark_written(w)
            if _needs(b):
                _mark_written(b)
        elif ctx.ks == 1 and need_dx and (parts is not None or M > 4096 or SYNC_BN is not None) and \
                _bwd_data_bn_ok(M, Cout, Cin, y.dtype, ctx.ipro):
            # the deep expand convs (64 -> 384, 96 -> 576, 160 -> 960, conv_blocks.py:263-294): the
            # backward-data GEMM forms dy = the BatchNorm-backward apply in its loader and writes it
            # once for the weight gradient (rod_conv_bwd_data_bn) — no rod_bn_bwd_apply launch
            if parts is not None:
                coef = bn_bwd_coef_from_parts(parts, M, Cout, rstd, gamma, beta, _needs(gamma), _needs(beta))
            else:
                coef = bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, ctx.act, _needs(gamma), _needs(beta))
            dy, dx = conv_bwd_data_bn(dz, y, mean, rstd, gamma, beta, ctx.act, coef, w)
            _conv_bwd_from_dy(x, w, b, ctx.ks, dy, ctx.ipro, False)
        else:
            if parts is not None:
                coef = bn_bwd_coef_from_parts(parts, M, Cout, rstd, gamma, beta, _needs(gamma), _needs(beta))
                dy = _bn_bwd_apply(dz, y, mean, rstd, gamma, beta, ctx.act, coef)
            else:
                dy = bn_bwd_dy(dz, y, mean, rstd, gamma, beta, ctx.act, _needs(gamma), _needs(beta))
            dx = _conv_bwd_from_dy(x, w, b, ctx.ks, dy, ctx.ipro, need_dx)
        return dx, None, None, None, None, None, None


class _DWBN(torch.autograd.Function):
    """DepthwiseConv2dNative 3x3 (TF-SAME, stride s) + slim.batch_norm as one node
    (conv_blocks.py:238-247); the input may be an owned Pending (ipro)."""

    @staticmethod
    def forward(ctx, x, w, stride, ipro, obn):
        gamma, beta, mm, mv, act, training, decay, eps = obn
        N, H, W, C = x.shape
        Ho, pt = same_pad(H, stride)
        Wo, pl = same_pad(W, stride)
        y = torch.empty((N, Ho, Wo, C), dtype=x.dtype, device=x.device)
        parts = None
        if training:
            nparts = _abi.lib().rod_dw3x3_fwd_stat_parts(N, Ho, Wo, C, stride, dtcode(x))
            parts = torch.empty((nparts, 3, C), dtype=torch.float32, device=x.device)
        nostore = getattr(x, "_rod_nostore", False)
        rc = dw_rc_ok(x, N, H, W, C, stride) if ipro is not None and ipro[4] == ROD_ACT_RELU6 else None
        if nostore:
            rc = x._rod_expand   # the input was never written: recompute (checked by _nostore_ok)
        ctx.rc_src = rc if nostore else None
        if rc is not None:
            # the expanded input recomputed from the block input, never read (ABI 23)
            xin, xpro, wt0, Cin = rc
            _abi.call("rod_dw3x3_fwd_rc", xin, *_pro_args(xpro), wt0, Cin, *_pro_args(ipro), w, y, parts, N, H, W, C,
                      stride, pt, pl, Ho, Wo, dtcode(x), stream())
        else:
            _abi.call("rod_dw3x3_fwd", x, *_pro_args(ipro), w, y, parts, N, H, W, C, stride, pt, pl, Ho, Wo,
                      dtcode(x), stream())
        y._rod_dw = (stride, ipro[4] if ipro is not None else -1)   # for the consumer's backward (dw_pw_ok)
        mean, rstd = bn_statistics(y, mm, mv, training, decay, eps, parts)
        ctx.save_for_backward(x, w, y, mean, rstd)
        ctx.geo = (N, H, W, C, stride, pt, pl, Ho, Wo)
        ctx.ipro, ctx.gb, ctx.act, ctx.training = ipro, (gamma, beta), act, training
        ctx.mark_non_differentiable(mean, rstd)
        ctx.set_materialize_grads(False)
        return y, mean, rstd

    @staticmethod
    def backward(ctx, dz, *_):
        if dz is None:
            return None, None, None, None, None
        if not ctx.training:
            raise RuntimeError("BatchNorm backward in inference mode is not part of the reference graph")
        x, w, y, mean, rstd = ctx.saved_tensors
        gamma, beta = ctx.gb
        N, H, W, C, s, pt, pl, Ho, Wo = ctx.geo
        # the BatchNorm-backward sums of (dz, y) when the consumer's backward-data formed them
        # (the project conv's streaming kernel, _conv_bwd_from_dy)
        parts = _take_bn_parts(dz)
        recipe = _take_dz_recipe(dz)   # dz unmaterialised: dy_p, W_p^T of the project (ABI 20)
        if recipe is not None and _needs(w) and ctx.needs_input_grad[0] and s == 1 and ctx.ipro is not None and \
                _dw_fused_ok(N, Ho, Wo, C, x.dtype, s):
            coef = bn_bwd_coef_from_parts(parts, N * Ho * Wo, C, rstd, gamma, beta, _needs(gamma), _needs(beta)) \
                if parts is not None else None
            if coef is not None:
                dyp, wt1, cout = recipe
                dx = torch.empty_like(x)
                gparts = torch.empty((_abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, 1, 1, 1), 2, C),
                                     dtype=torch.float32, device=x.device)
                ws = workspace(_abi.query("rod_dw3x3_bwd_fused_workspace", N, H, W, C, 1, 1, 1), x.device)
                det = lambda t: None if t is None else t.detach()
                _abi.call("rod_dw3x3_bwd_fused_pw", x, *_pro_args(ctx.ipro), dyp, wt1, cout, y, mean, rstd,
                          det(gamma), det(beta), ctx.act, coef, w, dx, grad_slot(w), gparts, ws, N, H, W, C,
                          dtcode(x), stream())
                _mark_written(w)
                _put_bn_parts(dx, gparts)
                return dx, None, None, None, None
        if recipe is not None:   # any other path: the dz the project would have written
            dz = _materialize_dz(recipe, (N, Ho, Wo, C), y.dtype)
            if parts is not None:
                _put_bn_parts(dz, parts)
                parts = _take_bn_parts(dz)

        def coef_d():
            if parts is not None:
                return bn_bwd_coef_from_parts(parts, N * Ho * Wo, C, rstd, gamma, beta, _needs(gamma), _needs(beta))
            return bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, ctx.act, _needs(gamma), _needs(beta))
        if ctx.rc_src is not None:
            # the input (the expand's output) was never written: the stride-2 fused backward
            # recomputes it from the block input (ABI 23)
            if not (_needs(w) and ctx.needs_input_grad[0] and ctx.ipro is not None and s == 2):
                raise RuntimeError("depthwise over an unwritten expand output needs the fused stride-2 backward")
            xin, xpro, wt0, Cin = ctx.rc_src
            dz = dz.contiguous()
            coef = coef_d()
            dx = torch.empty(x.shape, dtype=x.dtype, device=x.device)
            gparts = torch.empty((_abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, s, pt, pl), 2, C),
                                 dtype=torch.float32, device=x.device)
            ws = workspace(_abi.query("rod_dw3x3_bwd_fused_workspace", N, H, W, C, s, pt, pl), x.device)
            det = lambda t: None if t is None else t.detach()
            _abi.call("rod_dw3x3_bwd_fused_rc", xin, *_pro_args(xpro), wt0, Cin, *_pro_args(ctx.ipro), dz, y, mean, rstd,
                      det(gamma), det(beta), ctx.act, coef, w, dx, grad_slot(w), gparts, ws, N, H, W, C, s, pt, pl,
                      Ho, Wo, dtcode(dz), stream())
            _mark_written(w)
            _put_bn_parts(dx, gparts)
            return dx, None, None, None, None
        if _needs(w) and ctx.needs_input_grad[0] and _dw_fused_ok(N, Ho, Wo, C, x.dtype, s):
            # one pass: BN_d backward apply + backward-data + filter gradient (+ the input
            # BatchNorm's backward sums, handed to the producer) — rod_dw3x3_bwd_fused
            # (ABI 12 stride 1, ABI 13 stride 2)
            dz = dz.contiguous()
            coef = coef_d()
            dx = torch.empty_like(x)
            gparts = None
            if ctx.ipro is not None:
                gparts = torch.empty((_abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, s, pt, pl), 2, C),
                                     dtype=torch.float32, device=x.device)
            ws = workspace(_abi.query("rod_dw3x3_bwd_fused_workspace", N, H, W, C, s, pt, pl), x.device)
            det = lambda t: None if t is None else t.detach()
            _abi.call("rod_dw3x3_bwd_fused", x, *_pro_args(ctx.ipro), dz, y, mean, rstd, det(gamma), det(beta),
                      ctx.act, coef, w, dx, grad_slot(w), gparts, ws, N, H, W, C, s, pt, pl, Ho, Wo, dtcode(x),
                      stream())
            _mark_written(w)
            if gparts is not None:
                _put_bn_parts(dx, gparts)
            return dx, None, None, None, None
        if _needs(w) and N * Ho * Wo > 4096 and "dwbn" in _ENABLE:
            # opt-in (ROD_ENABLE=dwbn): the BatchNorm-backward apply runs inside the filter
            # gradient, which writes dy for the backward-data pass (rod_dw3x3_bwd_filter_bn).
            # Bit-identical, but measured no faster per step: the apply pass it
            # removes (-1.59 ms) comes back as filter-gradient time (+1.22 ms, VALU-bound)
            dz = dz.contiguous()
            coef = coef_d()
            dy = torch.empty_like(y)
            ws = workspace(_abi.query("rod_dw3x3_bwd_filter_workspace", N, Ho, Wo, C), x.device)
            det = lambda t: None if t is None else t.detach()
            _abi.call("rod_dw3x3_bwd_filter_bn", x, *_pro_args(ctx.ipro), dz, y, mean, rstd, det(gamma), det(beta),
                      ctx.act, coef, dy, grad_slot(w), ws, N, H, W, C, s, pt, pl, Ho, Wo, dtcode(x), stream())
            _mark_written(w)
            dx = None
            if ctx.needs_input_grad[0]:
                dx = torch.empty_like(x)
                _abi.call("rod_dw3x3_bwd_data", dy, w, dx, *_gred_args(None), N, H, W, C, s, pt, pl, Ho, Wo,
                          dtcode(x), stream())
            return dx, None, None, None, None
        if parts is not None:
            dy = _bn_bwd_apply(dz, y, mean, rstd, gamma, beta, ctx.act, coef_d())
        else:
            dy = bn_bwd_dy(dz, y, mean, rstd, gamma, beta, ctx.act, _needs(gamma), _needs(beta))
        if _needs(w):
            def filt():
                ws = workspace(_abi.query("rod_dw3x3_bwd_filter_workspace", N, Ho, Wo, C), x.device)
                _abi.call("rod_dw3x3_bwd_filter", x, *_pro_args(ctx.ipro), dy, grad_slot(w), ws, N, H, W, C, s, pt,
                          pl, Ho, Wo, dtcode(x), stream())
            SIDE.run(filt, x, dy, ctx.ipro)
            _mark_written(w)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _abi.call("rod_dw3x3_bwd_data", dy, w, dx, *_gred_args(None), N, H, W, C, s, pt, pl, Ho, Wo, dtcode(x),
                      stream())
        return dx, None, None, None, None


def _dw_fused_ok(N, Ho, Wo, C, dtype, stride=1):
    """rod_dw3x3_bwd_fused for a depthwise backward (ROD_DISABLE=dwfused: the unfused chain;
    ROD_DISABLE=dwfused2: stride 1 only); output maps of <= DW_FUSED_MIN rows keep the
    one-launch small-tensor BatchNorm backward."""
    if stride == 2 and "dwfused2" in _DISABLE:
        return False
    return "dwfused" not in _DISABLE and C % 4 == 0 and N * Ho * Wo > DW_FUSED_MIN and \
        dtype in (torch.float32, torch.bfloat16)


DW_FUSED_MIN = int(os.environ.get("ROD_DW_FUSED_MIN", "4096"))


def _in_pro(x):
    """(tensor, prologue tuple or None) of a node input: plain tensor or owned Pending."""
    if isinstance(x, Pending):
        if not x.owned:
            raise ValueError("conv2d_bn / dw3x3_bn take plain tensors or owned Pendings")
        det = lambda t: None if t is None else t.detach()
        return x.y, (x.mean, x.rstd, det(x.gamma), det(x.beta), x.act)
    return x, None


def conv2d_bn(x, w, b, ksize, gamma, beta, mmean, mvar, act, training, decay, eps=1e-3, dw_stride=0):
    """slim.conv2d + slim.batch_norm(+act), left Pending (owned) for the consumer's prologue.
    dw_stride: the conv is an inverted-residual block's expand feeding a depthwise of that stride
    (its output may then stay unwritten: _nostore_ok)."""
    xt, ipro = _in_pro(x)
    y, mean, rstd = _ConvBN.apply(xt, w, b, ksize, ipro, (gamma, beta, mmean, mvar, act, training, decay, eps),
                                  dw_stride)
    return Pending(y, mean, rstd, gamma, beta, act, training, owned=True)


def _cinpad_weights(w, cp, dtype):
    """GEMM operand of a [Cout, 3, 3, Cin] weight zero-padded to Cin = cp (inference): cached on the
    weight, refreshed when the weight changes (its version counter)."""
    key = (w._version, cp, dtype)
    hit = getattr(w, "_rod_cinpad", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    Cout, k, _, Cin = w.shape
    wp = torch.zeros((Cout, k, k, cp), dtype=torch.float32, device=w.device)
    wp[..., :Cin] = w.detach()
    wt = torch.empty((Cout, k * k * cp), dtype=dtype, device=w.device)
    _abi.call("rod_conv_weight_prep", wp, wt, Cout, cp, k, 0, dtcode(wt), stream())
    w._rod_cinpad = (key, wt)
    return wt


def conv2d_bn_act(x, w, b, ksize, gamma, beta, mmean, mvar, act, training, decay, eps=1e-3, residual=None):
    """conv2d_bn + materialize: act(BN(conv(x))) (+ residual) written out.  Inference in bf16:
    ONE launch, rod_conv_fwd_bnact (ABI 21) — the conv's epilogue applies the eval BatchNorm
    (moving statistics), the activation and the residual, bit-identical to conv -> rod_bn_apply
    with y never written; otherwise (training, fp32, ROD_DISABLE=bnepi) the owned Pending and
    rod_bn_apply."""
    xt, ipro = _in_pro(x)
    if training or xt.dtype != torch.bfloat16 or "bnepi" in _DISABLE or torch.is_grad_enabled() and \
            (xt.requires_grad or w.requires_grad):
        return materialize(conv2d_bn(x, w, b, ksize, gamma, beta, mmean, mvar, act, training, decay, eps), residual)
    N, H, W, Cin = xt.shape
    Cout = w.shape[0]
    if ksize == 1 and b is None and (ipro is None or Cin <= 32) and \
            _abi.lib().rod_conv_fwd_stream_ok(N * H * W, Cin, Cout, dtcode(xt)):
        # the streaming 1x1 kernel (no epilogue form) beats the tiled GEMM with the epilogue here
        return materialize(conv2d_bn(x, w, b, ksize, gamma, beta, mmean, mvar, act, training, decay, eps), residual)
    cp = -(-Cin // 8) * 8
    if ksize == 3 and ipro is not None and Cin != cp and "cinpad" not in _DISABLE:
        # the heads' last 3x3 convs (Cin = classes x anchors: 99, 66, 36): act(BN(x)) written once
        # into a zero-padded [.., Cin rounded up to 8] tensor and the weights zero-padded to match,
        # so the implicit GEMM's rows are 16-byte aligned (1080p b8 99 -> 99 at 34x60: 124 us
        # unpadded, 31 us for 128 -> 128 on the same map, tools/conv_bench.py).  The padded k
        # columns add exact zeros; the k-chunking of the sum differs (a rounding-level change).
        xb = torch.zeros((N, H, W, cp), dtype=xt.dtype, device=xt.device)
        im, ir, ig, ib, ia = ipro
        _abi.call("rod_bn_apply", xt, im, ir, ig, ib, None, xb, N * H * W, Cin, 0, 0, cp, ia, dtcode(xt), stream())
        xt, ipro = xb, None
        wt = _cinpad_weights(w, cp, xt.dtype)
        Cin = cp
    elif ksize == 3 and ipro is not None and N * H * W >= 16384 and "pro3" not in _DISABLE:
        # as _ConvBN.forward: a 3x3 gathers every input element 9 times, so act(BN(x)) is written
        # once instead of applied in the load prologue (the same rounded values)
        xb = torch.empty_like(xt)
        im, ir, ig, ib, ia = ipro
        _abi.call("rod_bn_apply", xt, im, ir, ig, ib, None, xb, N * H * W, Cin, 0, 0, 0, ia, dtcode(xt), stream())
        xt, ipro = xb, None
        wt = _prep(w, 0, xt.dtype, Cout, Cin, ksize)
    else:
        wt = _prep(w, 0, xt.dtype, Cout, Cin, ksize)
    z = torch.empty((N, H, W, Cout), dtype=xt.dtype, device=xt.device)
    mean, rstd = bn_statistics(z, mmean, mvar, False, decay, eps)
    nb = 0 if "splitk" in _DISABLE else _abi.query("rod_conv_fwd_workspace", N, H, W, Cin, Cout, ksize)
    ws = workspace(nb, xt.device) if nb else None
    res = residual.contiguous() if residual is not None else None
    det = lambda t: None if t is None else t.detach()
    _abi.call("rod_conv_fwd_bnact", xt, *_pro_args(ipro), wt, det(b), z, ws, mean, rstd, det(gamma), det(beta), act,
              res, 0, N, H, W, Cin, Cout, ksize, 0, 0, dtcode(xt), stream())
    return z


def dw3x3_bn(x, w, stride, gamma, beta, mmean, mvar, act, training, decay, eps=1e-3):
    """depthwise 3x3 + slim.batch_norm(+act), left Pending (owned)."""
    xt, ipro = _in_pro(x)
    y, mean, rstd = _DWBN.apply(xt, w, stride, ipro, (gamma, beta, mmean, mvar, act, training, decay, eps))
    return Pending(y, mean, rstd, gamma, beta, act, training, owned=True)


class _BNApplyOwned(torch.autograd.Function):
    """Write act(BN(y)) (+ residual) of an owned Pending; the producer node does the BatchNorm
    backward, so the gradient passes through to y (and to the residual) unchanged."""

    @staticmethod
    def forward(ctx, y, residual, mean, rstd, gamma, beta, act):
        N, H, W, C = y.shape
        out = torch.empty_like(y)
        _abi.call("rod_bn_apply", y, mean, rstd, gamma, beta, residual, out, N * H * W, C, 0, 0, 0, act, dtcode(y),
                  stream())
        ctx.has_res = residual is not None
        return out

    @staticmethod
    def backward(ctx, g):
        return g, (g if ctx.has_res else None), None, None, None, None, None


# ----------------------------------------------------------------------------- fused IR block (inference)
def ir_block_supported(Cin, inner, Cout, stride, residual, dtype):
    return "irblock" not in _DISABLE and bool(_abi.lib().rod_ir_block_supported(
        int(Cin), int(inner), int(Cout), int(stride), int(bool(residual)), _DT[dtype]))


def ir_block_preferred(Cin, inner, Cout, stride, residual, dtype):
    """Whether the eval backbone should take the fused block: where it measured faster than
    the unfused chain on MI355X (tools/irblock_bench.py, b8 720p / 1080p; DESIGN.md §6,
    profiles/r2s3_irblock_bench.txt) — the persistent variant (parameters resident in LDS) at
    stride 1, or at stride 2 on a 16-channel input.  Elsewhere (the deep blocks' parameters do
    not fit in LDS, the stride-2 blocks with wider inputs) the unfused chain is faster; the
    stride-2 24- and 32-channel blocks measure 1.03-1.14x fused at b8 but lose at the predict
    path's b32 (18.76 -> 18.88 ms per batch with them fused)."""
    if not ir_block_supported(Cin, inner, Cout, stride, residual, dtype):
        return False
    if rc_eval_ok(Cin, inner, stride, dtype):   # the chain with the expand output recomputed
        return False
    if "irblock_all" in _ENABLE:
        return True
    pers = bool(_abi.lib().rod_ir_block_persistent(int(Cin), int(inner), int(Cout), int(stride),
                                                      int(bool(residual)), _DT[dtype]))
    return pers and (stride == 1 or Cin <= 16)


IR_PERSIST, IR_EXACT = 1, 2


def ir_block_set_mode(mode):
    """rod_ir_block_set_mode: bit IR_PERSIST = persistent resident-parameter launch where it fits
    (default on), bit IR_EXACT = the unfused chain's rounding, bit for bit (default off: one
    rounding per expanded value).  Returns the previous mode."""
    return int(_abi.lib().rod_ir_block_set_mode(int(mode)))


def _eval_cached(mmean, mvar, eps):
    st = getattr(mmean, "_rod_store", None)
    if st is None or getattr(mvar, "_rod_store", None) is not st:
        return None
    return st.eval_views(mmean, mvar, eps)


def eval_stats(mmean, mvar, eps):
    hit = _eval_cached(mmean, mvar, eps)
    if hit is not None:
        return hit
    C = mmean.numel()
    mean = torch.empty(C, dtype=torch.float32, device=mmean.device)
    rstd = torch.empty(C, dtype=torch.float32, device=mmean.device)
    _abi.call("rod_bn_eval_stats", mmean, mvar, eps, mean, rstd, C, stream())
    return mean, rstd


def ir_block_fwd(x, we, bn_e, wd, bn_d, wp, bn_p, stride, residual):
    """rod_ir_block_fwd: expand -> BN+ReLU6 -> dw3x3 -> BN+ReLU6 -> project -> BN (+ x), one
    launch (inference).  we / wp: fp32 master weights [inner,1,1,Cin] / [Cout,1,1,inner];
    bn_*: (mean, rstd, gamma, beta) eval statistics."""
    N, H, W, Cin = x.shape
    inner, Cout = we.shape[0], wp.shape[0]
    wet = _prep(we, 0, x.dtype, inner, Cin, 1)
    wpt = _prep(wp, 0, x.dtype, Cout, inner, 1)
    y = torch.empty((N, -(-H // stride), -(-W // stride), Cout), dtype=x.dtype, device=x.device)
    _abi.call("rod_ir_block_fwd", x.contiguous(), wet, *bn_e, wd, *bn_d, wpt, *bn_p, int(bool(residual)), y, N, H, W,
              Cin, inner, Cout, int(stride), dtcode(x), stream())
    return y


# ----------------------------------------------------------------------------- levels
class _LevelsConcat(torch.autograd.Function):
    """[B, fh, fw, A*k] per level -> [B, sum(fh*fw*A), k] (tf.concat of reshaped levels)."""

    @staticmethod
    def forward(ctx, k, *levels):
        B = levels[0].shape[0]
        sizes = [lv.numel() // B for lv in levels]
        tot = sum(sizes)
        out = torch.empty((B, tot // k, k), dtype=levels[0].dtype, device=levels[0].device)
        es = out.element_size()
        off = 0
        for lv, n in zip(levels, sizes):
            lv = lv.contiguous()
            copy2d(lv, n * es, out, tot * es, B, n * es, 0, off * es)
            off += n
        ctx.shapes = [lv.shape for lv in levels]
        ctx.sizes = sizes
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        B = g.shape[0]
        tot = sum(ctx.sizes)
        es = g.element_size()
        outs = []
        off = 0
        for shp, n in zip(ctx.shapes, ctx.sizes):
            d = torch.empty(shp, dtype=g.dtype, device=g.device)
            copy2d(g, tot * es, d, n * es, B, n * es, off * es, 0)
            outs.append(d)
            off += n
        return (None, *outs)


def levels_concat(levels, k):
    return _LevelsConcat.apply(k, *levels)


# ----------------------------------------------------------------------------- losses
class _SmoothL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, mask, lvl_off, scale):
        B, A, _ = pred.shape
        L = len(lvl_off) - 1
        loss = torch.empty(L + 1, dtype=torch.float32, device=pred.device)
        grad = torch.empty_like(pred) if ctx.needs_input_grad[0] else None
        grad_t = torch.empty_like(target) if ctx.needs_input_grad[1] else None
        ws = workspace(_abi.query("rod_smoothl1_workspace", B, A), pred.device)
        _abi.call("rod_smoothl1_masked", pred, target, mask, np.ascontiguousarray(lvl_off, dtype=np.int32), L,
                  float(scale), loss, grad, grad_t, ws, B, A, dtcode(pred), stream())
        ctx.save_for_backward(grad, grad_t)
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(loss)
        return loss, loss[L]

    @staticmethod
    def backward(ctx, g_vec, g_tot):
        grad, grad_t = ctx.saved_tensors
        if g_tot is None:
            return None, None, None, None, None
        # the total is the training loss and its seed is 1 (graph.backward); any other
        # upstream weight would need a scale kernel, which no caller of the reference uses
        return grad, grad_t, None, None, None


def smooth_l1_masked(pred, target, mask, lvl_off, scale):
    """Returns ([L+1] fp32 per-level sum(smooth_l1((t - p)*m))/scale + total, total as a
    differentiable 0-d view).  The gradient is produced in the forward launch."""
    return _SmoothL1.apply(pred, target, mask, lvl_off, scale)


# ----------------------------------------------------------------------------- targets
def boxes_convert(boxes: torch.Tensor, to_center: bool) -> torch.Tensor:
    b = boxes.contiguous()
    out = torch.empty_like(b)
    _abi.call("rod_boxes_convert", b, out, b.numel() // 4, 1 if to_center else 0, stream())
    return out


def match_anchors(anc_corner, anc_center, lvl_off, thr, gt_center, gt_lbl, gt_n, nearest=False):
    """rod_match_anchors (JACCARD_BIGGER, thresholds thr) or, nearest=True, rod_match_anchors_nn
    (NEAREST_NEIGHBOR, thr unused)."""
    B, G, _ = gt_center.shape
    A = anc_corner.shape[0]
    dev = gt_center.device
    off = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
    cbox = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
    lbl = torch.empty((B, A), dtype=torch.int32, device=dev)
    pos = torch.empty((B, A), dtype=torch.int32, device=dev)
    lo = np.ascontiguousarray(lvl_off, dtype=np.int32)
    if nearest:
        _abi.call("rod_match_anchors_nn", anc_corner, anc_center, lo, len(lvl_off) - 1, gt_center.contiguous(),
                  gt_lbl.contiguous(), gt_n.contiguous(), off, cbox, lbl, pos, B, A, G, stream())
    else:
        _abi.call("rod_match_anchors", anc_corner, anc_center, lo, np.ascontiguousarray(thr, dtype=np.float32),
                  len(lvl_off) - 1, gt_center.contiguous(), gt_lbl.contiguous(), gt_n.contiguous(), off, cbox, lbl,
                  pos, B, A, G, stream())
    return off, cbox, lbl, pos


# ----------------------------------------------------------------------------- optimiser
def sgd_clip_(param_flat: torch.Tensor, grad_flat: torch.Tensor, lr: float, clip: float = 5.0):
    _abi.call("rod_sgd_clip", param_flat, grad_flat, param_flat.numel(), float(lr), float(clip), stream())


# ----------------------------------------------------------------------------- deconv pyramid
class _Resize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ho, wo):
        N, H, W, C = x.shape
        y = torch.empty((N, ho, wo, C), dtype=x.dtype, device=x.device)
        _abi.call("rod_resize_bilinear", x.contiguous(), y, N, H, W, C, ho, wo, dtcode(x), stream())
        ctx.geo = (N, H, W, C, ho, wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C, ho, wo = ctx.geo
        dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
        _abi.call("rod_resize_bilinear_bwd", dy.contiguous(), dx, N, H, W, C, ho, wo, dtcode(dy), stream())
        return dx, None, None


def resize_bilinear(x, size):
    """tf.image.resize_images(BILINEAR, align_corners=False), TF1 legacy scaling."""
    return _Resize.apply(x, int(size[0]), int(size[1]))


class _Deconv2x2(torch.autograd.Function):
    """conv2d_transpose(stride 2, SAME, 2x2 kernel [2, 2, F, Cin]) (catch_net.py:189-197)."""

    @staticmethod
    def forward(ctx, x, w, ho, wo):
        N, h, wd, Cin = x.shape
        F = w.shape[2]
        assert w.shape == (2, 2, F, Cin)
        x = x.contiguous()
        wt = _prep(w, 0, x.dtype, 4 * F, Cin, 1)
        z = torch.empty((N, h, wd, 4 * F), dtype=x.dtype, device=x.device)
        conv_fwd_raw(x, wt, None, z, N, h, wd, Cin, 4 * F, 1)
        y = torch.empty((N, ho, wo, F), dtype=x.dtype, device=x.device)
        _abi.call("rod_depth_to_space2", z, y, N, h, wd, F, ho, wo, 0, dtcode(x), stream())
        ctx.save_for_backward(x, w)
        ctx.geo = (N, h, wd, Cin, F, ho, wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, h, wd, Cin, F, ho, wo = ctx.geo
        dz = torch.empty((N, h, wd, 4 * F), dtype=dy.dtype, device=dy.device)
        _abi.call("rod_space_to_depth2", dy.contiguous(), dz, N, h, wd, F, ho, wo, 0, dtcode(dy), stream())
        dx = None
        if ctx.needs_input_grad[0]:
            wt1 = _prep(w, 1, dy.dtype, 4 * F, Cin, 1)
            dx = torch.empty_like(x)
            conv_fwd_raw(dz, wt1, None, dx, N, h, wd, 4 * F, Cin, 1)
        if ctx.needs_input_grad[1]:
            ws = workspace(_abi.query("rod_conv_wgrad_workspace", N, h, wd, Cin, 4 * F, 1), x.device)
            _abi.call("rod_conv_wgrad", x, *_pro_args(None), dz, grad_slot(w), None, ws, N, h, wd, Cin, 4 * F, 1,
                      0, 0, dtcode(x), stream())
            _mark_written(w)
        return dx, None, None, None


def deconv2x2(x, w, size):
    # TF's conv2d_transpose (SAME, stride 2) requires in = ceil(out / 2); it raises otherwise
    # (e.g. VGG-16's VALID chain at 720x1280: 4x8 -> 6x10)
    if x.shape[1] != -(-int(size[0]) // 2) or x.shape[2] != -(-int(size[1]) // 2):
        raise ValueError('conv2d_transpose: input %s does not match output %s (stride 2, SAME)' %
                         (tuple(x.shape[1:3]), tuple(size)))
    return _Deconv2x2.apply(x, w, int(size[0]), int(size[1]))


class _ChannelConcat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        N, H, W = xs[0].shape[:3]
        cs = [x.shape[3] for x in xs]
        Ct = sum(cs)
        out = torch.empty((N, H, W, Ct), dtype=xs[0].dtype, device=xs[0].device)
        es = out.element_size()
        off = 0
        for x, c in zip(xs, cs):
            copy2d(x.contiguous(), c * es, out, Ct * es, N * H * W, c * es, 0, off * es)
            off += c
        ctx.cs = cs
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        N, H, W, Ct = g.shape
        es = g.element_size()
        outs, off = [], 0
        for c in ctx.cs:
            d = torch.empty((N, H, W, c), dtype=g.dtype, device=g.device)
            copy2d(g, Ct * es, d, c * es, N * H * W, c * es, off * es, 0)
            outs.append(d)
            off += c
        return tuple(outs)


def channel_concat(xs):
    """tf.concat(xs, axis=-1) on NHWC tensors."""
    return _ChannelConcat.apply(*xs)


class _Add(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        assert a.shape == b.shape and a.dtype == b.dtype
        c = torch.empty_like(a)
        _abi.call("rod_add", a, b, c, a.numel(), dtcode(a), stream())
        return c

    @staticmethod
    def backward(ctx, g):
        return g, g


def add(a, b):
    return _Add.apply(a, b)


# ----------------------------------------------------------------------------- ODM / inference
def decode(anc_center, off_a, off_b=None, to_corner=False):
    """[B, A, 4] offsets (+ second offsets) -> fp32 boxes (centre or corner form)."""
    B, A = off_a.shape[0], off_a.shape[1]
    out = torch.empty((B, A, 4), dtype=torch.float32, device=off_a.device)
    _abi.call("rod_decode", anc_center, off_a.contiguous(), None if off_b is None else off_b.contiguous(), out, B, A,
              1 if to_corner else 0, dtcode(off_a), stream())
    return out


def _det_targets_raw(anc_center, refine_out, refine_gt, cbox, label, refine_pos, lvl_off, thr):
    B, A = refine_out.shape[0], refine_out.shape[1]
    dev = refine_out.device
    det_gt = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
    det_pos = torch.empty((B, A), dtype=torch.int32, device=dev)
    det_lbl = torch.empty((B, A), dtype=torch.int32, device=dev)
    iou = torch.empty((B, A), dtype=torch.float32, device=dev)
    _abi.call("rod_det_targets", anc_center, refine_out, refine_gt, cbox, label, refine_pos,
              np.ascontiguousarray(lvl_off, dtype=np.int32), np.ascontiguousarray(thr, dtype=np.float32),
              len(lvl_off) - 1, det_gt, det_pos, det_lbl, iou, B, A, dtcode(refine_out), stream())
    return det_gt, det_pos, det_lbl, iou


class _DetTargets(torch.autograd.Function):
    """det_groundtruth (net_tools.py:431-475) differentiable wrt refine_out: det_gt and iou
    depend on it (no stop-gradient in the reference); the masks and labels do not."""

    @staticmethod
    def forward(ctx, refine_out, anc_center, refine_gt, cbox, label, refine_pos, lvl_off, thr):
        det_gt, det_pos, det_lbl, iou = _det_targets_raw(anc_center, refine_out, refine_gt, cbox, label, refine_pos,
                                                         lvl_off, thr)
        ctx.save_for_backward(refine_out, anc_center, cbox, det_pos)
        ctx.mark_non_differentiable(det_pos, det_lbl)
        ctx.set_materialize_grads(False)
        return det_gt, det_pos, det_lbl, iou

    @staticmethod
    def backward(ctx, g_gt, g_pos, g_lbl, g_iou):
        refine_out, anc_center, cbox, det_pos = ctx.saved_tensors
        if g_gt is None and g_iou is None:
            return (None,) * 8
        B, A = refine_out.shape[0], refine_out.shape[1]
        g_ro = torch.empty_like(refine_out)
        _abi.call("rod_det_targets_bwd", anc_center, refine_out, cbox, det_pos,
                  None if g_gt is None else g_gt.contiguous(), None if g_iou is None else g_iou.contiguous(), g_ro,
                  B, A, dtcode(refine_out), stream())
        return (g_ro,) + (None,) * 7


def det_targets(anc_center, refine_out, refine_gt, cbox, label, refine_pos, lvl_off, thr):
    """(det_gt, det_pos, det_lbl, iou); differentiable wrt refine_out when it requires grad."""
    ro = refine_out.contiguous()
    if torch.is_grad_enabled() and ro.requires_grad:
        return _DetTargets.apply(ro, anc_center, refine_gt, cbox, label, refine_pos, lvl_off, thr)
    return _det_targets_raw(anc_center, ro, refine_gt, cbox, label, refine_pos, lvl_off, thr)


def _iou_factor_grad(logits, det_lbl, det_pos, iou, lvl_off, bs):
    """d clf_loss / d iou through the IoU focal factor (rod_iou_factor_bwd)."""
    B, A, K = logits.shape
    g = torch.empty((B, A), dtype=torch.float32, device=logits.device)
    _abi.call("rod_iou_factor_bwd", logits, det_lbl, det_pos, iou.contiguous(),
              np.ascontiguousarray(lvl_off, dtype=np.int32), len(lvl_off) - 1, float(bs), g, B, A, K,
              dtcode(logits), stream())
    return g


def softmax(logits, K):
    rows = logits.numel() // K
    out = torch.empty(logits.shape, dtype=torch.float32, device=logits.device)
    _abi.call("rod_softmax", logits.contiguous(), out, rows, K, dtcode(logits), stream())
    return out


class _SoftmaxCEHNM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, det_lbl, det_pos, iou, lvl_off, bs):
        B, A, K = logits.shape
        L = len(lvl_off) - 1
        out = torch.empty(8, dtype=torch.float32, device=logits.device)
        grad = torch.empty_like(logits) if ctx.needs_input_grad[0] else None
        ws = workspace(_abi.query("rod_softmax_ce_hnm_workspace", B, A, L), logits.device)
        _abi.call("rod_softmax_ce_hnm", logits.contiguous(), det_lbl, det_pos, iou,
                  np.ascontiguousarray(lvl_off, dtype=np.int32), L, float(bs), out, grad, ws, B, A, K,
                  dtcode(logits), stream())
        ctx.save_for_backward(grad, logits, det_lbl, det_pos, iou)
        ctx.hnm = (lvl_off, bs)
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(out)
        return out, out[2]

    @staticmethod
    def backward(ctx, g_vec, g_loss):
        grad, logits, det_lbl, det_pos, iou = ctx.saved_tensors
        if g_loss is None:
            return None, None, None, None, None, None
        # clf_loss enters the training loss with weight 1 (net_tools.det_clf_loss); the IoU
        # factor passes gradient to iou when refine_out is trained (fix_refine=False)
        g_iou = _iou_factor_grad(logits, det_lbl, det_pos, iou, *ctx.hnm) if ctx.needs_input_grad[3] else None
        return grad, None, None, g_iou, None, None


def softmax_ce_hnm(logits, det_lbl, det_pos, iou, lvl_off, bs):
    """([8] pos_loss, neg_loss, clf_loss, max_hard_pred, n_pos, k, n_neg_selected, 0;
    clf_loss as a differentiable 0-d view)."""
    return _SoftmaxCEHNM.apply(logits, det_lbl, det_pos, iou, lvl_off, bs)


def hnm_lockstep(shards, lvl_off, bs, B_global, allreduce, want_grad=True):
    """Hard-negative mining over a batch split into shards: rod_hnm_* for every
    shard in lock step, `allreduce(list_of_int32_tensors)` summing each exchange tensor over
    ALL shards of the global batch (in place) at the two exchange points — the counts, then
    the four 256-bin radix histograms.  In data-parallel training each process holds one
    shard and allreduce is an RCCL all-reduce on the compute stream; the sums are integers,
    so k and the threshold equal the single-process ones bit for bit.
    shards: [(logits [B,A,K], det_lbl, det_pos, iou)]; returns [(out [8], grad or None)]."""
    L = len(lvl_off) - 1
    lo = np.ascontiguousarray(lvl_off, dtype=np.int32)
    st = []
    for (logits, lbl, pos, iou) in shards:
        B, A, K = logits.shape
        dev = logits.device
        ws = workspace(_abi.query("rod_hnm_workspace", B, A, L), dev)
        counts = torch.empty(2, dtype=torch.int32, device=dev)
        state = torch.empty(8, dtype=torch.int32, device=dev)
        hist = torch.empty(256, dtype=torch.int32, device=dev)
        logits = logits.contiguous()
        _abi.call("rod_hnm_rows", logits, pos, ws, counts, B, A, K, L, dtcode(logits), stream())
        st.append((logits, lbl, pos, iou, ws, counts, state, hist, B, A, K))
    allreduce([x[5] for x in st])
    for x in st:
        _abi.call("rod_hnm_begin", x[5], int(B_global), x[6], x[7], stream())
    for shift in (24, 16, 8, 0):
        for x in st:
            _abi.call("rod_hnm_radix_hist", x[4], x[8], x[9], L, shift, x[6], x[7], stream())
        allreduce([x[7] for x in st])
        for x in st:
            _abi.call("rod_hnm_radix_scan", shift, x[6], x[7], stream())
    res = []
    for (logits, lbl, pos, iou, ws, counts, state, hist, B, A, K) in st:
        out = torch.empty(8, dtype=torch.float32, device=logits.device)
        grad = torch.empty_like(logits) if want_grad else None
        _abi.call("rod_hnm_loss", logits, lbl, pos, iou, lo, L, float(bs), state, out, grad, ws, B, A, K,
                  dtcode(logits), stream())
        res.append((out, grad))
    return res


class _SoftmaxCEHNMDP(torch.autograd.Function):
    """softmax_ce_hnm for one data-parallel shard (hnm_lockstep with the process group)."""

    @staticmethod
    def forward(ctx, logits, det_lbl, det_pos, iou, lvl_off, bs, B_global, allreduce):
        ((out, grad),) = hnm_lockstep([(logits, det_lbl, det_pos, iou)], lvl_off, bs, B_global, allreduce,
                                      want_grad=ctx.needs_input_grad[0])
        ctx.save_for_backward(grad, logits, det_lbl, det_pos, iou)
        ctx.hnm = (lvl_off, bs)
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(out)
        return out, out[2]

    @staticmethod
    def backward(ctx, g_vec, g_loss):
        grad, logits, det_lbl, det_pos, iou = ctx.saved_tensors
        if g_loss is None:
            return None, None, None, None, None, None, None, None
        g_iou = _iou_factor_grad(logits, det_lbl, det_pos, iou, *ctx.hnm) if ctx.needs_input_grad[3] else None
        return grad, None, None, g_iou, None, None, None, None


def softmax_ce_hnm_dp(logits, det_lbl, det_pos, iou, lvl_off, bs, B_global, allreduce):
    """softmax_ce_hnm with the hard negatives selected over the GLOBAL batch of a data-parallel
    job (allreduce: in-place SUM of a list of device int32 tensors over the ranks)."""
    return _SoftmaxCEHNMDP.apply(logits, det_lbl, det_pos, iou, lvl_off, bs, B_global, allreduce)


def select_topk_nms(probs, boxes, select_threshold, top_k, keep_top_k, nms_threshold, compact=True):
    """rod_select_topk_nms.  compact: pass the candidate-list workspace (one row-wise pass over
    probs; used when select_threshold > 0) — False forces the direct column-wise kernel."""
    B, A, K = probs.shape
    dev = probs.device
    scores = torch.empty((B, K - 1, keep_top_k), dtype=torch.float32, device=dev)
    bxs = torch.empty((B, K - 1, keep_top_k, 4), dtype=torch.float32, device=dev)
    ws = workspace(_abi.query("rod_select_topk_nms_workspace", B, A, K), dev) if compact else None
    _abi.call("rod_select_topk_nms", probs.contiguous(), boxes.contiguous(), B, A, K, float(select_threshold),
              int(top_k), int(keep_top_k), float(nms_threshold), scores, bxs, ws, stream())
    return scores, bxs


# ----------------------------------------------------------------------------- VGG-16 ops (F3)
# slim.conv2d with activation_fn and no normaliser (vgg_arg_scope: relu, nets/backbone/vgg.py:58):
# the conv's output y is left as an owned Pending with an identity BatchNorm (mean 0, rstd 1,
# no gamma / beta) and act = RELU, so consumers apply relu(y*1 + 0) = relu(y) exactly in their
# load prologue and the node's backward forms dy = dz * relu'(y) itself (rod_bn_bwd_apply with
# coefficients (1, 0, 0): dy = 1 * (g - 0 - yhat * 0) = g).
_IDENT = {}


def _ident_bn(C, device):
    key = (int(C), str(device))
    if key not in _IDENT:
        zeros = torch.zeros(C, dtype=torch.float32, device=device)
        ones = torch.ones(C, dtype=torch.float32, device=device)
        coef = torch.zeros(3 * C, dtype=torch.float32, device=device)
        coef[:C] = 1.0
        _IDENT[key] = (zeros, ones, coef)
    return _IDENT[key]


def _prep_flat(w, mode, dtype):
    """GEMM operand of a [Cout, 3, 3, Cin] weight viewed as a 1x1 conv over 9*Cin columns:
    mode 0 -> [Cout][9*Cin], mode 1 -> [9*Cin][Cout] (rod_conv_weight_prep, ksize 1)."""
    Cout, K = w.shape[0], w[0].numel()
    wt = torch.empty((Cout, K) if mode == 0 else (K, Cout), dtype=dtype, device=w.device)
    _abi.call("rod_conv_weight_prep", w, wt, Cout, K, 1, mode, dtcode(wt), stream())
    return wt


class _ConvAct(torch.autograd.Function):
    """slim.conv2d(+bias, activation_fn=act) as one node; geo None = SAME stride 1 (implicit
    GEMM, ksize 1 / 3), else (stride, pad_t, pad_l, Ho, Wo) for a 3x3 conv through the column
    matrix (rod_im2col3x3 -> GEMM with ksize 1; vgg.py:116-131)."""

    @staticmethod
    def forward(ctx, x, w, b, ks, ipro, act, geo):
        N, H, W, Cin = x.shape
        Cout = w.shape[0]
        col = None
        if geo is None:
            wt = _prep(w, 0, x.dtype, Cout, Cin, ks)
            y = torch.empty((N, H, W, Cout), dtype=x.dtype, device=x.device)
            conv_fwd_raw(x, wt, b, y, N, H, W, Cin, Cout, ks, None, ipro)
        else:
            s, pt, pl, Ho, Wo = geo
            col = torch.empty((N, Ho, Wo, 9 * Cin), dtype=x.dtype, device=x.device)
            _abi.call("rod_im2col3x3", x, *_pro_args(ipro), col, N, H, W, Cin, s, pt, pl, Ho, Wo, dtcode(x), stream())
            y = torch.empty((N, Ho, Wo, Cout), dtype=x.dtype, device=x.device)
            conv_fwd_raw(col, _prep_flat(w, 0, x.dtype), b, y, N, Ho, Wo, 9 * Cin, Cout, 1)
        ctx.save_for_backward(x, w, b, y, col)
        ctx.ks, ctx.ipro, ctx.act, ctx.geo = ks, ipro, act, geo
        ctx.set_materialize_grads(False)
        return y

    @staticmethod
    def backward(ctx, dz):
        if dz is None:
            return (None,) * 7
        x, w, b, y, col = ctx.saved_tensors
        C = y.shape[-1]
        zeros, ones, coef = _ident_bn(C, y.device)
        dy = torch.empty_like(y)
        _abi.call("rod_bn_bwd_apply", dz.contiguous(), y, zeros, ones, None, None, coef, dy, y.numel() // C, C,
                  ctx.act, dtcode(y), stream())
        need_dx = ctx.needs_input_grad[0]
        if ctx.geo is None:
            return _conv_bwd_from_dy(x, w, b, ctx.ks, dy, ctx.ipro, need_dx), None, None, None, None, None, None
        N, H, W, Cin = x.shape
        s, pt, pl, Ho, Wo = ctx.geo
        Cout = w.shape[0]
        dx = None
        if need_dx:
            dcol = torch.empty_like(col)
            conv_fwd_raw(dy, _prep_flat(w, 1, x.dtype), None, dcol, N, Ho, Wo, Cout, 9 * Cin, 1)
            dx = torch.empty_like(x)
            _abi.call("rod_col2im3x3", dcol, dx, N, H, W, Cin, s, pt, pl, Ho, Wo, dtcode(x), stream())
        need_w, need_bias = _needs(w), _needs(b)
        if need_w or need_bias:
            gw = grad_slot(w) if need_w else torch.empty(w.shape, dtype=torch.float32, device=x.device)
            gb = grad_slot(b) if need_bias else None
            ws = workspace(_abi.query("rod_conv_wgrad_workspace", N, Ho, Wo, 9 * Cin, Cout, 1), x.device)
            _abi.call("rod_conv_wgrad", col, *_pro_args(None), dy, gw, gb, ws, N, Ho, Wo, 9 * Cin, Cout, 1, 0, 0,
                      dtcode(x), stream())
            if need_w:
                _mark_written(w)
            if need_bias:
                _mark_written(b)
        return dx, None, None, None, None, None, None


def conv2d_act(x, w, b, ksize, act=ROD_ACT_RELU, stride=1, padding='SAME', pad=0, training=True):
    """slim.conv2d(x, Cout, [k, k], stride, padding, activation_fn=act) with no normaliser.
    padding 'SAME' with stride 1 runs the implicit GEMM; 'VALID' (after an explicit symmetric
    `pad`, custom_layers.pad2d) or stride 2 runs through the column matrix.  Returns an owned
    Pending (identity BatchNorm + act) for the consumer's load prologue."""
    xt, ipro = _in_pro(x)
    N, H, W, Cin = xt.shape
    geo = None
    if not (padding == 'SAME' and stride == 1 and pad == 0):
        assert ksize == 3, 'strided / VALID convs are 3x3 in the reference (vgg.py:116-131)'
        if padding == 'SAME':
            Ho, pt = same_pad(H, stride)
            Wo, pl = same_pad(W, stride)
        else:   # explicit pad then VALID
            Ho, Wo = (H + 2 * pad - 3) // stride + 1, (W + 2 * pad - 3) // stride + 1
            pt = pl = pad
        if Ho <= 0 or Wo <= 0:
            raise ValueError('conv2d_act: input %dx%d too small for a 3x3 VALID conv' % (H, W))
        geo = (stride, pt, pl, Ho, Wo)
    y = _ConvAct.apply(xt, w, b, ksize, ipro, act, geo)
    zeros, ones, _ = _ident_bn(y.shape[-1], y.device)
    return Pending(y, zeros, ones, None, None, act, training, owned=True)


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, H, W, C = x.shape
        x = x.contiguous()
        y = torch.empty((N, H // 2, W // 2, C), dtype=x.dtype, device=x.device)
        am = torch.empty((N, H // 2, W // 2, C), dtype=torch.uint8, device=x.device)
        _abi.call("rod_maxpool2x2", x, y, am, N, H, W, C, dtcode(x), stream())
        ctx.save_for_backward(am)
        ctx.geo = (N, H, W, C)
        ctx.mark_non_differentiable(am)
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        N, H, W, C = ctx.geo
        dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
        _abi.call("rod_maxpool2x2_bwd", dy.contiguous(), am, dx, N, H, W, C, dtcode(dy), stream())
        return dx


def max_pool2x2(x):
    """slim.max_pool2d(x, [2, 2]) — stride 2, VALID (vgg.py:93-101)."""
    return _MaxPool.apply(materialize(x))


_DROPOUT_CALLS = [0]
DROPOUT_RANK = [0, 1]   # (rank, world) of a data-parallel job (set by rod.trainer.Trainer)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, keep, seed):
        x = x.contiguous()
        y = torch.empty_like(x)
        mask = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
        _abi.call("rod_dropout", x, y, mask, x.numel(), float(keep), int(seed), dtcode(x), stream())
        ctx.save_for_backward(mask)
        ctx.keep = keep
        ctx.mark_non_differentiable(mask)
        return y, mask

    @staticmethod
    def backward(ctx, dy, _dmask):
        (mask,) = ctx.saved_tensors
        dx = torch.empty_like(dy)
        _abi.call("rod_dropout_bwd", dy.contiguous(), mask, dx, dy.numel(), float(ctx.keep), dtcode(dy), stream())
        return dx, None, None


def dropout(x, rate, training, seed=None):
    """tf.layers.dropout(x, rate, training) (vgg.py:106, 111).  Returns (y, mask or None); the
    seed defaults to a per-process call counter (every call draws a fresh mask), interleaved
    over the ranks of a data-parallel job so that no two ranks draw the same mask pattern for
    their shards (one device drawing over the global batch would not correlate them)."""
    x = materialize(x)
    if not training or rate == 0.0:
        return x, None
    if seed is None:
        _DROPOUT_CALLS[0] += 1
        rank, world = DROPOUT_RANK
        seed = 0x5EED0000 + _DROPOUT_CALLS[0] * world + rank
    return _Dropout.apply(x, 1.0 - float(rate), seed)


# ----------------------------------------------------------------------------- PREORDER_MSF ops (F4)
class _Pad2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, top, left):
        N, H, W, C = x.shape
        y = torch.empty((N, H + top, W + left, C), dtype=x.dtype, device=x.device)
        _abi.call("rod_pad2d", x.contiguous(), y, N, H, W, C, top, left, H + top, W + left, 0, dtcode(x), stream())
        ctx.geo = (N, H, W, C, top, left)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C, top, left = ctx.geo
        dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
        _abi.call("rod_pad2d", dy.contiguous(), dx, N, H, W, C, top, left, H + top, W + left, 1, dtcode(dy),
                  stream())
        return dx, None, None


def pad_top_left(x, top, left):
    """tf.pad(x, [[0, 0], [top, 0], [left, 0], [0, 0]]) (catch_net.py:135-136)."""
    x = materialize(x)
    return x if top == 0 and left == 0 else _Pad2d.apply(x, int(top), int(left))


class _SpaceToDepth(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r):
        N, H, W, C = x.shape
        y = torch.empty((N, H // r, W // r, r * r * C), dtype=x.dtype, device=x.device)
        _abi.call("rod_space_to_depth", x.contiguous(), y, N, H, W, C, r, 0, dtcode(x), stream())
        ctx.geo = (N, H, W, C, r)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C, r = ctx.geo
        dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
        _abi.call("rod_space_to_depth", dy.contiguous(), dx, N, H, W, C, r, 1, dtcode(dy), stream())
        return dx, None


def space_to_depth(x, block):
    """tf.space_to_depth(x, block_size) (catch_net.py:142)."""
    return _SpaceToDepth.apply(materialize(x), int(block))


class _SE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        N, H, W, C = x.shape
        C8 = w1.shape[1]
        x = x.contiguous()
        dev = x.device
        sq = torch.empty((N, C), dtype=torch.float32, device=dev)
        hid = torch.empty((N, C8), dtype=torch.float32, device=dev)
        e = torch.empty((N, C), dtype=torch.float32, device=dev)
        y = torch.empty_like(x)
        _abi.call("rod_se_fwd", x, w1, b1, w2, b2, sq, hid, e, y, N, H * W, C, C8, dtcode(x), stream())
        ctx.save_for_backward(x, w1, w2, sq, hid, e)
        ctx.params = (w1, b1, w2, b2)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w1, w2, sq, hid, e = ctx.saved_tensors
        N, H, W, C = x.shape
        C8 = w1.shape[1]
        dev = x.device
        de = torch.empty((N, C), dtype=torch.float32, device=dev)
        dsq = torch.empty((N, C), dtype=torch.float32, device=dev)
        dx = torch.empty_like(x)
        pw1, pb1, pw2, pb2 = ctx.params
        slots = [grad_slot(p) if _needs(p) else None for p in (pw1, pb1, pw2, pb2)]
        _abi.call("rod_se_bwd", dy.contiguous(), x, w1, w2, sq, hid, e, de, dsq, *slots, dx, N, H * W, C, C8,
                  dtcode(x), stream())
        for p, s in zip((pw1, pb1, pw2, pb2), slots):
            if s is not None:
                _mark_written(p)
        return dx, None, None, None, None


def se_block(x, w1, b1, w2, b2):
    """attention_module.se_block (attention_module.py:3-33): x * sigmoid(dense(relu(dense(mean_HW x))));
    w1 [C, C/8], w2 [C/8, C] fp32 (tf.layers.dense kernels)."""
    return _SE.apply(materialize(x), w1, b1, w2, b2)
