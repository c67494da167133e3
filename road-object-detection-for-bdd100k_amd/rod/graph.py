"""Graph helpers that keep PyTorch arithmetic off the product path.

When one activation feeds several consumers (a residual input, a tapped backbone endpoint,
a deconv output that also feeds the merge), autograd would sum the branch gradients with
its own elementwise add kernel.  `fork(x, n)` hands out n aliases of x through a custom
Function whose backward sums the branch gradients with rod_add (librod), so every
gradient byte is produced by librod kernels.  `scalar_sum` does the same for losses.
"""
import torch

from . import _abi
from .ops import dtcode, stream


def _sum(grads):
    gs = [g for g in grads if g is not None]
    if not gs:
        return None
    acc = gs[0].contiguous()
    for g in gs[1:]:
        out = torch.empty_like(acc)
        _abi.call("rod_add", acc, g.contiguous(), out, acc.numel(), dtcode(acc), stream())
        acc = out
    return acc


class _Fork(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, n):
        ctx.set_materialize_grads(False)    # unused branches hand back None, not zero tensors
        return tuple(x.view_as(x) for _ in range(n))

    @staticmethod
    def backward(ctx, *grads):
        return _sum(grads), None


def fork(x, n=2):
    """n aliases of x; their gradients are summed by rod_add in backward."""
    if not (torch.is_grad_enabled() and x.requires_grad):
        return tuple(x for _ in range(n))
    return _Fork.apply(x, n)


class _ScalarSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        ctx.n = len(xs)
        return _sum(list(xs))

    @staticmethod
    def backward(ctx, g):
        return tuple(g for _ in range(ctx.n))


def scalar_sum(*xs):
    """Sum of loss tensors (e.g. det_loss + clf_loss, train.py:163) with rod_add."""
    return _ScalarSum.apply(*xs)


_ONES = {}


def backward(loss):
    """loss.backward() seeded from a cached 1.0 tensor (no fill kernel per step)."""
    key = (loss.device, loss.dtype, tuple(loss.shape))
    if key not in _ONES:
        _ONES[key] = torch.ones_like(loss)
    ok = False
    try:
        torch.autograd.backward(loss, grad_tensors=_ONES[key])
        ok = True
    finally:
        from .ops import clear_bn_parts
        left = clear_bn_parts()   # BatchNorm sums / gradient recipes handed between nodes live for one backward
    if ok and left:
        raise RuntimeError("%d unmaterialised depthwise-input gradient(s) reached a node other than their "
                           "depthwise (rod.ops._DZ_RECIPE)" % left)
