"""utils/tf_extended/tensors.py: get_shape (34-56) and pad_axis (59-86) for numpy / torch."""
import numpy as np

__all__ = ['get_shape', 'pad_axis']


def get_shape(x, rank=None):
    return list(x.shape)


def pad_axis(x, offset, size, axis=0, name=None):
    """Zero-pad `x` on `axis` with `offset` leading entries up to `size` entries."""
    x = np.asarray(x)
    n = x.shape[axis]
    new = max(size - offset - n, 0)
    pad = [(0, 0)] * x.ndim
    pad[axis] = (offset, new)
    return np.pad(x, pad, mode='constant')
