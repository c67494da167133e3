"""utils/tf_extended/math.py: safe_divide (25-38) and cummax (41-67), numpy."""
import numpy as np

__all__ = ['safe_divide', 'cummax']


def safe_divide(numerator, denominator, name=None):
    """numerator / denominator where denominator > 0, else 0."""
    n = np.asarray(numerator)
    d = np.asarray(denominator)
    with np.errstate(divide='ignore', invalid='ignore'):
        q = n / d
    return np.where(d > 0, q, np.zeros_like(q))


def cummax(x, reverse=False, name=None):
    x = np.asarray(x)
    if reverse:
        return np.maximum.accumulate(x[::-1])[::-1]
    return np.maximum.accumulate(x)
