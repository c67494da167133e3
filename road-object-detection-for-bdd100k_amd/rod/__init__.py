"""rod — MI355X-native runtime for the road-object detector (HIP kernels via librod.so)."""
from . import _abi  # noqa: F401
