"""ctypes binding of librodio.so (include/rodio.h): CRC32C and the TFRecord scan.

Host-only native code (no device); the CLIs' data and checkpoint readers call it.  A
missing library raises at first use, like librod.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RODIO_LIB", os.path.join(os.path.dirname(_HERE), "lib", "librodio.so"))
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "rodio.h")

_SIG = {
    "rodio_abi_version": (ctypes.c_int, []),
    "rodio_last_error": (ctypes.c_char_p, []),
    "rodio_crc32c_extend": (ctypes.c_uint, [ctypes.c_uint, ctypes.c_void_p, ctypes.c_size_t]),
    "rodio_masked_crc32c": (ctypes.c_uint, [ctypes.c_void_p, ctypes.c_size_t]),
    "rodio_tfrecord_scan": (ctypes.c_long, [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long,
                                            ctypes.c_int]),
}
_lock = threading.Lock()
_cdll = None


def lib():
    global _cdll
    if _cdll is None:
        with _lock:
            if _cdll is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(f"librodio.so not found at {LIB_PATH}: build it with "
                                       f"`make -C {os.path.join(os.path.dirname(_HERE), 'csrc')}`")
                c = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in _SIG.items():
                    fn = getattr(c, name)
                    fn.restype, fn.argtypes = res, args
                _cdll = c
    return _cdll


def _buf(data):
    """(address, nbytes, keepalive) of a bytes-like object."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data)
        return a.ctypes.data, a.nbytes, a
    mv = memoryview(data).cast('B')
    if mv.readonly:
        a = np.frombuffer(mv, dtype=np.uint8)
        return a.ctypes.data, a.nbytes, a
    a = (ctypes.c_char * len(mv)).from_buffer(mv)
    return ctypes.addressof(a), len(mv), a


def crc32c(data, crc=0) -> int:
    p, n, _keep = _buf(data)
    return int(lib().rodio_crc32c_extend(crc, p, n))


def masked_crc32c(data) -> int:
    p, n, _keep = _buf(data)
    return int(lib().rodio_masked_crc32c(p, n))


def mask(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xa282ead8) & 0xFFFFFFFF


def unmask(masked: int) -> int:
    rot = (masked - 0xa282ead8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


def tfrecord_scan(path: str, verify_data=True):
    """(offsets, lengths) int64 arrays of every record payload in a TFRecord file."""
    L = lib()
    cap = 4096
    while True:
        off = np.empty(cap, np.int64)
        ln = np.empty(cap, np.int64)
        n = L.rodio_tfrecord_scan(os.fsencode(path), off.ctypes.data, ln.ctypes.data, cap, int(bool(verify_data)))
        if n < 0:
            raise IOError(L.rodio_last_error().decode(errors='replace'))
        if n <= cap:
            return off[:n].copy(), ln[:n].copy()
        cap = n


def exported_symbols():
    import re
    text = re.sub(r"/\*.*?\*/", " ", open(HEADER_PATH).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(rodio_\w+)\s*\(", text)))
