"""ctypes binding of librod.so (the C ABI declared in include/rod.h).

The prototypes are read from the header itself, so the header is the single source
of truth for argument types; every call checks the return code and raises
RuntimeError with rod_last_error() on failure.  There is no fallback: if the library
is missing the import of any op fails loudly (the product path never routes through
a CPU implementation).

Argument conversion for pointer parameters:
  torch.Tensor  -> data_ptr()   (device tensors for device buffers; CPU tensors are
                                  accepted only where the header documents a host array)
  numpy.ndarray -> host pointer (host arrays such as lvl_off / thr)
  None          -> NULL
  int           -> raw address
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("ROD_LIB", os.path.join(PKG_ROOT, "lib", "librod.so"))
HEADER_PATH = os.path.join(REPO_ROOT, "include", "rod.h")

ROD_F32 = 0
ROD_BF16 = 1
ROD_ACT_NONE = 0
ROD_ACT_RELU6 = 1
ROD_ACT_LEAKY = 2
ROD_ACT_RELU = 3

_CTYPE = {
    "int": ctypes.c_int,
    "long": ctypes.c_long,
    "uint64_t": ctypes.c_uint64,
    "float": ctypes.c_float,
    "size_t": ctypes.c_size_t,
    "ptr": ctypes.c_void_p,
    "cstr": ctypes.c_char_p,
    "void": None,
}

_PROTO_RE = re.compile(
    r"^\s*(const\s+char\s*\*|int|size_t|void)\s+(rod_\w+)\s*\(([^)]*)\)\s*;", re.M | re.S)


def parse_header(path: str = HEADER_PATH):
    """Return {name: (restype, [(argtype, argname), ...])} for every rod_* prototype."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    protos = {}
    for m in _PROTO_RE.finditer(text):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        ret = "cstr" if "char" in ret else ret.strip()
        argl = []
        a = " ".join(args.split())
        if a and a != "void":
            for piece in a.split(","):
                piece = piece.strip()
                if "*" in piece:
                    argl.append(("ptr", piece.split("*")[-1].strip()))
                else:
                    toks = piece.replace("const ", "").split()
                    argl.append((toks[0], toks[1]))
        protos[name] = (ret, argl)
    return protos


class _Lib:
    def __init__(self):
        self._lock = threading.Lock()
        self._cdll = None
        self.protos = None

    def load(self):
        if self._cdll is not None:
            return self._cdll
        with self._lock:
            if self._cdll is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"librod.so not found at {LIB_PATH}: build it with "
                        f"`make -C {os.path.join(PKG_ROOT, 'csrc')}` (or __graft_entry__.build())")
                cdll = ctypes.CDLL(LIB_PATH)
                protos = parse_header()
                for name, (ret, args) in protos.items():
                    fn = getattr(cdll, name)  # AttributeError => header/library mismatch
                    fn.restype = _CTYPE[ret]
                    fn.argtypes = [_CTYPE[t] for t, _ in args]
                self.protos = protos
                self._cdll = cdll
        return self._cdll


_LIB = _Lib()


def lib():
    return _LIB.load()


def _ptr(v):
    if v is None:
        return None
    if isinstance(v, int):
        return v
    if isinstance(v, np.ndarray):
        if not v.flags["C_CONTIGUOUS"]:
            raise ValueError("host array must be C-contiguous")
        return v.ctypes.data
    dp = getattr(v, "data_ptr", None)
    if dp is not None:
        return dp()
    raise TypeError(f"cannot pass {type(v)} as a pointer")


class Probe:
    """Live per-kernel timing for the roofline report (bench.py): when `name` matches,
    HIP events are recorded on the launching stream around every call and the
    algorithmic byte / flop count of the call (rod.roofline) is accumulated."""

    def __init__(self):
        self.names = frozenset()
        self.all = False
        self.records = []

    def arm(self, names):
        """names: one entry name, an iterable of names, or '*' (every entry)."""
        self.all = names == '*'
        self.names = frozenset([names] if isinstance(names, str) else names)
        self.records = []

    def disarm(self):
        self.names, self.all = frozenset(), False

    def wants(self, name):
        return self.all or name in self.names

    def table(self, by_shape=False):
        """{entry (or (entry, scalar args) when by_shape): (launches, total_ms, alg_bytes,
        alg_flops)} over the recorded calls."""
        out = {}
        for name, e0, e1, (b, f, _), shape in self.records:
            key = (name, shape) if by_shape else name
            n, ms, bb, ff = out.get(key, (0, 0.0, 0, 0))
            out[key] = (n + 1, ms + e0.elapsed_time(e1), bb + b, ff + f)
        return out

    def design_table(self):
        """{entry: design bytes} (rod.roofline.design_bytes: the bytes the kernels are built to
        move, >= the algorithmic bytes where a design re-reads a tensor)."""
        out = {}
        for name, _, _, (_, _, d), _ in self.records:
            out[name] = out.get(name, 0) + d
        return out


PROBE = Probe()


def _capturing():
    """True while a HIP graph is being captured: timing events recorded into a capture belong
    to the graph and cannot be read back, so the probe skips those calls."""
    import torch
    return torch.cuda.is_current_stream_capturing()


# entries whose parameter-gradient sums rod_slab_defer(1) may queue (include/rod.h, ABI 11)
DEFERRING = frozenset(("rod_conv_wgrad", "rod_dw3x3_bwd_filter", "rod_dw3x3_bwd_filter_bn", "rod_pw_bwd",
                       "rod_pw_bwd_rc", "rod_pw_bwd_gred", "rod_pw_bwd_gred_rc", "rod_pw_bwd_gred_dyp", "rod_stem_wgrad_bn", "rod_dw3x3_bwd_fused",
                       "rod_dw3x3_bwd_fused_pw", "rod_dw3x3_bwd_fused_rc"))
# while sums are deferred: every tensor handed to such an entry (partial slabs, gradient outputs)
# is kept referenced until rod_slab_flush has been enqueued (rod.ops.SlabDefer).  With WATCH_DEFER
# every other entry is checked against the queue length (rod_slab_pending) around the call: one
# that queued a sum has its tensors kept too and its name recorded in DEFER_UNLISTED (a registry
# gap, which tests/test_gpu_defer.py asserts never happens over REFINE / ALL steps).  On by default
# (ROD_DEFER_WATCH=0 turns it off): it costs two ctypes calls per entry of an EAGER backward only —
# a graph replay runs no Python — and a gap corrupts weight gradients silently (round 6 found one:
# rod_dw3x3_bwd_fused_rc, its slab freed and reused before the deferred flush read it, caught as
# run-to-run different steps by tools/rc_step_diag.py), while the watch keeps such a call correct.
KEEP = None
DEFER_UNLISTED = set()
WATCH_DEFER = os.environ.get("ROD_DEFER_WATCH", "1") != "0"


def call(name: str, *args):
    """Call rod_<name>; raise RuntimeError on a non-zero return code."""
    L = lib()
    fn = getattr(L, name)
    ret, argspec = _LIB.protos[name]
    if len(args) != len(argspec):
        raise TypeError(f"{name} expects {len(argspec)} args, got {len(args)}")
    watch = False
    if KEEP is not None:
        if name in DEFERRING:
            KEEP.extend(a for a in args if hasattr(a, "data_ptr"))
        elif WATCH_DEFER:
            watch = True
            pend0 = L.rod_slab_pending()
    conv = [(_ptr(a) if t == "ptr" else a) for (t, _), a in zip(argspec, args)]
    if PROBE.wants(name) and not _capturing():
        import torch
        from . import roofline
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        rc = fn(*conv)
        e1.record(s)
        shape = tuple(a for a in args if isinstance(a, (int, float)) and not isinstance(a, bool))
        PROBE.records.append((name, e0, e1, roofline.cost(name, args) + (roofline.design_bytes(name, args),), shape))
    else:
        rc = fn(*conv)
    if watch and L.rod_slab_pending() > pend0:
        KEEP.extend(a for a in args if hasattr(a, "data_ptr"))
        DEFER_UNLISTED.add(name)
    if ret == "int" and rc != 0:
        msg = L.rod_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")
    return rc


def query(name: str, *args) -> int:
    """Call a size_t workspace query."""
    return int(getattr(lib(), name)(*args))


def exported_symbols():
    return sorted(parse_header().keys())
