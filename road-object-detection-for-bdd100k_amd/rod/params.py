"""Flat parameter / gradient storage.

All trainable tensors live in one contiguous fp32 buffer (16-byte aligned slices) and
their gradients in a second buffer of identical layout.  Each parameter is a leaf
tensor viewing its slice; the rod.ops kernels write its gradient straight into the
matching grad slice (`p._rod_grad`), so the SGD update is one rod_sgd_clip launch over
the whole buffer and data-parallel reduction works on contiguous byte ranges.

Names follow the reference's TF/slim variable names (e.g.
``backbone/MobilenetV2/expanded_conv_3/depthwise/depthwise_weights``) so a checkpoint
importer maps 1:1; the weight layout differs from TF's [kh, kw, Cin, Cout] and is
[Cout, kh, kw, Cin] here (depthwise: [3, 3, C] for TF's [3, 3, C, 1]).
"""
from __future__ import annotations

import collections
import math

import numpy as np
import torch

ALIGN = 4  # fp32 elements (16 bytes)


def trunc_normal(rng: np.random.Generator, shape, std: float) -> np.ndarray:
    """tf.truncated_normal_initializer: N(0, std) redrawn outside +-2 std."""
    out = rng.standard_normal(size=shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(size=int(bad.sum()))
        bad = np.abs(out) > 2.0
    return (out * std).astype(np.float32)


def xavier_uniform(rng: np.random.Generator, shape_ohwi) -> np.ndarray:
    """slim default initializers.xavier_initializer() for a [Cout, kh, kw, Cin] conv."""
    co, kh, kw, ci = shape_ohwi
    fan_in, fan_out = kh * kw * ci, kh * kw * co
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape_ohwi).astype(np.float32)


class ParamStore:
    """Registry of parameters (trainable, fp32) and buffers (BN moving statistics)."""

    def __init__(self):
        self._specs = collections.OrderedDict()   # name -> (shape, init ndarray)
        self._buffers = collections.OrderedDict()  # name -> init ndarray
        self.params = collections.OrderedDict()
        self.buffers = collections.OrderedDict()
        self.flat = None
        self.flat_grad = None
        self.offsets = {}
        self.device = None
        self.version = 0          # bumped whenever parameter values change (SGD step, load)
        self._prep = {}           # (name, mode, dtype) -> [prepped tensor, version, entry]
        self._prep_tables = {}    # dtype -> (device table, n, total) or None when stale

    # ---- registration (host) ------------------------------------------------------
    def add(self, name: str, init: np.ndarray):
        assert name not in self._specs, f"duplicate parameter {name}"
        self._specs[name] = np.ascontiguousarray(init, dtype=np.float32)
        return name

    def add_buffer(self, name: str, init: np.ndarray):
        assert name not in self._buffers, f"duplicate buffer {name}"
        self._buffers[name] = np.ascontiguousarray(init, dtype=np.float32)
        return name

    # ---- materialisation (device) ---------------------------------------------------
    def finalize(self, device):
        self.device = torch.device(device)
        off = 0
        for name, arr in self._specs.items():
            self.offsets[name] = (off, arr.size)
            off += -(-arr.size // ALIGN) * ALIGN
        self.numel = off
        host = np.zeros(off, dtype=np.float32)
        for name, arr in self._specs.items():
            o, n = self.offsets[name]
            host[o:o + n] = arr.reshape(-1)
        self.flat = torch.from_numpy(host).to(self.device)
        self.flat_grad = torch.zeros(off, dtype=torch.float32, device=self.device)
        for name, arr in self._specs.items():
            o, n = self.offsets[name]
            p = self.flat[o:o + n].view(arr.shape).detach().requires_grad_(True)
            p._rod_grad = self.flat_grad[o:o + n].view(arr.shape)
            p._rod_name = name
            p._rod_store = self
            self.params[name] = p
        # BatchNorm moving statistics: views of ONE flat buffer, so the eval-mode (mean, rstd) of
        # every BatchNorm comes from a single rod_bn_eval_stats launch per forward (eval_refresh)
        nb = sum(arr.size for arr in self._buffers.values())
        hb = np.concatenate([arr.reshape(-1) for arr in self._buffers.values()]) if nb else np.zeros(1, np.float32)
        self.flat_buf = torch.from_numpy(hb).to(self.device)
        self._eval_out = torch.empty((2, max(nb, 1)), dtype=torch.float32, device=self.device)
        self._eval_eps = None
        o = 0
        for name, arr in self._buffers.items():
            b = self.flat_buf[o:o + arr.size].view(arr.shape)
            b._rod_store = self
            self.buffers[name] = b
            o += arr.size
        return self

    # ---- eval-mode BatchNorm statistics -----------------------------------------------
    def eval_refresh(self, eps):
        """(mean, rstd) = (moving_mean, 1/sqrt(moving_var + eps)) of EVERY buffer element in one
        launch (rod_bn_eval_stats over the flat buffer); until eval_release(), eval_views serves
        each BatchNorm's slices from it instead of a launch per BatchNorm."""
        from . import _abi
        from .ops import stream
        n = self.flat_buf.numel()
        _abi.call("rod_bn_eval_stats", self.flat_buf, self.flat_buf, eps, self._eval_out[0], self._eval_out[1], n,
                  stream())
        self._eval_eps = eps

    def eval_release(self):
        self._eval_eps = None

    def eval_views(self, mmean, mvar, eps):
        """The refreshed (mean, rstd) slices of one BatchNorm, or None outside a refresh."""
        if self._eval_eps is None or eps != self._eval_eps:
            return None
        base, n = self.flat_buf.data_ptr(), self.flat_buf.numel()
        C = mmean.numel()
        offs = []
        for t in (mmean, mvar):
            d = t.data_ptr() - base
            # a buffer rebound outside flat_buf (instead of updated in place) would otherwise
            # read the wrong slice: fall back to the per-BatchNorm path
            if t.numel() != C or t.dtype != self.flat_buf.dtype or d % 4 or not 0 <= d // 4 <= n - C:
                return None
            offs.append(d // 4)
        om, ov = offs
        return self._eval_out[0, om:om + C], self._eval_out[1, ov:ov + C]

    def set_trainable(self, predicate):
        """requires_grad per parameter name (train.py:160-166 trainable-var filtering)."""
        for name, p in self.params.items():
            p.requires_grad_(bool(predicate(name)))

    def trainable_count(self):
        return int(sum(p.numel() for p in self.params.values() if p.requires_grad))

    def zero_grad(self):
        self.flat_grad.zero_()

    # ---- derived weight layouts (rod_conv_weight_prep) -------------------------------
    def prepped(self, p, mode, dtype, Cout, Cin, ks):
        """The GEMM operand layout `mode` of conv weight p in `dtype` (rod_conv_weight_prep):
        built once, then refreshed for EVERY registered weight by one batched launch
        (rod_conv_weight_prep_batch) the first time it is asked for after the parameters
        changed (self.version)."""
        from . import _abi
        from .ops import dtcode, stream
        key = (p._rod_name, mode, dtype)
        e = self._prep.get(key)
        if e is None:
            wt = torch.empty((Cout, ks * ks * Cin) if mode == 0 else (Cin, ks * ks * Cout), dtype=dtype,
                             device=p.device)
            _abi.call("rod_conv_weight_prep", p, wt, Cout, Cin, ks, mode, dtcode(wt), stream())
            self._prep[key] = [wt, self.version, (p.data_ptr(), wt.data_ptr(), Cout, Cin, ks, mode)]
            self._prep_tables[dtype] = None
            return wt
        if e[1] != self.version:
            self._refresh_prep(dtype)
        return e[0]

    def build_prep_tables(self):
        """Upload the device tables of rod_conv_weight_prep_batch now (host -> device copies),
        e.g. before a HIP-graph capture, which may contain the refresh launch but no copy."""
        for dtype in {d for (_, _, d) in self._prep}:
            self._prep_table(dtype)

    def _prep_table(self, dtype):
        tab = self._prep_tables.get(dtype)
        if tab is None:
            ents = [e for (n, m, d), e in self._prep.items() if d == dtype]
            rec = np.zeros(len(ents), dtype=np.dtype([('w', '<u8'), ('wt', '<u8'), ('start', '<i8'), ('Cout', '<i4'),
                                                       ('Cin', '<i4'), ('ks', '<i4'), ('mode', '<i4')]))
            start = 0
            for i, e in enumerate(ents):
                wp, tp, Cout, Cin, ks, mode = e[2]
                rec[i] = (wp, tp, start, Cout, Cin, ks, mode)
                start += Cout * ks * ks * Cin
            dev = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)
            tab = (dev, len(ents), start, ents)
            self._prep_tables[dtype] = tab
        return tab

    def _refresh_prep(self, dtype):
        from . import _abi
        from .ops import dtcode, stream
        dev, n, total, ents = self._prep_table(dtype)
        _abi.call("rod_conv_weight_prep_batch", dev, n, total, dtcode(ents[0][0]), stream())
        for e in ents:
            e[1] = self.version

    # ---- checkpointing -------------------------------------------------------------
    def state_dict(self):
        sd = {n: p.detach().cpu().clone() for n, p in self.params.items()}
        sd.update({n: b.detach().cpu().clone() for n, b in self.buffers.items()})
        return sd

    def load_state_dict(self, sd, strict=True, names_regex=None):
        import re
        pat = re.compile(names_regex) if names_regex else None
        missing = []
        with torch.no_grad():
            for n, p in list(self.params.items()) + list(self.buffers.items()):
                if pat is not None and not pat.match(n):
                    continue
                if n not in sd:
                    missing.append(n)
                    continue
                p.copy_(sd[n].to(p.device).view(p.shape))
        self.version += 1
        if strict and missing:
            raise KeyError(f"missing entries in checkpoint: {missing[:5]}{'...' if len(missing) > 5 else ''}")
        return missing
