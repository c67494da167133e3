"""ORACLE — CPU restatement of the reference's hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / the timed CPU baseline — never as the product path
(the product path is librod.so via rod/, and fails loudly when that is missing).

Each function cites the reference file:line it restates.  Pinning: the anchor tables,
spec table and channel rounding are checked against fixtures produced by the reference
itself (tests/golden/make_golden.py imports the reference's pure-numpy code under a
stub `tensorflow`).  The TF-op arithmetic (IoU, encode/decode, BN, conv, losses, NMS,
AP) cannot run here (TensorFlow 1.x/slim is not installable): those parts restate the
documented TF-1.x op semantics and are pinned by hand-derived known-answer tests
(tests/test_oracle_semantics.py) — "parity unpinned" against the TF binary itself.

Numerical conventions shared with the kernels: float32 elementwise arithmetic with one
rounding per op (numpy float32), transcendental functions correctly rounded
(float64 evaluation, one cast), integer decisions (pos masks, argmax, NMS keep) exact.
"""
