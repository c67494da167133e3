"""Data-parallel gradient reduction over RCCL (torch.distributed 'nccl' = RCCL on ROCm).

The flat gradient buffer of rod.params.ParamStore is cut into contiguous buckets of
~`bucket_mb` MB aligned to parameter boundaries.  Every rod.ops kernel that writes a
parameter gradient calls the parameter's `_rod_on_grad` hook; when the last trainable
parameter of a bucket has been written, that bucket's all-reduce (sum) is issued
immediately, on a communication stream that waits (event) for the compute stream's work so
far, so the reduction of the head / late-backbone buckets overlaps the early-backbone
(depthwise) backward that is still running.  `__call__` (after backward) issues any bucket
not yet launched and makes the compute stream wait for all of them before the SGD update —
clipping happens after the sum (net_tools.py:649).

Transports:
  * native (the N > 1 default over RCCL, `make_reducer`): the library's own communicator
    (include/rod.h ABI 16/19: rod_allreduce_bucket, rod_allgather), created from a unique id
    handed over through torch.distributed's key-value store — no device collective of
    torch.distributed runs in a training step, so no ProcessGroupNCCL watchdog ever polls an
    event of a stream that is being captured, and the whole step (buckets, hard-negative
    exchange, SyncBatchNorm gathers) is captured into one HIP graph ('full', rod.trainer);
  * torch.distributed (gloo in the CPU tests and the one-GPU rehearsal): the same buckets via
    dist.all_reduce(async_op=True); a graphed step then captures only the collective-free
    compute ('split').

xGMI note: 8 GPUs are fully connected point-to-point; a 22 MB (REFINE) / 35 MB (ALL) fp32
gradient in ~4 MB buckets gives RCCL messages large enough to run its multi-channel rings
at link bandwidth while leaving room to overlap.
"""
import os

import torch
import torch.distributed as dist

_UID_KEY = 'rod_rccl_uid'
# Buckets completed on a detector-head chain stream wait for the end of backward and launch from
# the optimizer's stream.  ROD_DDP_CHAIN_DEFER=0 launches them where they complete instead (the
# communication stream forked from the chain stream by an event, joined at the optimizer's stream):
# that crashed hipStreamEndCapture (a segfault inside the HIP runtime) in round 6 too, on a 1-rank
# group (gpurun_out/r6b_tests.log), although the communication stream is now joined at the
# optimizer's stream — so the communication stream is never forked from a chain stream.
CHAIN_DEFER = os.environ.get('ROD_DDP_CHAIN_DEFER', '1') == '1'


def native_comm_init(rank, world, group=None):
    """The C-ABI reduce point (include/rod.h ABI 16: rod_rccl_unique_id / rod_rccl_init): rank 0
    makes the RCCL unique id and puts it in torch.distributed's key-value store (a host-side
    TCP store: no device collective, nothing for a watchdog to poll), every rank reads it and
    creates the library's communicator.  Idempotent: an existing communicator of this size is
    kept (one per process).  rod_rccl_destroy frees it."""
    import ctypes
    from . import _abi
    if _abi.lib().rod_rccl_world() == world:
        return
    if _abi.lib().rod_rccl_world() > 0:
        _abi.call('rod_rccl_destroy')
    uid = (ctypes.c_char * 128)()
    if rank == 0:
        _abi.call('rod_rccl_unique_id', ctypes.addressof(uid))
    if world > 1:
        store = dist.distributed_c10d._get_default_store()
        gen = getattr(native_comm_init, '_gen', 0) + 1    # a fresh key per communicator
        native_comm_init._gen = gen
        key = f'{_UID_KEY}_{gen}'
        if rank == 0:
            store.set(key, bytes(uid))
        else:
            ctypes.memmove(uid, store.get(key), 128)
    _abi.call('rod_rccl_init', rank, world, ctypes.addressof(uid))


def make_reducer(world, rank=None, group=None, bucket_mb=4.0):
    """The data-parallel reducer a job uses: over RCCL ('nccl' process group) the library's
    communicator (native), over any other backend (gloo) torch.distributed."""
    rank = dist.get_rank(group) if rank is None else rank
    if dist.get_backend(group) == 'nccl':
        native_comm_init(rank, world, group)
        return GradReducer(world, bucket_mb, group, native=True)
    return GradReducer(world, bucket_mb, group)


# Every collective a native reducer issues, in host order, when set to a list (tests): tuples
# (entry, element count, dtype code, stream role).  The role is 'comm' when the call was enqueued
# on the reducer's communication stream — the only stream a native collective may run on.
TRACE = None


class NativeComm(object):
    """The library's communicator (include/rod.h ABI 16/19) driven from ONE stream.

    RCCL requires every rank to issue a communicator's collectives in the same order, and two
    streams driving one communicator concurrently may interleave differently on different ranks
    (a cross-rank deadlock).  So every native collective of a step — the gradient buckets, the
    SyncBatchNorm all-gathers, the hard-negative count / histogram sums — is enqueued here, on
    this one communication stream, in host order: the stream first waits for everything the
    calling stream has queued (an event), the collective runs, and a done event joins it back —
    either right away (`run`: a collective whose result the calling stream consumes next) or
    when the optimizer needs the sums (`launch`: a gradient bucket, overlapping backward).
    Under HIP-graph capture the events are graph edges; no host synchronisation anywhere.

    record=True (tests): the entries are logged in TRACE but not called, and an all-gather
    replicates the local part (as if every rank held the same data) — so the collective
    sequence of a real step can be compared across ranks that share one GPU."""

    def __init__(self, record=False):
        self.stream = None
        self.record = bool(record)

    def _enqueue(self, entry, args, count, code):
        t = args[0]
        if not t.is_cuda:          # record mode on CPU tensors (the gloo unit tests)
            if TRACE is not None:
                TRACE.append((entry, int(count), int(code), 'comm'))
            if not self.record:
                raise RuntimeError('native collectives need device tensors')
            if entry == 'rod_allgather':
                args[1].copy_(args[0].reshape(-1)[:count].repeat(args[1].numel() // count).view_as(args[1]))
            return None, None
        cur = torch.cuda.current_stream(t.device)
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=t.device)
        comm = self.stream
        ready = torch.cuda.Event()
        ready.record(cur)            # the inputs are written
        comm.wait_event(ready)
        if TRACE is not None:
            TRACE.append((entry, int(count), int(code), 'comm'))
        if self.record:
            if entry == 'rod_allgather':
                with torch.cuda.stream(comm):
                    n = args[1].numel() // count
                    args[1].view(n, count).copy_(args[0].reshape(-1)[:count].expand(n, count))
        else:
            from . import _abi
            _abi.call(entry, *args, comm.cuda_stream)
        done = torch.cuda.Event()
        done.record(comm)
        return done, cur

    def run(self, entry, *args, count, code):
        """A collective whose result the calling stream reads next: joined right away."""
        done, cur = self._enqueue(entry, args, count, code)
        if done is not None:
            cur.wait_event(done)

    def launch(self, entry, *args, count, code):
        """A gradient bucket: returns the handle the optimizer's stream waits on."""
        done, cur = self._enqueue(entry, args, count, code)
        return _Done() if done is None else _Joined(done, cur)


class GradReducer(object):
    def __init__(self, world_size, bucket_mb=4.0, group=None, native=False, record=False):
        self.world = world_size
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.group = group
        # native=True: every collective goes through the library's own communicator, all of
        # them on ONE communication stream in host order (NativeComm): the buckets joined at
        # the optimizer, the hard-negative sums and SyncBatchNorm gathers joined right away;
        # otherwise torch.distributed (async work handles)
        self.native = bool(native)
        self.comm = NativeComm(record) if self.native else None
        self.store = None
        self.buckets = []
        # True while Trainer.step_graphed captures a 'split' step: the captured backward launches
        # no collective, every bucket is reduced after the replay (__call__)
        self.defer = False

    def attach(self, store):
        """Build buckets over the trainable parameters (in reverse registration order,
        i.e. roughly the order backward produces their gradients)."""
        self.store = store
        trainable = [(n, p) for n, p in store.params.items() if p.requires_grad]
        spans = sorted(((store.offsets[n][0], store.offsets[n][1], p) for n, p in trainable), key=lambda t: -t[0])
        self.buckets = []
        cur = None
        for off, n, p in spans:
            if cur is None or (cur['hi'] - off) * 4 > self.bucket_bytes:
                cur = {'lo': off, 'hi': off + n, 'params': [], 'pending': 0, 'work': None, 'streams': []}
                self.buckets.append(cur)
            cur['lo'] = min(cur['lo'], off)
            cur['params'].append(p)
            p._rod_bucket = cur
            p._rod_on_grad = self._on_grad
        self.reset()
        return self

    def reset(self):
        for b in self.buckets:
            b['pending'] = len(b['params'])
            b['work'] = None
            b['streams'] = []
            for p in b['params']:
                p._rod_seen = False

    def _launch(self, b):
        if b['work'] is None:
            from . import ops
            view = self.store.flat_grad[b['lo']:b['hi']]
            # gradients of one bucket may be written on several streams (the detector heads run
            # per level on their own, ops.LEVELS): the launching stream waits for all of them
            if view.is_cuda:
                cur = torch.cuda.current_stream(view.device)
                for st in b['streams']:
                    if st != cur:
                        cur.wait_stream(st)
            b['streams'] = []
            # the deferred weight-gradient sums INTO this bucket land before it is reduced; the
            # rest of the step's sums stay queued for the batched flush at the end of backward
            ops.SLAB.flush_range(view)
            b['work'] = self._allreduce(view)

    def _on_grad(self, p):
        b = getattr(p, '_rod_bucket', None)
        if b is None or p._rod_seen or self.defer:
            return
        p._rod_seen = True
        if torch.cuda.is_available() and p.is_cuda:
            st = torch.cuda.current_stream(p.device)
            if st not in b['streams']:
                b['streams'].append(st)
        b['pending'] -= 1
        if b['pending'] == 0 and not (CHAIN_DEFER and self._on_chain_stream(p)):
            self._launch(b)

    @staticmethod
    def _on_chain_stream(p):
        """A gradient written on a detector-head chain stream (ops.LEVELS): a bucket completed
        there is launched after backward, from the stream that runs the optimizer (__call__).
        Forking the communication stream from a chain stream crashes the end of a HIP-graph
        capture (hipStreamEndCapture, a segfault inside the runtime; tests/native_comm_worker.py
        and graph_dp_worker.py, rounds 5 and 6), while the same step with those buckets deferred
        captures and replays bit-identically."""
        if not (torch.cuda.is_available() and p.is_cuda):
            return False
        from . import ops
        return torch.cuda.current_stream(p.device) in ops.LEVELS.pool.values()

    def spans(self):
        """The buckets' ranges of the flat gradient merged where they touch: [(lo, hi)]."""
        out = []
        for lo, hi in sorted((b['lo'], b['hi']) for b in self.buckets):
            if out and out[-1][1] == lo:
                out[-1] = (out[-1][0], hi)
            else:
                out.append((lo, hi))
        return out

    def __call__(self, flat_grad):
        if self.store is None:
            raise RuntimeError('GradReducer.attach(store) was not called')
        if all(b['work'] is None for b in self.buckets):
            # nothing launched from inside backward (a 'split' graph replay, or hooks that never
            # fired): nothing left to overlap with, so one all-reduce per contiguous span (one
            # for the usual contiguous trainable set) instead of one per bucket
            from . import ops
            ops.SLAB.flush()
            works = [self._allreduce(self.store.flat_grad[lo:hi]) for lo, hi in self.spans()]
            for w in works:
                w.wait()
            self.reset()
            return
        for b in self.buckets:
            self._launch(b)
        for b in self.buckets:
            b['work'].wait()
        self.reset()

    def _allreduce(self, view):
        if not self.native:
            return dist.all_reduce(view, group=self.group, async_op=True)
        return self.comm.launch('rod_allreduce_bucket', view, view.numel(), 0, count=view.numel(), code=0)

    def hnm_allreduce(self, tensors):
        """In-place SUM of small device int32 tensors over the ranks (the hard-negative exchange
        of net_tools.det_clf_loss); native: on the communication stream, joined right away."""
        if self.native:
            for t in tensors:
                assert t.dtype == torch.int32 and t.is_contiguous()
                self.comm.run('rod_allreduce_bucket', t, t.numel(), 2, count=t.numel(), code=2)   # ROD_I32
            return
        for t in tensors:
            dist.all_reduce(t, group=self.group)

    def bn_allgather(self, parts):
        """[world * nparts, ...] = every rank's BatchNorm partial statistics in rank order
        (SyncBatchNorm)."""
        return allgather(parts, self.world, self.group, comm=self.comm)

    def launched(self):
        return sum(1 for b in self.buckets if b['work'] is not None)


class _Done(object):
    """The handle of a stream-ordered (already enqueued) reduction."""

    def wait(self):
        return None


class _Joined(object):
    """A bucket summed on the communication stream: wait() makes the stream current at the
    wait — the one that runs the optimizer step — wait for it (an event edge: a graph
    dependency under capture), no host synchronisation.  Not the stream current at the launch:
    a bucket may be launched from inside backward on a detector-head chain stream (ops.LEVELS)
    that nothing joins afterwards; joining the communication stream there left it unjoined at
    the end of a HIP-graph capture (a crash in capture_end, round 5)."""

    def __init__(self, done, stream):
        self.done, self.device = done, stream.device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.done)


def allgather(t, world, group=None, comm=None):
    """All-gather of a small device tensor into one [world * n, ...] buffer, rank-major
    (comm = a NativeComm: rod_allgather on its communication stream, joined right away; else
    RCCL all_gather_into_tensor on the compute stream; the list form for gloo)."""
    t = t.contiguous()
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if comm is not None:
        code = {torch.float32: 0, torch.bfloat16: 1, torch.int32: 2}[t.dtype]
        comm.run('rod_allgather', t, out, t.numel(), code, count=t.numel(), code=code)
    elif dist.get_backend(group) == 'nccl':
        dist.all_gather_into_tensor(out, t, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), t, group=group)
    return out


class SyncBatchNorm(object):
    """BatchNorm statistics over the global batch of a data-parallel job (rod.ops.SYNC_BN).
    Forward: each rank's partial statistics [nparts][3][C] (count, mean, M2) are all-gathered
    and every rank merges the same array (rod_bn_finalize, f64, fixed order), so mean, rstd and
    the moving averages are identical on all ranks and equal a single process holding the whole
    batch up to the merge order.  Backward: the partial sums (sum g, sum g*yhat) are gathered the
    same way for the dx coefficients; dgamma / dbeta stay per-rank sums, which the gradient
    all-reduce adds up.  One all-gather of 3*C (forward) / 2*C (backward) floats per part and
    BatchNorm: a few KB to ~1 MB per layer, latency-bound on xGMI."""

    def __init__(self, world, group=None, comm=None):
        self.world = world
        self.group = group
        self.comm = comm   # the reducer's NativeComm (the one communication stream) or None

    def gather(self, parts):
        return allgather(parts, self.world, self.group, comm=self.comm)
