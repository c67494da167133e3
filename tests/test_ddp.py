"""Data-parallel plumbing on CPU with the gloo backend, world_size 2 (the GPU runs use the
same code over RCCL): bucket construction, launch-during-backward, sum semantics, and the
global-batch loss normalisation that makes the reduced gradient equal the single-process
one (net_tools.py:513 divides by bs)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _store():
    from rod.params import ParamStore
    st = ParamStore()
    rng = np.random.default_rng(0)
    for i in range(12):
        st.add('layer_%d/weights' % i, rng.standard_normal((64, 3 + i)).astype(np.float32))
    st.add('frozen/w', np.zeros(100, np.float32))
    return st.finalize('cpu')


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from rod.ddp import GradReducer
        st = _store()
        st.params['frozen/w'].requires_grad_(False)
        red = GradReducer(world, bucket_mb=2 * 64 * 8 * 4 / (1 << 20)).attach(st)  # ~2 params per bucket
        nb = len(red.buckets)
        results = []
        for step in range(2):
            launched_midway = 0
            names = [n for n in st.params if n != 'frozen/w']
            for i, n in enumerate(reversed(names)):          # backward order
                p = st.params[n]
                p._rod_grad.copy_(torch.full(p.shape, float((rank + 1) * (i + 1) + step)))
                p._rod_on_grad(p)
                if i == len(names) // 2:
                    launched_midway = red.launched()
            red(st.flat_grad)
            results.append((launched_midway, st.flat_grad.clone()))
        # SyncBatchNorm gather: every rank gets the same rank-major concatenation
        from rod.ddp import SyncBatchNorm
        parts = torch.full((3, 2, 5), float(rank + 1))
        got = SyncBatchNorm(world).gather(parts)
        assert got.shape == (3 * world, 2, 5)
        for r in range(world):
            assert bool((got[3 * r:3 * r + 3] == r + 1).all())
        # global-batch normalisation: per-rank mean over its shard / world == global mean
        x = torch.arange(8, dtype=torch.float64).reshape(world, -1)[rank]
        local = (x.sum() / (x.numel() * world)).reshape(1)
        dist.all_reduce(local)
        q.put((rank, nb, [(m, g.numpy()) for m, g in results], float(local.item())))
    finally:
        dist.destroy_process_group()


def test_grad_reducer_gloo_world2():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    st = _store()
    names = [n for n in st.params if n != 'frozen/w']
    for rank, nb, results, gmean in out:
        assert nb >= 4
        assert gmean == pytest.approx(np.arange(8).mean())
        for step, (mid, flat) in enumerate(results):
            assert 0 < mid < nb  # some buckets were already reducing while "backward" ran
            for i, n in enumerate(reversed(names)):
                o, k = st.offsets[n]
                expect = sum((r + 1) * (i + 1) + step for r in range(world))
                np.testing.assert_array_equal(flat[o:o + k], np.full(k, expect, np.float32))
            o, k = st.offsets['frozen/w']
            np.testing.assert_array_equal(flat[o:o + k], 0)
    np.testing.assert_array_equal(out[0][2][1][1], out[1][2][1][1])


def _order_worker(rank, world, port, q):
    """The native reducer's collective sequence with the calls recorded, not made: buckets
    launched from the gradient hooks, the hard-negative sums and SyncBatchNorm gathers issued
    between them.  Every call must be on the one communication stream, and the (entry, count,
    dtype) sequence must be the same on every rank."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from rod import ddp
        st = _store()
        st.params['frozen/w'].requires_grad_(False)
        red = ddp.GradReducer(world, bucket_mb=2 * 64 * 8 * 4 / (1 << 20), native=True, record=True).attach(st)
        sbn = ddp.SyncBatchNorm(world, comm=red.comm)
        ddp.TRACE = []
        names = [n for n in st.params if n != 'frozen/w']
        for step in range(2):
            red.hnm_allreduce([torch.zeros(2, dtype=torch.int32)])        # ALL mode: counts in the loss
            for i, n in enumerate(reversed(names)):
                p = st.params[n]
                p._rod_grad.fill_(float(rank + i))
                p._rod_on_grad(p)
                if i % 3 == 1:       # a SyncBatchNorm backward gather between two gradient writes
                    g = sbn.gather(torch.full((2, 2, 3 + i), float(rank)))
                    assert g.shape == (2 * world, 2, 3 + i)
            red(st.flat_grad)
        q.put((rank, list(ddp.TRACE)))
    finally:
        ddp.TRACE = None
        dist.destroy_process_group()


def test_native_collective_order_identical_across_ranks():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_order_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    t0, t1 = out[0], out[1]
    assert len(t0) > 10 and t0 == t1
    assert {e[3] for e in t0} == {'comm'}
    entries = [e[0] for e in t0]
    assert 'rod_allgather' in entries and entries.count('rod_allreduce_bucket') > 4
    # buckets launched from inside "backward", interleaved with the gathers, not all at the end
    first_gather = entries.index('rod_allgather')
    assert any(e == 'rod_allreduce_bucket' and c > 2 for e, c, _, _ in t0[:first_gather + 6])


def test_cli_flag_surface():
    """train/evaluate/predict accept the reference's flag names and defaults."""
    import train
    import evaluate
    import predict
    t = train.parse([])
    assert (t.batch_size, t.learning_rate, t.log_every_n_steps, t.summary_every_n_steps, t.save_every_n_steps,
            t.fix_refine, t.num_readers, t.num_preprocessing_threads) == (20, 1e-3, 20, 20, 2000, True, 4, 4)
    assert t.checkpoint_refine == 'checkpoint/mbn_none53x35/refine/mobilenet_v2.model' and t.checkpoint_all is None
    assert train.parse(['--checkpoint_refine=None', '--fix_refine=False']).checkpoint_refine is None
    assert train.parse(['--fix_refine=False']).fix_refine is False
    e = evaluate.parse([])
    assert (e.select_threshold, e.select_top_k, e.keep_top_k, e.nms_threshold, e.matching_threshold,
            e.batch_size, e.checkpoint_path) == (0.3, 400, 200, 0.4, 0.5, 1, 'checkpoint/')
    p = predict.parse([])
    assert (p.checkpoint_all, p.vis_height, p.vis_width, p.vis_groundtruth) == \
        ('checkpoint/mobilenet_v2.model', 720, 1080, True)
