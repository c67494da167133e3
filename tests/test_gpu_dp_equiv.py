"""Data-parallel step equivalence: one training step of
2 ranks x (B/2) images — gradient all-reduce, global-batch loss normalisation, global
hard-negative selection (ALL), and SyncBatchNorm — against ONE process holding all B images.

With sync_bn the losses, the moving averages and the SGD result must match the single
process within fp32 reordering (1e-4), the SGD step is bit-exact given the reduced gradient,
and every parameter gradient and moving average within
max(1e-4, 4x the step's own fp32 sensitivity) normwise — the sensitivity being how far the
single-process gradient moves under 1e-6 / 1e-5 relative noise on its input: ReLU6 /
leaky kinks near zero and BatchNorm over the few rows of the deepest maps (3x5 at 320x576) make
single gradient entries move by percents under ANY fp32 reordering (the kernels also pick
other split-K / slab plans for B/2 rows), as in test_gpu_train.py.  Without sync_bn (the per-rank default) the deviation is
real and is only reported.  The ranks
share cuda:0 over gloo (RCCL refuses two ranks on one device); the transport is the only
difference from an 8-GPU RCCL run."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, 'tests', 'dp_step_worker.py')
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(out, world, train_range, sync, perturb_seed=None, amp=1e-6, extra=()):
    args = [WORKER, '--out', out, '--train_range', train_range] + (['--sync_bn'] if sync else []) + \
        (['--perturb', str(amp), '--perturb_seed', str(perturb_seed)] if perturb_seed is not None else []) + \
        list(extra)
    if world == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(world),
               '--master-addr', '127.0.0.1', '--master-port', str(_port())] + args
    r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, MASTER_ADDR='127.0.0.1'), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(out, weights_only=True)


def _nerr(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize('train_range', ['REFINE', 'ALL'])
def test_two_ranks_equal_one_process(train_range, tmp_path, dev):
    one = _run(str(tmp_path / 'one.pt'), 1, train_range, False)
    # sensitivity: 1e-6 and 1e-5 relative input noise, two draws each.  In ALL mode the det /
    # clf head gradients are sums over the few ODM-positive rows, so one leaky-ReLU sign flip
    # at those rows moves a whole head tensor by percents
    pert = [_run(str(tmp_path / f'p{s}_{a}.pt'), 1, train_range, False, perturb_seed=s, amp=a)
            for s in (11, 12) for a in (1e-6, 1e-5)]
    two = _run(str(tmp_path / 'two.pt'), 2, train_range, True)
    per = _run(str(tmp_path / 'per.pt'), 2, train_range, False)
    print(f"{train_range}: decisions (ODM positives, k, selected negatives): one {one['decisions'].tolist()} "
          f"two {two['decisions'].tolist()} noise {[p['decisions'].tolist() for p in pert]}")
    lo, lt = one['losses'], two['losses']
    assert torch.allclose(lt, lo, rtol=1e-4, atol=0), (lt, lo)
    bad, rows = [], []
    for name in one['trainable']:
        o, k = one['offsets'][name]
        g1 = one['grad'][o:o + k]
        if g1.abs().max() == 0:
            continue
        e_sync, e_per = (_nerr(r['grad'][o:o + k], g1) for r in (two, per))
        e_floor = max(_nerr(r['grad'][o:o + k], g1) for r in pert)
        rows.append((e_sync, e_floor, e_per))
        if e_sync > max(1e-4, 4 * e_floor):
            bad.append((name, e_sync, e_floor, e_per))
    assert not bad, bad[:10]
    # clip after the all-reduce, then SGD (net_tools.py:645-651): bit-exact given the reduced gradient
    ref = (two['flat0'].numpy() - np.float32(1e-2) * np.clip(two['grad'].numpy(), -5, 5)).astype(np.float32)
    np.testing.assert_array_equal(two['flat'].numpy(), ref)
    assert torch.equal(two['flat0'], one['flat0'])
    for k, v in one['buffers'].items():   # moving averages: same conditioning-aware bound
        e_floor = max(_nerr(r['buffers'][k], v) for r in pert)
        assert _nerr(two['buffers'][k], v) <= max(1e-4, 4 * e_floor), (k, _nerr(two['buffers'][k], v), e_floor)
    t = torch.tensor(rows)
    print(f'{train_range}: {len(rows)} gradients; normwise error vs one process, median / max: '
          f'sync {t[:, 0].median():.2g} / {t[:, 0].max():.2g}, input-noise floor {t[:, 1].median():.2g} / '
          f'{t[:, 1].max():.2g}, per-rank BatchNorm {t[:, 2].median():.2g} / {t[:, 2].max():.2g}')


def _cos_err(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return 1.0 - float(torch.nn.functional.cosine_similarity(a, b, dim=0))


def test_c3_per_rank_bf16_720p_two_by_four_equals_one_by_eight(tmp_path, dev):
    """BASELINE configs[2] (C3: bf16 at 1280x720, 8 images per rank) at the arithmetic one rank
    does: a REFINE step of 2 ranks x 4 images with SyncBatchNorm against one process holding
    all 8, both bf16 at 720x1280 (ref train.py:116-127, net_tools.py:557-587; 8 ranks x 8 is
    the same per-rank work over the same exchange).  Bound: bf16 itself.  Each gradient tensor's
    angular error (1 - cos) against the one-process step must stay within
    max(1e-3, 4x) that of the one-process step re-run with bf16-sized input noise (4e-3 relative:
    most inputs move by one bf16 ulp), and the loss within max(1e-3, 4x the noise floor)
    relative; the SGD update is bit-exact given the reduced gradient, and every moving statistic
    is within max(1e-3, 4x the noise floor) normwise."""
    ex = ['--dtype', 'bf16', '--hw', '720', '1280', '--batch', '8']
    one = _run(str(tmp_path / 'one.pt'), 1, 'REFINE', False, extra=ex)
    pert = [_run(str(tmp_path / f'p{s}.pt'), 1, 'REFINE', False, perturb_seed=s, amp=4e-3, extra=ex)
            for s in (11, 12)]
    two = _run(str(tmp_path / 'two.pt'), 2, 'REFINE', True, extra=ex)
    lo, lt = one['losses'], two['losses']
    lp = max(float((p['losses'] - lo).abs().max() / lo.abs().max()) for p in pert)
    print('C3 bf16 720p losses: one', lo.tolist(), 'two x four (sync)', lt.tolist(), 'noise floor', lp)
    assert float((lt - lo).abs().max() / lo.abs().max()) <= max(1e-3, 4 * lp)
    bad, rows = [], []
    for name in one['trainable']:
        o, k = one['offsets'][name]
        g1 = one['grad'][o:o + k]
        if g1.abs().max() == 0:
            continue
        e_sync = _cos_err(two['grad'][o:o + k], g1)
        e_floor = max(_cos_err(p['grad'][o:o + k], g1) for p in pert)
        rows.append((e_sync, e_floor))
        if e_sync > max(1e-3, 4 * e_floor):
            bad.append((name, e_sync, e_floor))
    assert len(rows) > 100 and not bad, bad[:10]
    ref = (two['flat0'].numpy() - np.float32(1e-2) * np.clip(two['grad'].numpy(), -5, 5)).astype(np.float32)
    np.testing.assert_array_equal(two['flat'].numpy(), ref)
    assert torch.equal(two['flat0'], one['flat0'])
    badm = []
    for k, v in one['buffers'].items():   # normwise (moving statistics are fp32 accumulations)
        e_floor = max(_nerr(p['buffers'][k], v) for p in pert)
        if _nerr(two['buffers'][k], v) > max(1e-3, 4 * e_floor):
            badm.append((k, _nerr(two['buffers'][k], v), e_floor))
    assert not badm, badm[:5]
    t = torch.tensor(rows)
    print(f'C3: {len(rows)} gradients; 1 - cos vs one process, median / max: sync {t[:, 0].median():.2g} / '
          f'{t[:, 0].max():.2g}, bf16 input-noise floor {t[:, 1].median():.2g} / {t[:, 1].max():.2g}')
