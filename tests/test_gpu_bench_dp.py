"""Rehearsal of bench.py's N>1 path on a one-GPU box: two ranks launched by
torch.distributed.run exactly as the driver does for --gpus 2, sharing cuda:0 over the gloo
backend (ROD_DIST_BACKEND=gloo; RCCL refuses two ranks on one device).  Covers the barrier /
max-over-ranks timing, the bucketed gradient reducer launched from inside backward, the
global-batch loss normalisation and, in ALL mode, the hard-negative count/histogram
exchange — everything of the 8-GPU run except the transport."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize('train_range', ['REFINE', 'ALL'])
def test_bench_two_ranks(train_range, dev):
    env = dict(os.environ, ROD_DIST_BACKEND='gloo', MASTER_ADDR='127.0.0.1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_port()), os.path.join(ROOT, 'bench.py'),
           '--gpus', '2', '--steps', '2', '--warmup', '1', '--height', '160', '--width', '288', '--batch', '2',
           '--train_range', train_range, '--no-cpu-baseline', '--no-inference']
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints exactly one JSON line
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['steps'] == 2 and out['warmup'] == 1
    assert out['config']['global_batch'] == 4 and out['config']['parallelism'] == 'dp2'
    assert out['config']['dist_backend'] == 'gloo'
    assert out['value'] > 0 and out['loss'] == out['loss']  # finite, not NaN
    assert abs(out['value'] - 4 * 2 / (out['ms_per_step'] * 2 / 1e3)) / out['value'] < 1e-2


@pytest.mark.gpu
def test_bench_two_ranks_inference_replicas(dev):
    """The inference legs at N > 1: every rank runs the predict path on its own batch; the
    line reports all ranks' images over the slowest rank's time."""
    env = dict(os.environ, ROD_DIST_BACKEND='gloo', MASTER_ADDR='127.0.0.1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_port()), os.path.join(ROOT, 'bench.py'),
           '--gpus', '2', '--steps', '1', '--warmup', '1', '--height', '160', '--width', '288', '--batch', '2',
           '--no-cpu-baseline', '--no-inference-1080', '--kernel-steps', '0']
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    inf = json.loads(lines[0])['inference']
    assert inf['n_gpus'] == 2 and inf['img_hw'] == [160, 288] and inf['batch'] == 32
    assert abs(inf['value'] - 2 * 32 * 1e3 / inf['ms_per_batch']) / inf['value'] < 1e-2
