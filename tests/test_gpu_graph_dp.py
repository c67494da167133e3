"""The data-parallel step as a HIP graph (Trainer.step_graphed with a GradReducer).

'full' (the N > 1 default over RCCL, what bench.py --gpus N replays: rod.ddp.make_reducer, the
library's communicator): captured on a 1-rank RCCL group on one MI355X — the bucketed
all-reduces launched from inside backward on their side stream, the SyncBatchNorm all-gathers
and (ALL mode) the hard-negative exchange go into the graph — and replayed over alternating
input batches: parameters, moving statistics and losses bit-identical to the eager
data-parallel step (ref net_tools.py:642-651: clip after the reduction).

'split' (torch.distributed reducers — the gloo rehearsal): two ranks over gloo on one GPU."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, 'tests', 'graph_dp_worker.py')
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('train_range', ['REFINE', 'ALL'])
def test_dp_step_graph_capture_bit_identical(train_range, tmp_path, dev):
    out = str(tmp_path / 'r.pt')
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_port()), RANK='0', WORLD_SIZE='1',
               LOCAL_RANK='0')
    r = subprocess.run([sys.executable, WORKER, '--out', out, '--train_range', train_range], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = torch.load(out, weights_only=True)
    print(train_range, d)
    assert d['ok'], d


SPLIT_WORKER = os.path.join(ROOT, 'tests', 'split_dp_worker.py')


def test_split_graph_dp_two_ranks(tmp_path, dev):
    """The torch.distributed graph mode ('split': forward + backward replayed, the bucketed
    all-reduce + SGD issued after the replay) with TWO ranks (gloo on one GPU): bit-identical
    to the eager DP step on each rank, ranks hold identical parameters; ALL mode stays eager."""
    out = str(tmp_path / 's.pt')
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_port()), SPLIT_WORKER, '--out', out]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = torch.load(out, weights_only=True)
    print(d)
    assert d['ok'], d


NATIVE_WORKER = os.path.join(ROOT, 'tests', 'native_comm_worker.py')


def test_native_comm_one_rank(tmp_path, dev):
    """rod_rccl_init / rod_allreduce_bucket (the C-ABI reduce point) on a 1-rank communicator:
    identity sums, graph capture and replay, and a training step reduced through it."""
    out = str(tmp_path / 'n.pt')
    r = subprocess.run([sys.executable, NATIVE_WORKER, '--out', out], cwd=ROOT, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = torch.load(out, weights_only=True)
    print(d)
    assert d['ok'], d


ORDER_WORKER = os.path.join(ROOT, 'tests', 'dp_order_worker.py')


def test_native_collective_order_two_ranks(tmp_path, dev):
    """Two ranks on one GPU (gloo rendezvous), the native reducer recording its collectives:
    REFINE, ALL (fix_refine=False: the hard-negative exchange) and ALL + SyncBatchNorm issue the
    same (entry, count, dtype) sequence on both ranks, eager and
    under capture, every call on the one communication stream (rod.ddp.NativeComm)."""
    out = str(tmp_path / 'o.pt')
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_port()), ORDER_WORKER, '--out', out]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    d = torch.load(out, weights_only=True)
    print({k: ({kk: vv for kk, vv in v.items() if kk != 'entries'} if isinstance(v, dict) else v)
           for k, v in d.items()})
    assert d['ok'], d
