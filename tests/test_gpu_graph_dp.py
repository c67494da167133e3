"""The data-parallel step as a HIP graph (Trainer.step_graphed with a GradReducer): bench.py
--gpus N replays it on every rank.  Captured on a 1-rank RCCL group on one MI355X — the
bucketed all-reduces launched from inside backward, the SyncBatchNorm all-gathers and (ALL)
the hard-negative count / histogram all-reduces all go into the graph — and replayed over
alternating input batches: parameters, moving statistics and losses bit-identical to the
eager data-parallel step (ref net_tools.py:642-651: clip after the reduction)."""
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
