"""Worker of tests/test_gpu_graph_dp.py::test_native_comm_one_rank: the C-ABI reduce point
(rod_rccl_unique_id / rod_rccl_init / rod_allreduce_bucket, include/rod.h ABI 16) on a 1-rank
communicator — in-place bucket sums (fp32 and bf16, identity at one rank), the same call captured
into a HIP graph and replayed, and a REFINE training step whose GradReducer sums through the
library (native=True: buckets on a side stream, the whole step captured, 'full') bit-identical
to the step without a reducer; ABI 19: int32 sums and rod_allgather (identity at one rank).  Writes
{'ok': bool, ...} to <out>."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    from rod import _abi, ops
    from rod.data import synthetic_batch
    from rod.ddp import GradReducer, native_comm_init
    from rod.trainer import Trainer
    native_comm_init(0, 1)
    det = {}
    x = torch.randn(1 << 20, device=dev)
    ref = x.clone()
    _abi.call('rod_allreduce_bucket', x, x.numel(), 0, ops.stream())
    xb = torch.randn(4099, device=dev).to(torch.bfloat16)
    refb = xb.clone()
    _abi.call('rod_allreduce_bucket', xb, xb.numel(), 1, ops.stream())
    torch.cuda.synchronize()
    xi = torch.randint(-1000, 1000, (1031,), device=dev, dtype=torch.int32)
    refi = xi.clone()
    _abi.call('rod_allreduce_bucket', xi, xi.numel(), 2, ops.stream())
    src = torch.randn(3, 517, device=dev)
    dst = torch.empty_like(src)
    _abi.call('rod_allgather', src, dst, src.numel(), 0, ops.stream())
    torch.cuda.synchronize()
    det['i32_identity'] = bool(torch.equal(xi, refi))
    det['allgather_identity'] = bool(torch.equal(src, dst))
    det['world'] = int(_abi.lib().rod_rccl_world())
    det['f32_identity'] = bool(torch.equal(x, ref))
    det['bf16_identity'] = bool(torch.equal(xb, refb))
    g = torch.cuda.CUDAGraph()
    y = torch.zeros(4096, device=dev)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        y.add_(1.0)
        _abi.call('rod_allreduce_bucket', y, y.numel(), 0, ops.stream())
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    det['graph_replay'] = bool((y == 3.0).all())
    H, W, B = 160, 288, 2
    batches = [synthetic_batch(B, H, W, dev, seed=90 + i) for i in range(2)]
    flats = []
    for red in (None, GradReducer(1, bucket_mb=1.0, native=True)):
        tr = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=4, world_size=1, reducer=red)
        for i in range(4):
            tr.step_graphed(*batches[i % 2])
        torch.cuda.synchronize()
        flats.append(tr.net.store.flat.detach().clone())
        det['mode_' + ('none' if red is None else 'native')] = tr.graph_mode()
    det['step_equal'] = bool(torch.equal(flats[0], flats[1]))
    _abi.call('rod_rccl_destroy')
    det['ok'] = det['f32_identity'] and det['bf16_identity'] and det['i32_identity'] and det['allgather_identity'] \
        and det['world'] == 1 and det['graph_replay'] and det['step_equal'] and det['mode_native'] == 'full'
    torch.save(det, a.out)


if __name__ == '__main__':
    main()
