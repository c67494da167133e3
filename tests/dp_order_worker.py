"""Worker of tests/test_gpu_graph_dp.py::test_native_collective_order_two_ranks: the N > 1
default data-parallel step (the library's communicator, NativeComm) on TWO ranks sharing one
MI355X.  RCCL refuses two ranks on one device, so the native collectives are recorded instead of
called (GradReducer(record=True)): the real model's backward fires the bucket hooks, the ALL-mode
hard-negative exchange and the SyncBatchNorm gathers exactly as on 8 GPUs, eager and captured
into the step graph.  Each rank writes its (entry, count, dtype, stream role) sequence; rank 0
compares them (gloo carries the comparison) and writes {'ok': bool, ...} to <out>.
Launched with torch.distributed.run --nproc-per-node 2."""
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
    ap.add_argument('--steps', type=int, default=3)
    a = ap.parse_args()
    import torch.distributed as dist
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    import config
    from rod import ddp
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    H, W, B = 160, 288, 2
    cases = {'REFINE': dict(train_range=config.train_range.REFINE),
             'ALL': dict(train_range=config.train_range.ALL, fix_refine=False),
             'ALL_sync_bn': dict(train_range=config.train_range.ALL, fix_refine=False, sync_bn=True)}
    res = {}
    for name, kw in cases.items():
        batches = [synthetic_batch(B, H, W, dev, seed=70 + 10 * rank + i) for i in range(2)]
        red = ddp.GradReducer(world, bucket_mb=1.0, native=True, record=True)
        tr = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=4, world_size=world, reducer=red, **kw)
        seqs = []
        for i in range(a.steps):
            ddp.TRACE = []
            tr.step_graphed(*batches[i % 2])   # step 0 eager, step 1 captures, step 2 replays
            torch.cuda.synchronize()
            seqs.append(list(ddp.TRACE))
        ddp.TRACE = None
        res[name] = {'mode': tr.graph_mode(), 'eager': seqs[0], 'captured': seqs[1], 'replay': seqs[2]}
    got = [None] * world
    dist.all_gather_object(got, res)
    if rank == 0:
        det = {'ok': True}
        for name in cases:
            r0, r1 = got[0][name], got[1][name]
            e, c = r0['eager'], r0['captured']
            d = {'mode': r0['mode'], 'n_eager': len(e), 'n_captured': len(c), 'n_replay': len(r0['replay']),
                 'same_across_ranks': r0['eager'] == r1['eager'] and r0['captured'] == r1['captured'],
                 'eager_equals_captured': e == c,
                 'one_stream': {x[3] for x in e + c} == {'comm'},
                 'entries': sorted(set(x[0] for x in e)),
                 'buckets': sum(1 for x in e if x[0] == 'rod_allreduce_bucket' and x[2] == 0)}
            d['ok'] = d['mode'] == 'full' and d['same_across_ranks'] and d['eager_equals_captured'] and \
                d['one_stream'] and d['n_replay'] == 0 and d['buckets'] > 3
            if name != 'REFINE':
                d['ok'] = d['ok'] and any(x[0] == 'rod_allreduce_bucket' and x[2] == 2 for x in e)
            if name == 'ALL_sync_bn':
                d['ok'] = d['ok'] and 'rod_allgather' in d['entries']
            det[name] = d
            det['ok'] = det['ok'] and d['ok']
        torch.save(det, a.out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
