"""Worker of tests/test_gpu_graph_dp.py: the data-parallel training step as the N > 1 default
runs it (rod.ddp.make_reducer over an RCCL process group: the library's communicator — bucketed
gradient all-reduces launched from inside backward on a side stream, SyncBatchNorm all-gathers
via rod_allgather, the global hard-negative exchange in ALL mode via int32 rod_allreduce_bucket)
captured as ONE HIP graph and replayed (Trainer.step_graphed, 'full'), against the same step run
eager, on a 1-rank group ('nccl' backend on cuda:0).  Writes {'ok': bool, 'detail': ...} to <out>."""
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
    ap.add_argument('--train_range', default='REFINE')
    ap.add_argument('--steps', type=int, default=4)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    import torch.distributed as dist
    dist.init_process_group('nccl', device_id=dev)
    import config
    from rod.data import synthetic_batch
    from rod import _abi
    from rod.ddp import make_reducer
    from rod.trainer import Trainer
    H, W, B = 160, 288, 2
    tr_range = getattr(config.train_range, a.train_range)
    batches = [synthetic_batch(B, H, W, dev, seed=60 + i) for i in range(2)]
    runs = {}
    for mode in ('eager', 'graphed'):
        tr = Trainer((H, W), B, dtype=torch.bfloat16, train_range=tr_range, device=dev, seed=4, world_size=1,
                     reducer=make_reducer(1, 0, bucket_mb=1.0), sync_bn=True)
        step = tr.step if mode == 'eager' else tr.step_graphed
        losses = []
        for i in range(a.steps):
            losses.append(step(*batches[i % 2])[0].detach().clone())   # new inputs every replay
        torch.cuda.synchronize()
        runs[mode] = (tr.net.store.flat.detach().clone(), {k: v.clone() for k, v in tr.net.store.buffers.items()},
                      torch.stack([l.reshape(()) for l in losses]), tr)
    fe, be, le, te = runs['eager']
    fg, bg, lg, tg = runs['graphed']
    detail = {'captured': getattr(tg, '_graph', None) is not None, 'buckets': len(tg.reducer.buckets),
              'params_equal': bool(torch.equal(fe, fg)), 'losses_equal': bool(torch.equal(le, lg)),
              'buffers_equal': all(torch.equal(v, bg[k]) for k, v in be.items()),
              'losses': le.float().tolist(), 'global_step': [te.opt.global_step, tg.opt.global_step]}
    # every collective through the library's communicator: REFINE and ALL (its hard-negative
    # exchange inside the step) are both captured whole
    detail['mode'] = tg.graph_mode()
    detail['native'] = bool(tg.reducer.native)
    detail['ok'] = detail['mode'] == 'full' and detail['native'] and detail['captured'] and detail['params_equal'] and \
        detail['losses_equal'] and detail['buffers_equal'] and detail['buckets'] > 3 and \
        te.opt.global_step == tg.opt.global_step == a.steps
    torch.save(detail, a.out)
    _abi.call('rod_rccl_destroy')
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
