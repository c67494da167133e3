"""Worker of tests/test_gpu_graph_dp.py: the data-parallel training step (bucketed RCCL
gradient all-reduce launched from inside backward, SyncBatchNorm all-gathers, the global
hard-negative exchange in ALL mode) captured as a HIP graph and replayed (Trainer.step_graphed),
against the same step run eager, on a 1-rank RCCL process group ('nccl' backend on cuda:0).
Writes {'ok': bool, 'detail': ...} to <out>."""
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
    # the step is captured with its RCCL collectives (Trainer.step_graphed): no event of an eager
    # collective may be recycled into the capture while the watchdog still polls it
    os.environ.setdefault('TORCH_NCCL_CUDA_EVENT_CACHE', '0')
    dist.init_process_group('nccl', device_id=dev)
    import config
    from rod.data import synthetic_batch
    from rod.ddp import GradReducer
    from rod.trainer import Trainer
    H, W, B = 160, 288, 2
    tr_range = getattr(config.train_range, a.train_range)
    batches = [synthetic_batch(B, H, W, dev, seed=60 + i) for i in range(2)]
    runs = {}
    for mode in ('eager', 'graphed'):
        tr = Trainer((H, W), B, dtype=torch.bfloat16, train_range=tr_range, device=dev, seed=4, world_size=1,
                     reducer=GradReducer(1, bucket_mb=1.0), sync_bn=True, graph_dp=True)
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
    # ALL mode: the hard-negative exchange keeps the step eager even with graph_dp (Trainer.graph_mode)
    detail['mode'] = tg.graph_mode()
    want = 'full' if a.train_range == 'REFINE' else 'eager'
    detail['ok'] = detail['mode'] == want and detail['captured'] == (want == 'full') and detail['params_equal'] and \
        detail['losses_equal'] and detail['buffers_equal'] and detail['buckets'] > 3 and \
        te.opt.global_step == tg.opt.global_step == a.steps
    torch.save(detail, a.out)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
