"""Worker of tests/test_gpu_graph_dp.py::test_split_graph_dp_two_ranks: launched by
torch.distributed.run with 2 ranks (gloo, both on cuda:0 — RCCL refuses two ranks on one
device).  Each rank runs the data-parallel step eager and through Trainer.step_graphed in its
default 'split' mode (forward + backward replayed as a graph holding no collective, then the
bucketed gradient all-reduce and SGD issued eagerly) over its own alternating batches.
Checks: replayed parameters, moving statistics and losses bit-identical to the eager DP step
on every rank, and parameters identical across the ranks (the all-reduce ran).  ALL mode (a
hard-negative exchange inside the step) must fall back to eager.  Rank 0 writes the result."""
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
    ap.add_argument('--steps', type=int, default=4)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    import torch.distributed as dist
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    import config
    from rod.data import synthetic_batch
    from rod.ddp import GradReducer
    from rod.trainer import Trainer
    H, W, B = 160, 288, 2
    batches = [synthetic_batch(B, H, W, dev, seed=80 + 10 * rank + i) for i in range(2)]
    runs, modes = {}, {}
    for mode in ('eager', 'graphed'):
        tr = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=4, world_size=world,
                     reducer=GradReducer(world, bucket_mb=1.0))
        step = tr.step if mode == 'eager' else tr.step_graphed
        losses = []
        for i in range(a.steps):
            losses.append(step(*batches[i % 2])[0].detach().clone())
        torch.cuda.synchronize()
        modes[mode] = tr.graph_mode()
        runs[mode] = (tr.net.store.flat.detach().clone(), {k: v.clone() for k, v in tr.net.store.buffers.items()},
                      torch.stack([l.reshape(()) for l in losses]), tr)
    fe, be, le, te = runs['eager']
    fg, bg, lg, tg = runs['graphed']
    # parameters identical on both ranks: max and min over ranks of a checksum vector agree
    ck = fg.view(-1)[:: max(1, fg.numel() // 4096)].double()
    hi, lo = ck.clone(), ck.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    # ALL mode: the global hard-negative exchange is a collective inside the step -> eager
    ta = Trainer((H, W), B, dtype=torch.bfloat16, device=dev, seed=4, world_size=world,
                 reducer=GradReducer(world, bucket_mb=1.0), train_range=config.train_range.ALL)
    all_mode = ta.graph_mode()
    detail = {'rank': rank, 'mode': modes['graphed'], 'all_mode': all_mode,
              'captured': len(getattr(tg, '_graphs', {})) == 1,
              'params_equal': bool(torch.equal(fe, fg)), 'losses_equal': bool(torch.equal(le, lg)),
              'buffers_equal': all(torch.equal(v, bg[k]) for k, v in be.items()),
              'ranks_agree': bool(torch.equal(hi, lo)), 'losses': lg.float().tolist(),
              'global_step': [te.opt.global_step, tg.opt.global_step]}
    detail['ok'] = detail['mode'] == 'split' and all_mode == 'eager' and detail['captured'] and \
        detail['params_equal'] and detail['losses_equal'] and detail['buffers_equal'] and detail['ranks_agree'] and \
        te.opt.global_step == tg.opt.global_step == a.steps
    res = [None] * world
    dist.all_gather_object(res, detail)
    if rank == 0:
        torch.save({'ok': all(r['ok'] for r in res), 'ranks': res}, a.out)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
