"""One training step of rod.trainer.Trainer for the data-parallel equivalence test
(tests/test_gpu_dp_equiv.py).  Launched by torch.distributed.run (WORLD_SIZE ranks sharing
cuda:0 over gloo) or directly (one process, the whole batch).  The global batch is one fixed
synthetic batch; rank r takes images [r*B/world, (r+1)*B/world).  Writes the reduced flat
gradient, the parameters after SGD, the moving statistics and the loss terms (summed over
ranks) to <out>."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--batch', type=int, default=4, help='global batch')
    ap.add_argument('--hw', type=int, nargs=2, default=(320, 576))
    ap.add_argument('--train_range', default='REFINE')
    ap.add_argument('--sync_bn', action='store_true')
    ap.add_argument('--perturb', type=float, default=0.0,
                    help='relative noise on the normalised input (sensitivity probe of the step itself)')
    ap.add_argument('--perturb_seed', type=int, default=0)
    ap.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'])
    a = ap.parse_args()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    reducer = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('gloo')
        from rod.ddp import GradReducer
        reducer = GradReducer(world)
    import config
    from rod import graph
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    tr_range = getattr(config.train_range, a.train_range)
    bl = a.batch // world
    dtype = torch.bfloat16 if a.dtype == 'bf16' else torch.float32
    tr = Trainer(tuple(a.hw), bl, dtype=dtype, train_range=tr_range, learning_rate=1e-2, device=dev,
                 seed=7, world_size=world, reducer=reducer, sync_bn=a.sync_bn)
    img, corner, labels, n = synthetic_batch(a.batch, a.hw[0], a.hw[1], dev, seed=8)
    # every run feeds the same normalised fp32 input ((2/255)x - 1, train.py:126, on the host)
    # so that a perturbed run differs from the others by the noise alone
    x = torch.from_numpy(np.float32(2.0 / 255.0) * img.cpu().numpy().astype(np.float32) - np.float32(1.0))
    if a.perturb:
        g = torch.Generator().manual_seed(a.perturb_seed)
        x = x * (1 + a.perturb * torch.randn(x.shape, generator=g))
    img = x.to(dev)
    sl = slice(rank * bl, (rank + 1) * bl)
    flat0 = tr.net.store.flat.detach().clone()
    losses = tr.losses(img[sl], corner[sl], labels[sl], n[sl])
    graph.backward(losses[0])
    if reducer is not None:
        reducer(tr.net.store.flat_grad)
    grad = tr.net.store.flat_grad.detach().clone()
    tr.opt.step()
    lv = torch.stack([l.detach().reshape(()).double() for l in losses])
    # integer decisions of the step (ALL): ODM positives (sum over ranks) and the global
    # hard-negative k / selected count (rod_softmax_ce_hnm stats [5], [6]; identical on all ranks)
    dec = torch.zeros(3, dtype=torch.float64, device=dev)
    if tr_range is config.train_range.ALL:
        import utils.net_tools as nt
        dec[0] = tr.last_targets[1].flat[1].sum().double()
        st = nt.det_clf_loss.last_stats.double()
        dec[1], dec[2] = st[5], st[6]
    if world > 1:
        torch.distributed.all_reduce(lv)
        dec[1] /= world                   # k is global already (identical on every rank)
        torch.distributed.all_reduce(dec)
    torch.cuda.synchronize()
    if rank == 0:
        store = tr.net.store
        torch.save({'grad': grad.cpu(), 'flat': store.flat.detach().cpu(), 'flat0': flat0.cpu(), 'offsets': dict(store.offsets),
                    'buffers': {k: v.detach().cpu() for k, v in store.buffers.items()},
                    'trainable': [k for k, p in store.params.items() if p.requires_grad],
                    'losses': lv.cpu(), 'decisions': dec.cpu()}, a.out)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
