"""Time the oracle step evaluations used by the full-size parity tests (analysis only):
fp64 on the CPU, bf16 / fp32 with PyTorch ops on the GPU, at 720x1280 b8 (REFINE step)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import test_gpu_fullsize as T
    from rod.data import SEED, synthetic_batch
    from rod.trainer import Trainer
    dev = torch.device('cuda', 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    tr = Trainer((720, 1280), B, dtype=torch.bfloat16, device=dev)
    img, corner, labels, n = synthetic_batch(B, 720, 1280, dev, seed=SEED)
    snap = ({k: v.detach().cpu().clone() for k, v in tr.net.store.params.items()},
            {k: v.detach().cpu().clone() for k, v in tr.net.store.buffers.items()})
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    for name, dt, d in (('gpu fp32', torch.float32, dev), ('gpu bf16', torch.bfloat16, dev),
                        ('cpu fp64', torch.float64, 'cpu')):
        t0 = time.perf_counter()
        P, mov, ref, loss = T._oracle_refine_step(tr, snap, img, corner, labels, n, B, dt, device=d)
        torch.cuda.synchronize()
        print(f'{name}: {time.perf_counter() - t0:.1f} s  loss {float(loss):.6f}', flush=True)
        del P, mov, ref, loss
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
