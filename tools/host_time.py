"""Host dispatch cost of an eager training step (the N > 1 path runs eager): wall time to
issue K steps without synchronising (host side) vs the time until the GPU finishes them.
If the issue time approaches the total, the eager step is host-bound.
usage: python tools/host_time.py [--steps 10] [--train_range REFINE|ALL]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--train_range', default='REFINE')
    a = ap.parse_args()
    import config
    from rod.data import SEED, synthetic_batch
    from rod.trainer import Trainer
    dev = torch.device('cuda')
    tr = Trainer((720, 1280), 8, dtype=torch.bfloat16, device=dev,
                 train_range=getattr(config.train_range, a.train_range))
    batch = synthetic_batch(8, 720, 1280, dev, seed=SEED)
    for _ in range(3):
        tr.step(*batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.step(*batch)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print({'host_issue_ms_per_step': round((t1 - t0) / a.steps * 1e3, 3),
           'total_ms_per_step': round((t2 - t0) / a.steps * 1e3, 3)}, flush=True)


if __name__ == '__main__':
    main()
